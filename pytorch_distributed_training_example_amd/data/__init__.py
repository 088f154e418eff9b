"""Data: datasets (MNIST real/synthetic, synthetic images/tokens) and device-side loaders."""
from .datasets import (MNIST, MNIST_MEAN, MNIST_STD, RandomTensorDataset, SyntheticImages, SyntheticMNIST,
                       SyntheticTokens, mnist)
from .loader import PrefetchLoader, ResidentLoader, SyntheticBatches, reference_loader

__all__ = ["MNIST", "MNIST_MEAN", "MNIST_STD", "RandomTensorDataset", "SyntheticImages", "SyntheticMNIST",
           "SyntheticTokens", "mnist", "PrefetchLoader", "ResidentLoader", "SyntheticBatches", "reference_loader"]
