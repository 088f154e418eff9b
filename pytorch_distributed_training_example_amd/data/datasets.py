"""Datasets: MNIST (real IDX files when present, else deterministic synthetic), synthetic
ImageNet-shaped images, synthetic token streams, random tensors.

Reference: torchvision ``datasets.MNIST('./data', download=True)`` with
``ToTensor() + Normalize((0.1307,), (0.3081,))`` (/root/reference/train.py:85-91). There is no
network and no torchvision here, so:
  * ``MNIST`` reads the standard IDX files (``{root}/MNIST/raw/*-ubyte[.gz]``, torchvision's
    layout) if they exist and applies the same normalisation;
  * otherwise ``SyntheticMNIST`` produces a deterministic 60k/10k set of 28×28 uint8 digits-like
    images (per-class prototype strokes + noise + jitter), so a model can actually learn and
    accuracy is meaningful; same shapes, dtype and normalisation as the real thing.
"""
from __future__ import annotations

import gzip
import os
import struct
from typing import Optional, Tuple

import numpy as np
import torch
from torch.utils.data import Dataset

MNIST_MEAN, MNIST_STD = 0.1307, 0.3081


def _read_idx(path: str) -> np.ndarray:
    op = gzip.open if path.endswith(".gz") else open
    with op(path, "rb") as f:
        data = f.read()
    magic = struct.unpack(">I", data[:4])[0]
    nd = magic & 0xFF
    dims = struct.unpack(">" + "I" * nd, data[4:4 + 4 * nd])
    return np.frombuffer(data, dtype=np.uint8, offset=4 + 4 * nd).reshape(dims)


def _find(root: str, stem: str) -> Optional[str]:
    for d in (os.path.join(root, "MNIST", "raw"), root):
        for ext in ("", ".gz"):
            p = os.path.join(d, stem + ext)
            if os.path.exists(p):
                return p
    return None


class _NormalizedImages(Dataset):
    def __init__(self, images: np.ndarray, labels: np.ndarray):
        self.images = torch.from_numpy(np.array(images, dtype=np.uint8, copy=True))  # uint8 [N, 28, 28]
        self.targets = torch.from_numpy(labels.astype(np.int64))

    def __len__(self) -> int:
        return self.images.shape[0]

    def __getitem__(self, idx: int) -> Tuple[torch.Tensor, int]:
        img = self.images[idx].float().div_(255.0).sub_(MNIST_MEAN).div_(MNIST_STD).unsqueeze(0)
        return img, int(self.targets[idx])

    def tensors(self) -> Tuple[torch.Tensor, torch.Tensor]:
        """Whole set as (normalized float [N,1,28,28], int64 [N]) for on-device loading."""
        x = self.images.float().div_(255.0).sub_(MNIST_MEAN).div_(MNIST_STD).unsqueeze(1)
        return x, self.targets


def synthetic_mnist_arrays(n: int, seed: int) -> Tuple[np.ndarray, np.ndarray]:
    rng = np.random.default_rng(seed)
    proto_rng = np.random.default_rng(12345)  # class prototypes shared by train/test
    protos = np.zeros((10, 28, 28), np.float32)
    yy, xx = np.mgrid[0:28, 0:28]
    for c in range(10):
        for _ in range(3):  # three random strokes per class
            cx, cy = proto_rng.uniform(8, 20, 2)
            ang = proto_rng.uniform(0, np.pi)
            length = proto_rng.uniform(6, 12)
            t = (xx - cx) * np.cos(ang) + (yy - cy) * np.sin(ang)
            d = np.abs(-(xx - cx) * np.sin(ang) + (yy - cy) * np.cos(ang))
            protos[c] += np.exp(-d ** 2 / 2.0) * (np.abs(t) < length / 2)
        protos[c] /= protos[c].max()
    labels = rng.integers(0, 10, n)
    shifts = rng.integers(-2, 3, (n, 2))
    imgs = np.empty((n, 28, 28), np.uint8)
    for i in range(n):
        p = np.roll(protos[labels[i]], tuple(shifts[i]), axis=(0, 1))
        v = p * rng.uniform(0.7, 1.0) + rng.normal(0, 0.08, (28, 28))
        imgs[i] = np.clip(v * 255, 0, 255).astype(np.uint8)
    return imgs, labels


class SyntheticMNIST(_NormalizedImages):
    def __init__(self, train: bool = True, n: Optional[int] = None, seed: int = 0):
        n = n if n is not None else (60000 if train else 10000)
        imgs, labels = synthetic_mnist_arrays(n, seed + (0 if train else 1_000_003))
        super().__init__(imgs, labels)
        self.synthetic = True


class MNIST(_NormalizedImages):
    """Real MNIST from local IDX files (no download: there is no network)."""

    FILES = {True: ("train-images-idx3-ubyte", "train-labels-idx1-ubyte"),
             False: ("t10k-images-idx3-ubyte", "t10k-labels-idx1-ubyte")}

    def __init__(self, root: str = "./data", train: bool = True):
        fi, fl = (_find(root, s) for s in self.FILES[train])
        if fi is None or fl is None:
            raise FileNotFoundError(f"MNIST IDX files not found under {root}")
        super().__init__(_read_idx(fi), _read_idx(fl))
        self.synthetic = False


def mnist(root: str = "./data", train: bool = True, synthetic: Optional[bool] = None, n: Optional[int] = None,
          seed: int = 0) -> _NormalizedImages:
    if synthetic is None:
        try:
            return MNIST(root, train)
        except FileNotFoundError:
            synthetic = True
    if synthetic:
        return SyntheticMNIST(train, n=n, seed=seed)
    return MNIST(root, train)


class RandomTensorDataset(Dataset):
    """Random (x, y) pairs for the 2-layer MLP plumbing config (BASELINE.json config 1)."""

    def __init__(self, n: int = 1024, in_features: int = 32, out_features: int = 8, seed: int = 0,
                 classification: bool = False):
        g = torch.Generator().manual_seed(seed)
        self.x = torch.randn(n, in_features, generator=g)
        self.y = torch.randint(0, out_features, (n,), generator=g) if classification \
            else torch.randn(n, out_features, generator=g)

    def __len__(self) -> int:
        return self.x.shape[0]

    def __getitem__(self, i):
        return self.x[i], self.y[i]


class SyntheticImages(Dataset):
    """ImageNet-shaped random images with random labels (deterministic per index)."""

    def __init__(self, n: int = 1281167, image_size: int = 224, num_classes: int = 1000, seed: int = 0):
        self.n, self.s, self.k, self.seed = n, image_size, num_classes, seed

    def __len__(self) -> int:
        return self.n

    def __getitem__(self, i):
        g = torch.Generator().manual_seed(self.seed * 1_000_003 + i)
        return torch.randn(3, self.s, self.s, generator=g), int(torch.randint(0, self.k, (1,), generator=g))


class SyntheticTokens(Dataset):
    """Random token sequences of length ``seq_len + 1`` (inputs, shifted targets)."""

    def __init__(self, n: int = 100000, seq_len: int = 1024, vocab: int = 50257, seed: int = 0):
        self.n, self.t, self.v, self.seed = n, seq_len, vocab, seed

    def __len__(self) -> int:
        return self.n

    def __getitem__(self, i):
        g = torch.Generator().manual_seed(self.seed * 1_000_003 + i)
        tok = torch.randint(0, self.v, (self.t + 1,), generator=g)
        return tok[:-1], tok[1:]
