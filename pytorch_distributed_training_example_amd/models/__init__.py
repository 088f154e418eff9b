"""Model zoo: LeNet (reference model), MLP (plumbing), ResNet, ViT, GPT-2."""
from __future__ import annotations

from typing import Callable, Dict

from torch import nn

from .lenet import MLP, LeNet
from .resnet import ResNet, resnet18, resnet50, resnet101

_REGISTRY: Dict[str, Callable[..., nn.Module]] = {
    "lenet": LeNet,
    "mlp": MLP,
    "resnet18": resnet18,
    "resnet50": resnet50,
    "resnet101": resnet101,
}


def register(name: str, fn: Callable[..., nn.Module]) -> None:
    _REGISTRY[name] = fn


def get_model(name: str, **kw) -> nn.Module:
    _lazy()
    if name not in _REGISTRY:
        raise KeyError(f"unknown model {name}; have {sorted(_REGISTRY)}")
    return _REGISTRY[name](**kw)


def _lazy():
    try:
        from . import vit, gpt2  # noqa: F401  (register themselves)
    except ImportError:
        pass


__all__ = ["MLP", "LeNet", "ResNet", "resnet18", "resnet50", "resnet101", "get_model", "register"]
