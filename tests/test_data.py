"""Partitioner / sampler / dataset math (CPU)."""
import importlib.util
import math
import os

import numpy as np
import pytest
import torch
from hypothesis import given, settings
from hypothesis import strategies as st

from pytorch_distributed_training_example_amd.data import RandomTensorDataset, SyntheticMNIST, mnist
from pytorch_distributed_training_example_amd.data.datasets import MNIST, _read_idx
from pytorch_distributed_training_example_amd.parallel import DistributedSampler, SplitDataset, rank_partition

REF = "/root/reference/splitdataset.py"


class _Range(torch.utils.data.Dataset):
    def __init__(self, n):
        self.n = n

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        return i


@pytest.mark.parametrize("world", list(range(1, 65)))
@pytest.mark.parametrize("n", [60000, 10000, 7, 1000003])
def test_split_covers_disjoint_in_bounds(world, n):
    ds = _Range(n)
    seen = []
    for r in range(world):
        s = rank_partition(ds, r, world)
        assert abs(len(s) - n / world) <= 1.0
        if len(s):
            seen.append((s[0], s[len(s) - 1], len(s)))
        with pytest.raises(IndexError):
            s[len(s)]
    covered = sum(c for _, _, c in seen)
    assert covered == n  # every sample exactly once (reference drops / overruns for 6,7,9,11,14)
    spans = sorted((a, b) for a, b, _ in seen)
    for (a0, b0), (a1, b1) in zip(spans, spans[1:]):
        assert b0 < a1


@pytest.mark.skipif(not os.path.exists(REF), reason="reference not mounted")
@pytest.mark.parametrize("world", [2, 3, 4, 5, 8])
def test_split_matches_reference_layout(world):
    """Where the reference works, shard offsets/lengths are identical (lexicographic names)."""
    spec = importlib.util.spec_from_file_location("ref_splitdataset", REF)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    ds = _Range(60000)
    parts = {str(i): 1 / world for i in range(world)}
    ref = mod.SplitDataset(ds, parts)
    ours = SplitDataset(ds, parts)
    for r in range(world):
        ref.select(str(r))
        ours.select(str(r))
        assert len(ref) == len(ours)
        assert ref[0] == ours[0] and ref[len(ref) - 1] == ours[len(ours) - 1]


def test_split_integer_sizes_and_errors():
    ds = _Range(100)
    s = SplitDataset(ds, {"train": 80, "val": 20}, initial_partition="val")
    assert len(s) == 20 and s[0] == 80
    with pytest.raises(ValueError):
        SplitDataset(ds, {"a": 1.5, "b": 2})
    with pytest.raises(ValueError):
        SplitDataset(ds, {"a": 90, "b": 20})
    with pytest.raises(ValueError):
        len(SplitDataset(ds, {"a": 0.5, "b": 0.5}))
    one = SplitDataset(ds, {"0": 1.0}, initial_partition="0")  # world_size 1 works
    assert len(one) == 100


@settings(max_examples=200, deadline=None)
@given(n=st.integers(1, 5000), world=st.integers(1, 64), shuffle=st.booleans(), drop_last=st.booleans(),
       seed=st.integers(0, 1000), epoch=st.integers(0, 5))
def test_sampler_matches_torch(n, world, shuffle, drop_last, seed, epoch):
    if drop_last and n < world:
        return
    ds = _Range(n)
    for r in range(world):
        ours = DistributedSampler(ds, world, r, shuffle=shuffle, seed=seed, drop_last=drop_last)
        ref = torch.utils.data.DistributedSampler(ds, world, r, shuffle=shuffle, seed=seed, drop_last=drop_last)
        ours.set_epoch(epoch)
        ref.set_epoch(epoch)
        assert list(ours) == list(ref)
        assert len(ours) == len(ref)


def test_sampler_resume_mid_epoch():
    ds = _Range(100)
    s = DistributedSampler(ds, 4, 1, seed=3)
    s.set_epoch(2)
    full = list(s)
    s.set_start_index(10)
    assert list(s) == full[10:]
    sd = s.state_dict()
    s2 = DistributedSampler(ds, 4, 1)
    s2.load_state_dict(sd)
    assert list(s2) == full[10:]


def test_synthetic_mnist_shapes_and_determinism():
    a = SyntheticMNIST(train=True, n=200, seed=0)
    b = SyntheticMNIST(train=True, n=200, seed=0)
    x, y = a[5]
    assert x.shape == (1, 28, 28) and x.dtype == torch.float32 and 0 <= y < 10
    assert torch.equal(a.images, b.images) and torch.equal(a.targets, b.targets)
    xs, ys = a.tensors()
    assert xs.shape == (200, 1, 28, 28)
    torch.testing.assert_close(xs[5], x)


def _write_idx(path, arr):
    arr = np.asarray(arr, dtype=np.uint8)
    with open(path, "wb") as f:
        f.write(bytes([0, 0, 8, arr.ndim]))
        for d in arr.shape:
            f.write(int(d).to_bytes(4, "big"))
        f.write(arr.tobytes())


def test_mnist_idx_reader(tmp_path):
    raw = tmp_path / "MNIST" / "raw"
    raw.mkdir(parents=True)
    imgs = np.random.default_rng(0).integers(0, 256, (12, 28, 28))
    labels = np.arange(12) % 10
    _write_idx(raw / "t10k-images-idx3-ubyte", imgs)
    _write_idx(raw / "t10k-labels-idx1-ubyte", labels)
    assert _read_idx(str(raw / "t10k-images-idx3-ubyte")).shape == (12, 28, 28)
    ds = MNIST(str(tmp_path), train=False)
    x, y = ds[3]
    assert y == 3
    ref = (torch.tensor(imgs[3], dtype=torch.float32) / 255 - 0.1307) / 0.3081  # reference transform
    torch.testing.assert_close(x[0], ref)
    assert mnist(str(tmp_path), train=False).synthetic is False
    assert mnist(str(tmp_path / "none"), train=False, n=10).synthetic is True


def test_random_tensor_dataset():
    d = RandomTensorDataset(64, 32, 8)
    x, y = d[0]
    assert x.shape == (32,) and y.shape == (8,)
