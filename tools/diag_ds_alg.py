"""Diagnostic: per-tensor gradient error of two ResNet bottlenecks (downsample + identity, as
tests/test_conv1x1_ours_gpu.py::test_bottleneck_chain_takes_bn_backward_stats) against an fp32 oracle of the same
weights / input, for the shortcut on the ALG backward (PDT_DS_ALG), on its old path, and with the BN-backward
hand-off off (no ALG at all).

    PDT_BWD_ALG_MIN_M=0 python tools/diag_ds_alg.py
"""
import copy
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from pytorch_distributed_training_example_amd.config import SW  # noqa: E402
from pytorch_distributed_training_example_amd.models import resnet as R  # noqa: E402
from pytorch_distributed_training_example_amd.models.precision import to_bf16_mixed  # noqa: E402


def run(net, x0, env, fp32=False):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    SW.reload()
    try:
        net.zero_grad(set_to_none=True)
        x = x0.clone().requires_grad_(True)
        y = net(x)
        y.backward((torch.ones_like(y) * 0.01 + y.detach() * 0.1))
        return [("x", x.grad.double())] + [(n, p.grad.double().clone()) for n, p in net.named_parameters()]
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        SW.reload()


def main():
    torch.manual_seed(0)
    ds = R._Downsample(R.conv1x1(64, 256, 1), R._bn(256))
    base = torch.nn.Sequential(R.Bottleneck(64, 64, 1, ds), R.Bottleneck(256, 64, 1, None)).cuda()
    net = to_bf16_mixed(copy.deepcopy(base).to(memory_format=torch.channels_last))
    ref = copy.deepcopy(base).to(memory_format=torch.channels_last)
    x0 = torch.randn(8, 64, 28, 28, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    g32 = run(ref, x0.float(), {"PDT_DISABLE_NATIVE": "1"})
    cfgs = {"ds_alg": {"PDT_CONV1X1": "ours", "PDT_DS_ALG": "512"},
            "ds_old": {"PDT_CONV1X1": "ours", "PDT_DS_ALG": "0"},
            "no_handoff": {"PDT_CONV1X1": "ours", "PDT_BN_BWD_STATS": "0"}}
    res = {k: run(net, x0, v) for k, v in cfgs.items()}
    print(f"{'tensor':32s} " + " ".join(f"{k:>11s}" for k in cfgs))
    for i, (n, g) in enumerate(g32):
        errs = [float((res[k][i][1] - g).norm() / g.norm().clamp_min(1e-30)) for k in cfgs]
        print(f"{n:32s} " + " ".join(f"{e:11.3e}" for e in errs))


if __name__ == "__main__":
    main()
