"""Sweep BN fwd/bwd over every (N,C,H,W,relu,res) that ResNet-50 produces; report errors."""
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
from pytorch_distributed_training_example_amd.models import get_model  # noqa: E402
from pytorch_distributed_training_example_amd.ops import batchnorm as bnm  # noqa: E402

shapes = set()
orig = bnm.batch_norm_act


def spy(x, residual, *a, **k):
    shapes.add((tuple(x.shape), residual is not None, bool(a[-1])))
    return orig(x, residual, *a, **k)


bnm.batch_norm_act = spy
B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
S = int(sys.argv[2]) if len(sys.argv) > 2 else 64
m = get_model("resnet50").cuda().to(memory_format=torch.channels_last)
from pytorch_distributed_training_example_amd.models.precision import to_bf16_mixed  # noqa: E402
m = to_bf16_mixed(m)
x = torch.randn(B, 3, S, S, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
m(x).float().sum().backward()
bnm.batch_norm_act = orig
for (shape, res, relu) in sorted(shapes):
    torch.manual_seed(0)
    xx = torch.randn(shape, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    r = torch.randn_like(xx) if res else None
    C = shape[1]
    w, b = torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda")
    xs = xx.clone().requires_grad_(True)
    rs = r.clone().requires_grad_(True) if res else None
    ws, bs = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    y = orig(xs, rs, ws, bs, None, None, True, 0.1, 1e-5, relu)
    xf = xx.float().requires_grad_(True)
    rf = r.float().requires_grad_(True) if res else None
    wf, bf = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    yf = F.batch_norm(xf, None, None, wf, bf, True, 0.1, 1e-5)
    if res:
        yf = yf + rf
    if relu:
        yf = F.relu(yf)
    g = torch.randn_like(yf)
    y.backward(g.bfloat16())
    yf.backward(g.bfloat16().float())
    e = lambda a, b_: ((a.float() - b_).norm() / (b_.norm() + 1e-9)).item()
    print(f"{str(shape):24s} res={res:d} relu={relu:d}  y={e(y, yf):.4f} dx={e(xs.grad, xf.grad):.4f} "
          f"dw={e(ws.grad, wf.grad):.4f} db={e(bs.grad, bf.grad):.4f}" + (f" dr={e(rs.grad, rf.grad):.4f}" if res else ""),
          flush=True)
