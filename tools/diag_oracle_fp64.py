"""Diagnostic: how far is an fp32 ResNet-50 gradient from the fp64 gradient of the same model and batch,
with our native ops on (fp32 kernels where they exist) and off (stock PyTorch)? The stock fp32 error
is the fp32 reduction-order noise floor that bounds tests/test_models_gpu.py's native-vs-stock check.

    python tools/diag_oracle_fp64.py [--hw 96] [--n 8]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from pytorch_distributed_training_example_amd.config import SW  # noqa: E402
from pytorch_distributed_training_example_amd.models import get_model  # noqa: E402


def run(dtype, disable_native, hw, n, model="resnet50", res_scale=None, amp16=False):
    if disable_native:
        os.environ["PDT_DISABLE_NATIVE"] = "1"
    SW.reload()
    try:
        torch.manual_seed(0)
        m = get_model(model).cuda().to(memory_format=torch.channels_last).to(dtype)
        if res_scale is not None:  # SkipInit-style: each residual branch's last BN starts at gamma = res_scale
            from pytorch_distributed_training_example_amd.models.resnet import BasicBlock, Bottleneck
            for b in m.modules():
                if isinstance(b, (Bottleneck, BasicBlock)):
                    torch.nn.init.constant_((b.bn3 if isinstance(b, Bottleneck) else b.bn2).weight, res_scale)
        g = torch.Generator(device="cuda").manual_seed(1)
        x = torch.randn(n, 3, hw, hw, device="cuda", generator=g).to(dtype).contiguous(memory_format=torch.channels_last)
        y = torch.randint(0, 1000, (n,), device="cuda", generator=g)
        with torch.autocast("cuda", dtype=torch.float16, enabled=amp16):
            out = m(x)
        loss = torch.nn.functional.cross_entropy(out.float(), y)
        loss.backward()
        return float(loss), {k: p.grad.double().clone() for k, p in m.named_parameters()}
    finally:
        os.environ.pop("PDT_DISABLE_NATIVE", None)
        SW.reload()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--hw", type=int, default=96)
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--res-scale", type=float, default=None)
    a = ap.parse_args()
    kw = dict(model=a.model, res_scale=a.res_scale)
    l64, g64 = run(torch.float64, True, a.hw, a.n, **kw)
    ln, gn = run(torch.float32, False, a.hw, a.n, **kw)
    ls, gs = run(torch.float32, True, a.hw, a.n, **kw)
    lh, gh = run(torch.float32, False, a.hw, a.n, amp16=True, **kw)
    ref_max = max(float(v.norm()) for v in g64.values())
    print(f"{a.model} res_scale {a.res_scale} hw {a.hw} n {a.n} loss fp64 {l64:.8f} native fp32 {ln:.8f} stock fp32 {ls:.8f}")
    rows = []
    for k, v in g64.items():
        d = float(v.norm())
        rows.append((k, d, float((gn[k] - v).norm()) / max(d, 1e-300), float((gs[k] - v).norm()) / max(d, 1e-300),
                     float((gn[k] - gs[k]).norm()) / max(float(gs[k].norm()), 1e-300),
                     float((gh[k] - v).norm()) / max(d, 1e-300)))
    big = [r for r in rows if r[1] > 1e-6 * ref_max]
    en = torch.tensor([r[2] for r in big])
    es = torch.tensor([r[3] for r in big])
    ens = torch.tensor([r[4] for r in big])
    eh = torch.tensor([r[5] for r in big])
    print(f"{len(big)}/{len(rows)} params with |g| > 1e-6 max|g|")
    for name, e in (("native fp32 vs fp64", en), ("stock fp32 vs fp64", es), ("native vs stock fp32", ens), ("ours amp_fp16 vs fp64", eh)):
        print(f"  {name:22s} median {float(e.median()):.3e} p90 {float(e.quantile(0.9)):.3e} max {float(e.max()):.3e}")
    print("worst 10 (native vs stock):")
    for r in sorted(big, key=lambda r: -r[4])[:10]:
        print(f"  {r[0]:40s} |g64| {r[1]:.3e} nat-vs-64 {r[2]:.3e} stock-vs-64 {r[3]:.3e} nat-vs-stock {r[4]:.3e}")


if __name__ == "__main__":
    main()
