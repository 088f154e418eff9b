"""Diagnostic (one-off): ResNet-50 gradients, fp32 with our native ops enabled vs disabled (stock PyTorch),
and bf16-mixed native vs fp32 stock, to check the fp32 oracle itself."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from pytorch_distributed_training_example_amd.config import SW  # noqa: E402
from pytorch_distributed_training_example_amd.models import get_model  # noqa: E402
from pytorch_distributed_training_example_amd.models.precision import to_bf16_mixed  # noqa: E402


def run(fp32, disable_native, hw=96, n=8):
    if disable_native:
        os.environ["PDT_DISABLE_NATIVE"] = "1"
    else:
        os.environ.pop("PDT_DISABLE_NATIVE", None)
    SW.reload()
    torch.manual_seed(0)
    m = get_model("resnet50").cuda().to(memory_format=torch.channels_last)
    if not fp32:
        m = to_bf16_mixed(m)
    x = torch.randn(n, 3, hw, hw, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (n,), device="cuda")
    if fp32:
        x = x.float()
    out = m(x).float()
    loss = torch.nn.functional.cross_entropy(out, y)
    loss.backward()
    g = {k: p.grad.float().clone() for k, p in m.named_parameters()}
    os.environ.pop("PDT_DISABLE_NATIVE", None)
    SW.reload()
    return float(loss), out.detach(), g


def rel(ga, gb):
    return torch.tensor([float((ga[k] - gb[k]).norm() / gb[k].norm().clamp_min(1e-12)) for k in gb])


l_nat32, o_nat32, g_nat32 = run(True, False)
l_st32, o_st32, g_st32 = run(True, True)
l_natb, o_natb, g_natb = run(False, False)
l_stb, o_stb, g_stb = run(False, True)
print(f"loss fp32 native {l_nat32:.5f} fp32 stock {l_st32:.5f} bf16 native {l_natb:.5f} bf16 stock {l_stb:.5f}")
for name, g in (("fp32 native", g_nat32), ("bf16 native", g_natb), ("bf16 stock", g_stb)):
    e = rel(g, g_st32)
    print(f"{name:12s} vs fp32 stock: median {float(e.median()):.4f} max {float(e.max()):.4f} "
          f"stem |g| {float(g['conv1.weight'].norm()):.4e} (fp32 stock {float(g_st32['conv1.weight'].norm()):.4e})")
print("logits native fp32 vs stock fp32 max abs diff", float((o_nat32 - o_st32).abs().max()))
e = rel(g_nat32, g_st32)
names = list(g_st32)
for i in list(range(4)) + list(range(len(names) - 8, len(names))):
    k = names[i]
    print(f"  {k:36s} rel {float(e[i]):.4f} |g| native {float(g_nat32[k].norm()):.4e} stock {float(g_st32[k].norm()):.4e}")
