"""Is the ResNet-50 native-vs-reference grad gap a bug or bf16 sensitivity? Compare both to fp32."""
import copy
import os
import sys

import torch

sys.path.insert(0, ".")
from pytorch_distributed_training_example_amd.models import get_model  # noqa: E402
from pytorch_distributed_training_example_amd.models.precision import to_bf16_mixed  # noqa: E402
from pytorch_distributed_training_example_amd.ops.cross_entropy import cross_entropy  # noqa: E402


def grads(m, x, y):
    m.zero_grad(set_to_none=True)
    loss = cross_entropy(m(x), y)
    loss.backward()
    return float(loss), {n: p.grad.float().clone() for n, p in m.named_parameters()}


name = sys.argv[1] if len(sys.argv) > 1 else "resnet50"
torch.manual_seed(0)
base = get_model(name).cuda().to(memory_format=torch.channels_last)
x32 = torch.randn(16, 3, 64, 64, device="cuda").contiguous(memory_format=torch.channels_last)
y = torch.randint(0, 1000, (16,), device="cuda")
f32 = copy.deepcopy(base)
os.environ["PDT_DISABLE_NATIVE"] = "1"
l32, g32 = grads(f32, x32, y)
lref, gref = grads(to_bf16_mixed(copy.deepcopy(base)), x32.bfloat16(), y)
lref2, gref2 = grads(to_bf16_mixed(copy.deepcopy(base)), (x32 * (1 + 1e-3)).bfloat16(), y)
os.environ.pop("PDT_DISABLE_NATIVE")
lnat, gnat = grads(to_bf16_mixed(copy.deepcopy(base)), x32.bfloat16(), y)
print("loss fp32 %.5f ref-bf16 %.5f ref-bf16-perturbed %.5f native-bf16 %.5f" % (l32, lref, lref2, lnat))
e = lambda a, b: ((a - b).norm() / (b.norm() + 1e-12)).item()
for n in list(g32)[:6] + list(g32)[-6:]:
    print(f"{n:30s} ref/fp32 {e(gref[n], g32[n]):.3f}  nat/fp32 {e(gnat[n], g32[n]):.3f}  nat/ref {e(gnat[n], gref[n]):.3f}"
          f"  ref/refpert {e(gref2[n], gref[n]):.3f}  |g| {g32[n].norm().item():.3e}")
