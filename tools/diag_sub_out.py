import torch, sys, os
sys.path.insert(0, "/root/repo")
os.environ.setdefault("PDT_BWD_ALG_MIN_M", "0")
from pytorch_distributed_training_example_amd.models import get_model
from pytorch_distributed_training_example_amd.models.precision import to_bf16_mixed
torch.manual_seed(0)
m = to_bf16_mixed(get_model("resnet50", num_classes=10).cuda().to(memory_format=torch.channels_last))
x = torch.randn(4, 3, 112, 112, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
y = torch.randint(0, 10, (4,), device="cuda")
def step():
    m.zero_grad(set_to_none=True)
    out = m(x)
    torch.nn.functional.cross_entropy(out.float(), y).backward()
    return [("out", out.detach())] + [(n, p.grad.clone()) for n, p in m.named_parameters()]
a = step(); a2 = step()
print("on vs on:", [n for (n, u), (_, v) in zip(a, a2) if not torch.equal(u, v)][:5])
for blk in (m.layer1[-1], m.layer2[-1], m.layer3[-1]): blk.emit_sub = 0
b = step(); b2 = step()
print("off vs off:", [n for (n, u), (_, v) in zip(b, b2) if not torch.equal(u, v)][:5])
print("on vs off:", [(n, float((u.float()-v.float()).norm()/v.float().norm())) for (n, u), (_, v) in zip(a, b) if not torch.equal(u, v)][:8])
