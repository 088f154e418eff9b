"""Diagnostic: accuracy of fp16 autocast (with loss scaling) and of fp32 GEMM paths on this stack.

  * ResNet-18 / ViT-tiny gradients, ours (native ops on) and stock (PDT_DISABLE_NATIVE) under fp16 autocast with
    a 2^12 loss scale, against the fp64 gradient of the same model and batch;
  * torch.mm / F.conv2d 1x1 in fp32 against fp64 (is any fp32 path running at reduced precision?).

    python tools/diag_amp16.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402
from pytorch_distributed_training_example_amd.config import SW  # noqa: E402
from pytorch_distributed_training_example_amd.models import get_model  # noqa: E402


def grads(model, dtype, amp16, native, scale=4096.0, res_scale=None):
    if not native:
        os.environ["PDT_DISABLE_NATIVE"] = "1"
    SW.reload()
    try:
        torch.manual_seed(0)
        if model == "resnet18":
            m = get_model("resnet18", num_classes=10).cuda().to(memory_format=torch.channels_last).to(dtype)
            if res_scale is not None:
                from pytorch_distributed_training_example_amd.models.resnet import BasicBlock
                for b in m.modules():
                    if isinstance(b, BasicBlock):
                        torch.nn.init.constant_(b.bn2.weight, res_scale)
            x = torch.randn(8, 3, 64, 64, device="cuda", generator=torch.Generator(device="cuda").manual_seed(1))
            x = x.to(dtype).contiguous(memory_format=torch.channels_last)
        else:
            m = get_model("vit_tiny", image_size=32, num_classes=10).cuda().to(dtype)
            torch.nn.init.normal_(m.heads.head.weight, std=0.02)
            x = torch.randn(8, 3, 32, 32, device="cuda", generator=torch.Generator(device="cuda").manual_seed(1)).to(dtype)
        y = torch.randint(0, 10, (8,), device="cuda", generator=torch.Generator(device="cuda").manual_seed(2))
        with torch.autocast("cuda", dtype=torch.float16, enabled=amp16):
            out = m(x)
        loss = F.cross_entropy(out.float(), y) * (scale if amp16 else 1.0)
        loss.backward()
        return {k: p.grad.double() / (scale if amp16 else 1.0) for k, p in m.named_parameters()}
    finally:
        os.environ.pop("PDT_DISABLE_NATIVE", None)
        SW.reload()


def rel(ga, gb):
    big = max(float(v.norm()) for v in gb.values())
    e = torch.tensor([float((ga[k] - gb[k]).norm() / gb[k].norm()) for k in gb if float(gb[k].norm()) > 1e-6 * big])
    return f"median {float(e.median()):.3e} p90 {float(e.quantile(0.9)):.3e} max {float(e.max()):.3e}"


def main():
    print("allow_tf32 matmul", torch.backends.cuda.matmul.allow_tf32, "cudnn", torch.backends.cudnn.allow_tf32,
          "fp32 precision", torch.get_float32_matmul_precision())
    a = torch.randn(4096, 1024, device="cuda", dtype=torch.float64)
    b = torch.randn(1024, 512, device="cuda", dtype=torch.float64)
    ref = a @ b
    print("mm fp32 vs fp64", float(((a.float() @ b.float()).double() - ref).norm() / ref.norm()))
    xc = torch.randn(16, 256, 14, 14, device="cuda", dtype=torch.float64).contiguous(memory_format=torch.channels_last)
    wc = torch.randn(512, 256, 1, 1, device="cuda", dtype=torch.float64)
    rc = F.conv2d(xc, wc)
    print("conv1x1 fp32 vs fp64", float((F.conv2d(xc.float(), wc.float()).double() - rc).norm() / rc.norm()))
    bm = torch.bmm(a.float().view(4, 1024, 1024).transpose(1, 2), a.float().view(4, 1024, 1024)).double()
    rb = torch.bmm(a.view(4, 1024, 1024).transpose(1, 2), a.view(4, 1024, 1024))
    print("bmm fp32 vs fp64", float((bm - rb).norm() / rb.norm()))
    for model, rs in (("resnet18", None), ("resnet18", 0.2), ("vit_tiny", None)):
        g64 = grads(model, torch.float64, False, False, res_scale=rs)
        g32n = grads(model, torch.float32, False, True, res_scale=rs)
        g16n = grads(model, torch.float32, True, True, res_scale=rs)
        g16s = grads(model, torch.float32, True, False, res_scale=rs)
        print(f"{model} res_scale {rs}: fp32 native {rel(g32n, g64)} | amp16 ours {rel(g16n, g64)} | amp16 stock {rel(g16s, g64)}")


if __name__ == "__main__":
    main()
