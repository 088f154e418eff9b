"""Our fp8 GEMM (csrc/kernels/gemm.hip F8) vs torch._scaled_mm (hipBLASLt, tuned by TunableOp when its table
is active) on the ViT-B/16 and GPT-2-medium Linear shapes (forward and data gradient: M = tokens).
One JSON line per shape: {"shape", "M", "N", "K", "ours_us", "lib_us", "speedup", "ours_tflops"}."""
import json
import os
import sys

import torch


def bench(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / iters


def main():
    sys.path.insert(0, ".")
    from pytorch_distributed_training_example_amd.ops._native import native
    n = native()
    shapes = {  # name: (M, N, K) of C[M, N] = A[M, K] B[N, K]^T
        "vit_qkv": (25216, 2304, 768), "vit_proj": (25216, 768, 768), "vit_fc1": (25216, 3072, 768),
        "vit_fc2": (25216, 768, 3072), "vit_qkv_dgrad": (25216, 768, 2304), "vit_fc1_dgrad": (25216, 768, 3072),
        "vit_fc2_dgrad": (25216, 3072, 768),
        "gpt2_qkv": (8192, 3072, 1024), "gpt2_proj": (8192, 1024, 1024), "gpt2_fc1": (8192, 4096, 1024),
        "gpt2_fc2": (8192, 1024, 4096), "sq8k": (8192, 8192, 8192),
        # weight gradients dW [out, in] = dY^T X over the tokens (split-K path)
        "vit_qkv_wgrad": (2304, 768, 25216), "vit_proj_wgrad": (768, 768, 25216), "vit_fc1_wgrad": (3072, 768, 25216),
        "vit_fc2_wgrad": (768, 3072, 25216), "gpt2_qkv_wgrad": (3072, 1024, 8192), "gpt2_proj_wgrad": (1024, 1024, 8192),
        "gpt2_fc1_wgrad": (4096, 1024, 8192), "gpt2_fc2_wgrad": (1024, 4096, 8192)}
    only = os.environ.get("SHAPES")
    if only:
        shapes = {k: v for k, v in shapes.items() if k in only.split(",")}
    g = torch.Generator(device="cuda").manual_seed(0)
    for name, (M, N, K) in shapes.items():
        a = (torch.randn(M, K, device="cuda", generator=g) * 4).to(torch.float8_e4m3fn)
        b = (torch.randn(N, K, device="cuda", generator=g) * 4).to(torch.float8_e4m3fn)
        sa = torch.tensor([0.02], device="cuda")
        sb = torch.tensor([0.03], device="cuda")
        ours = bench(lambda: n.gemm_nt_fp8(a, b, sa, sb))
        lib = bench(lambda: torch._scaled_mm(a, b.t(), scale_a=sa, scale_b=sb, out_dtype=torch.bfloat16))
        o, l = n.gemm_nt_fp8(a, b, sa, sb).float(), torch._scaled_mm(a, b.t(), scale_a=sa, scale_b=sb,
                                                                       out_dtype=torch.bfloat16).float()
        err = ((o - l).abs().max() / l.abs().max()).item()
        print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "ours_us": round(ours, 1), "lib_us": round(lib, 1),
                          "speedup": round(lib / ours, 3), "ours_tflops": round(2 * M * N * K / ours / 1e6, 1),
                          "rel_err_vs_lib": round(err, 5)}), flush=True)


if __name__ == "__main__":
    main()
