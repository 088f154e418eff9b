"""LayerNorm backward (layernorm.hip ln_bwd_kernel + finalize) at the ViT-B/16 / GPT-2-medium shapes, with the
residual-gradient input: us per call and effective HBM rate (dy, x, dres read + dx written). The workgroup
cap comes from PDT_LN_BWD_BLOCKS (read once per process)."""
import json
import os
import sys

import torch


def main():
    sys.path.insert(0, ".")
    from pytorch_distributed_training_example_amd.ops._native import native
    n = native()
    for name, (N, D) in {"vit_b16": (25216, 768), "gpt2_medium": (8192, 1024)}.items():
        g = torch.Generator(device="cuda").manual_seed(0)
        x = torch.randn(N, D, device="cuda", generator=g).bfloat16()
        dy = torch.randn(N, D, device="cuda", generator=g).bfloat16()
        dr = torch.randn(N, D, device="cuda", generator=g).bfloat16()
        w = torch.rand(D, device="cuda", generator=g) + 0.5
        mean = x.float().mean(1)
        rstd = (x.float().var(1, unbiased=False) + 1e-5).rsqrt()
        for _ in range(5):
            n.ln_bwd(dy, x, w, mean, rstd, dr)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(50):
            n.ln_bwd(dy, x, w, mean, rstd, dr)
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) * 1e3 / 50
        print(json.dumps({"shape": name, "blocks_cap": os.environ.get("PDT_LN_BWD_BLOCKS", "512"), "us": round(us, 1),
                          "TBps": round(4 * N * D * 2 / us / 1e6, 2)}), flush=True)


if __name__ == "__main__":
    main()
