"""Our Linear GEMM (csrc/kernels/gemm.hip) vs the library GEMM the bench would run (hipBLASLt through
F.linear, with the repo's TunableOp table) on the ViT-B/16 and GPT-2-medium Linear shapes.

Interleaved rounds in one process (cdna_hip_programming.md §5.4 rule 24), random operands
(rule 25). Per shape: median us and TF/s of each arm, and the error of ours against an fp32
reference. ``--epi gelu`` compares the fused H/G epilogue against F.linear + the standalone
bias+GELU kernel. One JSON line per shape on stdout.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = {  # name: (M, K, N)
    "gpt2_qkv": (8192, 1024, 3072), "gpt2_proj": (8192, 1024, 1024), "gpt2_fc1": (8192, 1024, 4096),
    "gpt2_fc2": (8192, 4096, 1024),
    "vit_qkv": (25216, 768, 2304), "vit_proj": (25216, 768, 768), "vit_fc1": (25216, 768, 3072),
    "vit_fc2": (25216, 3072, 768),
}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default=",".join(SHAPES))
    ap.add_argument("--epi", default="bias", choices=["none", "bias", "gelu"])
    ap.add_argument("--rounds", type=int, default=10)
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    from pytorch_distributed_training_example_amd.engine.gemm_tuning import use_repo_gemm_tuning
    use_repo_gemm_tuning()
    import torch
    import torch.nn.functional as F
    from pytorch_distributed_training_example_amd.ops._native import native
    C = native()
    torch.manual_seed(0)
    for name in args.shapes.split(","):
        M, K, N = SHAPES[name]
        x = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
        w = ((torch.rand(N, K, device="cuda") * 2 - 1) / K ** 0.5).bfloat16()
        b = (torch.rand(N, device="cuda") * 0.2 - 0.1).bfloat16()
        bf = b.float()
        tanh = name.startswith("gpt2")
        if args.epi == "none":
            ours = lambda: C.gemm_nt(x, w, None, 0, False)  # noqa: E731
            lib = lambda: F.linear(x, w)  # noqa: E731
        elif args.epi == "bias":
            ours = lambda: C.gemm_nt(x, w, b, 1, False)  # noqa: E731
            lib = lambda: F.linear(x, w, b)  # noqa: E731
        else:
            ours = lambda: C.gemm_nt(x, w, bf, 2, tanh)  # noqa: E731
            lib = lambda: C.bias_gelu_fwd(F.linear(x, w), bf, tanh)  # noqa: E731
        # numerics against fp32
        ref = x.float() @ w.float().t()
        if args.epi == "bias":
            ref = ref + b.float()
        got = ours()
        err = ((got[0].float() - ref).norm() / ref.norm()).item()
        if args.epi == "gelu":
            gref = F.gelu(got[0].float() + bf, approximate="tanh" if tanh else "none")
            gerr = ((got[1].float() - gref).norm() / gref.norm()).item()
            err = max(err, gerr)
        times = {"ours": [], "lib": []}
        for _ in range(args.rounds):
            for arm, fn in (("ours", ours), ("lib", lib)):
                for _ in range(3):
                    fn()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(args.iters):
                    fn()
                e.record()
                e.synchronize()
                times[arm].append(s.elapsed_time(e) * 1000 / args.iters)
        flop = 2.0 * M * N * K
        out = {"shape": name, "M": M, "K": K, "N": N, "epi": args.epi, "rel_err": round(err, 6)}
        for arm, t in times.items():
            t.sort()
            med = t[len(t) // 2]
            out[f"{arm}_us"] = round(med, 1)
            out[f"{arm}_tflops"] = round(flop / med / 1e6, 1)
        out["speedup"] = round(out["lib_us"] / out["ours_us"], 3)
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
