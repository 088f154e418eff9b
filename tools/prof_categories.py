"""Group a prof_window.py *_kernels.csv by kernel family (ms per step).

    python tools/prof_categories.py <kernels.csv> [steps] [--kind resnet|transformer]

The families follow the step's model: a window with attention / LayerNorm kernels is a transformer step
(ViT, GPT-2) and is broken out as GEMMs (hipBLASLt bf16 / fp8, ours), attention, LayerNorm, fp8 casts, bias+GELU,
bias-gradient column sums, cross-entropy, embedding, optimizer, PyTorch elementwise; otherwise the ResNet families
(1x1 / 3x3 / stem convs, BatchNorm, fused backward, library GEMMs).
"""
import csv
import re
import sys


def family_transformer(n):
    if n.startswith("Custom_Cijk") or n.startswith("Cijk"):
        fp8 = "F8" in n.split("_UserArgs")[0]
        return f"hipBLASLt GEMM ({'fp8 e4m3' if fp8 else 'bf16'}: qkv / proj / fc1 / fc2 / lm-head, fwd + dgrad + wgrad)"
    if "gemm_nt" in n or "splitk_reduce" in n:
        return "our GEMM (gemm.hip, MFMA)"
    if "attn_" in n:
        return "attention fwd / bwd (attention.hip, MFMA)"
    if "ln_" in n:
        return "LayerNorm (+residual add, +fp8 emit) fwd / bwd"
    if "fp8_" in n:
        return "fp8 casts / transposes / amax (incl. GELU+cast)"
    if "gelu" in n or "strip_kernel" in n:
        return "bias + GELU fwd / bwd (bf16)"
    if "colsum" in n or "slice_sum" in n:
        return "bias gradients (column sums)"
    if "ce_fwd" in n or "ce_bwd" in n:
        return "softmax cross-entropy"
    if "emb_" in n:
        return "embedding fwd / bwd"
    if "mt_kernel" in n:
        return "optimizer / multi-tensor copies"
    if "at::native" in n or "rocclr" in n:
        return "PyTorch elementwise / copies / reductions"
    return "other"


def family(n):
    if "conv1x1_bwd_fused" in n or "fb_reduce" in n:
        return "fused conv3 + BN3 backward (dgrad + wgrad + BN apply/reduction)"
    m = re.search(r"conv1x1_kernel<.*?G1<[^>]*>,(.*?)>\s*\(", n)  # <Cf, ACC, STATS, NT, BSTATS, ATR, APPLY[, STR]>
    if m and [f.strip() for f in m.group(1).split(",")][5:6] == ["true"]:
        return "1x1 GEMM + BN(+res)+ReLU apply epilogue (recomputed conv3)"
    m = re.search(r"conv1x1p_kernel<.*?G1<[^>]*>,(.*?)>\s*\(", n)  # persistent: <Cf, ACC, STATS, BSTATS, ATR, APPLY, STR>
    if m and [f.strip() for f in m.group(1).split(",")][4:5] == ["true"]:
        return "1x1 GEMM + BN(+res)+ReLU apply epilogue (recomputed conv3)"
    if "conv1x1_wgrad" in n:
        return "our 1x1 weight gradient (MFMA)"
    if "weight_prep" in n:
        return "batched weight transforms"
    if "bn_" in n or "maxpool" in n:
        return "our BN (+ReLU/residual/pool)"
    if "conv3x3" in n:
        return "our 3x3 conv (MFMA)"
    if "conv1x1_kernel" in n or "conv1x1p_kernel" in n:
        return "our 1x1 conv GEMM (MFMA, fused BN-stats epilogues)"
    if "stem_" in n:
        return "our 7x7 stem conv (MFMA)"
    if "Cijk" in n:
        return "hipBLASLt GEMM (1x1 convs, fc)"
    if any(s in n for s in ("igemm", "ck::", "_ZN2ck", "naive_conv", "SubTensor", "fillBuffer", "ranspose")):
        return "MIOpen conv (+fills)"
    if any(s in n for s in ("ce_", "mt_kernel", "sgd", "strip", "colsum")):
        return "our CE / optimizer"
    return "other"


def main():
    argv = [a for a in sys.argv[1:] if not a.startswith("--kind")]
    kind = next((a.split("=", 1)[1] for a in sys.argv[1:] if a.startswith("--kind=")), None)
    rows = list(csv.DictReader(open(argv[0])))
    steps = float(argv[1]) if len(argv) > 1 else 5.0
    if kind is None:
        kind = "transformer" if any("attn_" in r["Name"] or "ln_fwd" in r["Name"] for r in rows) else "resnet"
    fam = family_transformer if kind == "transformer" else family
    cat = {}
    other = []
    for r in rows:
        ms = float(r["TotalDurationNs"]) / 1e6 / steps
        f = fam(r["Name"])
        cat[f] = cat.get(f, 0.0) + ms
        if f == "other":
            other.append((ms, r["Name"][:80]))
    print("| family | ms/step |\n|---|---:|")
    for k, v in sorted(cat.items(), key=lambda x: -x[1]):
        print(f"| {k} | {v:.2f} |")
    print(f"| total busy | {sum(cat.values()):.2f} |")
    for ms, n in sorted(other, reverse=True)[:8]:
        print(f"  other: {ms:.3f} {n}", file=sys.stderr)


if __name__ == "__main__":
    main()
