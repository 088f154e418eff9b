"""Whole-model hipGraph check: forward+backward of the bench workload at fixed weights, eager vs a
captured-and-replayed graph of the same step (no optimizer, so both see identical weights).
Reports the loss both ways and the parameters whose gradients differ most (NaN counts first).

  python tools/diag_graph_model.py --model resnet50 --batch-size 1024
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    args = bench.parse(sys.argv[1:] + ["--graph", "1"])
    ctx = bench.setup(args)
    model, ddp, opt, precision = bench.build(args, ctx)
    from pytorch_distributed_training_example_amd.ops.cross_entropy import cross_entropy
    B = args.batch_size or bench.WORKLOADS[args.model][2]
    g = torch.Generator(device="cuda").manual_seed(7)
    is_lm = args.model.startswith("gpt")
    if is_lm:
        x = torch.randint(0, 50257, (B, args.seq_len), device="cuda", generator=g)
        y = torch.randint(0, 50257, (B, args.seq_len), device="cuda", generator=g)
    else:
        x = torch.randn(B, 3, args.image_size, args.image_size, device="cuda", generator=g).bfloat16()
        x = x.contiguous(memory_format=torch.channels_last)
        y = torch.randint(0, 1000, (B,), device="cuda", generator=g)
    params = [(n, p) for n, p in model.named_parameters() if p.requires_grad]

    snap = {}  # DIAG_HOOKS: copies of the fc input/output gradients taken inside the step

    def keep(name, t):
        if name not in snap:
            snap[name] = torch.empty_like(t)
        snap[name].copy_(t.detach())

    hooks = bool(os.environ.get("DIAG_HOOKS"))
    if hooks:
        model.fc.register_forward_hook(lambda m, i, o: [keep("fc.in", i[0]), keep("fc.out", o)] and None)

    def fb():
        for _, p in params:
            if p.grad is not None:
                p.grad.zero_()
        out = ddp(x)
        if hooks:
            out.register_hook(lambda gr: [keep("dlogits", gr), keep("dbias.sum0", gr.sum(0))] and None)
        if is_lm:
            loss = cross_entropy(out.reshape(-1, out.shape[-1]), y.reshape(-1))
        else:
            loss = cross_entropy(out, y, label_smoothing=0.1)
        loss.backward()
        if hooks:
            keep("fc.bias.grad", model.fc.bias.grad)
        return loss.detach()

    for _ in range(3):
        le = fb()
    torch.cuda.synchronize()
    ref = {n: p.grad.detach().float().clone() for n, p in params}
    ref_snap = {k: v.float().clone() for k, v in snap.items()}
    le = float(le)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fb()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, capture_error_mode=os.environ.get("DIAG_CAPMODE", "thread_local")):
        lg_t = fb()
    fcb = dict(params).get("fc.bias")
    if fcb is not None and os.environ.get("DIAG_NOCHURN"):
        # back-to-back replays into preallocated snapshots: no allocation between them
        snaps = [torch.empty_like(fcb.grad) for _ in range(3)]
        torch.cuda.synchronize()
        for r in range(3):
            graph.replay()
            snaps[r].copy_(fcb.grad)
        torch.cuda.synchronize()
        b = ref["fc.bias"]
        for r, a in enumerate(snaps):
            a = a.float()
            print(f"no-churn replay {r}: fc.bias relerr {float((a - b).norm() / b.norm()):.3e} "
                  f"|a| {float(a.abs().max()):.3e} |b| {float(b.abs().max()):.3e} "
                  f"a/b median {float((a / b).median()):.3f}", flush=True)
    for r in range(2):
        graph.replay()
        torch.cuda.synchronize()
        if fcb is not None:
            a, b = fcb.grad.float(), ref["fc.bias"]
            print(f"  fc.bias |a| {float(a.abs().max()):.3e} |b| {float(b.abs().max()):.3e} "
                  f"a/b median {float((a / b).median()):.3f} a-b max {float((a - b).abs().max()):.3e}")
        for k, v in snap.items():
            e = float((v.float() - ref_snap[k]).norm() / (ref_snap[k].norm() + 1e-12))
            print(f"  snapshot {k:18s} relerr {e:.3e}")
        rows = []
        for n, p in params:
            a, b = p.grad.detach().float(), ref[n]
            nan = int((~torch.isfinite(a)).sum())
            err = float((a - b).norm() / (b.norm() + 1e-12)) if nan == 0 else float("inf")
            rows.append((nan, err, n))
        rows.sort(key=lambda t: (-t[0], -t[1]))
        print(f"replay {r}: loss eager {le:.5f} graph {float(lg_t):.5f}; "
              f"{sum(1 for t in rows if t[0])} params with non-finite grads", flush=True)
        order = [n for n, _ in params]
        firsts = sorted((order.index(n), n, nan) for nan, _, n in rows if nan)
        if firsts:
            print("  non-finite grads, deepest-first param (backward reaches it first):", firsts[-1][1])
        for nan, err, n in rows[:12]:
            print(f"  {n:45s} nonfinite {nan:8d} relerr {err:.3e}")


if __name__ == "__main__":
    main()
