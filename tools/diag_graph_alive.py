"""What keeps a previous step's autograd graph alive? After a full forward+backward of the bench
workload (eager), list every live tensor that still has a ``grad_fn`` and every live custom-Function
context (``*Backward`` objects), with who refers to them. A node kept alive across steps keeps the
stream it was created on, which breaks hipGraph capture of the next step (torch's AccumulateGrad
stream-mismatch warning).

  python tools/diag_graph_alive.py --batch-size 1024
"""
import gc
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def describe(o):
    if isinstance(o, torch.Tensor):
        return f"Tensor{tuple(o.shape)} {o.dtype} grad_fn={type(o.grad_fn).__name__ if o.grad_fn else None}"
    if isinstance(o, dict):
        return f"dict(keys={list(o.keys())[:6]})"
    if isinstance(o, (list, tuple)):
        return f"{type(o).__name__}(len={len(o)})"
    return type(o).__name__


def main():
    args = bench.parse(sys.argv[1:] + ["--graph", "0"])
    ctx = bench.setup(args)
    model, ddp, opt, precision = bench.build(args, ctx)
    from pytorch_distributed_training_example_amd.ops.cross_entropy import cross_entropy
    B = args.batch_size or bench.WORKLOADS[args.model][2]
    x = torch.randn(B, 3, args.image_size, args.image_size, device="cuda").bfloat16()
    x = x.contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (B,), device="cuda")

    def fb():
        opt.zero_grad(set_to_none=True)
        loss = cross_entropy(ddp(x), y, label_smoothing=0.1)
        loss.backward()
        opt.step()
        return loss.detach()

    for _ in range(2):
        fb()
    torch.cuda.synchronize()
    gc.collect()
    live = [o for o in gc.get_objects() if isinstance(o, torch.Tensor) and o.grad_fn is not None]
    ctxs = [o for o in gc.get_objects() if type(o).__name__.endswith("Backward")
            and hasattr(o, "saved_tensors")]
    print(f"B={B}: {len(live)} live tensors with grad_fn, {len(ctxs)} live custom-Function contexts", flush=True)
    for o in live[:20] + ctxs[:20]:
        refs = [describe(r) for r in gc.get_referrers(o) if r is not live and r is not ctxs]
        print(f"  {describe(o)}  <- {refs[:4]}", flush=True)
        for r in gc.get_referrers(o):
            if isinstance(r, dict) and r is not globals():
                owners = [describe(q) for q in gc.get_referrers(r) if q is not live and q is not ctxs]
                print(f"      dict {list(r.keys())[:8]} <- {owners[:4]}", flush=True)


if __name__ == "__main__":
    main()
