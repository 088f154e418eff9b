"""Is a column sum (what nn.Linear's bias gradient is) replay-safe under hipGraph capture?
[rows, 1000] bf16/fp32 ``sum(0)`` captured once, replayed with allocator churn between replays,
against the eager result. Variants: torch sum, fp32-accumulating sum, and a GEMV against ones."""
import torch

torch.manual_seed(0)
for rows in (128, 1024, 4096):
    for dt in (torch.bfloat16, torch.float32):
        g = torch.randn(rows, 1000, device="cuda").to(dt)
        ones = torch.ones(rows, device="cuda", dtype=dt)
        fns = {"sum0": lambda: g.sum(0), "sum0_f32": lambda: g.sum(0, dtype=torch.float32),
               "gemv": lambda: torch.mv(g.t(), ones)}
        for name, fn in fns.items():
            ref = fn().float().clone()
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                for _ in range(3):
                    fn()
            torch.cuda.current_stream().wait_stream(s)
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                out = fn()
            errs = []
            for r in range(3):
                graph.replay()
                torch.cuda.synchronize()
                errs.append(float((out.float() - ref).norm() / ref.norm()))
                junk = [torch.randn(rows, 1000, device="cuda") for _ in range(4)]  # allocator churn
                del junk
            print(f"rows {rows:5d} {str(dt):15s} {name:9s} replay relerr {' '.join(f'{e:.2e}' for e in errs)}",
                  flush=True)
