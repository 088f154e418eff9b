"""Reduce vs apply kernel time of our BN at ResNet-50 shapes (batch 512) per bn_tune setting, from
torch.profiler device events; 4 rotating inputs per shape (> the 256-MiB Infinity Cache).
Variant 4 = v3 streaming only (no finalize: timing probe, outputs invalid)."""
import sys
from collections import defaultdict

import torch
from torch.profiler import ProfilerActivity, profile

sys.path.insert(0, ".")
from pytorch_distributed_training_example_amd.ops._native import native  # noqa: E402

C_ = native()
SHAPES = [(64, 56), (256, 56), (128, 28), (512, 28), (256, 14), (1024, 14), (512, 7), (2048, 7)]
TUNINGS = [(5, 512, 8, 4)]
B = 512
for C, h in SHAPES:
    xs = [torch.randn(B, C, h, h, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
          for _ in range(4)]
    dys = [torch.randn_like(x) for x in xs]
    w, b = torch.ones(C, device="cuda"), torch.zeros(C, device="cuda")
    rm, rv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
    line = f"C={C:5d} H={h:3d} {xs[0].numel() * 2 / 1e6:6.1f} MB |"
    for tu in TUNINGS:
        C_.bn_tune(*tu)
        outs = [C_.bn_fwd_train(x, None, w, b, rm, rv, 0.1, 1e-5, True) for x in xs]
        torch.cuda.synchronize()
        with profile(activities=[ProfilerActivity.CUDA]) as prof:
            for _ in range(3):
                for x, dy, o in zip(xs, dys, outs):
                    C_.bn_fwd_train(x, None, w, b, rm, rv, 0.1, 1e-5, True)
                    C_.bn_bwd_train(dy, x, o[1], w, o[2], o[3], True, False, True)
            torch.cuda.synchronize()
        t = defaultdict(list)
        for e in prof.events():
            if e.device_type == torch.autograd.DeviceType.CUDA and "bn_" in e.name:
                if "reduce" in e.name or "fin_kernel" in e.name:
                    key = "fr" if "<0" in e.name else "br"
                    if "fin_kernel" in e.name:
                        key += "f"
                else:
                    key = "ba" if "bwd_apply" in e.name else "fa"
                t[key].append(e.device_time)
        med = {k: sorted(v)[len(v) // 2] for k, v in t.items()}
        line += (f" {tu[0]},{tu[1]},{tu[2]},{tu[3]}: fr {med.get('fr', 0):5.1f}+{med.get('frf', 0):4.1f}"
                 f" br {med.get('br', 0):5.1f}+{med.get('brf', 0):4.1f} |")
    print(line, f"fa {med.get('fa', 0):5.1f} ba {med.get('ba', 0):5.1f}", flush=True)
    C_.bn_tune(5, 512, 8, 4)
    del xs, dys, outs
