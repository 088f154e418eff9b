"""Which MIOpen conv solvers are hipGraph-capture safe? Per ResNet-50 conv shape: run fwd /
dgrad / wgrad eagerly and as a replayed graph; report mismatches and eager time."""
import sys

import torch

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
torch.backends.cudnn.benchmark = bool(int(sys.argv[2])) if len(sys.argv) > 2 else True
SET = sys.argv[3] if len(sys.argv) > 3 else "r50"
# (c_in, c_out, kernel, stride, input size); r18s = ResNet-18 at 64x64 input (tests/test_graph_gpu.py)
R18S = [(3, 64, 7, 2, 64), (64, 64, 3, 1, 16), (64, 128, 3, 2, 16), (64, 128, 1, 2, 16), (128, 128, 3, 1, 8),
        (128, 256, 3, 2, 8), (128, 256, 1, 2, 8), (256, 256, 3, 1, 4), (256, 512, 3, 2, 4), (256, 512, 1, 2, 4),
        (512, 512, 3, 1, 2)]
shapes = [(3, 64, 7, 2, 224), (64, 64, 1, 1, 56), (64, 64, 3, 1, 56), (64, 256, 1, 1, 56), (256, 64, 1, 1, 56),
          (256, 128, 1, 1, 56), (128, 128, 3, 2, 56), (128, 512, 1, 1, 28), (256, 512, 1, 2, 56),
          (512, 128, 1, 1, 28), (128, 128, 3, 1, 28), (512, 256, 1, 1, 28), (256, 256, 3, 2, 28),
          (256, 1024, 1, 1, 14), (512, 1024, 1, 2, 28), (1024, 256, 1, 1, 14), (256, 256, 3, 1, 14),
          (1024, 512, 1, 1, 14), (512, 512, 3, 2, 14), (512, 2048, 1, 1, 7), (1024, 2048, 1, 2, 14),
          (2048, 512, 1, 1, 7), (512, 512, 3, 1, 7)]
if SET == "r18s":
    shapes = R18S
bad = []
tot = 0.0
for (ci, co, k, s, h) in shapes:
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(B, ci, h, h, device="cuda", generator=g).bfloat16().contiguous(memory_format=torch.channels_last)
    w = (torch.randn(co, ci, k, k, device="cuda", generator=g) * 0.05).bfloat16().contiguous(memory_format=torch.channels_last)
    pad = k // 2
    y = torch.nn.functional.conv2d(x, w, stride=s, padding=pad)
    gy = torch.randn(y.shape, device="cuda", generator=g).bfloat16().contiguous(memory_format=torch.channels_last)

    def ops():
        f = torch.nn.functional.conv2d(x, w, stride=s, padding=pad)
        dx, dw, _ = torch.ops.aten.convolution_backward(gy, x, w, None, [s, s], [pad, pad], [1, 1], False, [0, 0], 1,
                                                        [ci != 3, True, False])
        return f, dx, dw

    for _ in range(3):
        ref = ops()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        ops()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 5
    tot += ms
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(st):
        ops()
    torch.cuda.current_stream().wait_stream(st)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        out = ops()
    for _ in range(2):
        graph.replay()
    torch.cuda.synchronize()
    msg = []
    for name, a, b in zip(("fwd", "dgrad", "wgrad"), out, ref):
        if a is None:
            continue
        err = ((a.float() - b.float()).norm() / (b.float().norm() + 1e-9)).item()
        if err > 1e-2:
            msg.append(f"{name}:{err:.3f}")
            bad.append(((ci, co, k, s, h), name))
    print(f"{str((ci, co, k, s, h)):24s} eager {ms:7.3f} ms  {'BAD ' + ' '.join(msg) if msg else 'ok'}", flush=True)
print(f"TOTAL eager {tot:.2f} ms; {len(bad)} capture-unsafe ops: {bad}")
