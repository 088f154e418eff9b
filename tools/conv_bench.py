"""Per-shape ResNet-50 conv timing (batch 256, bf16, NHWC): MIOpen conv vs hipBLASLt GEMM for 1x1."""
import torch
import torch.nn.functional as F

torch.backends.cudnn.benchmark = True
B = 256
# (Cin, Cout, k, stride, H_in) for every distinct conv in ResNet-50 (v1.5) and its count
shapes = {}
def add(ci, co, k, s, h, n=1):
    shapes[(ci, co, k, s, h)] = shapes.get((ci, co, k, s, h), 0) + n
add(3, 64, 7, 2, 224)
for (w, blocks, h, ci) in [(64, 3, 56, 64), (128, 4, 56, 256), (256, 6, 28, 512), (512, 3, 14, 1024)]:
    s = 1 if w == 64 else 2
    ho = h // s
    add(ci, w, 1, 1, h); add(w, w, 3, s, h); add(w, 4 * w, 1, 1, ho); add(ci, 4 * w, 1, s, h)
    add(4 * w, w, 1, 1, ho, blocks - 1); add(w, w, 3, 1, ho, blocks - 1); add(w, 4 * w, 1, 1, ho, blocks - 1)


def t(fn, it=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it


tot_conv = tot_best = 0.0
print(f"{'shape':28s} n  conv_f  conv_bd  conv_bw | mm_f   mm_bd  mm_bw  (ms) TF/s(conv total)")
for (ci, co, k, s, h), n in sorted(shapes.items()):
    x = torch.randn(B, ci, h, h, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = torch.randn(co, ci, k, k, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    pad = k // 2
    y = F.conv2d(x, w, stride=s, padding=pad)
    gy = torch.randn_like(y)
    cf = t(lambda: F.conv2d(x, w, stride=s, padding=pad))
    cbd = t(lambda: torch.ops.aten.convolution_backward(gy, x, w, None, [s, s], [pad, pad], [1, 1], False, [0, 0], 1,
                                                          [True, False, False]))
    cbw = t(lambda: torch.ops.aten.convolution_backward(gy, x, w, None, [s, s], [pad, pad], [1, 1], False, [0, 0], 1,
                                                          [False, True, False]))
    flops = 2 * B * y.shape[2] * y.shape[3] * co * ci * k * k
    line = f"{str((ci, co, k, s, h)):28s} {n}  {cf:6.3f} {cbd:6.3f} {cbw:6.3f}"
    conv_t = cf + cbd + cbw
    best = conv_t
    if k == 1:
        xs = x[:, :, ::s, ::s] if s > 1 else x
        a = xs.permute(0, 2, 3, 1).reshape(-1, ci)
        wm = w.reshape(co, ci)
        g2 = gy.permute(0, 2, 3, 1).reshape(-1, co)
        mf = t(lambda: a @ wm.t())
        mbd = t(lambda: g2 @ wm)
        mbw = t(lambda: g2.t() @ a)
        line += f" | {mf:6.3f} {mbd:6.3f} {mbw:6.3f}"
        best = min(cf, mf) + min(cbd, mbd) + min(cbw, mbw)
    line += f"   {3 * flops / conv_t / 1e9:7.0f}"
    tot_conv += n * conv_t
    tot_best += n * best
    print(line, flush=True)
print(f"total conv ms/step: MIOpen {tot_conv:.2f}  best-of(MIOpen, GEMM for 1x1) {tot_best:.2f}")
