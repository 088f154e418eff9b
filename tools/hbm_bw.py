"""HBM bandwidth of plain read / write / copy patterns on one MI355X (torch kernels), to price
write-heavy kernels (a 1x1 conv with 4x more output than input) against what the memory does.

    python tools/hbm_bw.py
"""
import torch


def t(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / reps * 1e-3


def main():
    n = 1 << 30  # 1 Gi bf16 = 2 GiB
    x = torch.empty(n, dtype=torch.bfloat16, device="cuda").normal_()
    y = torch.empty_like(x)
    q = torch.empty(n // 4, dtype=torch.bfloat16, device="cuda").normal_()
    GB = 1e9
    rows = []
    s = t(lambda: y.fill_(1.0)); rows.append(("write only (fill)", 0, 2 * n, s))
    s = t(lambda: torch.amax(x)); rows.append(("read only (amax)", 2 * n, 0, s))
    s = t(lambda: y.copy_(x)); rows.append(("copy 1:1", 2 * n, 2 * n, s))
    s = t(lambda: y.view(-1, 4, 256).copy_(q.view(-1, 1, 256).expand(-1, 4, 256)))
    rows.append(("read 1 : write 4 (broadcast copy)", 2 * n // 4, 2 * n, s))
    s = t(lambda: torch.add(x, x, out=y)); rows.append(("read 1 (same tensor twice) : write 1", 2 * n, 2 * n, s))
    print(f"{'pattern':<40}{'GB read':>9}{'GB write':>9}{'us':>9}{'TB/s':>7}")
    for name, r, w, s in rows:
        print(f"{name:<40}{r / GB:9.2f}{w / GB:9.2f}{s * 1e6:9.1f}{(r + w) / s / 1e12:7.2f}")


if __name__ == "__main__":
    main()
