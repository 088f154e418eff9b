import sys, torch
sys.path.insert(0, "/root/repo/tests"); sys.path.insert(0, "/root/repo")
from test_bwd_alg_gpu import _deferred, _n
C4, CW = 256, 64
a, w, z, dy, bits, mean, coef = _deferred(900, C4, CW, C4 + 7)
wg = _n().conv1x1_wgrad_seg(a, dy, a)
s1 = dy.float().sum(0)
want = torch.stack((s1, -(mean * s1))).view(2, 1, C4).contiguous()
base = want.clone()
_n().bn_alg_fix_s2(want, wg, w)
got = _n().bn_alg_ds_part(s1, mean.contiguous(), wg, w)
d = (got - want).abs()
print("half0 maxdiff", float(d[0].max()), "half1 maxdiff", float(d[1].max()), "n diff", int((got != want).sum()))
i = int((got[1] != want[1]).nonzero()[0][1]) if (got[1] != want[1]).any() else -1
if i >= 0:
    print("idx", i, "got", got[1,0,i].item(), "want", want[1,0,i].item(), "base", base[1,0,i].item(), "s1", s1[i].item(), "mean", mean[i].item())
    rs = float(want[1,0,i] - base[1,0,i])
    print("want-base", rs, "got-(-mean*s1)", float(got[1,0,i]) - float(base[1,0,i]))
