"""One-off negative check of tests/test_models_gpu.py::test_resnet50_fp32_native_matches_fp64_oracle: the same check
with ONE channel of one BatchNorm's backward made wrong (a hook zeroes channel 5 of layer3.2.bn1's input gradient:
one of 256 channels dropped) must FAIL. Prints both verdicts.

    python tools/oracle_negative_check.py
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from test_models_gpu import check_fp32_native_against_fp64  # noqa: E402


def corrupt(m):
    bn = m.layer3[2].bn1

    def hook(module, gin, gout):
        g = gin[0]
        if g is None:
            return None
        g = g.clone()
        g[:, 5] = 0
        return (g,) + tuple(gin[1:])
    bn.register_full_backward_hook(hook)


ok, msg = check_fp32_native_against_fp64()
print("clean:", "PASS" if ok else "FAIL", msg, flush=True)
ok2, msg2 = check_fp32_native_against_fp64(corrupt)
print("one wrong channel in layer3.2.bn1's backward:", "PASS (check has no power!)" if ok2 else "FAIL (as it must)",
      msg2, flush=True)
sys.exit(0 if ok and not ok2 else 1)
