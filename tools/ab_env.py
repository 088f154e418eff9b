"""A/B of environment switches inside ONE process (same box, same warm caches): builds the bench
workload once per configuration and times it, cycling the configurations ``--reps`` times.

    python tools/ab_env.py --configs 'off:PDT_CONV1X1_OURS=none,PDT_CONV_BN_STATS=0' 'on:' [bench args]
"""
from __future__ import annotations

import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from pytorch_distributed_training_example_amd.config import SW  # noqa: E402


def apply_env(base: dict, env: dict) -> None:
    """Make a configuration's switches live: the PDT_* switches are read ONCE into config.SW (and a
    few decisions are cached per process), so editing os.environ alone changes nothing. Re-read SW,
    forget the per-shape 1x1 conv decisions (re-seeded from the table under the new switches) and
    re-read the import-time ResNet switch."""
    os.environ.clear()
    os.environ.update(base)
    os.environ.update(env)
    SW.reload()
    from pytorch_distributed_training_example_amd.ops import conv as conv_ops
    from pytorch_distributed_training_example_amd.models import resnet
    conv_ops._CHOICE.clear()
    conv_ops._TABLE_LOADED[0] = False
    resnet.DS_DEFER_APPLY[0] = os.environ.get("PDT_DS_DEFER", "1") != "0"
    resnet.PREP_WEIGHTS[0] = os.environ.get("PDT_PREP_WEIGHTS", "1") != "0"
    resnet.DS_FUSED_BWD[0] = os.environ.get("PDT_DS_FUSED_BWD", "1") != "0"
    from pytorch_distributed_training_example_amd.ops._native import native
    n = native()
    if hasattr(n, "conv1x1_persist"):
        n.conv1x1_persist(-1)  # re-read PDT_CONV1X1_PERSIST (the C side caches it)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", nargs="+", required=True, help="name:VAR=val;VAR=val")
    ap.add_argument("--reps", type=int, default=2)
    a, rest = ap.parse_known_args()
    args = bench.parse(rest)
    ctx = bench.setup(args)
    base = dict(os.environ)
    cfgs = []
    for c in a.configs:
        name, _, kv = c.partition(":")
        env = dict(p.split("=", 1) for p in kv.split(";") if p)
        cfgs.append((name, env))
    res = {n: [] for n, _ in cfgs}
    for rep in range(a.reps):
        for name, env in cfgs:
            apply_env(base, env)
            r = bench.run(args, ctx)
            res[name].append(r["value"])
            print(f"[ab] rep {rep} {name:>12}: {r['value']:9.1f} {r['config'].get('model')} "
                  f"{r['ms_per_step']:.3f} ms/step", flush=True)
            torch.cuda.empty_cache()
    for name, v in res.items():
        print(f"[ab] {name:>12}: " + " ".join(f"{x:.1f}" for x in v) + f"  best {max(v):.1f}", flush=True)


if __name__ == "__main__":
    main()
