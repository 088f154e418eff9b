#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PROBE=1
for b in tools/convbench/conv3x3_bench_c*; do echo "== $b"; timeout -k 5 60 $b 20 2>&1 | grep -E "N= 512|skip.*512" || true; done
