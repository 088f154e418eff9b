#!/bin/bash
# Kernel-name coverage gate: the GPU test tier under rocprofv3 --kernel-trace, then which kernels of the
# committed steady-state ResNet-50 step window (profiles/r6/steady_resnet50_b1024_final_kernels.csv) no test
# launched (tools/kernel_coverage.py). Report -> gpurun_out/kernel_coverage_resnet50.md.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf /tmp/p_cov; mkdir -p /tmp/p_cov
timeout -k 10 900 rocprofv3 --kernel-trace --output-format csv -d /tmp/p_cov -o cov -- python3 -m pytest tests -m gpu -q \
  -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t_cov.log 2>&1
rc=$?; echo "gpu tier under rocprof rc=$rc"; tail -3 gpurun_out/t_cov.log; [ $rc -eq 0 ] || exit $rc
python3 - <<'PY'
import csv, glob
rows = set()
for f in glob.glob("/tmp/p_cov/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        rows.add(r["Kernel_Name"])
with open("gpurun_out/cov_kernel_names.csv", "w", newline="") as f:
    w = csv.writer(f); w.writerow(["Kernel_Name"])
    for n in sorted(rows): w.writerow([n])
print(len(rows), "distinct kernels launched by the GPU tests")
PY
# profiles/ is gpurun-ignored (does not travel to the box): the gate runs where the step window is
if [ -f profiles/r6/steady_resnet50_b1024_final_kernels.csv ]; then
  python3 tools/kernel_coverage.py gpurun_out/cov_kernel_names.csv profiles/r6/steady_resnet50_b1024_final_kernels.csv \
    --out gpurun_out/kernel_coverage_resnet50.md
else
  echo "step window not here: run  python3 tools/kernel_coverage.py gpurun_out/cov_kernel_names.csv profiles/r6/steady_resnet50_b1024_final_kernels.csv  locally"
fi
