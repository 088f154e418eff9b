#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
( WGRAD=1 ONESX=1 timeout -k 10 60 tools/convbench/stem_bench_p0;
  WGRAD=1 ONESDY=1 timeout -k 10 60 tools/convbench/stem_bench_p0;
  WGRAD=1 ONESX=1 ONESDY=1 DUMP=1 timeout -k 10 60 tools/convbench/stem_bench_p0 ) > gpurun_out/stem_wgrad_dbg.log 2>&1
echo done
