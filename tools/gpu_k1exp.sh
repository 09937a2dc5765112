#!/bin/bash
# K1 (scan_exits) timed alone: the product's tail (target check + atomic append) vs a plain
# per-chunk exit list (tools/libscan_k1exp.so); rocprofv3 kernel trace of bench_scan with each
# diagnostic library (their scan results are not valid: only K1 runs).
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-k1exp}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for L in k1only k1exp; do
  NETC_GPU_LIB=$R/tools/libscan_$L.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_$L -o run -- python3 $R/tools/bench_scan.py --steps 20 > $OUT/$L.log 2>&1 || { echo FAIL $L; tail -20 $OUT/$L.log; exit 1; }
  grep scan_exits $OUT/trace_$L/run_kernel_stats.csv
done
echo done
