#!/bin/bash
# Round-3 A/B (through gpurun, from the repo root): the frame scan's K2 / K4 with 32 chunks per
# workgroup (tools/libblk32.so) against 16 (tools/libcur.so): the scan + ingest suites on the
# 32-chunk build, bench_scan alternating, a kernel trace of each at config 4.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r03h2
mkdir -p $OUT
ln -sf ../netc_amd/lib/libnetc.so tools/libnetc.so
NETC_GPU_LIB=tools/libblk32.so timeout -k 10 600 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_scan.py tests/test_gpu_ingest.py > $OUT/tests.log 2>&1 || { echo TESTFAIL; grep -E "FAILED|Error|assert" $OUT/tests.log | head -20; tail -20 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
LIBS="tools/libcur.so tools/libblk32.so" TOOL="tools/bench_scan.py --steps 50" ROUNDS=2 bash tools/gpu_ab_libs.sh r03h2_ab || exit 1
cd /tmp && export TMPDIR=/tmp
for L in cur blk32; do
  NETC_GPU_LIB=$R/tools/lib$L.so timeout -s KILL 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_$L -o run -- python3 $R/tools/bench_scan.py --steps 20 --workloads c4 > $OUT/trace_$L.log 2>&1 || { echo TRACEFAIL; tail -20 $OUT/trace_$L.log; exit 1; }
  echo "== $L c4"; grep scan_ $OUT/trace_$L/run_kernel_stats.csv | cut -d, -f1-4
done
echo done
