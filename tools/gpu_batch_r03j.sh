#!/bin/bash
# Round-3 A/B (through gpurun, from the repo root): the merged K3a + K3b launch up to 512 tiles
# with both rounds of tile records in the first trip (tools/libm512.so) against the merge up to
# 256 tiles (tools/libs32e64.so, separate launches at config 4): scan suite, bench_scan, C4 trace.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r03j
mkdir -p $OUT
ln -sf ../netc_amd/lib/libnetc.so tools/libnetc.so
NETC_GPU_LIB=tools/libm512.so timeout -k 10 600 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_scan.py > $OUT/tests.log 2>&1 || { echo TESTFAIL; grep -E "FAILED|Error|assert" $OUT/tests.log | head -20; tail -20 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
LIBS="tools/libs32e64.so tools/libm512.so" TOOL="tools/bench_scan.py --steps 50" ROUNDS=2 bash tools/gpu_ab_libs.sh r03j_ab || exit 1
cd /tmp && export TMPDIR=/tmp
for L in s32e64 m512; do
  NETC_GPU_LIB=$R/tools/lib$L.so timeout -s KILL 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_$L -o run -- python3 $R/tools/bench_scan.py --steps 20 --workloads c4 > $OUT/trace_$L.log 2>&1 || { echo TRACEFAIL; tail -20 $OUT/trace_$L.log; exit 1; }
  echo "== $L c4"; grep scan_ $OUT/trace_$L/run_kernel_stats.csv | cut -d, -f1-4
done
cd $R
timeout -k 10 300 python -u tools/mask_sweep.py --workloads c2 --unroll 1,2 --flags=-1,8,9,10,11 --reps 60 > $OUT/mask_sweep_c2.jsonl 2> $OUT/mask_sweep.err || { echo SWEEPFAIL; tail -20 $OUT/mask_sweep.err; exit 1; }
cut -c1-200 $OUT/mask_sweep_c2.jsonl
echo done
