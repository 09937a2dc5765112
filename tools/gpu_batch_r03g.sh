#!/bin/bash
# Round-3 A/B (through gpurun, from the repo root): the scan, ingest and UTF-8 suites on the
# product build (round-2 K1, K3a + K3b merged, DPP carry in the UTF-8 check); bench_scan against
# the build before the merge (tools/libk1_prev.so), bench_validate against the build before the
# DPP carry (tools/libk3m.so), and the SQ wait counters of both validate builds.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r03g
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_scan.py tests/test_gpu_ingest.py tests/test_gpu_utf8.py > $OUT/tests.log 2>&1 || { echo TESTFAIL; grep -E "FAILED|Error|assert" $OUT/tests.log | head -20; tail -20 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
ln -sf ../netc_amd/lib/libnetc.so tools/libnetc.so
LIBS="tools/libk1_prev.so tools/libcur.so" TOOL="tools/bench_scan.py --steps 50" ROUNDS=2 bash tools/gpu_ab_libs.sh r03g_scan || exit 1
LIBS="tools/libk3m.so tools/libcur.so" TOOL="tools/bench_validate.py --steps 30" ROUNDS=2 bash tools/gpu_ab_libs.sh r03g_val || exit 1
cd /tmp && export TMPDIR=/tmp
C2="SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY"
for L in k3m cur; do
  NETC_GPU_LIB=$R/tools/lib$L.so timeout -s KILL 120 rocprofv3 --pmc $C2 --kernel-include-regex "mask_np_kernel|utf8" --output-format csv -d $OUT/sq_$L -o run -- \
      python3 $R/tools/bench_validate.py --steps 5 > $OUT/sq_$L.log 2>&1 || { echo SQFAIL $L; tail -20 $OUT/sq_$L.log; exit 1; }
done
NETC_GPU_LIB=$R/tools/libcur.so timeout -s KILL 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_scan -o run -- python3 $R/tools/bench_scan.py --steps 20 --workloads c2 > $OUT/trace_scan.log 2>&1 || { echo TRACEFAIL; tail -20 $OUT/trace_scan.log; exit 1; }
grep scan_ $OUT/trace_scan/run_kernel_stats.csv | cut -d, -f1-4
cd $R && python3 tools/summarize_sq.py gpurun_out/r03g
echo done
