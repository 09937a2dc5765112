#!/bin/bash
# Round-3 A/B (through gpurun, from the repo root): the UTF-8 check out of place with each window
# checking its own first bytes (utf8_messages skips the seams) and 8 waves per SIMD for one-step
# windows (tools/libval_own.so = the product build) against tools/libval_new.so: the UTF-8 and
# ingest suites, bench_validate alternating, a kernel trace.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r03n
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_utf8.py tests/test_gpu_ingest.py tests/test_gpu_parity.py > $OUT/tests.log 2>&1 || { echo TESTFAIL; grep -E "FAILED|Error|assert" $OUT/tests.log | head -20; tail -20 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
ln -sf ../netc_amd/lib/libnetc.so tools/libnetc.so
LIBS="tools/libval_new.so tools/libval_own.so" TOOL="tools/bench_validate.py --steps 30" ROUNDS=2 bash tools/gpu_ab_libs.sh r03n_ab || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/tools/bench_validate.py --steps 10 > $OUT/trace.log 2>&1 || { echo TRACEFAIL; tail -20 $OUT/trace.log; exit 1; }
grep -E "utf8|mask_np" $OUT/trace/run_kernel_stats.csv | cut -d, -f1-4
echo done
