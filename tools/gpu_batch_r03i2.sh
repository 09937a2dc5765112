#!/bin/bash
# Round-3 (through gpurun, from the repo root): the scan + ingest suites on the product build
# (K2 32 chunks per block, K4 64), bench_scan A/B of K2/K4 chunks per block (16/16, 32/32, 32/64),
# and a C2 launch-shape sweep of the headline mask kernel (load / store policies).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r03i2
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_scan.py tests/test_gpu_ingest.py tests/test_gpu_epoll.py > $OUT/tests.log 2>&1 || { echo TESTFAIL; grep -E "FAILED|Error|assert" $OUT/tests.log | head -20; tail -20 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
ln -sf ../netc_amd/lib/libnetc.so tools/libnetc.so
LIBS="tools/libs16e16.so tools/libs32e32.so tools/libs32e64.so" TOOL="tools/bench_scan.py --steps 50" ROUNDS=2 bash tools/gpu_ab_libs.sh r03i2_ab || exit 1
timeout -k 10 300 python -u tools/mask_sweep.py --workloads c2 --unroll 1,2 --flags=-1,8,9,10,11 --reps 60 > $OUT/mask_sweep_c2.jsonl 2> $OUT/mask_sweep.err || { echo SWEEPFAIL; tail -20 $OUT/mask_sweep.err; exit 1; }
cut -c1-200 $OUT/mask_sweep_c2.jsonl
echo done
