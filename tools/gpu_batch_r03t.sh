#!/bin/bash
# Round-3 A/B (through gpurun, from the repo root): frame scan K1 with plain 16-B loads
# (tools/libk1plain.so) against the non-temporal ones (tools/libcur.so), three rounds.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r03t
mkdir -p $OUT
ln -sf ../netc_amd/lib/libnetc.so tools/libnetc.so
NETC_GPU_LIB=tools/libk1plain.so timeout -k 10 600 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_scan.py > $OUT/tests.log 2>&1 || { echo TESTFAIL; tail -20 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
LIBS="tools/libcur.so tools/libk1plain.so" TOOL="tools/bench_scan.py --steps 50" ROUNDS=3 bash tools/gpu_ab_libs.sh r03t_ab || exit 1
echo done
