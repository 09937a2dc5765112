#!/bin/bash
# Round-3 A/B (through gpurun, from the repo root): the unmask + UTF-8 kernel with plain payload
# loads and stores (tools/libvalplain.so) against the non-temporal default (tools/libvalnt.so):
# UTF-8 suite on plain, bench_validate alternating, three rounds.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r03w
mkdir -p $OUT
ln -sf ../netc_amd/lib/libnetc.so tools/libnetc.so
NETC_GPU_LIB=tools/libvalplain.so timeout -k 10 600 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_utf8.py > $OUT/tests.log 2>&1 || { echo TESTFAIL; tail -20 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
LIBS="tools/libvalnt.so tools/libvalplain.so" TOOL="tools/bench_validate.py --steps 30" ROUNDS=3 bash tools/gpu_ab_libs.sh r03w_ab || exit 1
echo done
