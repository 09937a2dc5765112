#!/bin/bash
# Round-3 final record (through gpurun, from the repo root): tools/gpu_round3.sh (the whole -m gpu
# suite, smoke, bench at C2 / C3 / C4 with rocprof traces and PMC passes, the SURVEY §8(f) rows,
# the C5 probe), then bench_validate: the product build against tools/libval_new.so.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
bash tools/gpu_round3.sh r03o || exit 1
ln -sf ../netc_amd/lib/libnetc.so tools/libnetc.so
LIBS="tools/libval_new.so tools/libval_own1.so" TOOL="tools/bench_validate.py --steps 30" ROUNDS=2 bash tools/gpu_ab_libs.sh r03o_val || exit 1
echo all done
