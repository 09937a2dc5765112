#!/bin/bash
# GPU-box profiling pass for one round (run through gpurun from the repo root):
#   1. bench.py (default workload) -> gpurun_out/bench_<wl>.json
#   2. rocprofv3 --kernel-trace --stats of the same bench command (CPU leg off)
#   3. two separate rocprofv3 --pmc passes: FETCH_SIZE, then WRITE_SIZE (TCC slots
#      cannot hold both; MI355X_MICROARCH.md "rocprofv3 PMC slots")
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
R=$PWD
OUT=$R/gpurun_out/prof_${TAG:-r01}
mkdir -p "$OUT"
WL=${WL:-c2}
STEPS=${STEPS:-200}
export TMPDIR=/tmp
timeout -k 10 400 python3 bench.py --workload $WL --steps $STEPS --warmup 20 > "$OUT/bench_$WL.json" 2> "$OUT/bench_$WL.err" || exit $?
cd /tmp || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_$WL" -o run -- \
    python3 "$R/bench.py" --workload $WL --steps $STEPS --warmup 20 --cpu-seconds 0 --no-copy-ceiling --no-pipelined-probe \
    > "$OUT/trace_$WL.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex mask_frames --output-format csv -d "$OUT/pmc_fetch_$WL" -o run -- \
    python3 "$R/bench.py" --workload $WL --steps 30 --warmup 5 --cpu-seconds 0 --no-copy-ceiling --no-pipelined-probe \
    > "$OUT/pmc_fetch_$WL.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex mask_frames --output-format csv -d "$OUT/pmc_write_$WL" -o run -- \
    python3 "$R/bench.py" --workload $WL --steps 30 --warmup 5 --cpu-seconds 0 --no-copy-ceiling --no-pipelined-probe \
    > "$OUT/pmc_write_$WL.log" 2>&1 || exit $?
echo "profile pass done: $OUT"
