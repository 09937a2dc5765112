#!/bin/bash
# rocprofv3 kernel trace of tools/bench_encode.py at config-2 shape (per-kernel durations
# of the assembly's launches); from the repo root, through gpurun
set -o pipefail
R=$PWD
OUT=$R/gpurun_out/trace_enc_${TAG:-x}
mkdir -p "$OUT"
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- \
    python3 "$R/tools/bench_encode.py" --workloads ${WL:-c2} --unroll 4 --steps 50 > "$OUT/bench.log" 2>&1) || exit $?
f=$(find "$OUT" -name '*kernel_stats.csv' | head -1)
cat "$f" | cut -d, -f1-8 | head -20
