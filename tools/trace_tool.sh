#!/bin/bash
# GPU-box kernel trace of one tool run (through gpurun, from the repo root):
#   TOOL=tools/<x>.py ARGS="..." TAG=... -> gpurun_out/trace_<TAG>/ (rocprofv3 --kernel-trace --stats)
set -o pipefail
R=$PWD
OUT=$R/gpurun_out/trace_${TAG:-r01}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- \
    python3 "$R/$TOOL" $ARGS > "$OUT/run.log" 2>&1 || exit $?
tail -3 "$OUT/run.log"
