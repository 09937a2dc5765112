#!/bin/bash
# GPU-box pass for the ingest ring (through gpurun, from the repo root): the ingest
# bench at two slot sizes, the scan bench, then one rocprofv3 kernel + copy trace of
# a short ingest run.  Each GPU step is time-limited; the chain stops at a failure.
set -o pipefail
R=$PWD
OUT=$R/gpurun_out/ingest_${TAG:-r01}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/bench_ingest.py > "$OUT/ingest_16.json" 2> "$OUT/ingest_16.err" || exit $?
cat "$OUT/ingest_16.json"
timeout -k 10 300 python3 tools/bench_ingest.py --slot-mib 64 > "$OUT/ingest_64.json" 2> "$OUT/ingest_64.err" || exit $?
cat "$OUT/ingest_64.json"
timeout -k 10 300 python3 tools/bench_scan.py > "$OUT/scan.json" 2> "$OUT/scan.err" || exit $?
cat "$OUT/scan.json"
cd /tmp || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 "$R/tools/bench_ingest.py" --gib 1 > "$OUT/trace.log" 2>&1 || exit $?
echo "ingest pass done: $OUT"
