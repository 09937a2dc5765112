#!/bin/bash
# GPU-box check pass (run through gpurun from the repo root).
#   STEPS  space-separated steps, run in order: a test file (tests/*.py), "smoke"
#          (__graft_entry__.smoke()), "bench" (bench.py, args in BENCH_ARGS), or a
#          tool script (tools/*.py, args in TOOL_ARGS)
#   TAG    output directory suffix (gpurun_out/check_$TAG)
# Every GPU step has its own time limit; the chain stops at the first failure and
# nothing else touches the GPU after it.
set -o pipefail
R=$PWD
OUT=$R/gpurun_out/check_${TAG:-r01}
mkdir -p "$OUT"
export TMPDIR=/tmp
STEPS=${STEPS:-"tests/test_gpu_parity.py smoke bench"}
for s in $STEPS; do
    echo "== $s"
    name=$(basename "$s" .py)
    case "$s" in
    smoke)
        timeout -k 10 300 python3 -c 'import __graft_entry__ as g; g.smoke()' > "$OUT/smoke.log" 2>&1
        rc=$?
        tail -3 "$OUT/smoke.log" ;;
    bench)
        timeout -k 10 400 python3 bench.py ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err"
        rc=$?
        cat "$OUT/bench.json"; tail -3 "$OUT/bench.err" ;;
    tests|tests/*)
        timeout -k 10 ${SUITE_TIMEOUT:-400} python3 -u -m pytest "$s" -m gpu -x -v --timeout 120 --timeout-method thread \
            > "$OUT/$name.log" 2>&1
        rc=$?
        tail -3 "$OUT/$name.log" ;;
    *)
        timeout -k 10 ${TOOL_TIMEOUT:-300} python3 -u "$s" ${TOOL_ARGS:-} > "$OUT/$name.json" 2> "$OUT/$name.err"
        rc=$?
        cat "$OUT/$name.json"; tail -3 "$OUT/$name.err" ;;
    esac
    [ $rc -eq 0 ] || { echo "step $s failed rc=$rc"; exit $rc; }
done
echo "check pass done: $OUT"
