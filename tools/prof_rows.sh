#!/bin/bash
# GPU-box profiling pass for the SURVEY.md §8(f) rows (through gpurun, from the repo
# root): for each tool -- frame assembly, fused unmask + UTF-8, frame scan -- the
# bench JSON, one rocprofv3 --kernel-trace --stats run, and two separate --pmc passes
# (FETCH_SIZE, then WRITE_SIZE) of the same command; then the C5 host stream.
# Every GPU step is time-limited; the chain stops at the first failure.
set -o pipefail
R=$PWD
OUT=$R/gpurun_out/rows_${TAG:-r01}
mkdir -p "$OUT"
export TMPDIR=/tmp
run_tool() {   # name, regex, args...
    local name=$1 rx=$2
    shift 2
    timeout -k 10 300 python3 "$R/tools/$name.py" "$@" > "$OUT/$name.json" 2> "$OUT/$name.err" || return $?
    cat "$OUT/$name.json"
    (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_$name" -o run -- \
        python3 "$R/tools/$name.py" "$@" > "$OUT/trace_$name.log" 2>&1) || return $?
    (cd /tmp && timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$rx" --output-format csv \
        -d "$OUT/pmc_fetch_$name" -o run -- python3 "$R/tools/$name.py" "$@" > "$OUT/pmc_fetch_$name.log" 2>&1) || return $?
    (cd /tmp && timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$rx" --output-format csv \
        -d "$OUT/pmc_write_$name" -o run -- python3 "$R/tools/$name.py" "$@" > "$OUT/pmc_write_$name.log" 2>&1) || return $?
}
run_tool bench_encode "encode|wire_offsets" --steps 50 --unroll 1 --entry scan,class || exit $?   # the default shapes
run_tool bench_validate "mask_np_kernel|utf8" --steps 30 || exit $?
run_tool bench_scan "scan_" --steps 20 || exit $?
timeout -k 10 400 python3 tools/bench_stream.py > "$OUT/bench_stream.json" 2> "$OUT/bench_stream.err" || exit $?
cat "$OUT/bench_stream.json"
echo "rows pass done: $OUT"
