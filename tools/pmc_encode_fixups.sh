#!/bin/bash
# where the frame assembly's excess counter traffic comes from at config 2.
# FETCH_SIZE and WRITE_SIZE (separate passes) and a kernel trace per variant (through gpurun,
# repo root):  class entry -- default, ENC_FIX=2 (header vectors by the assembly wavefronts after
# their windows), plain loads / stores (tune flags 8); general entry -- default, and the
# diagnostic build without header fixups (diag/libnetc_ws_gpu_nofix.so: wrong wire bytes, its
# parity check fails by design).
set -o pipefail
R=$PWD
OUT=$R/gpurun_out/${TAG:-r06_encfix}
mkdir -p $OUT
export TMPDIR=/tmp
run() {   # name, env, bench args
  local n=$1 e=$2; shift 2
  for c in FETCH_SIZE WRITE_SIZE; do
    (cd /tmp && env $e timeout -s KILL 200 rocprofv3 --pmc $c --kernel-include-regex "encode|wire_offsets" --output-format csv \
        -d $OUT/${n}_$c -o run -- python3 $R/tools/bench_encode.py --steps 20 --warmup 5 --workloads c2 --unroll 1 "$@" > $OUT/${n}_$c.log 2>&1) || [ "$n" = nofix ] || { echo PMCFAIL $n $c; tail -5 $OUT/${n}_$c.log; exit 1; }
  done
  (cd /tmp && env $e timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${n}_trace -o run -- \
      python3 $R/tools/bench_encode.py --steps 20 --warmup 5 --workloads c2 --unroll 1 "$@" > $OUT/${n}_trace.log 2>&1) || [ "$n" = nofix ] || { echo TRACEFAIL $n; exit 1; }
  echo "ran $n"
}
run class_default "X=1" --entry class
run class_fix2 "NETC_ENC_FIX=2" --entry class
run class_plain "X=1" --entry class --flags 8
run scan_default "X=1" --entry scan
run nofix "NETC_GPU_LIB=$R/diag/libnetc_ws_gpu_nofix.so" --entry scan
echo done
