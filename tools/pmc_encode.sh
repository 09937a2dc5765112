#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of the frame assembly at config 2 per environment variant (through gpurun,
# repo root): VARIANTS="NETC_ENC_PROBE=0 -" TAG=... bash tools/pmc_encode.sh
# ENTRY=class: netc_gpu_encode_frames_class (bench_encode.py --entry); TRACE=1 adds a --kernel-trace --stats pass
set -o pipefail
R=$PWD
OUT=$R/gpurun_out/${TAG:-pmc_encode}
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for V in ${VARIANTS:--}; do
  i=$((i + 1))
  ENVS=()
  [ "$V" != "-" ] && IFS=',' read -ra ENVS <<< "$V"
  for c in FETCH_SIZE WRITE_SIZE; do
    (cd /tmp && env "${ENVS[@]}" timeout -s KILL 200 rocprofv3 --pmc $c --kernel-include-regex "encode|wire_offsets" --output-format csv \
        -d $OUT/v${i}_$c -o run -- python3 $R/tools/bench_encode.py --steps 20 --warmup 5 --workloads c2 --unroll 1 --entry ${ENTRY:-scan} > $OUT/v${i}_$c.log 2>&1) || { echo PMCFAIL $V $c; tail -5 $OUT/v${i}_$c.log; exit 1; }
  done
  if [ -n "$TRACE" ]; then
    (cd /tmp && env "${ENVS[@]}" timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/v${i}_trace -o run -- \
        python3 $R/tools/bench_encode.py --steps 20 --warmup 5 --workloads c2 --unroll 1 --entry ${ENTRY:-scan} > $OUT/v${i}_trace.log 2>&1) || { echo TRACEFAIL $V; exit 1; }
  fi
  echo "$i $V" >> $OUT/variants.txt
done
echo done
