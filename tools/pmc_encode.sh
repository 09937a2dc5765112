#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of the frame assembly at config 2 per environment variant (through gpurun,
# repo root): VARIANTS="NETC_ENC_PROBE=0 -" TAG=... bash tools/pmc_encode.sh
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
        -d $OUT/v${i}_$c -o run -- python3 $R/tools/bench_encode.py --steps 20 --warmup 5 --workloads c2 --unroll 1 > $OUT/v${i}_$c.log 2>&1) || { echo PMCFAIL $V $c; tail -5 $OUT/v${i}_$c.log; exit 1; }
  done
  echo "$i $V" >> $OUT/variants.txt
done
echo done
