#!/bin/bash
# tools/pmc_shapes.py per source shift under separate FETCH_SIZE / WRITE_SIZE passes (through gpurun, repo root)
set -o pipefail
R=$PWD
OUT=$R/gpurun_out/${TAG:-pmc_shapes}
mkdir -p $OUT
export TMPDIR=/tmp
for s in 0 3 8; do
  (cd /tmp && timeout -k 10 200 python3 $R/tools/pmc_shapes.py --shift $s > $OUT/bench_$s.json 2> $OUT/bench_$s.err) || { echo BENCHFAIL $s; tail -5 $OUT/bench_$s.err; exit 1; }
  cat $OUT/bench_$s.json
  for c in FETCH_SIZE WRITE_SIZE; do
    (cd /tmp && timeout -s KILL 150 rocprofv3 --pmc $c --kernel-include-regex mask_np_kernel --output-format csv -d $OUT/pmc_${c}_$s -o run -- python3 $R/tools/pmc_shapes.py --shift $s > $OUT/pmc_${c}_$s.log 2>&1) || { echo PMCFAIL $s $c; tail -5 $OUT/pmc_${c}_$s.log; exit 1; }
  done
done
echo done
