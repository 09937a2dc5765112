#!/bin/bash
# Mask kernel: threads per workgroup (NETC_MASK_BLOCK) A/B at the headline workload,
# interleaved on one box.  Run through gpurun from the repo root.
# (The NETC_MASK_BLOCK launch knob was removed again with the experiment: DESIGN.md §4.)
set -o pipefail
OUT=gpurun_out/${TAG:-mblk}
mkdir -p $OUT
for rep in 1 2; do
  for bs in ${BLOCKS:-256 512 1024}; do
    NETC_MASK_BLOCK=$bs timeout -k 10 200 python3 bench.py --cpu-seconds 0 --no-copy-ceiling --no-pipelined-probe \
        > $OUT/b${bs}_$rep.json 2>> $OUT/err.txt || exit $?
    python3 -c "import json; d=json.load(open('$OUT/b${bs}_$rep.json')); print($bs, $rep, d['value'], d['roofline']['kernel_ms_mean'], d['roofline']['frac'])"
  done
done
