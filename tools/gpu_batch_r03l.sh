#!/bin/bash
# Round-3 (through gpurun, from the repo root): the fused unmask + UTF-8 window as 1, 2 or 4
# steps (knob VAL_STEPS), bench_validate each, two rounds.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r03l
mkdir -p $OUT
for i in 1 2; do
  for S in 1 2 4; do
    NETC_VAL_STEPS=$S timeout -k 10 300 python -u tools/bench_validate.py --steps 30 > $OUT/val_s${S}_$i.json 2> $OUT/val_s${S}_$i.err || { echo VALFAIL; tail -20 $OUT/val_s${S}_$i.err; exit 1; }
    echo "== steps $S round $i"; cut -c1-200 $OUT/val_s${S}_$i.json
  done
done
echo done
