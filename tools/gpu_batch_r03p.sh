#!/bin/bash
# Round-3 (through gpurun, from the repo root): the headline mask kernel at C2 with the default
# window order (flags -1) and with XCD-grouped windows (flags 43 = NT loads + NT stores + two steps
# + XCD groups): time (tools/mask_sweep.py) and HBM bytes (FETCH_SIZE and WRITE_SIZE, each its own
# rocprofv3 --pmc pass).
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r03p
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u tools/mask_sweep.py --workloads c2 --unroll 1 --flags=-1,43,-1,43 --reps 60 > $OUT/sweep.jsonl 2> $OUT/sweep.err || { echo SWEEPFAIL; tail -20 $OUT/sweep.err; exit 1; }
cat $OUT/sweep.jsonl
cd /tmp && export TMPDIR=/tmp
for F in -1 43; do
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex "mask_np_kernel" --output-format csv -d $OUT/pmc_${C}_f$F -o run -- python3 $R/tools/mask_sweep.py --workloads c2 --unroll 1 --flags=$F --reps 10 > $OUT/pmc_${C}_f$F.log 2>&1 || { echo PMCFAIL $F $C; tail -20 $OUT/pmc_${C}_f$F.log; exit 1; }
  done
done
echo done
