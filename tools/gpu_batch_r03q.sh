#!/bin/bash
# Round-3 (through gpurun, from the repo root): the small-frame rows (tools/bench_sizes.py) and the
# N-rank launcher rehearsed on one GPU: python bench.py --gpus 2 and --gpus 4 with every rank on
# device 0 (NETC_BENCH_DEVICE=0, gloo barrier), C4 shard leg included.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r03q
mkdir -p $OUT
timeout -k 10 400 python -u tools/bench_sizes.py > $OUT/sizes.jsonl 2> $OUT/sizes.err || { echo SIZESFAIL; tail -20 $OUT/sizes.err; exit 1; }
cut -c1-220 $OUT/sizes.jsonl
for N in 2 4; do
  NETC_BENCH_DEVICE=0 NETC_BENCH_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus $N --steps 20 --warmup 5 --c5-gib 0 --cpu-seconds 0 --no-copy-ceiling > $OUT/rehearse_n$N.json 2> $OUT/rehearse_n$N.err || { echo REHFAIL $N; tail -20 $OUT/rehearse_n$N.err; exit 1; }
  tail -1 $OUT/rehearse_n$N.json | cut -c1-400
done
echo done
