#!/bin/bash
# Round-3 (through gpurun, from the repo root): frame assembly with 2 KiB vs 4 KiB chunks
# (netc_gpu_tune unroll 4 vs 8), config 2 and config 4, three rounds.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r03r
mkdir -p $OUT
for i in 1 2 3; do
  timeout -k 10 300 python -u tools/bench_encode.py --unroll 4,8 --steps 50 > $OUT/enc_$i.jsonl 2> $OUT/enc_$i.err || { echo ENCFAIL; tail -20 $OUT/enc_$i.err; exit 1; }
  python3 -c "import json,sys; [print(sys.argv[1], d['workload'], d['unroll'], d['us_per_step']) for d in map(json.loads, open(sys.argv[1]))]" $OUT/enc_$i.jsonl
done
echo done
