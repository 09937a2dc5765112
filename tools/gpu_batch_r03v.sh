#!/bin/bash
# Round-3 (through gpurun, from the repo root): frame assembly with non-temporal payload loads and
# stores (the default) vs plain ones (tune flags 8), the default chunk, three rounds; the same for
# the unmask + UTF-8 check (mask_sweep-style policy only applies to the mask kernels, so VAL is
# not varied here).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r03v
mkdir -p $OUT
for i in 1 2 3; do
  timeout -k 10 300 python -u tools/bench_encode.py --unroll 1 --flags=-1,8 --steps 50 > $OUT/enc_$i.jsonl 2> $OUT/enc_$i.err || { echo ENCFAIL; tail -20 $OUT/enc_$i.err; exit 1; }
  python3 -c "import json,sys; [print(sys.argv[1][-11:], d['workload'], d['flags'], d['us_per_step']) for d in map(json.loads, open(sys.argv[1]))]" $OUT/enc_$i.jsonl
done
echo done
