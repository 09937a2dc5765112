#!/bin/bash
# Round-3 (through gpurun, from the repo root): the whole -m gpu suite and smoke on the final build
# (frame assembly's default chunk by batch size), then bench_encode at the default (unroll 1).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r03s
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 900 --timeout-method thread -m gpu tests > $OUT/gputest.log 2>&1 || { echo TESTFAIL; grep -E "FAILED|Error" $OUT/gputest.log | head -20; tail -30 $OUT/gputest.log; exit 1; }
tail -1 $OUT/gputest.log
timeout -k 10 300 python3 -c 'import __graft_entry__ as g; g.smoke()' > $OUT/smoke.log 2>&1 || { echo SMOKEFAIL; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
for i in 1 2; do
  timeout -k 10 300 python -u tools/bench_encode.py --unroll 1 --steps 50 > $OUT/enc_$i.jsonl 2> $OUT/enc_$i.err || { echo ENCFAIL; tail -20 $OUT/enc_$i.err; exit 1; }
  cut -c1-160 $OUT/enc_$i.jsonl
done
echo done
