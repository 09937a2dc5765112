#!/bin/bash
# One GPU session for round 3's record (through gpurun, from the repo root):
#   the whole -m gpu suite; smoke(); bench.py at the driver's shape (C2, every leg) and at
#   C3 / C4; per workload a rocprofv3 kernel trace + stats of the bench command, then its
#   FETCH_SIZE and WRITE_SIZE passes on their own (tools/summarize_round.py --src TAG_wl);
#   the SURVEY §8(f) rows pass (tools/prof_rows.sh); the C5 in-place probe.
#   bash tools/gpu_round3.sh TAG
set -o pipefail
TAG=${1:-r03}
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 900 --timeout-method thread -m gpu tests > $OUT/gputest.log 2>&1 || { echo TESTFAIL; grep -E "FAILED|Error" $OUT/gputest.log | head -20; tail -30 $OUT/gputest.log; exit 1; }
  tail -2 $OUT/gputest.log
  timeout -k 10 300 python3 -c 'import __graft_entry__ as g; g.smoke()' > $OUT/smoke.log 2>&1 || { echo SMOKEFAIL; tail -20 $OUT/smoke.log; exit 1; }
  tail -1 $OUT/smoke.log
fi
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_c2_full.json 2> $OUT/bench_c2_full.err || { echo BENCHFAIL; tail -30 $OUT/bench_c2_full.err; exit 1; }
cat $OUT/bench_c2_full.json
cd /tmp && export TMPDIR=/tmp
for WL in c2 c3 c4; do
  D=$R/gpurun_out/${TAG}_$WL
  mkdir -p $D
  CMD="python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --c5-gib 0 --cpu-seconds 0 --workload $WL"
  timeout -k 10 300 $CMD > $D/bench.json 2> $D/bench.err || { echo BENCH${WL}FAIL; tail -20 $D/bench.err; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- $CMD > $D/trace.log 2>&1 || { echo TRACEFAIL; tail -20 $D/trace.log; exit 1; }
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "mask_np_kernel" --output-format csv -d $D/pmc_fetch -o run -- $CMD --no-copy-ceiling > $D/pmc_fetch.log 2>&1 || { echo FETCHFAIL; tail -20 $D/pmc_fetch.log; exit 1; }
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "mask_np_kernel" --output-format csv -d $D/pmc_write -o run -- $CMD --no-copy-ceiling > $D/pmc_write.log 2>&1 || { echo WRITEFAIL; tail -20 $D/pmc_write.log; exit 1; }
  echo "$WL profiled"
done
cd $R
[ "${ROWS:-1}" = 1 ] && { TAG=$TAG bash tools/prof_rows.sh > $OUT/rows.log 2>&1 || { echo ROWSFAIL; tail -20 $OUT/rows.log; exit 1; }; tail -3 $OUT/rows.log; }
timeout -k 10 300 python -u tools/c5_inplace_probe.py --gib 4 > $OUT/c5_inplace.json 2> $OUT/c5_inplace.err || { echo C5PFAIL; tail -20 $OUT/c5_inplace.err; exit 1; }
cat $OUT/c5_inplace.json
echo done
