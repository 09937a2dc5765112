# One GPU session for a round's record (through gpurun, from the repo root):
#   the whole -m gpu suite; bench.py at the driver's shape (C2) and at C3 / C4 (CPU
#   baselines included); rocprofv3 kernel trace + stats of the C2 command, then its
#   FETCH_SIZE and WRITE_SIZE passes on their own; the SURVEY §8(f) rows pass.
#   bash tools/gpu_round2.sh TAG
set -o pipefail
TAG=${1:-r02}
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 900 --timeout-method thread -m gpu tests > $OUT/gputest.log 2>&1 || { echo TESTFAIL; grep -E "FAILED|Error" $OUT/gputest.log | head -20; tail -30 $OUT/gputest.log; exit 1; }
tail -2 $OUT/gputest.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { echo BENCHFAIL; tail -30 $OUT/bench_c2.err; exit 1; }
cat $OUT/bench_c2.json
for WL in c3 c4; do
  timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --workload $WL --c5-gib 0 > $OUT/bench_$WL.json 2> $OUT/bench_$WL.err || { echo BENCH${WL}FAIL; tail -30 $OUT/bench_$WL.err; exit 1; }
  cat $OUT/bench_$WL.json
done
cd /tmp && export TMPDIR=/tmp
PROFCMD="python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --c5-gib 0 --cpu-seconds 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- $PROFCMD > $OUT/trace.log 2>&1 || { echo TRACEFAIL; tail -20 $OUT/trace.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "mask_np_kernel" --output-format csv -d $OUT/pmc_fetch -o run -- $PROFCMD --no-copy-ceiling > $OUT/pmc_fetch.log 2>&1 || { echo FETCHFAIL; tail -20 $OUT/pmc_fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "mask_np_kernel" --output-format csv -d $OUT/pmc_write -o run -- $PROFCMD --no-copy-ceiling > $OUT/pmc_write.log 2>&1 || { echo WRITEFAIL; tail -20 $OUT/pmc_write.log; exit 1; }
[ "${ROWS:-1}" = 0 ] && { echo done; exit 0; }
cd $R && TAG=$TAG bash tools/prof_rows.sh > $OUT/rows.log 2>&1 || { echo ROWSFAIL; tail -20 $OUT/rows.log; exit 1; }
tail -3 $OUT/rows.log
echo done
