# One GPU session: the whole -m gpu suite, the driver's bench command, and the profiles of it
# (rocprofv3 kernel trace + stats, then FETCH_SIZE and WRITE_SIZE passes on their own).
#   bash tools/gpu_round.sh TAG [tests|notests]
set -o pipefail
TAG=${1:-r02}
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
if [ "${2:-tests}" = tests ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 900 --timeout-method thread -m gpu tests > $OUT/gputest.log 2>&1 || { echo TESTFAIL; grep -E "FAILED|Error|error" $OUT/gputest.log | head -20; tail -30 $OUT/gputest.log; exit 1; }
  tail -2 $OUT/gputest.log
fi
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { echo BENCHFAIL; tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
cd /tmp && export TMPDIR=/tmp
PROFCMD="python3 $GRAFT_REPO_ROOT/bench.py --gpus 1 --steps 20 --warmup 5 --c5-gib 0 --cpu-seconds 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- $PROFCMD > $OUT/trace.log 2>&1 || { echo TRACEFAIL; tail -20 $OUT/trace.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "mask_np_kernel" --output-format csv -d $OUT/pmc_fetch -o run -- $PROFCMD --no-copy-ceiling > $OUT/pmc_fetch.log 2>&1 || { echo FETCHFAIL; tail -20 $OUT/pmc_fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "mask_np_kernel" --output-format csv -d $OUT/pmc_write -o run -- $PROFCMD --no-copy-ceiling > $OUT/pmc_write.log 2>&1 || { echo WRITEFAIL; tail -20 $OUT/pmc_write.log; exit 1; }
echo done
