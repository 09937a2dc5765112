# GPU session for frame assembly: its parity suite, the C2/C4 encode bench, the small-frame
# sizes, and a kernel trace of the encode bench.
#   bash tools/gpu_encode.sh TAG
set -o pipefail
TAG=${1:-enc}
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_encode.py > $OUT/t.log 2>&1 || { echo TESTFAIL; grep -E "FAILED|Error|assert" $OUT/t.log | head -20; tail -30 $OUT/t.log; exit 1; }
tail -2 $OUT/t.log
timeout -k 10 300 python -u tools/bench_encode.py > $OUT/bench_encode.jsonl 2> $OUT/bench_encode.err || { echo BENCHFAIL; tail -20 $OUT/bench_encode.err; exit 1; }
cat $OUT/bench_encode.jsonl
timeout -k 10 300 python -u tools/bench_sizes.py --sizes 16,64,256,1024,4096 > $OUT/sizes.jsonl 2> $OUT/sizes.err || { echo SIZESFAIL; tail -20 $OUT/sizes.err; exit 1; }
cat $OUT/sizes.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_encode.py --steps 20 > $OUT/trace.log 2>&1 || { echo TRACEFAIL; tail -20 $OUT/trace.log; exit 1; }
echo done
