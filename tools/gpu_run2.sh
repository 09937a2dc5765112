# GPU session: C5 parity tests, the mask parity suite, then the bench (driver shape) + rocprof of it.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 900 --timeout-method thread -m gpu tests/test_gpu_stream.py > gpurun_out/t2_stream.log 2>&1 || { echo STREAMFAIL; tail -40 gpurun_out/t2_stream.log; exit 1; }
grep -E "C5|passed|failed" gpurun_out/t2_stream.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/b2.json 2> gpurun_out/b2.err || { echo BENCHFAIL; tail -30 gpurun_out/b2.err; exit 1; }
cat gpurun_out/b2.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof2 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 50 --warmup 5 --c5-gib 0 --cpu-seconds 0 > $GRAFT_REPO_ROOT/gpurun_out/prof2.log 2>&1 || { echo PROFFAIL; tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof2.log; exit 1; }
echo done
