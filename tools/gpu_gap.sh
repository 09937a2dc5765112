set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/gap; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gap/trace -o run -- python3 bench.py --steps 50 --warmup 5 --c5-gib 0 --cpu-seconds 0 > gpurun_out/gap/bench.json 2> gpurun_out/gap/trace.err || { echo TRACEFAIL; tail -20 gpurun_out/gap/trace.err; exit 1; }
T=$(find gpurun_out/gap/trace -name '*kernel_trace.csv' | head -1)
python3 tools/kernel_gaps.py "$T" mask_np_kernel --grid 2097152 | tee gpurun_out/gap/gaps.json
