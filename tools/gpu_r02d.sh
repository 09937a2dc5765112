# misaligned-path A/B + kernel-boundary gap of the headline loop (rocprofv3 kernel trace)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r02d; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py > gpurun_out/r02d/t.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/r02d/t.log; exit 1; }
tail -2 gpurun_out/r02d/t.log
for WL in c2 c3 c4; do timeout -k 10 300 python -u bench.py --workload $WL --steps 20 --warmup 5 --c5-gib 0 --cpu-seconds 0 > gpurun_out/r02d/b_$WL.json 2> gpurun_out/r02d/b_$WL.err || { echo BENCHFAIL; tail -20 gpurun_out/r02d/b_$WL.err; exit 1; }; python3 -c "
import json;d=json.load(open('gpurun_out/r02d/b_$WL.json'));r=d['roofline'];print('$WL', d['value'], d['ms_per_step'], r['kernel_ms_mean'], r['achieved'], r['shapes'], d['verified'])"; done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r02d/trace -o run -- python3 bench.py --steps 50 --warmup 5 --c5-gib 0 --cpu-seconds 0 > gpurun_out/r02d/trace_bench.json 2> gpurun_out/r02d/trace.err || { echo TRACEFAIL; tail -20 gpurun_out/r02d/trace.err; exit 1; }
T=$(find gpurun_out/r02d/trace -name '*kernel_trace.csv' | head -1)
python3 tools/kernel_gaps.py "$T" mask_np_kernel --grid 2097152 | tee gpurun_out/r02d/gaps.json
cat gpurun_out/r02d/trace_bench.json
