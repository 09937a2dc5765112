set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/mis
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_utf8.py tests/test_gpu_scan.py > gpurun_out/mis/t.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/mis/t.log; exit 1; }
tail -2 gpurun_out/mis/t.log
for WL in c2 c3 c4; do timeout -k 10 300 python -u bench.py --workload $WL --steps 20 --warmup 5 --c5-gib 0 --cpu-seconds 0 > gpurun_out/mis/b_$WL.json 2> gpurun_out/mis/b_$WL.err || { echo BENCHFAIL; tail -20 gpurun_out/mis/b_$WL.err; exit 1; }; python3 -c "
import json;d=json.load(open('gpurun_out/mis/b_$WL.json'));r=d['roofline'];print('$WL', r['achieved'], r['shapes'], d['verified'])"; done
