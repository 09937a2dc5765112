set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_utf8.py tests/test_gpu_scan.py tests/test_gpu_ingest.py > gpurun_out/t1.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/t1.log; exit 1; }
tail -3 gpurun_out/t1.log
for L in 0 16384 32768; do NETC_MASK_LDS=$L timeout -k 10 200 python -u tools/mask_sweep.py >> gpurun_out/sw1.jsonl 2>>gpurun_out/sw1.err || exit 1; done
timeout -k 10 200 python -u tools/mask_sweep.py --workloads c2,c4 --shift 3 --unroll 2,4 --flags=-1,11 >> gpurun_out/sw1.jsonl 2>>gpurun_out/sw1.err
