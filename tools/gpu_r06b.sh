set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
mkdir -p gpurun_out/r06b
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_scan.py tests/test_gpu_ingest.py > gpurun_out/r06b/tests.log 2>&1 || { tail -30 gpurun_out/r06b/tests.log; exit 1; }
tail -3 gpurun_out/r06b/tests.log
for r in 1 2 3; do for v in 1 0; do
NETC_SCAN_ONEPASS=$v timeout -k 10 120 python -u tools/bench_scan.py --steps 100 --no-cpu --workloads c2,c4 > gpurun_out/r06b/scan_op${v}_$r.log 2>&1 || exit 1
echo "op=$v round=$r"; cat gpurun_out/r06b/scan_op${v}_$r.log
done; done
