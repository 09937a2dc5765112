set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
D=gpurun_out/r06e; mkdir -p $D
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_scan.py tests/test_gpu_ingest.py > $D/tests.log 2>&1 || { tail -40 $D/tests.log; exit 1; }
tail -3 $D/tests.log
for r in 1 2 3; do for v in 1 0; do
NETC_SCAN_ONEPASS=$v timeout -k 10 120 python -u tools/bench_scan.py --steps 100 --no-cpu --workloads c2,c4 > $D/scan_op${v}_$r.log 2>&1 || exit 1
echo "op=$v r=$r $(grep -o '"workload": "c[24]"\|"us_per_scan": [0-9.]*\|"matches_oracle": [a-z]*\|"onepass": [a-z]*' $D/scan_op${v}_$r.log | tr '\n' ' ')"
done; done
