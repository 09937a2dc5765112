set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
D=$R/gpurun_out/${TAG:-r06j}; mkdir -p $D
for v in 1 0; do
NETC_SCAN_ONEPASS=$v timeout -k 10 120 python -u tools/bench_scan.py --steps 100 --no-cpu --workloads c2,c4 > $D/scan_op${v}.log 2>&1 || exit 1
echo "op=$v $(grep -o '"workload": "c[24]"\|"us_per_scan": [0-9.]*\|"matches_oracle": [a-z]*\|"onepass": [a-z]*' $D/scan_op${v}.log | tr '\n' ' ')"
done
cd /tmp && export TMPDIR=/tmp
NETC_SCAN_ONEPASS=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof -o run -- python3 $R/tools/bench_scan.py --steps 20 --no-cpu --workloads c2 > $D/prof.log 2>&1 || exit 1
f=$(find $D/prof -name '*kernel_stats.csv' | head -1); cut -d, -f1-4 $f | head -6
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_scan.py tests/test_gpu_ingest.py > $D/tests.log 2>&1 || { tail -40 $D/tests.log; exit 1; }
tail -2 $D/tests.log
