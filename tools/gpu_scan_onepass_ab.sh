#!/bin/bash
# The frame scan's one-pass path against the graph path (NETC_SCAN_ONEPASS=1 / 0): -m gpu scan and
# ingest tests, three interleaved bench_scan rounds at config 2 and 4 shapes, and a kernel trace of
# each path at config 2 (through gpurun, repo root)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
D=$R/gpurun_out/${TAG:-r06_onepass}; mkdir -p $D
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_scan.py tests/test_gpu_ingest.py > $D/tests.log 2>&1 || { tail -40 $D/tests.log; exit 1; }
tail -1 $D/tests.log
for r in 1 2 3; do for v in 1 0; do
NETC_SCAN_ONEPASS=$v timeout -k 10 120 python -u tools/bench_scan.py --steps 100 --no-cpu --workloads c2,c4 > $D/scan_op${v}_r$r.log 2>&1 || exit 1
echo "op=$v r=$r $(grep -o '"workload": "c[24]"\|"us_per_scan": [0-9.]*\|"matches_oracle": [a-z]*\|"onepass": [a-z]*' $D/scan_op${v}_r$r.log | tr '\n' ' ')"
done; done
cd /tmp && export TMPDIR=/tmp
for v in 1 0; do
NETC_SCAN_ONEPASS=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof_op$v -o run -- python3 $R/tools/bench_scan.py --steps 20 --no-cpu --workloads c2 > $D/prof_op$v.log 2>&1 || exit 1
f=$(find $D/prof_op$v -name '*kernel_stats.csv' | head -1); echo "op=$v"; cut -d, -f1-4 $f | grep scan_
done
