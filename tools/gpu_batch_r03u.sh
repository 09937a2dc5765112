#!/bin/bash
# Round-3 (through gpurun, from the repo root): the scan / ingest / epoll suites on the product
# build (K1 plain loads up to 128 MiB, non-temporal above) and bench_scan, two rounds.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r03u
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_scan.py tests/test_gpu_ingest.py tests/test_gpu_epoll.py > $OUT/tests.log 2>&1 || { echo TESTFAIL; grep -E "FAILED|Error|assert" $OUT/tests.log | head; tail -20 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for i in 1 2; do
  timeout -k 10 300 python -u tools/bench_scan.py --steps 50 > $OUT/scan_$i.json 2> $OUT/scan_$i.err || { echo SCANFAIL; tail -20 $OUT/scan_$i.err; exit 1; }
  cut -c1-140 $OUT/scan_$i.json
done
echo done
