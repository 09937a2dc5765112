#!/bin/bash
# Round-3 (through gpurun, from the repo root): the scan + ingest GPU suites (RSV1 accepted by the
# speculative pass), then the SQ passes and the K1 experiment (tools/gpu_batch_r03d.sh).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r03e
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_scan.py tests/test_gpu_ingest.py > $OUT/scan_tests.log 2>&1 || { echo SCANTESTFAIL; grep -E "FAILED|Error|assert" $OUT/scan_tests.log | head -20; tail -20 $OUT/scan_tests.log; exit 1; }
tail -1 $OUT/scan_tests.log
timeout -k 10 300 python -u tools/bench_scan.py --rsv1 --non-strict --steps 20 > $OUT/scan_rsv1.json 2> $OUT/scan_rsv1.err || { echo RSVFAIL; tail -10 $OUT/scan_rsv1.err; exit 1; }
cat $OUT/scan_rsv1.json
bash tools/gpu_batch_r03d.sh
