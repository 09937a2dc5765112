#!/bin/bash
# Round-3 (through gpurun, from the repo root): the scan + ingest GPU suites with the three-launch
# default, the scan's per-kernel stamps (c2, c4) and the headline mask launch's per-wave timeline.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r03c
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_scan.py tests/test_gpu_ingest.py > $OUT/scan_tests.log 2>&1 || { echo SCANTESTFAIL; grep -E "FAILED|Error|assert" $OUT/scan_tests.log | head -20; tail -20 $OUT/scan_tests.log; exit 1; }
tail -1 $OUT/scan_tests.log
timeout -k 10 300 python -u tools/scan_stamps.py > $OUT/scan_stamps.jsonl 2> $OUT/scan_stamps.err || { echo STAMPFAIL; tail -20 $OUT/scan_stamps.err; exit 1; }
cat $OUT/scan_stamps.jsonl | cut -c1-600
timeout -k 10 300 python -u tools/mask_timeline.py --workload c2 > $OUT/mask_timeline_c2.jsonl 2> $OUT/mask_timeline.err || { echo TLFAIL; tail -20 $OUT/mask_timeline.err; exit 1; }
cat $OUT/mask_timeline_c2.jsonl
echo done
