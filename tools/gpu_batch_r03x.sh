#!/bin/bash
# Round-3 (through gpurun, from the repo root): the UTF-8 and ingest suites and smoke on the final
# build (two-step VAL windows with plain payload accesses), then bench_validate.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r03x
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_utf8.py tests/test_gpu_ingest.py tests/test_gpu_parity.py > $OUT/tests.log 2>&1 || { echo TESTFAIL; grep -E "FAILED|Error|assert" $OUT/tests.log | head; tail -20 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 python3 -c 'import __graft_entry__ as g; g.smoke()' > $OUT/smoke.log 2>&1 || { echo SMOKEFAIL; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python -u tools/bench_validate.py --steps 30 > $OUT/val.json 2> $OUT/val.err || { echo VALFAIL; tail -20 $OUT/val.err; exit 1; }
cut -c1-160 $OUT/val.json
echo done
