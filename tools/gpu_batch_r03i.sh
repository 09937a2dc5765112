#!/bin/bash
# K1 (scan_exits) A/B (through gpurun, from the repo root): the scan GPU suite on the new build,
# tools/bench_scan.py new vs tools/libk1_prev.so (3 rounds), then one SQ pass over K1 of each
# build at both shapes (VALU instructions and busy cycles per dispatch).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r03i
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_scan.py tests/test_gpu_ingest.py > $OUT/scan_tests.log 2>&1 || { echo SCANTESTFAIL; grep -E "FAILED|Error|assert" $OUT/scan_tests.log | head -20; tail -20 $OUT/scan_tests.log; exit 1; }
tail -1 $OUT/scan_tests.log
LIBS="tools/libk1_new.so tools/libk1_prev.so" TOOL="tools/bench_scan.py --steps 50" ROUNDS=3 bash tools/gpu_ab_libs.sh r03i_ab || exit 1
for i in 1 2; do   # the new K1 with the three separate launches (knob SCAN_FUSE = 0)
  NETC_SCAN_FUSE=0 NETC_GPU_LIB=tools/libk1_new.so timeout -k 10 300 python -u tools/bench_scan.py --steps 50 > $OUT/nofuse_$i.json 2> $OUT/nofuse_$i.err || { echo NOFUSEFAIL; tail -20 $OUT/nofuse_$i.err; exit 1; }
  echo "== nofuse $i"; cat $OUT/nofuse_$i.json
done
timeout -k 10 300 python -u tools/bench_scan.py --steps 50 --non-strict > $OUT/nonstrict.json 2> $OUT/nonstrict.err || { echo NSFAIL; tail -20 $OUT/nonstrict.err; exit 1; }
echo "== non-strict"; cat $OUT/nonstrict.json
cd /tmp && export TMPDIR=/tmp
C="SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY"
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/tools/bench_scan.py --steps 20 > $OUT/trace.log 2>&1 || { echo TRACEFAIL; tail -20 $OUT/trace.log; exit 1; }
for L in new prev; do
  NETC_GPU_LIB=$R/tools/libk1_$L.so timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex "scan_exits" --output-format csv -d $OUT/sq_$L -o run -- python3 $R/tools/bench_scan.py --steps 5 --warmup 1 > $OUT/sq_$L.log 2>&1 || { echo SQFAIL $L; tail -20 $OUT/sq_$L.log; exit 1; }
done
echo done
