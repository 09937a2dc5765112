#!/bin/bash
# Round-3 K1 prefetch A/B (through gpurun, from the repo root): the scan + ingest suites on the
# new K1 (one resident round striding over the chunks, the next chunk's loads in flight), the
# scan suite on its 7-waves-per-SIMD build and on the K3a+K3b merged launch (libk3m), then bench_scan: previous K1, 6- and 7-wave builds,
# and the 6-wave build with one chunk per wavefront (NETC_SCAN_K1_BLOCKS).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r03f
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_scan.py tests/test_gpu_ingest.py > $OUT/scan_tests.log 2>&1 || { echo SCANTESTFAIL; grep -E "FAILED|Error|assert" $OUT/scan_tests.log | head -20; tail -20 $OUT/scan_tests.log; exit 1; }
tail -1 $OUT/scan_tests.log
ln -sf ../netc_amd/lib/libnetc.so tools/libnetc.so
NETC_GPU_LIB=tools/libk1_w7.so timeout -k 10 600 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_scan.py > $OUT/scan_tests_w7.log 2>&1 || { echo W7TESTFAIL; grep -E "FAILED|Error|assert" $OUT/scan_tests_w7.log | head -20; tail -20 $OUT/scan_tests_w7.log; exit 1; }
tail -1 $OUT/scan_tests_w7.log
NETC_GPU_LIB=tools/libk3m.so timeout -k 10 600 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_scan.py > $OUT/scan_tests_k3m.log 2>&1 || { echo K3MTESTFAIL; grep -E "FAILED|Error|assert" $OUT/scan_tests_k3m.log | head -20; tail -20 $OUT/scan_tests_k3m.log; exit 1; }
tail -1 $OUT/scan_tests_k3m.log
LIBS="tools/libk1_prev.so tools/libk1_w6.so tools/libk1_w7.so tools/libk3m.so" TOOL="tools/bench_scan.py --steps 50" ROUNDS=2 bash tools/gpu_ab_libs.sh r03f_ab || exit 1
NETC_SCAN_K1_BLOCKS=1073741824 NETC_GPU_LIB=tools/libk1_w6.so timeout -k 10 300 python -u tools/bench_scan.py --steps 50 > $OUT/w6_onechunk.json 2> $OUT/w6_onechunk.err || { echo ONEFAIL; tail -20 $OUT/w6_onechunk.err; exit 1; }
echo "== w6 one chunk per wave"; cat $OUT/w6_onechunk.json
cd /tmp && export TMPDIR=/tmp
NETC_GPU_LIB=$R/tools/libk1_w6.so timeout -s KILL 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_w6 -o run -- python3 $R/tools/bench_scan.py --steps 20 --workloads c2 > $OUT/trace_w6.log 2>&1 || { echo TRACEFAIL; tail -20 $OUT/trace_w6.log; exit 1; }
grep scan_ $OUT/trace_w6/run_kernel_stats.csv | cut -d, -f1-4
echo done
