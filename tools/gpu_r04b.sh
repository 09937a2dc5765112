#!/bin/bash
# Round-4 A/B pass (through gpurun, from the repo root): GPU suites on the new build, then the
# §8(f) row tools alternating abl/libnetc_ws_gpu_prev.so (the round-3 build) and the new
# library.  SUITES: the test files; TOOLS_AB: any of scan scan_ns enc val (default all).
#   TAG=r04x SUITES="tests/test_gpu_utf8.py" TOOLS_AB="val" bash tools/gpu_r04b.sh
# (the comparison build is untracked: git worktree add /tmp/prev <commit> && make -C /tmp/prev
#  netc_amd/lib/libnetc_ws_gpu.so, then copy it to the path below; PREV overrides the path)
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${TAG:-r04b}
mkdir -p gpurun_out/$T
ln -sf ../netc_amd/lib/libnetc.so abl/libnetc.so
timeout -k 10 800 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu ${SUITES:-tests/test_gpu_scan.py tests/test_gpu_encode.py tests/test_gpu_ingest.py tests/test_gpu_epoll.py} > gpurun_out/$T/tests.log 2>&1 || { echo TESTFAIL; grep -E "FAILED|Error|assert" gpurun_out/$T/tests.log | head -30; tail -40 gpurun_out/$T/tests.log; exit 1; }
tail -2 gpurun_out/$T/tests.log
L="${PREV:-abl/libnetc_ws_gpu_prev.so} netc_amd/lib/libnetc_ws_gpu.so"
for t in ${TOOLS_AB:-scan scan_ns enc val}; do
  case $t in
  scan)    LIBS="$L" TOOL="tools/bench_scan.py --steps 50" ROUNDS=2 bash tools/gpu_ab_libs.sh ${T}_scan || exit 1 ;;
  scan_ns) LIBS="$L" TOOL="tools/bench_scan.py --steps 50 --non-strict" ROUNDS=1 bash tools/gpu_ab_libs.sh ${T}_scan_ns || exit 1 ;;
  enc)     LIBS="$L" TOOL="tools/bench_encode.py --steps 50 --unroll 1" ROUNDS=2 bash tools/gpu_ab_libs.sh ${T}_enc || exit 1 ;;
  val)     LIBS="$L" TOOL="tools/bench_validate.py --steps 30" ROUNDS=3 bash tools/gpu_ab_libs.sh ${T}_val || exit 1 ;;
  esac
done
echo all done
