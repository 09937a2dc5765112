#!/bin/bash
# A/B of the fused unmask + UTF-8 kernel (through gpurun, from the repo root): the UTF-8 GPU
# suite on the new build; tools/bench_validate.py new vs tools/libnetc_ws_gpu_prev.so
# (NETC_GPU_LIB), twice each; then SQ_INSTS_VALU / SQ_WAVES per dispatch of both builds
# (one --pmc pass each, nothing else in the pass).
#   bash tools/gpu_ab_utf8.sh TAG
# (the comparison build is untracked: git worktree add /tmp/prev <commit> && make -C /tmp/prev
#  netc_amd/lib/libnetc_ws_gpu.so, then copy it to the path below; PREV overrides the path)
set -o pipefail
TAG=${1:-ab_utf8}
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_gpu_utf8.py > $OUT/gputest.log 2>&1 || { echo TESTFAIL; grep -E "FAILED|Error" $OUT/gputest.log | head -20; tail -30 $OUT/gputest.log; exit 1; }
tail -2 $OUT/gputest.log
for i in 1 2; do
  for K in ${VAL_STEPS_LIST:-1}; do
    NETC_VAL_STEPS=$K timeout -k 10 300 python -u tools/bench_validate.py --steps 30 > $OUT/new_k${K}_$i.json 2> $OUT/new_k${K}_$i.err || { echo NEWFAIL; tail -20 $OUT/new_k${K}_$i.err; exit 1; }
    echo "steps=$K"; cat $OUT/new_k${K}_$i.json
  done
  NETC_GPU_LIB=${PREV:-tools/libnetc_ws_gpu_prev.so} timeout -k 10 300 python -u tools/bench_validate.py --steps 30 > $OUT/prev_$i.json 2> $OUT/prev_$i.err || { echo PREVFAIL; tail -20 $OUT/prev_$i.err; exit 1; }
  echo prev; cat $OUT/prev_$i.json
done
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES --kernel-include-regex "mask_np_kernel" --output-format csv -d $OUT/valu_new -o run -- python3 $R/tools/bench_validate.py --steps 5 > $OUT/valu_new.log 2>&1 || { echo VALUFAIL; tail -20 $OUT/valu_new.log; exit 1; }
NETC_GPU_LIB=$R/${PREV:-tools/libnetc_ws_gpu_prev.so} timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES --kernel-include-regex "mask_np_kernel" --output-format csv -d $OUT/valu_prev -o run -- python3 $R/tools/bench_validate.py --steps 5 > $OUT/valu_prev.log 2>&1 || { echo VALUPFAIL; tail -20 $OUT/valu_prev.log; exit 1; }
echo done
