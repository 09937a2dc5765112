#!/bin/bash
# A/B of the mask kernel on one box (through gpurun, from the repo root):
#   the whole -m gpu suite on the new build; then bench.py C2 / C4 alternating the new
#   library and tools/libnetc_ws_gpu_prev.so (the previous kernel, NETC_GPU_LIB), 3 rounds;
#   then rocprofv3 kernel trace + FETCH_SIZE / WRITE_SIZE passes of the new C2 command.
#   bash tools/gpu_ab_mask.sh TAG
# (the comparison build is untracked: git worktree add /tmp/prev <commit> && make -C /tmp/prev
#  netc_amd/lib/libnetc_ws_gpu.so, then copy it to the path below; PREV overrides the path)
set -o pipefail
TAG=${1:-ab}
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 900 --timeout-method thread -m gpu tests > $OUT/gputest.log 2>&1 || { echo TESTFAIL; grep -E "FAILED|Error" $OUT/gputest.log | head -20; tail -30 $OUT/gputest.log; exit 1; }
  tail -2 $OUT/gputest.log
fi
B="python -u bench.py --gpus 1 --steps 200 --warmup 20 --c5-gib 0 --cpu-seconds 0"
for i in 1 2 3; do
  for WL in ${WLS:-c2 c4}; do
    timeout -k 10 300 $B --workload $WL > $OUT/new_${WL}_$i.json 2> $OUT/new_${WL}_$i.err || { echo NEWFAIL; tail -20 $OUT/new_${WL}_$i.err; exit 1; }
    NETC_GPU_LIB=${PREV:-tools/libnetc_ws_gpu_prev.so} timeout -k 10 300 $B --workload $WL > $OUT/prev_${WL}_$i.json 2> $OUT/prev_${WL}_$i.err || { echo PREVFAIL; tail -20 $OUT/prev_${WL}_$i.err; exit 1; }
  done
done
python3 - "$OUT" <<'EOF'
import glob, json, os, sys
out = sys.argv[1]
for f in sorted(glob.glob(os.path.join(out, "*_c?_?.json"))):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    r = d["roofline"]
    print(os.path.basename(f), "value", d["value"], "kern_us", round(r["kernel_ms_mean"] * 1e3, 2), "frac", r["frac"],
          "xor", r["ceilings"]["xor_inplace_GBps"], "mis", r["shapes"]["src_misaligned_3_GBps"], "oop", r["shapes"]["out_of_place_GBps"])
EOF
[ "${PROF:-1}" = 0 ] && { echo done; exit 0; }
cd /tmp && export TMPDIR=/tmp
PROFCMD="python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --c5-gib 0 --cpu-seconds 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- $PROFCMD > $OUT/trace.log 2>&1 || { echo TRACEFAIL; tail -20 $OUT/trace.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "mask_np_kernel" --output-format csv -d $OUT/pmc_fetch -o run -- $PROFCMD --no-copy-ceiling > $OUT/pmc_fetch.log 2>&1 || { echo FETCHFAIL; tail -20 $OUT/pmc_fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "mask_np_kernel" --output-format csv -d $OUT/pmc_write -o run -- $PROFCMD --no-copy-ceiling > $OUT/pmc_write.log 2>&1 || { echo WRITEFAIL; tail -20 $OUT/pmc_write.log; exit 1; }
echo done
