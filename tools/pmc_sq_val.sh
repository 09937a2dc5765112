#!/bin/bash
# GPU-box SQ counter pass for the fused unmask + UTF-8 check (VALU per dword of the
# rule at each step count): tools/bench_validate.py per workload, text kind and VAL_STEPS, one
# rocprofv3 --pmc run each (8 SQ counters fit one pass); the mask-only kernel of the same run
# (bench_validate times it beside) is the reference.  Summaries: tools/summarize_sq.py.
#   TAG=r04x bash tools/pmc_sq_val.sh
set -o pipefail
R=$PWD
OUT=$R/gpurun_out/sqval_${TAG:-r04}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
C="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
for run in "c2 dense 1" "c2 dense 2" "c2 dense 4" "c2 ascii 2" "c4 dense 1" "c4 ascii 1"; do
    set -- $run
    NETC_VAL_STEPS=$3 timeout -s KILL 150 rocprofv3 --pmc $C --kernel-include-regex "mask_np_kernel|utf8" --output-format csv \
        -d "$OUT/${1}_${2}_k$3" -o run -- python3 "$R/tools/bench_validate.py" --workloads $1 --text $2 --steps 8 \
        > "$OUT/${1}_${2}_k$3.log" 2>&1 || exit $?
    echo "done $run"
done
echo done
