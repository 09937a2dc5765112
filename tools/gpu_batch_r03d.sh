#!/bin/bash
# Round-3 SQ instruction-mix passes (through gpurun, from the repo root): the fused unmask +
# UTF-8 kernel against the plain unmask (tools/bench_validate.py), and the frame-assembly
# kernels at C2 (tools/bench_encode.py), one rocprofv3 --pmc run each (8 SQ counters fit).
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r03d
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp || exit 1
C="SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU"
timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex "mask_np_kernel|utf8" --output-format csv -d $OUT/val -o run -- \
    python3 $R/tools/bench_validate.py --steps 5 > $OUT/val.log 2>&1 || { echo VALFAIL; tail -20 $OUT/val.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex "encode|wire_offsets" --output-format csv -d $OUT/enc -o run -- \
    python3 $R/tools/bench_encode.py --workloads c2 --unroll 4 --steps 5 --warmup 2 > $OUT/enc.log 2>&1 || { echo ENCFAIL; tail -20 $OUT/enc.log; exit 1; }
C2="SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS SQ_WAVES SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM_RD SQ_INSTS_BRANCH SQ_ACTIVE_INST_ANY"
timeout -s KILL 120 rocprofv3 --pmc $C2 --kernel-include-regex "mask_np_kernel|utf8" --output-format csv -d $OUT/val2 -o run -- \
    python3 $R/tools/bench_validate.py --steps 5 > $OUT/val2.log 2>&1 || { echo VAL2FAIL; tail -20 $OUT/val2.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex "scan_exits|scan_links|scan_emit" --output-format csv -d $OUT/scan -o run -- \
    python3 $R/tools/bench_scan.py --steps 5 --warmup 2 > $OUT/scan.log 2>&1 || { echo SCANFAIL; tail -20 $OUT/scan.log; exit 1; }
cd $R && python3 tools/summarize_sq.py gpurun_out/r03d
# K1 alone: the product's tail (exit target check + returning atomic append) vs plain per-chunk lists
bash tools/gpu_k1exp.sh r03d_k1exp || true
echo done
