#!/bin/bash
# GPU-box SQ counter pass (through gpurun, from the repo root): instruction mix of the
# frame-assembly kernels (config 2 and config 4 shapes, separately) and of the mask
# kernel, one rocprofv3 --pmc run each (8 SQ counters fit one pass).
set -o pipefail
R=$PWD
OUT=$R/gpurun_out/sq_${TAG:-r01}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
C="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
for wl in c2 c4; do
    timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex "encode_frames|wire_offsets" --output-format csv \
        -d "$OUT/enc_$wl" -o run -- python3 "$R/tools/bench_encode.py" --workloads $wl --unroll 1 --steps 10 --warmup 2 \
        > "$OUT/enc_$wl.log" 2>&1 || exit $?
done
timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex "mask_np_kernel" --output-format csv -d "$OUT/mask" -o run -- \
    python3 "$R/bench.py" --steps 10 --warmup 2 --cpu-seconds 0 --c5-gib 0 --no-copy-ceiling --no-pipelined-probe --no-shard-leg > "$OUT/mask.log" 2>&1 || exit $?
echo done
