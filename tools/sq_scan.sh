set -o pipefail
R=$PWD
OUT=$R/gpurun_out/sq_scan
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
C="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex "scan_exits" --output-format csv -d "$OUT/k1" -o run -- \
    python3 "$R/tools/bench_scan.py" --workloads c2 --steps 5 --warmup 1 > "$OUT/k1.log" 2>&1 || exit $?
C2="SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_WAVES SQ_WAVE_CYCLES"
timeout -s KILL 120 rocprofv3 --pmc $C2 --kernel-include-regex "scan_exits" --output-format csv -d "$OUT/k1b" -o run -- \
    python3 "$R/tools/bench_scan.py" --workloads c2 --steps 5 --warmup 1 > "$OUT/k1b.log" 2>&1 || exit $?
echo done
