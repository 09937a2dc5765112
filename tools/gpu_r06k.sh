set -o pipefail
R=$GRAFT_REPO_ROOT; cd /tmp && export TMPDIR=/tmp
D=$R/gpurun_out/r06k; mkdir -p $D
for v in NOWALK NOCHUNK; do
NETC_GPU_LIB=$R/diag/lib_$v.so NETC_SCAN_ONEPASS=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D/$v -o run -- python3 $R/tools/bench_scan.py --steps 20 --no-cpu --workloads c2 > $D/$v.log 2>&1 || exit 1
f=$(find $D/$v -name '*kernel_stats.csv' | head -1); echo $v; cut -d, -f1-4 $f | grep scan_exits
done
