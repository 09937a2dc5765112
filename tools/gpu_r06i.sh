set -o pipefail
R=$GRAFT_REPO_ROOT; cd /tmp && export TMPDIR=/tmp
D=$R/gpurun_out/r06i; mkdir -p $D
NETC_GPU_LIB=$R/diag/lib_nowait0.so NETC_SCAN_ONEPASS=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D/nw -o run -- python3 $R/tools/bench_scan.py --steps 20 --no-cpu --workloads c2 > $D/nw.log 2>&1 || exit 1
f=$(find $D/nw -name '*kernel_stats.csv' | head -1); cut -d, -f1-4 $f | head -8
NETC_SCAN_ONEPASS=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D/g -o run -- python3 $R/tools/bench_scan.py --steps 20 --no-cpu --workloads c2 > $D/g.log 2>&1 || exit 1
f=$(find $D/g -name '*kernel_stats.csv' | head -1); cut -d, -f1-4 $f | head -8
