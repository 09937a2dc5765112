set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
D=$R/gpurun_out/r06h; mkdir -p $D
NETC_GPU_LIB=diag/libnetc_ws_gpu_trace.so timeout -k 10 120 python -u tools/scan_probe.py --cases dense1k_x5000,c2 --stamps > $D/stamps.log 2>&1 || { tail -20 $D/stamps.log; exit 1; }
cat $D/stamps.log
cd /tmp && export TMPDIR=/tmp
NETC_SCAN_ONEPASS=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof -o run -- python3 $R/tools/bench_scan.py --steps 20 --no-cpu --workloads c2 > $D/prof.log 2>&1 || exit 1
f=$(find $D/prof -name '*kernel_stats.csv' | head -1); cut -d, -f1-4 $f | head -12
