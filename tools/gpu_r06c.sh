set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
mkdir -p gpurun_out/r06c
NETC_GPU_LIB=diag/libnetc_ws_gpu_trace.so timeout -k 10 120 python -u tools/scan_probe.py --cases dense1k_x5000,c2 --stamps > gpurun_out/r06c/stamps.log 2>&1 || { tail -20 gpurun_out/r06c/stamps.log; exit 1; }
cat gpurun_out/r06c/stamps.log
