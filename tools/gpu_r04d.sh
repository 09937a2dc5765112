set -o pipefail
cd $GRAFT_REPO_ROOT
SUITES="tests/test_gpu_scan.py" AB=0 TAG=r04d bash tools/gpu_r04b.sh || exit 1
LIBS="abl/libnetc_ws_gpu_prev.so netc_amd/lib/libnetc_ws_gpu.so" TOOL="tools/bench_scan.py --steps 20" bash tools/gpu_prof_ab.sh r04d_scan || exit 1
LIBS="netc_amd/lib/libnetc_ws_gpu.so" TOOL="tools/bench_encode.py --steps 20 --unroll 1 --flags 0" bash tools/gpu_prof_ab.sh r04d_enc_plain || exit 1
