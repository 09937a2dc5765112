set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_encode.py > gpurun_out/t_enc.log 2>&1
for P in 16 8 4 2 1; do
  NETC_ENC_SCAN_PER=$P timeout -k 10 120 python -u tools/bench_encode.py --workloads c2,c4 --unroll 4 > gpurun_out/enc_per_$P.jsonl 2>&1
done
