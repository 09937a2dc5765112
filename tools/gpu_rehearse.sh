#!/bin/bash
# N-rank rehearsal of bench.py on a one-GPU box (every rank on device 0, gloo for the
# timing collectives), then the small-frame sizes sweep; through gpurun, from the repo root
set -o pipefail
mkdir -p gpurun_out/rehearse
for N in 2 4; do
  NETC_BENCH_DEVICE=0 NETC_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
      --nproc-per-node $N --master-addr 127.0.0.1 --master-port $((29500 + N)) bench.py --gpus $N --steps 20 \
      --warmup 5 --cpu-seconds 0 --c5-gib 0 > gpurun_out/rehearse/bench_n$N.json 2> gpurun_out/rehearse/bench_n$N.err || exit $?
  tail -1 gpurun_out/rehearse/bench_n$N.json | cut -c1-400
done
timeout -k 10 400 python -u tools/bench_sizes.py --sizes 8,16,32,64,256,1024 > gpurun_out/rehearse/sizes.jsonl 2> gpurun_out/rehearse/sizes.err || exit $?
cat gpurun_out/rehearse/sizes.jsonl
