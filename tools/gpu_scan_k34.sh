# scan K3a / K4 trip changes: parity + timing; then a 2-rank rehearsal of bench.py's N-GPU path on one GPU
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/${AB_TAG:-k34}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_scan.py tests/test_gpu_ingest.py > $O/t.log 2>&1 || { echo TESTFAIL; tail -40 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 300 python -u tools/bench_scan.py > $O/strict.jsonl 2> $O/b.err || { echo BENCHFAIL; tail -20 $O/b.err; exit 1; }
python3 -c "
import json
for l in open('$O/strict.jsonl'):
    d=json.loads(l); print(d['workload'], d['us_per_scan'], d['matches_oracle'], d['serial_fallback'])"
NETC_BENCH_DEVICE=0 NETC_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 3 --c5-gib 0 --cpu-seconds 0 > $O/rank2.json 2> $O/rank2.err || { echo RANK2FAIL; tail -20 $O/rank2.err; exit 1; }
cat $O/rank2.json | cut -c1-400
