set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
D=$R/gpurun_out/r06_encnt; mkdir -p $D
for r in 1 2 3; do
  timeout -k 10 300 python -u tools/bench_encode.py --steps 100 --warmup 10 --workloads c2,c4 --unroll 1 --flags=-1,8 --entry scan,class > $D/r$r.log 2>&1 || { tail -5 $D/r$r.log; exit 1; }
  python3 -c "
import json,sys
for l in open('$D/r$r.log'):
    if l.startswith('{'):
        d=json.loads(l); print($r, d['workload'], d['entry'], d['flags'], d.get('us_per_step', d.get('us')))
"
done
