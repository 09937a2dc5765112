# A/B of the default GPU library against netc_amd/lib/alt: encode parity on both, then the
# mask bench (C2 / C4) and the frame-assembly bench, interleaved, twice (same box).
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/${AB_TAG:-abenc}; mkdir -p $O; export TMPDIR=/tmp
ALT=$PWD/netc_amd/lib/alt/libnetc_ws_gpu.so
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_encode.py tests/test_gpu_parity.py > $O/t.log 2>&1 || { echo TESTFAIL; tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for R in 1 2; do for V in def alt; do
  if [ $V = alt ]; then export NETC_GPU_LIB=$ALT; else unset NETC_GPU_LIB; fi
  timeout -k 10 300 python -u tools/bench_encode.py --steps 50 --unroll 4 > $O/enc_${V}_$R.jsonl 2> $O/e.err || { echo ENCFAIL; tail -20 $O/e.err; exit 1; }
  python3 -c "
import json
for l in open('$O/enc_${V}_$R.jsonl'):
    d=json.loads(l); print('enc $V $R', {k:d[k] for k in d if k in ('workload','us_per_step','us','GBps','achieved_GBps','frac')} or d)"
  for WL in c2 c4; do
    timeout -k 10 300 python -u bench.py --workload $WL --steps 50 --warmup 5 --c5-gib 0 --cpu-seconds 0 > $O/b_${WL}_${V}_$R.json 2> $O/b.err || { echo BENCHFAIL; tail -20 $O/b.err; exit 1; }
    python3 -c "
import json;d=json.load(open('$O/b_${WL}_${V}_$R.json'));r=d['roofline'];print('$WL $V $R', d['value'], r['kernel_ms_mean'], r['achieved'], r['shapes'])"
  done
done; done
