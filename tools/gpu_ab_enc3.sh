# Frame-assembly occupancy A/B on one box: default library vs netc_amd/lib/alt6 and alt8
# (encode_frames_kernel at 6 / 8 waves per SIMD), encode parity on each, then
# tools/bench_encode.py interleaved, twice.
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/${AB_TAG:-abenc3}; mkdir -p $O; export TMPDIR=/tmp
for V in def alt6 alt8; do
  if [ $V = def ]; then unset NETC_GPU_LIB; else export NETC_GPU_LIB=$PWD/netc_amd/lib/$V/libnetc_ws_gpu.so; fi
  timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_encode.py > $O/t_$V.log 2>&1 || { echo TESTFAIL $V; tail -30 $O/t_$V.log; exit 1; }
  echo "$V $(tail -1 $O/t_$V.log)"
done
for R in 1 2; do for V in def alt6 alt8; do
  if [ $V = def ]; then unset NETC_GPU_LIB; else export NETC_GPU_LIB=$PWD/netc_amd/lib/$V/libnetc_ws_gpu.so; fi
  timeout -k 10 300 python -u tools/bench_encode.py --steps 50 --unroll 4 > $O/enc_${V}_$R.jsonl 2> $O/e.err || { echo ENCFAIL; tail -20 $O/e.err; exit 1; }
  python3 -c "
import json
for l in open('$O/enc_${V}_$R.jsonl'):
    d=json.loads(l); print('enc $V $R', d['workload'], d['us_per_step'], d['achieved_GBps'])"
done; done
