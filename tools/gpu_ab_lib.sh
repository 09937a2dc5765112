# A/B of the default GPU library against netc_amd/lib/alt (same box, interleaved)
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/${AB_TAG:-ab}; mkdir -p $O; export TMPDIR=/tmp
ALT=$PWD/netc_amd/lib/alt/libnetc_ws_gpu.so
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py > $O/t.log 2>&1 || { echo TESTFAIL; tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
NETC_GPU_LIB=$ALT timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py > $O/t_alt.log 2>&1 || { echo TESTFAIL_ALT; tail -30 $O/t_alt.log; exit 1; }
tail -1 $O/t_alt.log
for R in 1 2; do for WL in c2 c4; do for V in def alt; do
  if [ $V = alt ]; then export NETC_GPU_LIB=$ALT; else unset NETC_GPU_LIB; fi
  timeout -k 10 300 python -u bench.py --workload $WL --steps 20 --warmup 5 --c5-gib 0 --cpu-seconds 0 > $O/b_${WL}_${V}_$R.json 2> $O/b.err || { echo BENCHFAIL; tail -20 $O/b.err; exit 1; }
  python3 -c "
import json;d=json.load(open('$O/b_${WL}_${V}_$R.json'));r=d['roofline'];print('$WL $V $R', d['value'], r['kernel_ms_mean'], r['achieved'], r['ceilings']['xor_inplace_GBps'], r['shapes'], d['verified']['involution'] and d['verified']['keystream_all_frames'])"
done; done; done
