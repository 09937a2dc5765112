# Misaligned-source sweep: bench.py shapes (out of place aligned vs src = dst + 3) at C2 / C4
# for unroll 1 / 2 / 4 (windows of 2 / 4 / 8 x 1 KiB), twice each, on one box.
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/${TAG:-missweep}; mkdir -p $O; export TMPDIR=/tmp
for R in 1 2; do for WL in c2 c4; do for U in ${US:-1 2 4}; do
  timeout -k 10 300 python -u bench.py --workload $WL --steps 20 --warmup 5 --c5-gib 0 --cpu-seconds 0 --unroll $U > $O/b_${WL}_${U}_$R.json 2> $O/b.err || { echo BENCHFAIL; tail -20 $O/b.err; exit 1; }
  python3 -c "
import json;d=json.load(open('$O/b_${WL}_${U}_$R.json'));r=d['roofline'];s=r['shapes'];print(json.dumps({'wl':'$WL','unroll':$U,'rep':$R,'inplace':r['achieved'],**s,'ratio':round(s['src_misaligned_3_GBps']/s['out_of_place_GBps'],3)}))" | tee -a $O/sweep.jsonl
done; done; done
