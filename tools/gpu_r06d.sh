set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
D=gpurun_out/r06d; mkdir -p $D
for r in 1 2; do
 for v in 23ed8cb 29dfaa4 2abbf2a 51eb6b9 67fddae head0 head; do
  if [ $v = head ]; then L=; E=; elif [ $v = head0 ]; then L=; E=0; else L=diag/ab/lib_$v.so; E=; fi
  ( [ -n "$L" ] && export NETC_GPU_LIB=$L; [ -n "$E" ] && export NETC_SCAN_ONEPASS=$E; exec timeout -k 10 120 python -u tools/bench_scan.py --steps 100 --no-cpu --workloads c2,c4 > $D/$v.$r.log 2>&1 ) || { echo FAIL $v; tail -5 $D/$v.$r.log; exit 1; }
  echo "$v $r $(grep -o '"workload": "c[24]"\|"us_per_scan": [0-9.]*\|"matches_oracle": [a-z]*\|"onepass": [a-z]*' $D/$v.$r.log | tr '\n' ' ')"
 done
done
