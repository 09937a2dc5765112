set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
D=$R/gpurun_out/${TAG:-r06q}; mkdir -p $D
for r in 1 2; do for v in def 0; do
 ( [ $v = 0 ] && export NETC_SCAN_ONEPASS=0; exec timeout -k 10 120 python -u tools/bench_scan.py --steps 100 --no-cpu --workloads c2,c4s,c4 > $D/scan_$v.$r.log 2>&1 ) || exit 1
 echo "op=$v r=$r $(grep -o '"workload": "c[24]s*"\|"us_per_scan": [0-9.]*\|"matches_oracle": [a-z]*\|"onepass": [a-z]*' $D/scan_$v.$r.log | tr '\n' ' ')"
done; done
