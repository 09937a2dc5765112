set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for v in 1 0; do
  D=$R/gpurun_out/${TAG:-r06e}/op$v
  mkdir -p $D
  NETC_SCAN_ONEPASS=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python3 $R/tools/bench_scan.py --steps 50 --no-cpu --workloads ${WL:-c2} > $D/log 2>&1 || exit 1
done
