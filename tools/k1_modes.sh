# K1 timing floor: the scan bench's kernel trace with K1 doing everything (0), only the
# quick check (1), only its loads (2).  Modes 1 and 2 give wrong scans: timing only.
set -o pipefail
TAG=${1:-k1m}
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for m in ${MODES:-0 1 2}; do
  NETC_SCAN_K1_MODE=$m timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/m$m -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_scan.py --steps 20 > $OUT/m$m.log 2>&1 || { echo FAIL$m; tail -20 $OUT/m$m.log; exit 1; }
done
echo done
