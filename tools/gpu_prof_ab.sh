#!/bin/bash
# rocprofv3 kernel traces of one tool run per library (through gpurun, from the repo root):
# per-kernel durations of the A and B builds side by side.
#   LIBS="abl/a.so netc_amd/lib/libnetc_ws_gpu.so" TOOL="tools/bench_scan.py --steps 20" bash tools/gpu_prof_ab.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
T=${1:-prof_ab}
mkdir -p gpurun_out/$T
ln -sf ../netc_amd/lib/libnetc.so abl/libnetc.so
export TMPDIR=/tmp
for L in $LIBS; do
  n=$(basename $L .so)
  (cd /tmp && NETC_GPU_LIB=$R/$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$T/$n -o run -- python3 $R/$TOOL > $R/gpurun_out/$T/$n.log 2>&1) || { echo "FAIL $L"; tail -20 gpurun_out/$T/$n.log; exit 1; }
  echo "== $n"
  python3 - $R/gpurun_out/$T/$n <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(f"{r['Name'][:70]:70s} calls {r['Calls']:>5s} avg_us {float(r['AverageNs'])/1e3:9.2f}")
PY
done
echo done
