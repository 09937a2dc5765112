#!/bin/bash
# Frame scan: workgroups of the LDS kernels K2' / K4b' (NETC_SCAN_SLOW_BLOCKS) swept
# at 16 B and 64 B frames (tools/bench_sizes.py), then a kernel trace at 16 B.
# Run through gpurun from the repo root; every GPU step is time-limited.
set -o pipefail
mkdir -p gpurun_out/${TAG:-r01v}
for g in ${GRIDS:-1024 2048 4096 16384}; do
  NETC_SCAN_SLOW_BLOCKS=$g timeout -k 10 120 python3 tools/bench_sizes.py --sizes 16,64,1024 > gpurun_out/${TAG:-r01v}/g$g.json 2>> gpurun_out/${TAG:-r01v}/err.txt || exit $?
  echo "grid $g"; cat gpurun_out/${TAG:-r01v}/g$g.json | python3 -c "import sys,json; [print(json.loads(l)[\"frame_bytes\"], json.loads(l)[\"scan_us\"]) for l in sys.stdin]"
done
cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/${TAG:-r01v}/trace -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_sizes.py --sizes 16 > $GRAFT_REPO_ROOT/gpurun_out/${TAG:-r01v}/trace.log 2>&1
