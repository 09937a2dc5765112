#!/bin/bash
# Round-3 regression check (through gpurun, from the repo root): the encoder with the
# in-kernel header patch reverted (it spilled 10 VGPRs at <2,true,7>) and the frame scan with
# and without the fused K2+K3a+K3b launch, each against tools/libr03_prev.so (b32d238).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r03b
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_encode.py > $OUT/encode_tests.log 2>&1 || { echo ENCTESTFAIL; grep -E "FAILED|Error|assert" $OUT/encode_tests.log | head -20; tail -20 $OUT/encode_tests.log; exit 1; }
tail -1 $OUT/encode_tests.log
LIBS="tools/libr03_new.so tools/libr03_prev.so" TOOL="tools/bench_encode.py --unroll 4 --steps 50" ROUNDS=2 bash tools/gpu_ab_libs.sh r03b_enc || exit 1
LIBS="tools/libr03_new.so tools/libr03_prev.so" TOOL="tools/bench_scan.py --steps 50" ROUNDS=2 bash tools/gpu_ab_libs.sh r03b_scan || exit 1
for i in 1 2; do
  NETC_SCAN_FUSE=0 NETC_GPU_LIB=tools/libr03_new.so timeout -k 10 300 python -u tools/bench_scan.py --steps 50 > $OUT/nofuse_$i.json 2> $OUT/nofuse_$i.err || { echo NOFUSEFAIL; tail -20 $OUT/nofuse_$i.err; exit 1; }
  echo "== nofuse $i"; cat $OUT/nofuse_$i.json
done
cd /tmp && export TMPDIR=/tmp
for F in 1 0; do
  NETC_SCAN_FUSE=$F timeout -s KILL 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_fuse$F -o run -- python3 $R/tools/bench_scan.py --steps 20 > $OUT/trace_fuse$F.log 2>&1 || { echo TRACEFAIL; tail -20 $OUT/trace_fuse$F.log; exit 1; }
done
echo done
