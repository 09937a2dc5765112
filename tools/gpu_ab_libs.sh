#!/bin/bash
# A/B of whole-library builds on one box (through gpurun, from the repo root): a tool run
# alternately with each library named (NETC_GPU_LIB), ROUNDS times.
#   LIBS="tools/a.so tools/b.so" TOOL="tools/bench_validate.py --steps 30" bash tools/gpu_ab_libs.sh TAG
set -o pipefail
TAG=${1:-ab_libs}
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
ln -sf ../netc_amd/lib/libnetc.so tools/libnetc.so   # the copies in tools/ and abl/ find libnetc.so through $ORIGIN
ln -sf ../netc_amd/lib/libnetc.so abl/libnetc.so
for i in $(seq 1 ${ROUNDS:-2}); do
  for L in $LIBS; do
    n=$(basename $L .so)
    NETC_GPU_LIB=$L timeout -k 10 300 python -u $TOOL > $OUT/${n}_$i.json 2> $OUT/${n}_$i.err || { echo FAIL $L; tail -20 $OUT/${n}_$i.err; exit 1; }
    echo "== $n $i"; cat $OUT/${n}_$i.json
  done
done
echo done
