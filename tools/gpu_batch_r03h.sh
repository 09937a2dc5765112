#!/bin/bash
# round-3 batch (through gpurun, from the repo root): encoder GPU parity on the new build, then
# bench_encode new vs tools/libenc_prev.so (2 rounds), the RSV1 scan cliff, the C5 in-place probe.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r03h
mkdir -p $OUT
if [ "${ENC_TESTS:-1}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_encode.py > $OUT/encode_tests.log 2>&1 || { echo ENCTESTFAIL; grep -E "FAILED|Error|assert" $OUT/encode_tests.log | head -20; tail -20 $OUT/encode_tests.log; exit 1; }
  tail -1 $OUT/encode_tests.log
fi
LIBS="tools/libenc_new.so tools/libenc_prev.so" TOOL="tools/bench_encode.py --unroll 4 --steps 50" ROUNDS=2 bash tools/gpu_ab_libs.sh r03h_enc || exit 1
# persistent (library's block count) vs covering grid (one 2 KiB chunk per wavefront)
timeout -k 10 300 python -u tools/bench_encode.py --unroll 4 --max-blocks 0,100000000,0,100000000 --steps 50 > $OUT/enc_grid.jsonl 2> $OUT/enc_grid.err || { echo GRIDFAIL; tail -10 $OUT/enc_grid.err; exit 1; }
cut -c1-200 $OUT/enc_grid.jsonl
timeout -k 10 300 python -u tools/bench_scan.py --rsv1 --non-strict --steps 3 --warmup 1 > $OUT/scan_rsv1.json 2> $OUT/scan_rsv1.err || { echo RSVFAIL; tail -10 $OUT/scan_rsv1.err; exit 1; }
cat $OUT/scan_rsv1.json
timeout -k 10 300 python -u tools/c5_inplace_probe.py --gib 4 > $OUT/c5_inplace.json 2> $OUT/c5_inplace.err || { echo C5FAIL; tail -10 $OUT/c5_inplace.err; exit 1; }
cat $OUT/c5_inplace.json
for i in 1 2; do
  for S in auto spin; do
    timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --c5-gib 0 --cpu-seconds 0 --no-copy-ceiling --sync $S > $OUT/bench_sync_${S}_$i.json 2> $OUT/bench_sync_${S}_$i.err || { echo SYNCFAIL; tail -10 $OUT/bench_sync_${S}_$i.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['kernel_ms_mean'])" $OUT/bench_sync_${S}_$i.json $S
  done
done
echo done
