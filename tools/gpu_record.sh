#!/bin/bash
# GPU session driver of a round's record (through gpurun, from the repo root; round 4's
# tools/gpu_r04.sh, renamed in round 5).  STEPS picks the parts, in order:
#   tests     the whole -m gpu suite (one pytest process)        -> TAG/gputest.log
#   smoke     __graft_entry__.smoke()                             -> TAG/smoke.log
#   bench     bench.py with the driver's arguments                -> TAG/bench.json
#   taper     headline kernel A/B over NETC_MASK_TAPER            -> TAG_taper/ (tools/gpu_ab_env.sh)
#   sync      bench.py --sync auto vs spin at the driver's steps  -> TAG_sync/
#   prof      rocprofv3 trace + FETCH_SIZE / WRITE_SIZE passes of the headline, summarised into
#             profiles/ by tools/summarize_round.py on the CPU side afterwards  -> TAG_c2/
#   rows      the SURVEY §8(f) rows (tools/prof_rows.sh)          -> rows_TAG/
#   wl        bench.py --workload W (WLS, default "c3 c4") with FETCH_SIZE / WRITE_SIZE passes -> TAG_W/
#   routes    tools/bench_routes.py (the kept API over loopback TCP) -> TAG/routes.jsonl
#   hub       tools/bench_hub.py + a rocprofv3 trace of the hub leg  -> TAG/hub.jsonl, TAG_hub/
# Every GPU step runs under its own time limit; the chain stops at the first failure.
#   STEPS="tests bench" bash tools/gpu_record.sh TAG
set -o pipefail
TAG=${1:-r05}
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for s in ${STEPS:-tests smoke bench}; do
  echo "== $s"
  case $s in
  tests)
    timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu ${TESTS_SEL:-tests} > $OUT/gputest.log 2>&1 || { echo TESTFAIL; grep -E "FAILED|Error" $OUT/gputest.log | head -20; tail -30 $OUT/gputest.log; exit 1; }
    tail -2 $OUT/gputest.log ;;
  smoke)
    timeout -k 10 300 python3 -c 'import __graft_entry__ as g; g.smoke()' > $OUT/smoke.log 2>&1 || { echo SMOKEFAIL; tail -20 $OUT/smoke.log; exit 1; }
    tail -1 $OUT/smoke.log ;;
  bench)
    timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { echo BENCHFAIL; tail -30 $OUT/bench.err; exit 1; }
    cat $OUT/bench.json ;;
  taper)
    VARIANTS="${TAPERS:-- NETC_MASK_TAPER=1048576 NETC_MASK_TAPER=2097152 NETC_MASK_TAPER=4194304 NETC_MASK_TAPER=8388608}" \
    CMD="python -u bench.py --gpus 1 --steps 200 --warmup 20 --c5-gib 0 --cpu-seconds 0 --no-copy-ceiling --no-pipelined-probe" \
    ROUNDS=${ROUNDS:-3} bash tools/gpu_ab_env.sh ${TAG}_taper > $OUT/taper.log 2>&1 || { echo TAPERFAIL; tail -20 $OUT/taper.log; exit 1; }
    tail -40 $OUT/taper.log ;;
  sync)
    for i in 1 2 3; do
      for m in auto spin; do
        timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --c5-gib 0 --cpu-seconds 0 --no-copy-ceiling --sync $m > $OUT/sync_${m}_$i.json 2> $OUT/sync_${m}_$i.err || { echo SYNCFAIL; tail -20 $OUT/sync_${m}_$i.err; exit 1; }
        python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['kernel_ms_mean'], (d['pipelined_2stream'] or {}).get('value'))" $OUT/sync_${m}_$i.json $m
      done
    done ;;
  prof)
    D=$R/gpurun_out/${TAG}_c2
    mkdir -p $D
    CMD="python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --c5-gib 0 --cpu-seconds 0 --no-pipelined-probe --workload ${WL:-c2}"
    (cd /tmp && timeout -k 10 300 $CMD > $D/bench.json 2> $D/bench.err) || { echo PBENCHFAIL; tail -20 $D/bench.err; exit 1; }
    (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- $CMD > $D/trace.log 2>&1) || { echo TRACEFAIL; tail -20 $D/trace.log; exit 1; }
    (cd /tmp && timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "mask_np_kernel" --output-format csv -d $D/pmc_fetch -o run -- $CMD --no-copy-ceiling > $D/pmc_fetch.log 2>&1) || { echo FETCHFAIL; tail -20 $D/pmc_fetch.log; exit 1; }
    (cd /tmp && timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "mask_np_kernel" --output-format csv -d $D/pmc_write -o run -- $CMD --no-copy-ceiling > $D/pmc_write.log 2>&1) || { echo WRITEFAIL; tail -20 $D/pmc_write.log; exit 1; }
    echo "profiled ${WL:-c2}" ;;
  rows)
    TAG=$TAG bash tools/prof_rows.sh > $OUT/rows.log 2>&1 || { echo ROWSFAIL; tail -20 $OUT/rows.log; exit 1; }
    tail -3 $OUT/rows.log ;;
  wl)
    for W in ${WLS:-c3 c4}; do
    D=$R/gpurun_out/${TAG}_$W
    mkdir -p $D
    CMD="python3 $R/bench.py --gpus 1 --steps 10 --warmup 3 --c5-gib 0 --cpu-seconds 0 --no-pipelined-probe --workload $W"
    (cd /tmp && timeout -k 10 300 $CMD > $D/bench.json 2> $D/bench.err) || { echo WLFAIL; tail -20 $D/bench.err; exit 1; }
    (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- $CMD > $D/trace.log 2>&1) || { echo WLTRACEFAIL; tail -20 $D/trace.log; exit 1; }
    (cd /tmp && timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "mask_np_kernel" --output-format csv -d $D/pmc_fetch -o run -- $CMD --no-copy-ceiling > $D/pmc_fetch.log 2>&1) || { echo WLFETCHFAIL; tail -20 $D/pmc_fetch.log; exit 1; }
    (cd /tmp && timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "mask_np_kernel" --output-format csv -d $D/pmc_write -o run -- $CMD --no-copy-ceiling > $D/pmc_write.log 2>&1) || { echo WLWRITEFAIL; tail -20 $D/pmc_write.log; exit 1; }
    cut -c1-300 $D/bench.json
    done ;;
  routes)
    timeout -k 10 600 python3 -u tools/bench_routes.py --out $OUT/routes.jsonl > $OUT/routes.log 2>&1 || { echo ROUTESFAIL; tail -20 $OUT/routes.log; exit 1; }
    tail -2 $OUT/routes.log | cut -c1-200 ;;
  hub)
    timeout -k 10 600 python3 -u tools/bench_hub.py --out $OUT/hub.jsonl > $OUT/hub.log 2>&1 || { echo HUBFAIL; tail -20 $OUT/hub.log; exit 1; }
    D=$R/gpurun_out/${TAG}_hub
    mkdir -p $D
    (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- $R/tests/bin/ws_hub_server hub 256 400 1024 > $D/trace.log 2>&1) || { echo HUBTRACEFAIL; tail -20 $D/trace.log; exit 1; }
    tail -1 $D/trace.log | cut -c1-300 ;;
  hubs)
    # round 6: hub / hubcpu / cpu / ref at 256 and 1,024 connections, 0-1 KiB and 0-16 KiB, both sides and the echo
    timeout -k 10 600 python3 -u tools/bench_hub.py --configs ${RX_CFGS:-256x400x1024,1024x100x1024,256x100x16384,1024x25x16384} --chunks 65536 --repeat ${REPEAT:-2} --out $OUT/hub_rx.jsonl > $OUT/hub_rx.log 2>&1 || { echo HUBRXFAIL; tail -20 $OUT/hub_rx.log; exit 1; }
    timeout -k 10 600 python3 -u tools/bench_hub.py --send --send-configs ${TX_CFGS:-256x100x1024,1024x40x1024,256x40x16384,1024x10x16384} --bursts 1 --repeat ${REPEAT:-2} --out $OUT/hub_tx.jsonl > $OUT/hub_tx.log 2>&1 || { echo HUBTXFAIL; tail -20 $OUT/hub_tx.log; exit 1; }
    timeout -k 10 600 python3 -u tools/bench_hub.py --echo --echo-configs ${ECHO_CFGS:-256x200x1024x65536,1024x50x1024x65536,256x50x16384x65536,1024x12x16384x65536} --repeat ${REPEAT:-2} --out $OUT/hub_echo.jsonl > $OUT/hub_echo.log 2>&1 || { echo HUBECHOFAIL; tail -20 $OUT/hub_echo.log; exit 1; }
    wc -l $OUT/hub_*.jsonl ;;
  *)
    echo "unknown step $s"; exit 2 ;;
  esac
done
echo all done
