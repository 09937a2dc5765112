#!/bin/bash
# UTF-8 check (f3) per text kind (the ASCII early-out on dense and ASCII-heavy
# text): tools/bench_validate.py per --text, then a rocprofv3 kernel trace of each for the
# per-kernel split (VAL mask kernel, phase B utf8_messages, mask-only kernel).
#   bash tools/gpu_val_text.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
T=${1:-val_text}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
for k in dense sparse ascii; do
  timeout -k 10 300 python tools/bench_validate.py --steps 30 --text $k > gpurun_out/$T/$k.jsonl 2> gpurun_out/$T/$k.err || { echo "FAIL $k"; tail -20 gpurun_out/$T/$k.err; exit 1; }
  cat gpurun_out/$T/$k.jsonl
done
for k in dense sparse ascii; do
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$T/prof_$k -o run -- python3 $R/tools/bench_validate.py --steps 20 --text $k > $R/gpurun_out/$T/prof_$k.log 2>&1) || { echo "PROF FAIL $k"; tail -20 gpurun_out/$T/prof_$k.log; exit 1; }
  echo "== $k"
  python3 - $R/gpurun_out/$T/prof_$k <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(f"{r['Name'][:90]:90s} calls {r['Calls']:>5s} avg_us {float(r['AverageNs'])/1e3:9.2f}")
PY
done
echo done
