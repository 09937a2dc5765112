# rocprofv3 kernel trace of the frame assembly at C2 (per-kernel durations and gaps)
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/${AB_TAG:-enctr}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 tools/bench_encode.py --workloads c2 --unroll 4 --steps 40 --warmup 5 > $O/b.jsonl 2> $O/b.err || { echo TRACEFAIL; tail -20 $O/b.err; exit 1; }
python3 - $O <<'PY'
import csv, glob, sys, statistics
o = sys.argv[1]
f = glob.glob(f"{o}/trace/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted((r for r in csv.DictReader(open(f)) if "netc_gpu" in r["Kernel_Name"]), key=lambda r: int(r["Start_Timestamp"]))
rows = rows[-60:]
prev_end = None
per = {}
gaps = []
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("netc_gpu::", "")
    per.setdefault(name, []).append((e - s) / 1e3)
    if prev_end is not None: gaps.append((s - prev_end) / 1e3)
    prev_end = e
for k, v in per.items(): print(k, len(v), round(statistics.median(v), 2))
print("gap median", round(statistics.median(gaps), 2), "mean", round(statistics.mean(gaps), 2))
PY
cat $O/b.jsonl | cut -c1-160
