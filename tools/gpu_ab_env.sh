#!/bin/bash
# A/B of environment settings on one box (through gpurun, from the repo root): CMD run once per
# variant, ROUNDS times, variants interleaved so box drift hits every arm alike.  A variant is a
# comma-separated list of VAR=value assignments ("-" = none); each run's stdout goes to
# gpurun_out/TAG/<i>_<round>.json and its last JSON line is summarised at the end.
#   VARIANTS="- NETC_MASK_TAPER=2097152" CMD="python -u bench.py --steps 200 --cpu-seconds 0 --c5-gib 0" \
#   ROUNDS=3 bash tools/gpu_ab_env.sh TAG
set -o pipefail
TAG=${1:-ab_env}
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
for r in $(seq 1 ${ROUNDS:-3}); do
  i=0
  for V in $VARIANTS; do
    i=$((i + 1))
    ENVS=()
    [ "$V" != "-" ] && IFS=',' read -ra ENVS <<< "$V"
    env "${ENVS[@]}" timeout -k 10 ${RUN_TIMEOUT:-300} $CMD > $OUT/${i}_$r.json 2> $OUT/${i}_$r.err || { echo "FAIL $V"; tail -20 $OUT/${i}_$r.err; exit 1; }
    echo "== $V round $r"; tail -c 400 $OUT/${i}_$r.json; echo
  done
done
python3 - "$OUT" "$VARIANTS" <<'EOF'
import glob, json, os, sys
out, variants = sys.argv[1], sys.argv[2].split()
rows = {}
for f in sorted(glob.glob(os.path.join(out, "*_*.json"))):
    i, r = os.path.basename(f)[:-5].split("_")
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except (ValueError, IndexError):
        continue
    rows.setdefault(variants[int(i) - 1], []).append(d)
summary = {}
for v, ds in rows.items():
    s = {}
    if "roofline" in ds[0]:
        s["value"] = [d["value"] for d in ds]
        s["ms_per_step_us"] = [round(d["ms_per_step"] * 1e3, 2) for d in ds]
        s["kernel_us"] = [round(d["roofline"]["kernel_ms_mean"] * 1e3, 3) for d in ds]
        s["frac"] = [d["roofline"]["frac"] for d in ds]
    else:
        s["lines"] = ds
    summary[v] = s
print(json.dumps(summary, indent=1))
json.dump(summary, open(os.path.join(out, "summary.json"), "w"), indent=1)
EOF
echo done
