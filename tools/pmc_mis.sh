# HBM bytes of the aligned and src-misaligned mask launches in bench.py's shape points (2 --pmc passes)
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/${AB_TAG:-pmc_mis}; mkdir -p $O; export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex mask_np_kernel --output-format csv -d $O/pmc_$C -o run -- python3 bench.py --steps 5 --warmup 2 --c5-gib 0 --cpu-seconds 0 > $O/pmc_$C.json 2> $O/pmc_$C.err || { echo PMCFAIL; tail -20 $O/pmc_$C.err; exit 1; }
done
python3 - $O <<'PY'
import csv, glob, sys, collections
o = sys.argv[1]
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    f = glob.glob(f"{o}/pmc_{c}/**/*counter_collection.csv", recursive=True)[0]
    g = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if "mask_np_kernel" in r["Kernel_Name"] and r["Counter_Name"] == c:
            g[(r["Kernel_Name"].split("(")[0], r["Grid_Size_X"] if "Grid_Size_X" in r else r.get("Grid_Size"))].append(float(r["Counter_Value"]))
    for k, v in g.items():
        print(c, k, len(v), round(sum(v) / len(v)))
PY
