#!/usr/bin/env python3
"""Print the per-dispatch mean of each SQ counter per kernel from gpurun_out/sq_<tag>/ (tools/pmc_sq.sh)."""
import csv
import glob
import os
import statistics
import sys

src = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/sq_r01"
for d in sorted(glob.glob(os.path.join(src, "*", ""))):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        continue
    agg = {}
    for r in csv.DictReader(open(f[0])):
        k = (r["Kernel_Name"].split("(")[0].replace("void ", "").replace("netc_gpu::", ""), r["Counter_Name"])
        agg.setdefault(k, {}).setdefault(r["Dispatch_Id"], 0.0)
        agg[k][r["Dispatch_Id"]] += float(r["Counter_Value"])
    for (kn, c), v in sorted(agg.items()):
        vals = list(v.values())
        print(f"{os.path.basename(os.path.dirname(d))[:10]:10s} {kn[:40]:40s} {c:18s} {round(statistics.mean(vals[2:] or vals)):>14}")
