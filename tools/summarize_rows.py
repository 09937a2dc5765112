#!/usr/bin/env python3
"""Summarise a merged gpurun_out/rows_<tag>/ (tools/prof_rows.sh) directory into committed
evidence under profiles/:

  profiles/<tag>_<tool>_kernel_stats.csv   rocprofv3 --stats summary (as produced)
  profiles/<tag>_rows_summary.json         per tool: bench lines, and per (kernel, grid size)
                                           the dispatch count, mean duration and the mean
                                           HBM bytes from the separate FETCH_SIZE / WRITE_SIZE
                                           passes (gfx950 correction: 2 x FETCH_SIZE + WRITE_SIZE,
                                           KiB -> bytes; MI355X_MICROARCH.md §HBM)

Dispatches of one kernel with different grid sizes are the different workloads of
a tool (e.g. config 2 vs config 4 shapes), so they are kept apart.
"""
import argparse
import csv
import glob
import json
import os
import shutil
import statistics

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    return name.split("(")[0].replace("void ", "").replace("netc_gpu::", "")


def trace_groups(d):
    path = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    groups = {}
    if not path:
        return groups
    for r in csv.DictReader(open(path[0])):
        if "netc_gpu" not in r["Kernel_Name"]:
            continue
        key = (short(r["Kernel_Name"]), int(r["Grid_Size_X"]))
        groups.setdefault(key, []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    return groups


def pmc_groups(d, counter):
    path = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    groups = {}
    if not path:
        return groups
    per = {}
    for r in csv.DictReader(open(path[0])):
        if r.get("Counter_Name") != counter or "netc_gpu" not in r["Kernel_Name"]:
            continue
        key = (short(r["Kernel_Name"]), int(r["Grid_Size"]), r["Dispatch_Id"])
        per[key] = per.get(key, 0.0) + float(r["Counter_Value"])
    for (k, g, _), v in per.items():
        groups.setdefault((k, g), []).append(v)
    return groups


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--src", default=os.path.join(ROOT, "gpurun_out", "rows_r01e"))
    ap.add_argument("--tag", default="r01e")
    ap.add_argument("--tools", default="bench_encode,bench_validate,bench_scan")
    args = ap.parse_args()
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    out = {"tag": args.tag, "source": os.path.relpath(args.src, ROOT),
           "hbm_bytes": "2 x FETCH_SIZE + WRITE_SIZE (KiB x 1024), separate --pmc passes, per dispatch"}
    for tool in args.tools.split(","):
        rec = {}
        bj = os.path.join(args.src, f"{tool}.json")
        if os.path.exists(bj):
            rec["bench"] = [json.loads(line) for line in open(bj) if line.strip().startswith("{")]
        stats = glob.glob(os.path.join(args.src, f"trace_{tool}", "**", "*kernel_stats.csv"), recursive=True)
        if stats:
            shutil.copy(stats[0], os.path.join(ROOT, "profiles", f"{args.tag}_{tool}_kernel_stats.csv"))
        tr = trace_groups(os.path.join(args.src, f"trace_{tool}"))
        fe = pmc_groups(os.path.join(args.src, f"pmc_fetch_{tool}"), "FETCH_SIZE")
        wr = pmc_groups(os.path.join(args.src, f"pmc_write_{tool}"), "WRITE_SIZE")
        kern = []
        for key in sorted(set(tr) | set(fe)):
            d = tr.get(key, [])
            row = {"kernel": key[0], "grid": key[1], "dispatches": len(d),
                   "mean_us": round(statistics.mean(d) / 1e3, 3) if d else None}
            f, w = fe.get(key), wr.get(key)
            if f and w:
                row["hbm_bytes_mean"] = round(2 * statistics.mean(f) * 1024 + statistics.mean(w) * 1024)
            kern.append(row)
        rec["kernels"] = kern
        out[tool] = rec
    path = os.path.join(ROOT, "profiles", f"{args.tag}_rows_summary.json")
    json.dump(out, open(path, "w"), indent=1)
    for tool in args.tools.split(","):
        print(tool)
        for k in out[tool]["kernels"]:
            print("   ", k)


if __name__ == "__main__":
    main()
