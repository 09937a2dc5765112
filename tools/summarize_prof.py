#!/usr/bin/env python3
"""Turn a merged gpurun_out/prof_<tag>/ directory into the committed evidence under profiles/:

  profiles/<tag>_<wl>_kernel_stats.csv   rocprofv3 --stats summary (as produced)
  profiles/<tag>_<wl>_summary.json       mask-kernel launches, mean duration, PMC bytes
  profiles/pmc_traffic.json              per-workload HBM bytes per launch (read by bench.py)

PMC correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE and WRITE_SIZE are in KiB; on
gfx950 FETCH_SIZE reports half the bytes of a wide (16 B / lane) coalesced streaming
read, so HBM bytes = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024.
"""

import argparse
import csv
import glob
import json
import os
import shutil
import statistics

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def find(pattern):
    hits = sorted(glob.glob(pattern, recursive=True))
    return hits[0] if hits else None


def pmc_mean(d, counter):
    path = find(os.path.join(d, "**", "*counter_collection.csv"))
    if not path:
        return None, 0
    vals = {}
    for r in csv.DictReader(open(path)):
        if "mask_frames" not in r.get("Kernel_Name", ""):
            continue
        if r.get("Counter_Name") != counter:
            continue
        key = r.get("Dispatch_Id") or r.get("Correlation_Id")
        vals[key] = vals.get(key, 0.0) + float(r["Counter_Value"])
    if not vals:
        return None, 0
    v = list(vals.values())[5:] or list(vals.values())   # skip the first launches (warm-up)
    return statistics.mean(v), len(v)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--src", default=os.path.join(ROOT, "gpurun_out", "prof_r01"))
    ap.add_argument("--tag", default="r01")
    ap.add_argument("--workload", default="c2")
    args = ap.parse_args()
    wl, src = args.workload, args.src
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    stats = find(os.path.join(src, f"trace_{wl}", "**", "*kernel_stats.csv"))
    trace = find(os.path.join(src, f"trace_{wl}", "**", "*kernel_trace.csv"))
    out = {"workload": wl, "tag": args.tag}
    if stats:
        shutil.copy(stats, os.path.join(ROOT, "profiles", f"{args.tag}_{wl}_kernel_stats.csv"))
        for r in csv.DictReader(open(stats)):
            if "mask_frames" in r["Name"]:
                out["rocprof_mask_kernel"] = {"name": r["Name"], "calls": int(r["Calls"]),
                                              "average_ns": float(r["AverageNs"]), "min_ns": float(r["MinNs"]),
                                              "max_ns": float(r["MaxNs"])}
    if trace:
        rows = [r for r in csv.DictReader(open(trace)) if "mask_frames" in r["Kernel_Name"]]
        d = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows]
        if d:
            out["trace_duration_ns"] = {"mean": statistics.mean(d), "median": statistics.median(d), "n": len(d)}
            out["grid"] = {k: rows[0].get(k) for k in ("Grid_Size_X", "Workgroup_Size_X", "VGPR_Count", "SGPR_Count",
                                                        "LDS_Block_Size", "Scratch_Size")}
    fetch, nf = pmc_mean(os.path.join(src, f"pmc_fetch_{wl}"), "FETCH_SIZE")
    write, nw = pmc_mean(os.path.join(src, f"pmc_write_{wl}"), "WRITE_SIZE")
    bj = find(os.path.join(src, f"bench_{wl}.json"))
    bench = None
    if bj:
        for line in open(bj):
            line = line.strip()
            if line.startswith("{"):
                bench = json.loads(line)
        if bench:
            out["bench"] = {k: bench.get(k) for k in ("value", "ms_per_step", "roofline", "pipelined_2stream")}
            shutil.copy(bj, os.path.join(ROOT, "profiles", f"{args.tag}_{wl}_bench.json"))
    if fetch is not None and write is not None:
        hbm = 2 * fetch * 1024 + write * 1024
        out["pmc"] = {"FETCH_SIZE_KiB_mean": fetch, "WRITE_SIZE_KiB_mean": write, "launches": [nf, nw],
                      "hbm_bytes_per_launch": hbm, "correction": "2 x FETCH_SIZE (gfx950 half-count) + WRITE_SIZE, KiB"}
        if bench:
            alg = bench["roofline"]["algorithmic_bytes_per_launch"]
            out["pmc"]["traffic_over_algorithmic"] = hbm / alg
        tp = os.path.join(ROOT, "profiles", "pmc_traffic.json")
        allw = json.load(open(tp)) if os.path.exists(tp) else {}
        allw[wl] = {"hbm_bytes_per_launch": round(hbm), "source": f"profiles/{args.tag}_{wl}_summary.json"}
        json.dump(allw, open(tp, "w"), indent=1, sort_keys=True)
    json.dump(out, open(os.path.join(ROOT, "profiles", f"{args.tag}_{wl}_summary.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
