#!/usr/bin/env python3
"""gpurun_out/<tag>/ (tools/gpu_record.sh) -> the committed evidence under profiles/:

  profiles/<tag>_c2_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary, as produced
  profiles/<tag>_c2_summary.json       the mask kernel: launches, rocprof mean duration (all
                                       launches and the bench's timed ones), PMC HBM bytes,
                                       the bench line it was measured beside
  profiles/pmc_traffic.json            per-workload HBM bytes per launch (read by bench.py)

PMC correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE / WRITE_SIZE are KiB; on gfx950
FETCH_SIZE reports half the bytes of a wide (16 B / lane) coalesced streaming read, so
HBM bytes = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024.  Each counter comes from its own
rocprofv3 --pmc pass of the same bench command.
"""

import argparse
import csv
import json
import os
import shutil
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL = "mask_np_kernel<1, 2, true, true, false, netc_gpu::Args>"   # the headline instantiation
# (bench.py's shape points launch other instantiations; the out-of-place point runs this one,
# after the timed launches)


def pmc(path, counter):
    vals = {}
    for r in csv.DictReader(open(path)):
        if KERNEL in r["Kernel_Name"] and r["Counter_Name"] == counter:
            vals[r["Dispatch_Id"]] = vals.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    v = [vals[k] for k in sorted(vals, key=int)]
    return v


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("--workload", default="c2")
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--src", default=None, help="gpurun_out/ subdirectory (default: the tag)")
    args = ap.parse_args()
    src = os.path.join(ROOT, "gpurun_out", args.src or args.tag)
    prof = os.path.join(ROOT, "profiles")
    wl = args.workload
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"),
                os.path.join(prof, f"{args.tag}_{wl}_kernel_stats.csv"))
    bpath = os.path.join(src, "bench.json")
    if not os.path.exists(bpath):   # the record driver names it per workload
        bpath = os.path.join(src, f"bench_{wl}.json")
    bench = json.loads(open(bpath).read().strip().splitlines()[-1])
    total = bench["config"]["batch_bytes_per_gpu"]
    stats = {}
    for r in csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv"))):
        if KERNEL in r["Name"]:
            stats = {"name": r["Name"], "calls": int(r["Calls"]), "average_ns": float(r["AverageNs"]),
                     "min_ns": float(r["MinNs"]), "max_ns": float(r["MaxNs"])}
    durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) for r in
            csv.DictReader(open(os.path.join(src, "trace", "run_kernel_trace.csv"))) if KERNEL in r["Kernel_Name"]]
    first = 1 + args.warmup   # bench.py: one validated call through the Python mirror, then the warmup
    timed = durs[first: first + args.steps]
    fetch = pmc(os.path.join(src, "pmc_fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write = pmc(os.path.join(src, "pmc_write", "run_counter_collection.csv"), "WRITE_SIZE")
    ft = fetch[first: first + args.steps]
    wt = write[first: first + args.steps]
    hbm = 2 * statistics.mean(ft) * 1024 + statistics.mean(wt) * 1024
    out = {
        "tag": args.tag, "workload": wl, "kernel": stats.get("name"),
        "command": "python3 bench.py --gpus 1 --steps 20 --warmup 5 --c5-gib 0 --cpu-seconds 0 "
                   "(the driver's bench command with the C5 and CPU legs off: the C5 leg launches the "
                   "same kernel on 512 MiB slots, which would mix into the average)",
        "rocprof_stats": stats,
        "rocprof_timed_launches": len(timed),
        "rocprof_timed_mean_us": round(statistics.mean(timed) / 1e3, 3),
        "rocprof_timed_GBps": round(2 * total / statistics.mean(timed), 1),
        "bench_kernel_ms_mean": bench["roofline"]["kernel_ms_mean"],
        "bench_achieved_GBps": bench["roofline"]["achieved"],
        "algorithmic_bytes_per_launch": 2 * total,
        "pmc_fetch_kib_mean": round(statistics.mean(ft), 1),
        "pmc_write_kib_mean": round(statistics.mean(wt), 1),
        "hbm_bytes_per_launch": int(hbm),
        "hbm_over_algorithmic": round(hbm / (2 * total), 4),
        "correction": "HBM bytes = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024 (gfx950, MI355X_MICROARCH.md §HBM)",
        "bench_line": bench,
    }
    json.dump(out, open(os.path.join(prof, f"{args.tag}_{wl}_summary.json"), "w"), indent=1)
    tp = os.path.join(prof, "pmc_traffic.json")
    traffic = json.load(open(tp)) if os.path.exists(tp) else {}
    sys.path.insert(0, ROOT)
    from bench import kernel_source_hash   # the sources this pass measured (the tree it ran from)

    traffic[wl] = {"hbm_bytes_per_launch": int(hbm), "source": f"profiles/{args.tag}_{wl}_summary.json",
                   "kernel_source_sha256": kernel_source_hash()}
    json.dump(traffic, open(tp, "w"), indent=1)
    print(json.dumps({k: v for k, v in out.items() if k != "bench_line"}, indent=1))


if __name__ == "__main__":
    main()
