"""Back-to-back launch gaps of one kernel in a rocprofv3 kernel trace.

    python tools/kernel_gaps.py <kernel_trace.csv> <name substring> [--grid N]

For every pair of consecutive dispatches of the kernel (by start time) whose gap is
under 100 us (same timed loop), reports the kernel duration, the idle gap between
the end of one dispatch and the start of the next, and the period.  bench.py's
`ms_per_step` is the period; the roofline's kernel time is the duration -- the
difference is this gap (GPU-side dispatch / drain between two kernels on one stream
when the host is ahead), not host work.
"""
import csv
import json
import statistics
import sys


def main():
    path, name = sys.argv[1], sys.argv[2]
    grid = int(sys.argv[sys.argv.index("--grid") + 1]) if "--grid" in sys.argv else None
    rows = [r for r in csv.DictReader(open(path)) if name in r["Kernel_Name"]
            and (grid is None or int(r["Grid_Size_X"]) == grid)]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    durs, gaps, periods = [], [], []
    for a, b in zip(rows, rows[1:]):
        s0, e0, s1 = int(a["Start_Timestamp"]), int(a["End_Timestamp"]), int(b["Start_Timestamp"])
        if s1 - e0 > 100_000:
            continue
        durs.append(e0 - s0)
        gaps.append(s1 - e0)
        periods.append(s1 - s0)
    out = {
        "trace": path, "kernel": name, "grid": grid, "pairs": len(gaps),
        "duration_us_median": round(statistics.median(durs) / 1e3, 3) if durs else None,
        "gap_us_median": round(statistics.median(gaps) / 1e3, 3) if gaps else None,
        "gap_us_mean": round(statistics.mean(gaps) / 1e3, 3) if gaps else None,
        "period_us_median": round(statistics.median(periods) / 1e3, 3) if periods else None,
    }
    print(json.dumps(out))


if __name__ == "__main__":
    main()
