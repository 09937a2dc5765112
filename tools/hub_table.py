"""Tabulates tools/bench_hub.py JSON lines (receive, send, echo): per configuration, each leg's mean
rate over its repeats and its ratio to libnetc's CPU leg.  python tools/hub_table.py FILE..."""

import collections
import json
import sys


def key_of(d):
    if "msgs_per_conn" in d and "round_trips_per_s" in d:
        return "echo", f"{d['conns']} conns, 0-{d['max_bytes']} B, chunk {d['chunk']}", "round_trips_per_s"
    if "rounds" in d:
        return "send", f"{d['conns']} conns, 0-{d['max_bytes']} B, burst {d['burst']}", "msgs_per_s"
    return "receive", f"{d['conns']} conns, 0-{d['max_bytes']} B, chunk {d['chunk']}", "msgs_per_s"


def main(paths):
    rows = collections.OrderedDict()
    for p in paths:
        for line in open(p):
            line = line.strip()
            if not line.startswith("{"):
                continue
            d = json.loads(line)
            side, cfg, metric = key_of(d)
            rows.setdefault((side, cfg, metric), collections.defaultdict(list))[d["leg"]].append(d[metric])
    for (side, cfg, metric), legs in rows.items():
        mean = {l: sum(v) / len(v) for l, v in legs.items()}
        cpu = mean.get("cpu")
        cells = []
        for l in ("hub", "hubcpu", "cpu", "ref"):
            if l in mean:
                r = f" ({mean[l] / cpu:.2f}x)" if cpu else ""
                cells.append(f"{l} {mean[l]:,.0f}{r}")
        gpu_share = ""
        if "hub" in mean and "hubcpu" in mean:
            gpu_share = f" | hub/hubcpu {mean['hub'] / mean['hubcpu']:.2f}"
        print(f"| {side} | {cfg} | {metric} | " + " | ".join(cells) + gpu_share + " |")


if __name__ == "__main__":
    main(sys.argv[1:])
