"""Prints tools/bench_routes.py's JSON lines as a table (DESIGN_ROUNDS.md §15)."""
import json
import sys

for path in sys.argv[1:]:
    for line in open(path):
        r = json.loads(line)
        if r["route"] == "receive":
            print(f"recv {r['leg']:4s} {r['msg_bytes']:8d} closed={r['closed_loop']} n={r['count']:6d} "
                  f"{r['msgs_per_s']:10.0f} msg/s {r['gib_per_s']:7.3f} GiB/s p50 {r['lat_p50_us']:9.1f} "
                  f"p99 {r['lat_p99_us']:9.1f} us ev={r['events']} gpu={r['gpu_slots']} host={r['host_slots']}")
        else:
            print(f"send {r['leg']:12s} {r['msg_bytes']:8d} {r['msgs_per_s']:10.0f} msg/s {r['payload_GiBps']:7.3f} GiB/s")
