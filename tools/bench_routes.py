"""Rates of the routes through netc's kept C API over loopback TCP (VERDICT r4 "next" #6).

Receive: tests/bin/ws_route_bench (tests/drivers/ws_route_bench.c) -- netc's server loop, ONE
ws_parse_frame per EPOLLIN (reference src/tcp/server.c:72-75 -> src/web/server.c:86-98) -- per
message size and leg:
  cpu   libnetc's ws_parse_frame on the CPU
  gpu   the same call with the socket attached to a GPU ingest ring (netc_ws_gpu_attach)
  ref   the reference's own ws_parse_frame (oracle/_ref/libref_ws.so, its flags: -O0), a stated
        baseline
each open loop (messages back to back: rate, and latency under that load) and closed loop (one
message in flight: the latency of a message alone).
Send: tests/bin/ws_egress_bench over TCP: the GPU egress ring behind ws_send_message (DEFER),
libnetc's CPU ws_send_message, and the reference's own ws_send_message (TEXT payloads, since
its masked BINARY path overflows above 254 B, defect B1).

Writes one JSON line per run to stdout (and --out).

    python tools/bench_routes.py [--sizes 1024,65536,1048576] [--mib 256] [--out FILE]
"""

import argparse
import json
import os
import platform
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RECV = os.path.join(ROOT, "tests", "bin", "ws_route_bench")
SEND = os.path.join(ROOT, "tests", "bin", "ws_egress_bench")
REF = os.path.join(ROOT, "oracle", "_ref", "libref_ws.so")


def run(cmd, timeout=300):
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, cwd=ROOT)
    if r.returncode:
        raise RuntimeError(f"{cmd} failed ({r.returncode}): {r.stderr[-2000:]}")
    return [json.loads(line) for line in r.stdout.splitlines() if line.startswith("{")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="1024,65536,1048576")
    ap.add_argument("--mib", type=int, default=256, help="payload MiB per open-loop receive run and per send leg")
    ap.add_argument("--closed", type=int, default=2000, help="messages per closed-loop run")
    ap.add_argument("--legs", default="cpu,gpu,ref")
    ap.add_argument("--no-send", action="store_true")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    out = open(args.out, "a") if args.out else None
    legs = [l for l in args.legs.split(",") if l != "ref" or os.path.exists(REF)]
    head = {"host": platform.node(), "cpu": platform.processor() or platform.machine()}
    try:
        head["commit"] = subprocess.run(["git", "rev-parse", "--short", "HEAD"], capture_output=True, text=True,
                                        cwd=ROOT).stdout.strip() or None
    except OSError:
        head["commit"] = None

    def emit(rec):
        rec = {**head, **rec}
        line = json.dumps(rec)
        print(line, flush=True)
        if out:
            out.write(line + "\n")
            out.flush()

    for size in [int(s) for s in args.sizes.split(",")]:
        n = max(64, min(200000, (args.mib << 20) // size))
        for leg in legs:
            for rec in run([RECV, leg, str(size), str(n), "0"]):
                emit({"route": "receive", **rec})
            nc = max(32, min(args.closed, (64 << 20) // size))
            for rec in run([RECV, leg, str(size), str(nc), "1"]):
                emit({"route": "receive", **rec})
        if not args.no_send:
            send_legs = "route_socket,cpu_socket" + (",ref_socket" if os.path.exists(REF) else "")
            for rec in run([SEND, str(size), str(args.mib), "1", send_legs, "tcp"], timeout=600):
                emit({"route": "send", "transport": "tcp", **rec})
    if out:
        out.close()


if __name__ == "__main__":
    main()
