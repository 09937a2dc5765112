"""Send rates of the GPU egress ring (include/ws/egress.h) beside libnetc's CPU ws_send_message.

Runs tests/bin/ws_egress_bench (tests/drivers/ws_egress_bench.c) per message size and prints one
JSON line per (size, leg): ring_mem (queue -> GPU assembly -> pinned wire, host to host),
ring_socket (the same, then send() on a Unix socketpair), route_socket (libnetc's ws_send_message
with the ring attached, DEFER), cpu_socket (ws_send_message on the CPU), cpu_mem (the CPU path's
header + mask into memory).  Parity of the ring is tests/test_gpu_egress.py's.

    python tools/bench_egress.py [--sizes 1024,65536,1048576] [--mib 256] [--unmasked]
"""

import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "bin", "ws_egress_bench")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="1024,65536,1048576")
    ap.add_argument("--mib", type=int, default=256)
    ap.add_argument("--unmasked", action="store_true")
    ap.add_argument("--legs", default=None)
    args = ap.parse_args()
    if not os.path.exists(EXE):
        sys.exit(f"{EXE} missing: run make")
    for size in [int(s) for s in args.sizes.split(",")]:
        cmd = [EXE, str(size), str(args.mib), "0" if args.unmasked else "1"] + ([args.legs] if args.legs else [])
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
        if r.returncode:
            sys.exit(f"{cmd} failed ({r.returncode}): {r.stderr[-2000:]}")
        for line in r.stdout.splitlines():
            rec = json.loads(line)
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
