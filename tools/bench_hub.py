"""Many connections on one event loop: the GPU hub (include/ws/hub.h) against libnetc's CPU
ws_parse_frame and the reference's own parser (VERDICT r4 "next" #7).

Runs tests/bin/ws_hub_server (tests/drivers/ws_hub_server.c) per configuration and leg: CONNS
loopback TCP connections, MSGS messages each of 0..MAX bytes (1-3 fragments, PINGs), sent round
robin by 4 client threads with libnetc's ws_send_message; the server calls ws_parse_frame once per
readable socket per loop iteration (netc's loop, reference src/tcp/server.c:30-75 ->
src/web/server.c:69-98).  Per-connection delivery is checked by hash against what each client
sent.  One JSON line per run (stdout and --out).

--chunks 0,65536 adds prerendered client traffic (CHUNK bytes per send(), rendered before the clock
starts; tests/drivers/ws_hub_server.c): with 0 the 4 client threads run ws_send_message per message
inside the timed region, and "clients_seconds" in each line shows whether they, not the server,
set the pace.

    python tools/bench_hub.py [--configs 256x400x1024,1024x100x1024,64x200x16384] [--chunks 0] [--out FILE]

Legs: hub (the GPU hub), hubcpu (the SAME hub host code -- slots, peeks, sendmsg batching -- with its
device work done on the host: tests/bin/*_cpu linked to tests/bin/libnetc_hub_cpu.so, netc_ws_mask
for the XOR; the control that isolates what the GPU itself adds), cpu (libnetc's per-connection CPU
path), ref (the reference's own code).  --repeat N interleaves N passes of every leg.

--send runs the send side instead (tests/bin/ws_egress_hub_server, include/ws/egress_hub.h): CONNS
connections answered ROUNDS times each from one loop with netc's ws_send_message -- through one
GPU egress hub (flushed once per loop iteration), libnetc's CPU path, or the reference's own
ws_send_message; 4 client threads check every connection's bytes by hash.  --send-configs
CONNSxROUNDSxMAX.
"""

import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "bin", "ws_hub_server")
SEND_EXE = os.path.join(ROOT, "tests", "bin", "ws_egress_hub_server")
REF = os.path.join(ROOT, "oracle", "_ref", "libref_ws.so")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="256x400x1024,1024x100x1024,64x200x16384,16x100x262144")
    ap.add_argument("--legs", default="hub,hubcpu,cpu,ref")
    ap.add_argument("--repeat", type=int, default=1, help="passes over every leg, interleaved")
    ap.add_argument("--chunks", default="0,65536", help="client send chunk sizes (0: live ws_send_message)")
    ap.add_argument("--out", default=None)
    ap.add_argument("--send", action="store_true", help="the send side (egress hub) instead")
    ap.add_argument("--echo", action="store_true", help="the echo server (both hubs) instead: --echo-configs")
    ap.add_argument("--echo-configs", default="256x200x1024x0,256x200x1024x65536,1024x50x1024x65536,64x100x16384x65536")
    ap.add_argument("--send-configs", default="256x100x1024,1024x40x1024,64x100x16384,16x40x262144")
    ap.add_argument("--bursts", default="1,8", help="send side: messages per connection per loop iteration")
    ap.add_argument("--masked", type=int, default=0, help="send side: masked frames (the client side; no ref leg)")
    args = ap.parse_args()
    if args.send:
        return send_side(args)
    if args.echo:
        return echo(args)
    if not os.path.exists(EXE):
        sys.exit(f"{EXE} missing: run make")
    out = open(args.out, "a") if args.out else None
    for cfg in args.configs.split(","):
        conns, msgs, mx = cfg.split("x")
        for _, chunk, leg in [(i, c, l) for c in args.chunks.split(",") for i in range(args.repeat)
                              for l in args.legs.split(",")]:
            if leg == "ref" and not os.path.exists(REF):
                continue
            r = subprocess.run([exe_of(EXE, leg), leg, conns, msgs, mx, "0", "0", "-", chunk], capture_output=True,
                               text=True, timeout=600, cwd=ROOT)
            if r.returncode:
                sys.exit(f"{cfg} {leg}: rc {r.returncode}: {r.stderr[-2000:]}")
            rec = json.loads(r.stdout.strip().splitlines()[-1])
            rec.pop("conn_hash", None)
            line = json.dumps(rec)
            print(line, flush=True)
            if out:
                out.write(line + "\n")
                out.flush()


def exe_of(exe, leg):
    """the hubcpu leg runs the driver built against the host-backend hub library"""
    return exe + "_cpu" if leg == "hubcpu" else exe


def echo(args):
    exe = os.path.join(ROOT, "tests", "bin", "ws_echo_server")
    out = open(args.out, "a") if args.out else None
    for cfg in args.echo_configs.split(","):
        conns, msgs, mx, chunk = cfg.split("x")
        for _, leg in [(i, l) for i in range(args.repeat) for l in args.legs.split(",") if l != "ref"]:
            r = subprocess.run([exe_of(exe, leg), leg, conns, msgs, mx, chunk], capture_output=True, text=True,
                               timeout=600, cwd=ROOT)
            if r.returncode:
                sys.exit(f"echo {cfg} {leg}: rc {r.returncode}: {r.stderr[-2000:]}")
            line = r.stdout.strip().splitlines()[-1]
            print(line, flush=True)
            if out:
                out.write(line + "\n")
                out.flush()


def send_side(args):
    if not os.path.exists(SEND_EXE):
        sys.exit(f"{SEND_EXE} missing: run make")
    out = open(args.out, "a") if args.out else None
    for cfg in args.send_configs.split(","):
        conns, rounds, mx = cfg.split("x")
        for _, burst, leg in [(i, b, l) for b in args.bursts.split(",") for i in range(args.repeat)
                              for l in args.legs.split(",")]:
            if leg == "ref" and (args.masked or not os.path.exists(REF)):
                continue
            r = subprocess.run([exe_of(SEND_EXE, leg), leg, conns, str(max(1, int(rounds) // int(burst))), mx, str(args.masked), "0",
                                "-", burst], capture_output=True, text=True, timeout=600, cwd=ROOT)
            if r.returncode:
                sys.exit(f"send {cfg} {leg}: rc {r.returncode}: {r.stderr[-2000:]}")
            line = r.stdout.strip().splitlines()[-1]
            print(line, flush=True)
            if out:
                out.write(line + "\n")
                out.flush()


if __name__ == "__main__":
    main()
