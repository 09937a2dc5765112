#!/usr/bin/env python3
"""Launch-shape sweep for the masking kernel (diagnostic; interleaved rounds in ONE process).

For every variant: R rotating device batches (>= 1 GiB distinct, so the 256 MiB
Infinity Cache cannot serve them), `reps` back-to-back launches, throughput from
events around the whole run, and mean per-launch kernel time (1-stream runs).
Also times tools/libdiag_stream.so's constant-key XOR stream and torch's copy as
practical ceilings for the same bytes.
"""

import argparse
import ctypes
import itertools
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c2")
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--rotation-bytes", type=int, default=2 << 30)
    ap.add_argument("--variants", default="4:0:0,4:0:3,4:0:1,4:0:2,2:0:0,2:0:3,1:0:3,8:0:3,4:2048:0,4:1024:3")
    ap.add_argument("--streams", default="1,2")
    args = ap.parse_args()

    import torch

    from netc_amd import _lib, synth
    from netc_amd import mask as nm

    dev = torch.device("cuda", 0)
    lib = _lib.gpu()
    diag = ctypes.CDLL(os.path.join(ROOT, "tools", "libdiag_stream.so"))
    diag.diag_stream.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                 ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    sink = torch.zeros(1 << 20, dtype=torch.int32, device=dev)
    off, keys, total = synth.config(args.workload)
    nb = max(2, -(-args.rotation_bytes // total))
    off_t = torch.from_numpy(off.view(np.int64)).to(dev)
    keys_t = torch.from_numpy(keys.view(np.int32)).to(dev)
    bufs = [torch.randint(0, 256, (total,), dtype=torch.uint8, device=dev) for _ in range(nb)]
    ptrs = [b.data_ptr() for b in bufs]
    streams = [torch.cuda.Stream(dev) for _ in range(4)]
    n = keys.size

    def run(launch, nstreams, reps, per_kernel=False):
        ss = streams[:nstreams]
        start = torch.cuda.Event(enable_timing=True)
        end = torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        start.record(ss[0])
        for s in ss[1:]:
            s.wait_event(start)
        ev = []
        for i in range(reps):
            s = ss[i % nstreams]
            if per_kernel:
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(s)
            launch(ptrs[i % nb], s.cuda_stream)
            if per_kernel:
                b.record(s)
                ev.append((a, b))
        for s in ss[1:]:
            e = torch.cuda.Event()
            e.record(s)
            ss[0].wait_event(e)
        end.record(ss[0])
        torch.cuda.synchronize()
        ms = start.elapsed_time(end)
        kms = float(np.mean([a.elapsed_time(b) for a, b in ev])) if ev else None
        return ms / reps, kms

    variants = []
    for v in args.variants.split(","):
        parts = [int(x) for x in v.split(":")]
        u, mb, fl = parts[:3]
        oop = parts[3] if len(parts) > 3 else 0
        variants.append(("mask" if not oop else "mask_oop", u, mb, fl))
    # diag: in-place XOR, grid-stride (contig 0) / wave-contiguous (1), nt (flags 1) -- see tools/diag_stream.hip
    variants += [("diag", 0, 0, 1), ("diag", 0, 1, 1), ("diag", 0, 0, 0)]
    stream_counts = [int(x) for x in args.streams.split(",")]
    results = {}
    for rnd in range(args.rounds):
        for (kind, u, mb, fl), ns in itertools.product(variants, stream_counts):
            if kind in ("mask", "mask_oop"):
                nm.tune(u, mb, fl)
                oop = kind == "mask_oop"

                def launch(p, s, oop=oop):
                    d = ptrs[(ptrs.index(p) + 1) % nb] if oop else p
                    rc = lib.netc_gpu_mask_batch(0, d, p, total, off_t.data_ptr(), keys_t.data_ptr(), n, s)
                    assert rc == 0
            elif kind == "diag":
                def launch(p, s, contig=mb, nt=fl):
                    diag.diag_stream(0, nt, contig, p, p, total, 0x5A5A5A5A, 2048, sink.data_ptr(), s)
            else:
                def launch(p, s):
                    j = ptrs.index(p)
                    with torch.cuda.stream(torch.cuda.ExternalStream(s)):
                        bufs[(j + 1) % nb].copy_(bufs[j])
            run(launch, ns, 10)
            ms, kms = run(launch, ns, args.reps, per_kernel=(ns == 1))
            key = f"{kind} U={u} blocks={mb} flags={fl} streams={ns}"
            results.setdefault(key, []).append((ms, kms))
    nm.tune()
    out = []
    for key, vals in results.items():
        step = [v[0] for v in vals]
        ker = [v[1] for v in vals if v[1] is not None]
        best = min(step)
        rec = {"variant": key, "step_us_med": round(1e3 * float(np.median(step)), 2), "step_us_min": round(1e3 * best, 2),
               "GBps_traffic_best": round(2 * total / (best * 1e-3) / 1e9, 1),
               "kernel_us_med": round(1e3 * float(np.median(ker)), 2) if ker else None}
        out.append(rec)
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
