#!/usr/bin/env python3
"""Device frame-boundary scan (netc_gpu_scan_frames) throughput, one GPU.

Wire streams of configs 2 and 4 shape (masked client frames, built on the host by
the oracle encoder), strict mode (--non-strict: the reference's semantics; --unmasked).  Per step: one full scan of the stream (all of
its kernels).  Bytes = wire bytes read by the scan's per-chunk passes (reported as
GB/s of stream scanned).  GPU time from two events around K steps on one stream.
The result of the last step is checked against the oracle scan.
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workloads", default="c2,c4", help="c2, c4 (256 MiB of the config-4 mix), c4s (64 MiB of it)")
    ap.add_argument("--non-strict", action="store_true", help="flags 0: the reference's semantics (speculative pass)")
    ap.add_argument("--unmasked", action="store_true", help="unmasked frames (server-to-client direction)")
    ap.add_argument("--rsv1", action="store_true",
                    help="every frame with RSV1 set (as permessage-deflate sends them): strict rejects the stream; "
                         "non-strict keeps the speculative parallel pass (it filters RSV2 / RSV3 only since round 3; "
                         "ADVICE r2 measured the serial-walk cliff it replaced)")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU walks (A/B runs)")
    args = ap.parse_args()
    flags = 0 if args.non_strict else 1

    import torch

    from netc_amd import _lib, synth
    from netc_amd import mask as nm
    from oracle import oracle as orc

    dev = torch.device("cuda", 0)
    entry = _lib.gpu().netc_gpu_scan_frames
    s = torch.cuda.Stream(dev)
    sh = s.cuda_stream
    for wl in args.workloads.split(","):
        off, keys, total = synth.config("c4" if wl == "c4s" else wl)
        if wl in ("c4", "c4s"):   # 256 MiB of the config-4 size mix keeps the host-side encode short
            cut = int(np.searchsorted(off, (256 if wl == "c4" else 64) << 20))   # c4s: 64 MiB of it
            off, keys = off[: cut + 1], keys[:cut]
        rng = np.random.default_rng(5)
        payload = rng.integers(0, 256, int(off[-1]), dtype=np.uint8)
        b0 = np.full(keys.size, 0xC2, dtype=np.uint8) if args.rsv1 else None
        wire, wo = orc.encode_batch(payload, off, keys, b0, not args.unmasked)
        if args.unmasked:
            keys = np.zeros_like(keys)
        n = keys.size
        w = torch.from_numpy(wire).to(dev)
        hdr = torch.empty(n + 1, dtype=torch.int64, device=dev)
        kk = torch.empty(n, dtype=torch.int32, device=dev)
        b0 = torch.empty(n, dtype=torch.uint8, device=dev)
        res = torch.empty(3, dtype=torch.int64, device=dev)
        torch.cuda.synchronize()

        def step():
            rc = entry(0, w.data_ptr(), wire.size, 0, flags, hdr.data_ptr(), kk.data_ptr(), b0.data_ptr(), n,
                       res.data_ptr(), sh)
            if rc:
                raise RuntimeError(_lib.gpu().netc_gpu_strerror())

        for _ in range(args.warmup):
            step()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        for _ in range(args.steps):
            step()
        b.record(s)
        torch.cuda.synchronize()
        us = a.elapsed_time(b) / args.steps * 1e3
        r = res.cpu().numpy()
        ok = (int(r[0]) == n and int(r[1]) == wire.size
              and np.array_equal(hdr.cpu().numpy()[:n].view(np.uint64), wo[:n])
              and np.array_equal(kk.cpu().numpy().view(np.uint32), keys))
        # CPU baseline: the oracle's serial header walk (oracle_scan_frames, -O2, 1 thread) on the same stream
        import ctypes
        import time

        ch = np.zeros(n + 1, dtype=np.uint64)
        ck = np.zeros(n + 1, dtype=np.uint32)
        cb = np.zeros(n + 1, dtype=np.uint8)
        cons, err = ctypes.c_uint64(0), ctypes.c_uint64(0)
        reps, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < (0.0 if args.no_cpu else 2.0) or reps == 0:
            orc.lib().oracle_scan_frames(wire.ctypes.data, wire.size, 0, flags, ch.ctypes.data, ck.ctypes.data,
                                         cb.ctypes.data, n + 1, ctypes.addressof(cons), ctypes.addressof(err))
            reps += 1
        cpu_s = (time.perf_counter() - t0) / reps
        # the product's host walk (netc_ws_scan_frames_host, libnetc.so -O3): what the ingest ring uses
        hres = np.zeros(3, dtype=np.uint64)
        hl = _lib.host().netc_ws_scan_frames_host
        reps, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < (0.0 if args.no_cpu else 2.0) or reps == 0:
            hl(wire.ctypes.data, wire.size, 0, flags, ch.ctypes.data, ck.ctypes.data, cb.ctypes.data, n + 1,
               hres.ctypes.data)
            reps += 1
        host_s = (time.perf_counter() - t0) / reps
        print(json.dumps({"workload": wl, "strict": bool(flags), "masked": not args.unmasked, "rsv1": args.rsv1, "frames": int(n), "wire_bytes": int(wire.size), "us_per_scan": round(us, 2),
                          "wire_GBps": round(wire.size / (us * 1e-6) / 1e9, 1),
                          "frames_per_s": round(n / (us * 1e-6), 1), "matches_oracle": bool(ok),
                          "serial_fallback": hex(nm.scan_diag(s)), "onepass": nm.scan_onepass(s),
                          "cpu_serial_us": round(cpu_s * 1e6, 1),
                          "cpu_serial_frames_per_s": round(n / cpu_s, 1),
                          "host_walk_us": round(host_s * 1e6, 1), "host_walk_ok": int(hres[0]) == n}), flush=True)
        del w
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
