#!/usr/bin/env python3
"""Small frames: the rows at uniform frame sizes below config 2's 1 KiB.

64 MiB of payload cut into frames of S bytes (S = 16 .. 4096), per size: the mask
kernel (netc_gpu_mask_batch, in place), frame assembly (netc_gpu_encode_frames), and
the frame scan of the assembled wire (netc_gpu_scan_frames, strict).  GPU time from
events around K calls on one stream; the scan result is checked (frame count and
consumed bytes).  One JSON line per size; GB/s counts payload read + written for
mask / encode (wire written), wire read for the scan."""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="16,64,256,1024,4096")
    ap.add_argument("--mib", type=int, default=64)
    ap.add_argument("--steps", type=int, default=20)
    args = ap.parse_args()

    import torch

    from netc_amd import mask as nm

    dev = torch.device("cuda", 0)
    total = args.mib << 20
    src = torch.randint(0, 256, (total,), dtype=torch.uint8, device=dev)

    def timed(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.steps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1000.0 / args.steps

    for size in (int(x) for x in args.sizes.split(",")):
        n = total // size
        off = torch.arange(0, n + 1, dtype=torch.int64, device=dev) * size
        keys = torch.randint(-2**31, 2**31 - 1, (n,), dtype=torch.int32, device=dev)
        buf = src[: n * size].clone()
        t_mask = timed(lambda: nm.mask_batch(buf, buf, off, keys))
        bound = n * size + 14 * n + 64
        wire = torch.empty(bound, dtype=torch.uint8, device=dev)
        wo = torch.empty(n + 1, dtype=torch.int64, device=dev)
        t_enc = timed(lambda: nm.encode_frames(wire, wo, buf, off, keys))
        wlen = int(wo[-1].item())
        hdr = torch.empty(n + 1, dtype=torch.int64, device=dev)
        kk = torch.empty(n, dtype=torch.int32, device=dev)
        b0 = torch.empty(n, dtype=torch.uint8, device=dev)
        res = torch.empty(3, dtype=torch.int64, device=dev)
        t_scan = timed(lambda: nm.scan_frames(wire, hdr, kk, b0, res, length=wlen))
        r = res.cpu().tolist()
        payload = n * size
        print(json.dumps({"frame_bytes": size, "frames": n, "payload_bytes": payload, "wire_bytes": wlen,
                          "mask_us": round(t_mask, 2), "mask_GBps": round(2 * payload / t_mask / 1e3, 1),
                          "encode_us": round(t_enc, 2), "encode_GBps": round((payload + wlen) / t_enc / 1e3, 1),
                          "scan_us": round(t_scan, 2), "scan_GBps": round(wlen / t_scan / 1e3, 1),
                          "scan_ok": r[0] == n and r[1] == wlen}), flush=True)


if __name__ == "__main__":
    main()
