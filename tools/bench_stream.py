#!/usr/bin/env python3
"""BASELINE config 5: host-resident frames through netc_gpu_mask_stream_host (pinned slots,
overlapped H2D / kernel / D2H on separate HIP streams).  Reports the host-to-host rate
(payload GiB/s, PCIe-inclusive) for DESIGN.md -- it is never bench.py's `value`.

Default: 16 GiB of 4 KiB frames, in place in one pinned host buffer, 2 slots of 512 MiB
(the fastest shape of a sweep over 32 MiB - 2 GiB slots and 2 - 16 slots).
A sample of frames is checked against the oracle after the timed call.
"""

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=16.0)
    ap.add_argument("--frame", type=int, default=4096)
    ap.add_argument("--slot-mib", type=int, default=512)
    ap.add_argument("--slots", type=int, default=2)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--pageable", action="store_true", help="plain malloc'd host memory instead of pinned")
    args = ap.parse_args()

    import torch

    from netc_amd import mask as nm
    from netc_amd import synth
    from oracle import oracle as orc

    total = int(args.gib * (1 << 30)) // args.frame * args.frame
    nframes = total // args.frame
    off = synth.uniform_offsets(nframes, args.frame)
    keys = synth.random_keys(nframes, stream=500)
    t_alloc = time.perf_counter()
    host = torch.empty(total, dtype=torch.uint8, pin_memory=not args.pageable)
    buf = host.numpy()
    # cheap deterministic fill (content does not change the transfer rate): 64-bit counter pattern
    buf.view(np.uint64)[:] = np.arange(total // 8, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15)
    t_alloc = time.perf_counter() - t_alloc
    picks = synth.rng(7).choice(nframes, size=64, replace=False)
    before = {int(k): buf[int(off[k]):int(off[k + 1])].copy() for k in picks}

    nm.gpu_init(0)
    slot = args.slot_mib << 20
    times = []
    for r in range(args.reps):
        t0 = time.perf_counter()
        nm.mask_stream_host(buf, buf, off, keys, slot_bytes=slot, nslots=args.slots)
        times.append(time.perf_counter() - t0)
    # after an even number of in-place passes the buffer is back to the input; check one more pass
    nm.mask_stream_host(buf, buf, off, keys, slot_bytes=slot, nslots=args.slots)
    bad = 0
    for k, src in before.items():
        exp = orc.mask_batch(src, np.array([0, src.size], dtype=np.uint64), keys[k:k + 1])
        if args.reps % 2 == 0 and not np.array_equal(buf[int(off[k]):int(off[k + 1])], exp):
            bad += 1
    best = min(times)
    print(json.dumps({
        "config": f"c5: {total / (1 << 30):.1f} GiB of {args.frame} B frames, host-resident "
                  f"({'pageable' if args.pageable else 'pinned'}), in place",
        "slots": args.slots, "slot_MiB": args.slot_mib,
        "host_to_host_GiBps": round(total / best / (1 << 30), 3),
        "seconds": [round(t, 3) for t in times],
        "sample_frames_checked": len(before), "sample_frames_wrong": bad,
        "fill_seconds": round(t_alloc, 2),
    }), flush=True)


if __name__ == "__main__":
    main()
