#!/usr/bin/env python3
"""Send-side frame assembly (netc_gpu_encode_frames) throughput, one GPU.

Per step: the wire-offset scan + the assembly kernel over one batch (configs 2 and 4
shapes: 65,536 x 1 KiB, and 1 GiB of 256 B..64 KiB frames), masked.  --entry class times
netc_gpu_encode_frames_class instead (one launch: affine wire offsets) on the workloads whose
frames are all in one length class (config 2).  Algorithmic
bytes = payload read + wire written (+ 8 B/frame offsets read, + 8 B/frame wire
offsets written, reported, not counted).  GPU time from two events around K steps
on one stream; batches rotate over >= 1 GiB of distinct payload.  One JSON line per
workload.
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--workloads", default="c2,c4")
    ap.add_argument("--unroll", default="4,8", help="netc_gpu_tune unroll values to time (4: 2 KiB chunks, the default; 8: 4 KiB)")
    ap.add_argument("--max-blocks", default="0", help="netc_gpu_tune max_blocks values (0: the library's choice; "
                                                       "a huge value: one chunk per wavefront over a covering grid)")
    ap.add_argument("--flags", default="-1", help="netc_gpu_tune flags values (-1: auto, non-temporal payload "
                                                  "loads and stores; 8: plain loads and stores)")
    ap.add_argument("--entry", default="scan", help="comma list: scan (netc_gpu_encode_frames), class "
                                                    "(netc_gpu_encode_frames_class, one-class workloads only)")
    args = ap.parse_args()

    import torch

    from netc_amd import _lib, synth
    from netc_amd import mask as nm

    dev = torch.device("cuda", 0)
    lib = _lib.gpu()
    s = torch.cuda.Stream(dev)
    sh = s.cuda_stream
    for wl in args.workloads.split(","):
        off, keys, total = synth.config(wl)
        n = keys.size
        nb = max(2, (1 << 30) // total)
        srcs = [torch.randint(0, 256, (total,), dtype=torch.uint8, device=dev) for _ in range(nb)]
        cap = nm.wire_bound(total, n, True)
        wires = [torch.empty(cap, dtype=torch.uint8, device=dev) for _ in range(2)]
        wo = torch.empty(n + 1, dtype=torch.int64, device=dev)
        off_t = torch.from_numpy(off.view(np.int64)).to(dev)
        keys_t = torch.from_numpy(keys.view(np.int32)).to(dev)
        wire_len = nm.wire_size(off, True)
        torch.cuda.synchronize()

        cls = nm.length_class(off)

        def step(i):
            if entry == "class":
                rc = lib.netc_gpu_encode_frames_class(0, wires[i % 2].data_ptr(), cap, wo.data_ptr(),
                                                      srcs[i % nb].data_ptr(), total, off_t.data_ptr(),
                                                      keys_t.data_ptr(), None, n, 1, cls, sh)
            else:
                rc = lib.netc_gpu_encode_frames(0, wires[i % 2].data_ptr(), cap, wo.data_ptr(), srcs[i % nb].data_ptr(),
                                                total, off_t.data_ptr(), keys_t.data_ptr(), None, n, 1, sh)
            if rc:
                raise RuntimeError(nm._lib.gpu().netc_gpu_strerror())

        for entry, unroll, mb, fl in [(e, int(u), int(m), int(f)) for e in args.entry.split(",")
                                      for u in args.unroll.split(",") for m in args.max_blocks.split(",")
                                      for f in args.flags.split(",")]:
            if entry == "class" and cls is None:
                continue
            nm.tune(unroll, mb, fl)
            K = args.steps if wl == "c2" else max(10, args.steps // 5)
            with torch.cuda.stream(s):
                for i in range(args.warmup):
                    step(i)
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(s)
                for i in range(K):
                    step(i)
                b.record(s)
            torch.cuda.synchronize()
            us = a.elapsed_time(b) / K * 1e3
            # spot check the last step against the oracle on a few frames
            from oracle import oracle as orc

            wire = wires[(K - 1) % 2][:wire_len].cpu().numpy()   # the last timed step is step(K - 1)
            wo_h = wo.cpu().numpy().view(np.uint64)
            src_h = srcs[(K - 1) % nb].cpu().numpy()
            bad = 0
            for k in np.linspace(0, n - 1, 16).astype(np.int64):
                lo, hi = int(off[k]), int(off[k + 1])
                exp = orc.encode_frame(src_h[lo:hi].tobytes(), 2, int(keys[k]).to_bytes(4, "little"))
                bad += wire[int(wo_h[k]): int(wo_h[k + 1])].tobytes() != exp
            alg = total + wire_len
            print(json.dumps({"workload": wl, "entry": entry, "unroll": unroll, "max_blocks": mb, "flags": fl, "frames": int(n), "payload_bytes": int(total), "wire_bytes": int(wire_len),
                              "us_per_step": round(us, 2), "achieved_GBps": round(alg / (us * 1e-6) / 1e9, 1),
                              "frac_of_8TBps": round(alg / (us * 1e-6) / 8e12, 4),
                              "payload_GiBps": round(total / (us * 1e-6) / 2**30, 1),
                              "sampled_frames_wrong": int(bad)}), flush=True)
        nm.tune()
        del srcs, wires
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
