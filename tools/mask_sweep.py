#!/usr/bin/env python3
"""Launch-shape sweep of the product mask kernel (diagnostic): netc_gpu_tune(unroll, 0, flags)
over the workloads, HIP-event timed over a >= 2 GiB rotation, one JSON line per point.
NETC_MASK_LDS (read once per process) is reported with each line."""

import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workloads", default="c2,c4,c3")
    ap.add_argument("--unroll", default="1,2,4")
    ap.add_argument("--flags", default="-1,11,19,27,7", help="netc_gpu_tune flags values")
    ap.add_argument("--reps", type=int, default=60)
    ap.add_argument("--shift", type=int, default=0, help="src = dst + shift (out of place when != 0)")
    args = ap.parse_args()
    import torch

    from netc_amd import _lib, synth

    g = _lib.gpu()
    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream(dev)
    lds = os.environ.get("NETC_MASK_LDS", "0")
    for wl in args.workloads.split(","):
        off, keys, total = synth.config(wl)
        nb = max(3, (2 << 30) // total + 1)
        bufs = [torch.randint(0, 256, (total + 64,), dtype=torch.uint8, device=dev) for _ in range(nb)]
        off_t = torch.from_numpy(off.view(np.int64)).to(dev)
        keys_t = torch.from_numpy(keys.view(np.int32)).to(dev)
        reps = args.reps if total < (1 << 30) else max(8, args.reps // 6)
        for unroll in [int(x) for x in args.unroll.split(",")]:
            for flags in [int(x) for x in args.flags.split(",")]:
                assert g.netc_gpu_tune(unroll, 0, flags) == 0

                def fn(i):
                    b = bufs[i % nb].data_ptr()
                    if args.shift:
                        src, dst = bufs[(i + nb // 2) % nb].data_ptr() + args.shift, b
                    else:
                        src = dst = b
                    assert g.netc_gpu_mask_batch(0, dst, src, total, off_t.data_ptr(), keys_t.data_ptr(), keys.size,
                                                 s.cuda_stream) == 0
                with torch.cuda.stream(s):
                    for i in range(4):
                        fn(i)
                    torch.cuda.synchronize()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(s)
                    for i in range(reps):
                        fn(4 + i)
                    e1.record(s)
                    torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / reps
                print(json.dumps({"wl": wl, "unroll": unroll, "flags": flags, "lds": int(lds), "shift": args.shift,
                                  "us": round(ms * 1e3, 2), "GBps": round(2 * total / (ms * 1e-3) / 1e9, 1)}),
                      flush=True)
        g.netc_gpu_tune(2, 0, -1)
        del bufs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
