#!/usr/bin/env python3
"""Diagnostic: frame-table size of the masking kernel (adaptive vs pinned 64 / 16 entries),
single stream, back-to-back launches over rotating batches, GPU time from two events."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    from netc_amd import _lib, synth
    from netc_amd import mask as nm

    dev = torch.device("cuda", 0)
    entry = _lib.gpu().netc_gpu_mask_batch
    s = torch.cuda.Stream(dev)
    sh = s.cuda_stream
    for wl in ("c2", "c3", "c4"):
        off, keys, total = synth.config(wl)
        nb = max(2, (2 << 30) // total)
        bufs = [torch.randint(0, 256, (total,), dtype=torch.uint8, device=dev) for _ in range(nb)]
        ptrs = [b.data_ptr() for b in bufs]
        off_t = torch.from_numpy(off.view(np.int64)).to(dev)
        keys_t = torch.from_numpy(keys.view(np.int32)).to(dev)
        torch.cuda.synchronize()
        K = 200 if wl == "c2" else 20

        def timed(flags):
            nm.tune(4, 0, flags)

            def f(i):
                entry(0, ptrs[i % nb], ptrs[i % nb], total, off_t.data_ptr(), keys_t.data_ptr(), keys.size, sh)

            for i in range(5):
                f(i)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            for i in range(K):
                f(i)
            b.record(s)
            torch.cuda.synchronize()
            return a.elapsed_time(b) / K * 1e3

        for rnd in range(3):
            for name, flags in (("adaptive", -1), ("table64", 3 | 4), ("table16", 3 | 8)):
                us = timed(flags)
                print(f"{wl} round{rnd} {name:9s} {us:8.2f} us  {2 * total / (us * 1e-6) / 1e9:7.1f} GB/s", flush=True)
        nm.tune()
        del bufs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
