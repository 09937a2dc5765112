#!/usr/bin/env python3
"""Diagnostic: walk order of an in-place XOR stream (tools/diag_order.hip) vs the masking kernel,
single stream, back-to-back launches, GPU time from two events around the whole loop."""
import ctypes
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
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "libdiag_order.so"))
    lib.diag_order.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int,
                               ctypes.c_void_p, ctypes.c_void_p]
    ds = ctypes.CDLL(os.path.join(ROOT, "tools", "libdiag_stream.so"))
    ds.diag_stream.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                               ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    entry = _lib.gpu().netc_gpu_mask_batch
    ticket = torch.zeros(16, dtype=torch.int64, device=dev)
    sink = torch.zeros(1 << 20, dtype=torch.int32, device=dev)
    s = torch.cuda.Stream(dev)
    sh = s.cuda_stream
    for wl in ("c2", "c4"):
        off, keys, total = synth.config(wl)
        nb = max(2, (2 << 30) // total)
        bufs = [torch.randint(0, 256, (total,), dtype=torch.uint8, device=dev) for _ in range(nb)]
        ptrs = [b.data_ptr() for b in bufs]
        off_t = torch.from_numpy(off.view(np.int64)).to(dev)
        keys_t = torch.from_numpy(keys.view(np.int32)).to(dev)
        torch.cuda.synchronize()
        K = 200 if wl == "c2" else 20

        def timed(fn):
            for i in range(5):
                fn(i)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            for i in range(K):
                fn(i)
            b.record(s)
            torch.cuda.synchronize()
            return a.elapsed_time(b) / K * 1e3

        variants = []
        for order in (1, 2, 3):
            for blocks in (1024, 2048):
                variants.append((f"order{order} blocks{blocks}",
                                 lambda i, o=order, bl=blocks: lib.diag_order(o, ptrs[i % nb], total, 0x5A5A5A5A, bl,
                                                                             ticket.data_ptr(), sh)))
        variants.append(("diag gridstride nt", lambda i: ds.diag_stream(0, 1, 0, ptrs[i % nb], ptrs[i % nb], total,
                                                                        0x5A5A5A5A, 2048, sink.data_ptr(), sh)))
        for flags in (7, 3):
            def f(i, fl=flags):
                entry(0, ptrs[i % nb], ptrs[i % nb], total, off_t.data_ptr(), keys_t.data_ptr(), keys.size, sh)
            variants.append((f"mask flags{flags}", (lambda fl: (lambda i: (nm.tune(4, 0, fl), f(i, fl))))(flags)))
        for rnd in range(3):
            for name, fn in variants:
                us = timed(fn)
                print(f"{wl} round{rnd} {name:22s} {us:8.2f} us  {2 * total / (us * 1e-6) / 1e9:7.1f} GB/s", flush=True)
        del bufs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
