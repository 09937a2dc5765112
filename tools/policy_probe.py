#!/usr/bin/env python3
"""Diagnostic: cache-policy bits (sc0 / nt / sc1) of an in-place XOR stream (tools/diag_policy.hip)
against the masking kernel, single stream, back-to-back launches, GPU time from two events."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CASES = [(0, 0), (2, 2), (2, 0), (0, 2), (2, 16), (2, 17), (2, 18), (0, 16), (1, 2), (2, 1), (16, 2), (3, 3)]


def main():
    import torch

    from netc_amd import _lib, synth

    dev = torch.device("cuda", 0)
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "libdiag_policy.so"))
    lib.diag_policy.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
                                ctypes.c_int, ctypes.c_void_p]
    entry = _lib.gpu().netc_gpu_mask_batch
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
        body = total // 4096 * 4096

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
        for la, sa in CASES:
            for blocks in (1024, 2048):
                variants.append((f"l{la:02d} s{sa:02d} b{blocks}", body,
                                 lambda i, la=la, sa=sa, bl=blocks: lib.diag_policy(la, sa, ptrs[i % nb], ptrs[i % nb], total,
                                                                                    0x5A5A5A5A, bl, sh)))
        for la, sa in ((2, 2), (0, 0), (2, 16)):
            variants.append((f"oop l{la:02d} s{sa:02d}", body,
                             lambda i, la=la, sa=sa: lib.diag_policy(la, sa, ptrs[(i + 1) % nb], ptrs[i % nb], total,
                                                                     0x5A5A5A5A, 1024, sh)))
        variants.append(("mask oop", total,
                         lambda i: entry(0, ptrs[(i + 1) % nb], ptrs[i % nb], total, off_t.data_ptr(),
                                         keys_t.data_ptr(), keys.size, sh)))
        variants.append(("mask kernel", total,
                         lambda i: entry(0, ptrs[i % nb], ptrs[i % nb], total, off_t.data_ptr(), keys_t.data_ptr(),
                                         keys.size, sh)))
        for rnd in range(2):
            for name, nbytes, fn in variants:
                us = timed(fn)
                print(f"{wl} round{rnd} {name:18s} {us:8.2f} us  {2 * nbytes / (us * 1e-6) / 1e9:7.1f} GB/s",
                      flush=True)
        del bufs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
