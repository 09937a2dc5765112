#!/usr/bin/env python3
"""Diagnostic: cost of unaligned 16-B source loads (tools/diag_policy.hip diag_shift) in an
out-of-place XOR stream, by source byte shift; single stream, rotating 1 GiB of buffers."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    dev = torch.device("cuda", 0)
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "libdiag_policy.so"))
    lib.diag_shift.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_uint32,
                               ctypes.c_int, ctypes.c_void_p]
    s = torch.cuda.Stream(dev)
    for size in (64 << 20, 1 << 30):
        nb = max(2, (2 << 30) // size)
        bufs = [torch.randint(0, 256, (size + 4096,), dtype=torch.uint8, device=dev) for _ in range(nb)]
        K = 100 if size < (1 << 30) else 10
        for shift in (0, 1, 4, 8, 13):
            for blocks in (1024, 2048):
                def f(i):
                    lib.diag_shift(bufs[(i + 1) % nb].data_ptr(), bufs[i % nb].data_ptr(), size, shift, 0x5A5A5A5A,
                                   blocks, s.cuda_stream)
                for i in range(5):
                    f(i)
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(s)
                for i in range(K):
                    f(i)
                b.record(s)
                torch.cuda.synchronize()
                us = a.elapsed_time(b) / K * 1e3
                print(f"{size >> 20} MiB shift {shift:2d} blocks {blocks}: {us:8.2f} us  {2 * size / (us * 1e-6) / 1e9:7.1f} GB/s",
                      flush=True)
        del bufs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
