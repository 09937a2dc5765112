#!/usr/bin/env python3
"""Diagnostic: host-side launch loop shapes for the masking kernel (1 vs 2 streams, events)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    from netc_amd import _lib, synth
    from netc_amd import mask as nm

    dev = torch.device("cuda", 0)
    off, keys, total = synth.config("c2")
    nb = 32
    bufs = [torch.randint(0, 256, (total,), dtype=torch.uint8, device=dev) for _ in range(nb)]
    off_t = torch.from_numpy(off.view(np.int64)).to(dev)
    keys_t = torch.from_numpy(keys.view(np.int32)).to(dev)
    torch.cuda.synchronize()
    entry = _lib.gpu().netc_gpu_mask_batch
    ptrs = [b.data_ptr() for b in bufs]
    o, k, n = off_t.data_ptr(), keys_t.data_ptr(), keys.size
    sA, sB = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    K = 400

    def loop(streams, events=False):
        hs = [s.cuda_stream for s in streams]
        ev = []
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(K):
            s = streams[i % len(streams)]
            if events:
                a = torch.cuda.Event(enable_timing=True)
                a.record(s)
            entry(0, ptrs[i % nb], ptrs[i % nb], total, o, k, n, hs[i % len(hs)])
            if events:
                b = torch.cuda.Event(enable_timing=True)
                b.record(s)
                ev.append((a, b))
        t_host = time.perf_counter() - t0
        torch.cuda.synchronize()
        t = time.perf_counter() - t0
        km = np.mean([a.elapsed_time(b) for a, b in ev]) * 1e3 if ev else None
        return t / K * 1e6, t_host / K * 1e6, km

    for rnd in range(2):
        for name, ss, ev in [("1 stream", [sA], False), ("1 stream + events", [sA], True),
                             ("2 streams", [sA, sB], False), ("2 streams + events", [sA, sB], True),
                             ("NULL stream", [torch.cuda.default_stream(dev)], False)]:
            us, host_us, km = loop(ss, ev)
            print(f"round {rnd} {name:22s} step {us:7.2f} us  host {host_us:7.2f} us  kernel {km}", flush=True)
    for flags in (3, 7):
        nm.tune(4, 0, flags)
        for name, ss in [("1 stream", [sA]), ("2 streams", [sA, sB])]:
            us, host_us, km = loop(ss)
            print(f"flags {flags} {name:12s} step {us:7.2f} us host {host_us:7.2f}", flush=True)


if __name__ == "__main__":
    main()
