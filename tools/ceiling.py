#!/usr/bin/env python3
"""HBM ceilings for the masking access pattern + per-wave timing of the masking kernel (diagnostic).

1. tools/libdiag_stream.so: in-place XOR / read-only / write-only / copy streams,
   wave-contiguous vs grid-stride, plain vs non-temporal, at 64 MiB (rotating
   over >= 1 GiB) and 1 GiB; plus hipMemcpyAsync device-to-device.
2. tools/libnetc_ws_gpu_stamps.so (the product kernel built with per-wave
   s_memrealtime stamps): distribution of wave start / end times inside one launch.
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
    ap.add_argument("--part", default="streams,stamps")
    ap.add_argument("--reps", type=int, default=50)
    args = ap.parse_args()
    import torch

    dev = torch.device("cuda", 0)
    torch.cuda.init()
    s = torch.cuda.current_stream()
    res = []

    def timeit(fn, reps):
        for i in range(3):
            fn(i)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        a.record()
        for i in range(reps):
            fn(i)
        b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b) / reps

    if "streams" in args.part:
        diag = ctypes.CDLL(os.path.join(ROOT, "tools", "libdiag_stream.so"))
        diag.diag_stream.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                     ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
        hip = ctypes.CDLL("libamdhip64.so.7")
        hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
        sink = torch.zeros(1 << 20, dtype=torch.int32, device=dev)
        for size in (64 << 20, 1 << 30):
            nb = max(2, (2 << 30) // size)
            bufs = [torch.randint(0, 256, (size,), dtype=torch.uint8, device=dev) for _ in range(nb)]
            traffic = {0: 2, 1: 1, 2: 1, 3: 2}
            for mode in (0, 1, 2, 3):
                for nt in (0, 1):
                    for contig in (1, 0):
                        for blocks in (2048, 1024):
                            def fn(i):
                                src = bufs[i % nb]
                                dst = bufs[(i + 1) % nb] if mode == 3 else src
                                rc = diag.diag_stream(mode, nt, contig, dst.data_ptr(), src.data_ptr(), size,
                                                      0x5A5A5A5A, blocks, sink.data_ptr(), s.cuda_stream)
                                assert rc == 0
                            ms = timeit(fn, args.reps if size < (1 << 30) else 10)
                            r = {"size_MiB": size >> 20, "mode": ["xor_inplace", "read", "write", "copy"][mode],
                                 "nt": nt, "contig": contig, "blocks": blocks, "us": round(ms * 1e3, 2),
                                 "GBps": round(traffic[mode] * size / (ms * 1e-3) / 1e9, 1)}
                            res.append(r)
                            print(json.dumps(r), flush=True)

            def cp(i):
                hip.hipMemcpyAsync(bufs[(i + 1) % nb].data_ptr(), bufs[i % nb].data_ptr(), size, 3, s.cuda_stream)
            ms = timeit(cp, args.reps if size < (1 << 30) else 10)
            r = {"size_MiB": size >> 20, "mode": "hipMemcpyAsync_D2D", "us": round(ms * 1e3, 2),
                 "GBps": round(2 * size / (ms * 1e-3) / 1e9, 1)}
            print(json.dumps(r), flush=True)
            del bufs
            torch.cuda.empty_cache()

    if "stamps" in args.part:
        from netc_amd import synth

        lib = ctypes.CDLL(os.path.join(ROOT, "tools", "libnetc_ws_gpu_stamps.so"))
        lib.netc_gpu_mask_batch.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
        lib.netc_gpu_debug_stamps.argtypes = [ctypes.c_void_p]
        lib.netc_gpu_tune.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int]
        for wl in ("c2", "c4"):
            off, keys, total = synth.config(wl)
            # two words for every window the launch can have (a window is >= 1 KiB)
            stamps = torch.zeros(2 * (total // 1024 + 1024), dtype=torch.int64, device=dev)
            assert lib.netc_gpu_debug_stamps(stamps.data_ptr()) == 0
            nb = max(2, (2 << 30) // total)
            bufs = [torch.randint(0, 256, (total,), dtype=torch.uint8, device=dev) for _ in range(nb)]
            off_t = torch.from_numpy(off.view(np.int64)).to(dev)
            keys_t = torch.from_numpy(keys.view(np.int32)).to(dev)
            for flags in (0, 3):
                lib.netc_gpu_tune(4, 0, flags)
                for i in range(6):
                    stamps.zero_()
                    p = bufs[i % nb].data_ptr()
                    assert lib.netc_gpu_mask_batch(0, p, p, total, off_t.data_ptr(), keys_t.data_ptr(), keys.size,
                                                   s.cuda_stream) == 0
                    torch.cuda.synchronize()
                st = stamps.view(-1, 2).cpu().numpy()
                st = st[st[:, 1] > 0]
                t0 = st[:, 0].min()
                start = (st[:, 0] - t0) * 10e-3   # us (100 MHz)
                end = (st[:, 1] - t0) * 10e-3
                dur = end - start
                q = lambda x: [round(float(v), 2) for v in np.percentile(x, [0, 10, 50, 90, 99, 100])]
                r = {"workload": wl, "flags": flags, "waves": int(st.shape[0]),
                     "span_us": round(float(end.max()), 2),
                     "start_pct_0_10_50_90_99_100": q(start), "end_pct": q(end), "dur_pct": q(dur),
                     "bytes_GBps_over_span": round(2 * total / (end.max() * 1e-6) / 1e9, 1)}
                print(json.dumps(r), flush=True)
            del bufs
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
