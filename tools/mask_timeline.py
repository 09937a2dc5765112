#!/usr/bin/env python3
"""Diagnostic: per-wave start / end timeline of ONE headline mask launch.

Loads tools/libnetc_ws_gpu_stamps.so (`make diag`: the product sources built with
-DNETC_MASK_STAMPS, each wavefront of mask_np_kernel writes s_memrealtime at entry and exit,
100 MHz) and launches netc_gpu_mask_batch with the library's default launch shape on the
config-2 batch (64 MiB, 65,536 x 1 KiB frames, in place), rotating over 2 GiB of batches like
bench.py.  The stamp buffer holds two words for every window of the launch (a window is at
least 1 KiB, so total / 1024 + 1024 windows bound the wave index).

Output: one JSON line per launch shape: the launch span (first wave start -> last wave end),
percentiles of wave start, end and duration, the ramp (time until 99 % of the waves have
started) and the tail (time from 90 % of the waves ended to the last), and the rate over the
span.
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
    ap.add_argument("--workload", default="c2", choices=("c2", "c3"))
    ap.add_argument("--reps", type=int, default=8)
    args = ap.parse_args()

    import torch

    from netc_amd import synth

    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream(dev)
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "libnetc_ws_gpu_stamps.so"))
    lib.netc_gpu_mask_batch.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
    lib.netc_gpu_debug_stamps.argtypes = [ctypes.c_void_p]
    off, keys, total = synth.config(args.workload)
    nwin_max = total // 1024 + 1024
    stamps = torch.zeros(2 * nwin_max, dtype=torch.int64, device=dev)
    assert lib.netc_gpu_debug_stamps(stamps.data_ptr()) == 0
    nb = max(2, (2 << 30) // total)
    bufs = [torch.randint(0, 256, (total,), dtype=torch.uint8, device=dev) for _ in range(nb)]
    off_t = torch.from_numpy(off.view(np.int64)).to(dev)
    keys_t = torch.from_numpy(keys.view(np.int32)).to(dev)
    torch.cuda.synchronize()
    rows = []
    for i in range(args.reps):
        stamps.zero_()
        torch.cuda.synchronize()
        p = bufs[i % nb].data_ptr()
        assert lib.netc_gpu_mask_batch(0, p, p, total, off_t.data_ptr(), keys_t.data_ptr(), keys.size,
                                       s.cuda_stream) == 0
        torch.cuda.synchronize()
        st = stamps.view(-1, 2).cpu().numpy()
        st = st[st[:, 1] > 0]
        t0 = st[:, 0].min()
        start = (st[:, 0] - t0) * 10e-3   # us (100 MHz)
        end = (st[:, 1] - t0) * 10e-3
        rows.append((start, end))
    q = lambda x: [round(float(v), 2) for v in np.percentile(x, [0, 1, 10, 50, 90, 99, 100])]
    for i, (start, end) in enumerate(rows):
        if i < 2:
            continue   # warm-up launches
        dur = end - start
        span = float(end.max())
        r = {"workload": args.workload, "launch": i, "waves": int(start.size), "span_us": round(span, 2),
             "start_pct_0_1_10_50_90_99_100": q(start), "end_pct": q(end), "dur_pct": q(dur),
             "ramp_us_99pct_started": round(float(np.percentile(start, 99)), 2),
             "tail_us_after_90pct_ended": round(span - float(np.percentile(end, 90)), 2),
             "GBps_over_span": round(2 * total / (span * 1e-6) / 1e9, 1)}
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
