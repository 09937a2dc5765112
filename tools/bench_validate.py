#!/usr/bin/env python3
"""Fused unmask + UTF-8 validation (netc_gpu_unmask_validate) vs plain unmask (netc_gpu_mask_batch).

TEXT payloads (mostly ASCII with multi-byte code points, as JSON-like text is), in
the config-2 frame shape (65,536 x 1 KiB) and a 1 GiB config-4 size mix, out of
place from masked text (so every step unmasks to text) into rotating buffers.
GPU time from two events around K steps on one stream over rotating batches.
Algorithmic bytes = 2 x payload (read + write) for both entries.
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=50)
    args = ap.parse_args()

    import torch

    from netc_amd import _lib, synth

    dev = torch.device("cuda", 0)
    lib = _lib.gpu()
    s = torch.cuda.Stream(dev)
    sh = s.cuda_stream
    rng = np.random.default_rng(9)
    pool = np.array([ord(c) for c in 'abcdefghijklmnopqrstuvwxyz {}[]":,0123456789'], dtype=np.uint8)
    for wl in ("c2", "c4"):
        off, keys, total = synth.config(wl)
        n = keys.size
        # text: ASCII from the pool with "é" (c3 a9) and "€" (e2 82 ac) sprinkled in
        text = pool[rng.integers(0, pool.size, total)]
        idx = rng.integers(0, total - 3, total // 64)
        text[idx], text[idx + 1] = 0xC3, 0xA9
        text[idx[::3]], text[idx[::3] + 1], text[idx[::3] + 2] = 0xE2, 0x82, 0xAC
        nb = max(2, (1 << 30) // total)
        t_text = torch.from_numpy(text).to(dev)
        off_t = torch.from_numpy(off.view(np.int64)).to(dev)
        keys_t = torch.from_numpy(keys.view(np.int32)).to(dev)
        src = torch.empty_like(t_text)   # the masked wire payload of the text
        lib.netc_gpu_mask_batch(0, src.data_ptr(), t_text.data_ptr(), total, off_t.data_ptr(), keys_t.data_ptr(), n,
                                None)
        bufs = [torch.empty_like(t_text) for _ in range(nb)]
        h0 = torch.full((n,), 0x81, dtype=torch.uint8, device=dev)
        valid = torch.empty(n, dtype=torch.uint8, device=dev)
        torch.cuda.synchronize()
        K = args.steps if wl == "c2" else max(10, args.steps // 5)

        def timed(fn):
            for i in range(3):
                fn(i)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            for i in range(K):
                fn(i)
            b.record(s)
            torch.cuda.synchronize()
            return a.elapsed_time(b) / K * 1e3

        def val(i):
            p = bufs[i % nb].data_ptr()
            rc = lib.netc_gpu_unmask_validate(0, p, src.data_ptr(), total, off_t.data_ptr(), keys_t.data_ptr(), h0.data_ptr(), n,
                                              valid.data_ptr(), sh)
            if rc:
                raise RuntimeError(lib.netc_gpu_strerror())

        def plain(i):
            p = bufs[i % nb].data_ptr()
            lib.netc_gpu_mask_batch(0, p, src.data_ptr(), total, off_t.data_ptr(), keys_t.data_ptr(), n, sh)

        us_v, us_m = timed(val), timed(plain)
        val(0)
        torch.cuda.synchronize()
        ok = bool(torch.equal(bufs[0], t_text))
        print(json.dumps({"workload": wl, "frames": int(n), "payload_bytes": int(total),
                          "validate_us": round(us_v, 2), "mask_only_us": round(us_m, 2),
                          "validate_GBps": round(2 * total / (us_v * 1e-6) / 1e9, 1),
                          "mask_only_GBps": round(2 * total / (us_m * 1e-6) / 1e9, 1),
                          "overhead": round(us_v / us_m - 1, 4), "output_is_the_text": ok,
                          "frames_invalid": int((valid == 0).sum().item())}), flush=True)
        del bufs, t_text, src
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
