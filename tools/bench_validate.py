#!/usr/bin/env python3
"""Fused unmask + UTF-8 validation (netc_gpu_unmask_validate) vs plain unmask (netc_gpu_mask_batch).

TEXT payloads (JSON-like ASCII with 2/3/4-byte code points; every frame a valid
one-frame message except 1 % with one broken byte), in the config-2 frame shape
(65,536 x 1 KiB) and a 1 GiB config-4 size mix, out of place from masked text (so
every step unmasks to text) into rotating buffers.  The verdicts are checked
against the oracle.
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


# share of multi-byte code points per --text kind: "dense" (the default, about one character in
# 16: every 1 KiB span of a wavefront holds some), "sparse" (one in 4,096: most spans are pure
# ASCII), "ascii" (none: the per-span ASCII early-out takes every span)
WIDE_SHARE = {"dense": 0.06, "sparse": 1 / 4096, "ascii": 0.0}


def valid_text(rng, off, total, kind="dense"):
    """UTF-8 text, every frame (a one-frame TEXT message) valid on its own: JSON-like ASCII
    with 2-, 3- and 4-byte code points (WIDE_SHARE[kind] of the characters), tiled from a 1 MiB
    sample; a code point cut by a frame edge is replaced by ASCII 'x' bytes."""
    ascii_toks = [c.encode() for c in 'abcdefghijklmnopqrstuvwxyz {}[]":,0123456789']
    wide_toks = [c.encode() for c in "éü€中😀"]
    toks = ascii_toks + wide_toks
    w = WIDE_SHARE[kind]
    p = [(1 - w) / len(ascii_toks)] * len(ascii_toks) + [w / len(wide_toks)] * len(wide_toks)
    pick = rng.choice(len(toks), size=1 << 20, p=p)
    sample = np.frombuffer(b"".join(toks[i] for i in pick), dtype=np.uint8)
    text = np.resize(sample, total).copy()
    x = np.uint8(ord("x"))
    starts = off[:-1].astype(np.int64)
    ends = off[1:].astype(np.int64)
    ends = ends[ends > starts]
    # a frame's last bytes: a lead byte whose sequence runs past the frame end
    for back, lead in ((1, 0xC0), (2, 0xE0), (3, 0xF0)):
        e = ends[ends - back >= 0] - back
        hit = e[(text[e] >= lead) & (e + back <= total)]
        for j in range(back):
            text[hit + j] = x
    # a frame's first bytes: continuation bytes with no lead in the frame
    s0 = starts[starts < total]
    run = np.ones(s0.size, dtype=bool)
    for j in range(3):
        q = np.minimum(s0 + j, total - 1)
        run &= (text[q] & 0xC0) == 0x80
        text[q[run]] = x
    return text


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--text", default="dense", choices=sorted(WIDE_SHARE))
    ap.add_argument("--workloads", default="c2,c4")
    args = ap.parse_args()

    import torch

    from netc_amd import _lib, synth

    dev = torch.device("cuda", 0)
    lib = _lib.gpu()
    s = torch.cuda.Stream(dev)
    sh = s.cuda_stream
    rng = np.random.default_rng(9)
    for wl in args.workloads.split(","):
        off, keys, total = synth.config(wl)
        n = keys.size
        text = valid_text(rng, off, total, args.text)
        # 1 % of the frames (messages) broken: one 0xFF byte somewhere in the frame
        bad = rng.choice(n, size=max(1, n // 100), replace=False)
        lens = (off[bad + 1] - off[bad]).astype(np.int64)
        pos = off[bad].astype(np.int64) + (rng.random(bad.size) * np.maximum(lens, 1)).astype(np.int64)
        text[pos[lens > 0]] = 0xFF
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
        from oracle import oracle as orc

        exp = orc.validate_batch(text, off, np.full(n, 0x81, dtype=np.uint8))
        print(json.dumps({"workload": wl, "text": args.text, "wide_share": WIDE_SHARE[args.text], "frames": int(n), "payload_bytes": int(total),
                          "validate_us": round(us_v, 2), "mask_only_us": round(us_m, 2),
                          "validate_GBps": round(2 * total / (us_v * 1e-6) / 1e9, 1),
                          "mask_only_GBps": round(2 * total / (us_m * 1e-6) / 1e9, 1),
                          "overhead": round(us_v / us_m - 1, 4), "output_is_the_text": ok,
                          "frames_invalid": int((valid == 0).sum().item()),
                          "verdicts_match_oracle": bool(np.array_equal(valid.cpu().numpy(), exp))}), flush=True)
        del bufs, t_text, src
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
