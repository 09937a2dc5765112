#!/usr/bin/env python3
"""Diagnostic: where the frame scan's time goes, from in-kernel wall-clock stamps.

Loads tools/libnetc_ws_gpu_stamps.so (`make diag`: the product sources built with
-DNETC_SCAN_STAMPS) and runs netc_gpu_scan_frames on the config-2 / config-4 shaped
streams of tools/bench_scan.py.  Each of the five kernels stamps, per block, its
start, its phase ends and its end (s_memrealtime, 100 MHz).  Per kernel the output
gives the span (first block start -> last block end), the gap to the next kernel,
and for the single-block / per-tile kernels the median duration of each phase.
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("NETC_GPU_LIB", os.path.join(ROOT, "tools", "libnetc_ws_gpu_stamps.so"))

NAMES = ["K1 scan_exits", "K2 scan_links", "K3a scan_tiles", "K3b scan_resolve", "K4 scan_emit"]
BLOCKS = 8192


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workloads", default="c2,c4")
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()

    import ctypes

    import torch

    from netc_amd import _lib, synth
    from oracle import oracle as orc

    lib = _lib.gpu()
    lib.netc_gpu_debug_scan_stamps.argtypes = [ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    stamps = torch.zeros(5 * BLOCKS * 8, dtype=torch.int64, device=dev)
    assert lib.netc_gpu_debug_scan_stamps(stamps.data_ptr()) == 0
    if hasattr(lib, "netc_gpu_debug_dense_phases"):
        lib.netc_gpu_debug_dense_phases.argtypes = [ctypes.c_void_p, ctypes.c_int]
    s = torch.cuda.Stream(dev)
    for wl in args.workloads.split(","):
        if wl.startswith("u"):   # uniform frames of int(wl[1:]) payload bytes, 64 MiB of payload
            fb = int(wl[1:])
            nf = (64 << 20) // fb
            off = np.arange(nf + 1, dtype=np.uint64) * np.uint64(fb)
            keys = np.random.default_rng(3).integers(0, 2**32, nf, dtype=np.uint64).astype(np.uint32)
        else:
            off, keys, total = synth.config(wl)
        if wl == "c4":
            cut = int(np.searchsorted(off, 256 << 20))
            off, keys = off[: cut + 1], keys[:cut]
        rng = np.random.default_rng(5)
        payload = rng.integers(0, 256, int(off[-1]), dtype=np.uint8)
        wire, _ = orc.encode_batch(payload, off, keys, None, True)
        n = keys.size
        w = torch.from_numpy(wire).to(dev)
        hdr = torch.empty(n + 1, dtype=torch.int64, device=dev)
        kk = torch.empty(n, dtype=torch.int32, device=dev)
        b0 = torch.empty(n, dtype=torch.uint8, device=dev)
        res = torch.empty(3, dtype=torch.int64, device=dev)

        def step():
            rc = lib.netc_gpu_scan_frames(0, w.data_ptr(), wire.size, 0, 1, hdr.data_ptr(), kk.data_ptr(),
                                          b0.data_ptr(), n, res.data_ptr(), s.cuda_stream)
            assert rc == 0, lib.netc_gpu_strerror()

        for _ in range(5):
            step()
        torch.cuda.synchronize()
        reps = []
        for _ in range(args.reps):
            stamps.zero_()
            torch.cuda.synchronize()
            step()
            torch.cuda.synchronize()
            st = stamps.view(5, BLOCKS, 8).cpu().numpy().astype(np.int64)
            reps.append(st)
        assert int(res[0].item()) == n
        out = {"workload": wl, "frames": int(n), "wire_bytes": int(wire.size), "unit": "us", "kernels": []}
        spans, gaps, phases = [], [], []
        for st in reps:
            t0 = None
            row_span, row_gap, row_ph = [], [], []
            prev_end = None
            for k in range(5):
                blk = st[k]
                live = blk[:, 0] > 0
                starts, ends = blk[live, 0], blk[live, 7]
                ends = ends[ends > 0]
                if starts.size == 0 or ends.size == 0:   # not launched (e.g. K3b inside K3a's launch)
                    row_span.append((None, None, 0))
                    row_gap.append(None)
                    row_ph.append([None] * 7)
                    continue
                if t0 is None:
                    t0 = starts.min()
                row_span.append(((starts.min() - t0) / 100.0, (ends.max() - starts.min()) / 100.0, int(live.sum())))
                row_gap.append(None if prev_end is None else (starts.min() - prev_end) / 100.0)
                prev_end = ends.max()
                # phase medians over the live blocks: stamps 0..7 where set
                ph = []
                for i in range(1, 8):
                    if i in (5, 6) and k in (2, 3):   # counts, not times (SCAN_VALUE)
                        ph.append(float(np.median(blk[live, i])))
                        continue
                    ok = live & (blk[:, i] > 0)
                    prev = np.zeros(BLOCKS, dtype=np.int64)
                    for j in range(i - 1, -1, -1):   # the last set stamp before i
                        if j in (5, 6) and k in (2, 3):
                            continue
                        sel = (prev == 0) & (blk[:, j] > 0)
                        prev[sel] = blk[sel, j]
                    d = (blk[ok, i] - prev[ok]) / 100.0
                    ph.append(float(np.median(d)) if d.size else None)
                row_ph.append(ph)
            spans.append(row_span)
            gaps.append(row_gap)
            phases.append(row_ph)
        for k in range(5):
            def med(vals):
                v = [x for x in vals if x is not None]
                return round(float(np.median(v)), 2) if v else None
            out["kernels"].append({
                "kernel": NAMES[k],
                "blocks": spans[0][k][2],
                "start_after_first_us": med([r[k][0] for r in spans]),
                "span_us": med([r[k][1] for r in spans]),
                "gap_before_us": med([r[k] for r in gaps]),
                "phase_median_us": [med([r[k][i] for r in phases]) for i in range(7)],
            })
        last = [r[4][0] + r[4][1] for r in spans if r[4][0] is not None]
        out["first_start_to_last_end_us"] = round(float(np.median(last)), 2)
        if hasattr(lib, "netc_gpu_debug_dense_phases"):   # K2's per-wavefront dense path, summed over the reps
            ph = (ctypes.c_ulonglong * 8)()
            lib.netc_gpu_debug_dense_phases(ph, 1)
            calls = ph[7]
            if calls:
                names = ["load", "quick_check+list", "successors", "doubling", "walk", "link_node"]
                out["dense_phase_us_per_chunk"] = {nm: round(ph[i] / 100.0 / calls, 3) for i, nm in enumerate(names)}
                out["dense_chunks_per_call"] = calls / (args.reps + 5)
        print(json.dumps(out), flush=True)
        del w
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
