"""Diagnostic: one scan per stream shape with its wall time and path (one pass or graph), flushed per
line -- for finding a slow or stuck case quickly on the GPU box.  With the trace build
(NETC_GPU_LIB=diag/libnetc_ws_gpu_trace.so) the one-pass kernels' progress words (host-mapped)
are printed while a scan runs, and a scan that does not finish within --limit seconds ends the
process after printing them."""
import argparse
import ctypes
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", default="tiny5,small,dense1k_x100,dense1k_x5000,mixed,c2")
    ap.add_argument("--limit", type=float, default=15.0)
    ap.add_argument("--stamps", action="store_true",
                    help="trace build: after each case, one more call with the one-pass timestamps (OP_STAMP) printed")
    args = ap.parse_args()
    import torch

    from netc_amd import _lib
    from netc_amd import mask as nm
    from tests.test_gpu_scan import _stream, run_scan

    trace = None
    lib = _lib.gpu()
    if hasattr(lib, "netc_gpu_debug_scan_trace"):
        trace = torch.zeros(16, dtype=torch.int32).pin_memory()
        lib.netc_gpu_debug_scan_trace.argtypes = [ctypes.c_void_p]
        assert lib.netc_gpu_debug_scan_trace(trace.data_ptr()) == 0
    rng = np.random.default_rng(1)
    cases = {
        "tiny5": lambda: np.frombuffer(bytes.fromhex("8185") + bytes(4) + b"Hello", dtype=np.uint8).copy(),
        "small": lambda: _stream(rng, rng.integers(0, 100, 10))[0],
        "dense1k_x100": lambda: _stream(rng, np.full(100, 1024))[0],
        "dense1k_x5000": lambda: _stream(rng, np.full(5000, 1024))[0],
        "mixed": lambda: _stream(rng, rng.integers(0, 5000, 300))[0],
        "c2": lambda: _stream(rng, np.full(65536, 1024))[0],
    }
    for name in args.cases.split(","):
        wire = cases[name]()
        if trace is not None:
            trace.zero_()
        box = {}

        def go():
            t0 = time.perf_counter()
            try:
                box["n"] = run_scan(torch, wire)
            except BaseException as e:   # (reported below)
                box["err"] = repr(e)
            box["dt"] = time.perf_counter() - t0

        th = threading.Thread(target=go, daemon=True)
        th.start()
        th.join(args.limit)
        tr = trace.tolist() if trace is not None else None
        if th.is_alive():
            print(f"{name}: STUCK after {args.limit} s; trace {tr}", flush=True)
            os._exit(3)
        print(f"{name}: {wire.size} B, {box.get('n')} frames, {box['dt'] * 1e3:.1f} ms, err {box.get('err')}, "
              f"onepass {nm.scan_onepass()}, diag {nm.scan_diag():#x}, trace {tr}", flush=True)
        if args.stamps and hasattr(lib, "netc_gpu_debug_scan_stamps"):
            stamps(torch, lib, run_scan, wire, name)


def stamps(torch, lib, run_scan, wire, name):
    """OP_STAMP words of one call (ws_scan_gpu.hip, trace build), in 100 MHz ticks -> us"""
    buf = torch.zeros(16, dtype=torch.int64, device="cuda")
    buf[0] = (1 << 62)
    lib.netc_gpu_debug_scan_stamps.argtypes = [ctypes.c_void_p]
    assert lib.netc_gpu_debug_scan_stamps(buf.data_ptr()) == 0
    run_scan(torch, wire)
    torch.cuda.synchronize()
    assert lib.netc_gpu_debug_scan_stamps(None) == 0
    v = buf.cpu().numpy()
    t0 = int(v[0])
    us = lambda t: (int(t) - t0) / 100.0 if t else None
    out = {"case": name, "k1_start": 0.0, "k1_last_wave_end": us(v[1]), "t_none": int(v[5]), "t_single": int(v[6]),
           "t_multi": int(v[7]), "t_fail": int(v[8])}
    import json
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
