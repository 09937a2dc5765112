#!/usr/bin/env python3
"""HBM stream ceilings on the box (diagnostic): netc_amd/lib/libnetc_ceiling.so swept over
mode x policy x chunk x workgroup size x grid, at 64 MiB (rotating over 2 GiB) and 1 GiB,
next to the product mask kernel at C2 / C4 in the same process.  One JSON line per point."""

import argparse
import ctypes
import itertools
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

MODES = {0: "copy", 1: "xor_inplace", 2: "xor_oop", 3: "read", 4: "write"}
TRAFFIC = {0: 2, 1: 2, 2: 2, 3: 1, 4: 1}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="64,1024", help="MiB")
    ap.add_argument("--modes", default="0,1")
    ap.add_argument("--nt", default="0,1")
    ap.add_argument("--u", default="1,2,4,8")
    ap.add_argument("--threads", default="256,512,1024")
    ap.add_argument("--blocks", default="0,-1", help="0 = one resident round, -1 = one chunk per wave, N = fixed")
    ap.add_argument("--reps", type=int, default=40)
    ap.add_argument("--mask", action="store_true", help="also time the product mask kernel (c2, c4)")
    ap.add_argument("--walk", action="store_true", help="sweep netc_ceiling_walk instead")
    ap.add_argument("--pipe", default="0,1")
    ap.add_argument("--k", default="1,2,4,8,16")
    ap.add_argument("--lds", default="4,16384,32768")
    args = ap.parse_args()
    import torch

    dev = torch.device("cuda", 0)
    torch.cuda.init()
    s = torch.cuda.Stream(dev)
    lib = ctypes.CDLL(os.path.join(ROOT, "netc_amd", "lib", "libnetc_ceiling.so"))
    lib.netc_ceiling_stream.argtypes = [ctypes.c_int] * 5 + [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                                             ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]
    lib.netc_ceiling_walk.argtypes = [ctypes.c_int] * 8 + [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                                           ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]
    sink = torch.zeros(1024, dtype=torch.int32, device=dev)

    def timeit(fn, reps):
        with torch.cuda.stream(s):
            for i in range(4):
                fn(i)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            a.record(s)
            for i in range(reps):
                fn(4 + i)
            b.record(s)
            torch.cuda.synchronize()
        return a.elapsed_time(b) / reps

    for size_mib in [int(x) for x in args.sizes.split(",")]:
        size = size_mib << 20
        nb = max(3, (2 << 30) // size + 1)
        bufs = [torch.randint(0, 256, (size,), dtype=torch.uint8, device=dev) for _ in range(nb)]
        reps = args.reps if size_mib < 1024 else max(6, args.reps // 4)
        if args.walk:
            walk(args, lib, bufs, nb, size, size_mib, reps, sink, s, timeit)
            del bufs
            torch.cuda.empty_cache()
            continue
        for mode, nt, u, th, bl in itertools.product([int(x) for x in args.modes.split(",")],
                                                     [int(x) for x in args.nt.split(",")],
                                                     [int(x) for x in args.u.split(",")],
                                                     [int(x) for x in args.threads.split(",")],
                                                     [int(x) for x in args.blocks.split(",")]):
            def fn(i):
                src = bufs[i % nb]
                dst = bufs[(i + nb // 2) % nb] if mode in (0, 2) else src   # not written by the last steps
                rc = lib.netc_ceiling_stream(mode, nt, u, th, bl, dst.data_ptr(), src.data_ptr(), size, 0x5A5A5A5A,
                                             sink.data_ptr(), s.cuda_stream)
                assert rc == 0, rc
            ms = timeit(fn, reps)
            print(json.dumps({"MiB": size_mib, "mode": MODES[mode], "nt": nt, "u": u, "threads": th, "blocks": bl,
                              "us": round(ms * 1e3, 2),
                              "GBps": round(TRAFFIC[mode] * size / (ms * 1e-3) / 1e9, 1)}), flush=True)
        del bufs
        torch.cuda.empty_cache()

    if args.mask:
        from netc_amd import _lib, synth
        g = _lib.gpu()
        for wl in ("c2", "c4"):
            off, keys, total = synth.config(wl)
            nb = max(3, (2 << 30) // total + 1)
            bufs = [torch.randint(0, 256, (total,), dtype=torch.uint8, device=dev) for _ in range(nb)]
            off_t = torch.from_numpy(off.view(np.int64)).to(dev)
            keys_t = torch.from_numpy(keys.view(np.int32)).to(dev)
            for unroll, mb in ((4, 0), (8, 0), (2, 0), (1, 0)):
                assert g.netc_gpu_tune(unroll, mb, -1) == 0

                def fn(i):
                    p = bufs[i % nb].data_ptr()
                    assert g.netc_gpu_mask_batch(0, p, p, total, off_t.data_ptr(), keys_t.data_ptr(), keys.size,
                                                 s.cuda_stream) == 0
                ms = timeit(fn, args.reps if total < (1 << 30) else 10)
                print(json.dumps({"mask": wl, "unroll": unroll, "max_blocks": mb, "us": round(ms * 1e3, 2),
                                  "GBps": round(2 * total / (ms * 1e-3) / 1e9, 1)}), flush=True)
            g.netc_gpu_tune(4, 0, -1)
            del bufs
            torch.cuda.empty_cache()


def walk(args, lib, bufs, nb, size, size_mib, reps, sink, s, timeit):
    ints = lambda x: [int(v) for v in x.split(",")]
    for mode, nt, u, pipe, th in itertools.product(ints(args.modes), ints(args.nt), ints(args.u), ints(args.pipe),
                                                   ints(args.threads)):
        for bl, k, lds in [(b, kk, l) for b in ints(args.blocks) for kk in (ints(args.k) if b < 0 else [1])
                           for l in ints(args.lds)]:
            def fn(i):
                src = bufs[i % nb]
                dst = bufs[(i + nb // 2) % nb] if mode in (0, 2) else src
                rc = lib.netc_ceiling_walk(mode, nt, u, pipe, k, th, bl, lds, dst.data_ptr(), src.data_ptr(), size,
                                           0x5A5A5A5A, sink.data_ptr(), s.cuda_stream)
                assert rc == 0, rc
            ms = timeit(fn, reps)
            print(json.dumps({"MiB": size_mib, "mode": MODES[mode], "nt": nt, "u": u, "pipe": pipe, "k": k,
                              "threads": th, "blocks": bl, "lds": lds, "us": round(ms * 1e3, 2),
                              "GBps": round(TRAFFIC[mode] * size / (ms * 1e-3) / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
