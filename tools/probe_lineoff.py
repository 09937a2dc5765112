"""Probe: does a 16-B-aligned but not 128-B-aligned source cost a stream copy time?

Times the in-bench float4 copy (netc_ceiling_walk mode 0, NT, 2 x 1 KiB per wavefront)
with the source pointer moved by 0 / 16 / 48 / 112 / 128 bytes from a 4 KiB boundary,
destination 4 KiB-aligned, at 64 MiB and 1 GiB.  Prints one JSON line per point.
A 16 KiB wave span read at an offset that is not a multiple of 128 touches 9 lines per
1 KiB instead of 8 (the question behind the misaligned mask path)."""
import ctypes
import json
import os

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    lib = ctypes.CDLL(os.path.join(ROOT, "netc_amd", "lib", "libnetc_ceiling.so"))
    lib.netc_ceiling_walk.argtypes = [ctypes.c_int] * 8 + [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                                           ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]
    dev = torch.device("cuda:0")
    stream = torch.cuda.Stream(dev)
    sink = torch.zeros(1024, dtype=torch.int32, device=dev)
    for total in (64 << 20, 1 << 30):
        nb = max(4, (2 << 30) // total)
        bufs = [torch.empty(total + 8192, dtype=torch.uint8, device=dev) for _ in range(nb)]
        n = total - 1024
        for off in (0, 16, 48, 112, 128, 0):
            def launch(i):
                src = bufs[i % nb].data_ptr() + off
                dst = bufs[(i + nb // 2) % nb].data_ptr()
                rc = lib.netc_ceiling_walk(0, 1, 1, 0, 2, 256, -1, 4, dst, src, n, 0x5A5A5A5A,
                                           sink.data_ptr(), stream.cuda_stream)
                assert rc == 0, rc
            for i in range(6):
                launch(i)
            steps = 40 if total < (1 << 30) else 20
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record(stream)
            for i in range(steps):
                launch(6 + i)
            e1.record(stream)
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / steps * 1e3
            print(json.dumps({"total": total, "src_off": off, "us": round(us, 2),
                              "GBps": round(2.0 * n / (us * 1e-6) / 1e9, 1)}), flush=True)
        del bufs


if __name__ == "__main__":
    main()
