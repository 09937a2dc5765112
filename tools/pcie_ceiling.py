#!/usr/bin/env python3
"""Host-link ceiling on the GPU box, for BASELINE config 5 and the ingest ring: pinned
host <-> device copies of 256 MiB (hipMemcpyAsync through torch), H2D alone, D2H
alone, and both directions at once on two streams (what an overlapped H2D / kernel /
D2H pipeline can reach at best).  One JSON line; GB/s = 1e9 bytes / s."""
import json
import time

import torch


def main():
    n = 256 << 20
    reps = 8
    dev = torch.device("cuda", 0)
    h_in = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    h_out = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    d_a = torch.empty(n, dtype=torch.uint8, device=dev)
    d_b = torch.empty(n, dtype=torch.uint8, device=dev)
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    for _ in range(2):   # warm-up
        d_a.copy_(h_in, non_blocking=True)
        h_out.copy_(d_b, non_blocking=True)
    torch.cuda.synchronize()

    def timed(fn):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / reps

    def h2d():
        with torch.cuda.stream(s1):
            d_a.copy_(h_in, non_blocking=True)

    def d2h():
        with torch.cuda.stream(s2):
            h_out.copy_(d_b, non_blocking=True)

    def both():
        h2d()
        d2h()

    t_h2d, t_d2h, t_both = timed(h2d), timed(d2h), timed(both)
    print(json.dumps({"bytes_per_copy": n, "h2d_GBps": round(n / t_h2d / 1e9, 2), "d2h_GBps": round(n / t_d2h / 1e9, 2),
                      "bidirectional_GBps_each_way": round(n / t_both / 1e9, 2),
                      "bidirectional_GiBps_each_way": round(n / t_both / 2**30, 2),
                      "note": "pinned host memory, 256 MiB per copy, torch non_blocking copies on dedicated streams"}),
          flush=True)


if __name__ == "__main__":
    main()
