#!/usr/bin/env python3
"""Diagnostic: frame-assembly launches at frame counts from 1 to 1M over 64 MiB of
payload, for the per-kernel durations under rocprofv3 (tools/trace_tool.sh).  One JSON
line per case with the whole call's event time."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from netc_amd import mask as nm  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    total = 64 << 20
    src = torch.randint(0, 256, (total,), dtype=torch.uint8, device=dev)
    for n in (1, 1024, 65536, 1 << 20):
        off = torch.linspace(0, total, n + 1, device=dev).to(torch.int64)
        off[-1] = total
        keys = torch.randint(-2**31, 2**31 - 1, (n,), dtype=torch.int32, device=dev)
        wire = torch.empty(total + 14 * n + 64, dtype=torch.uint8, device=dev)
        wo = torch.empty(n + 1, dtype=torch.int64, device=dev)
        for _ in range(3):
            nm.encode_frames(wire, wo, src, off, keys)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 20
        e0.record()
        for _ in range(reps):
            nm.encode_frames(wire, wo, src, off, keys)
        e1.record()
        torch.cuda.synchronize()
        print(json.dumps({"frames": n, "us_per_call": round(e0.elapsed_time(e1) * 1000 / reps, 2)}), flush=True)


if __name__ == "__main__":
    main()
