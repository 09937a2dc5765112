#!/usr/bin/env python3
"""Why BASELINE config 5 runs slower in place than out of place.

Two pinned host arrays A and B (netc_gpu_host_alloc), each `--gib` GiB of 4 KiB frames,
streamed through one persistent handle (2 x 512 MiB slots) in every source/destination
combination: A->B, B->A, A->A (in place), B->B (in place), best of 3 passes each, plus the
NUMA node each array's first page sits on (/proc/self/numa_maps, when readable).  If the
in-place rate follows the array rather than the in/out shape, the gap is where the host
memory lives, not the pipeline.  One JSON line.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def numa_node(addr: int):
    """the N<node>=<pages> fields of the mapping holding addr (the one with the largest start <= addr)"""
    try:
        best = None
        with open("/proc/self/numa_maps") as f:
            for line in f:
                parts = line.split()
                start = int(parts[0], 16)
                if start <= addr and (best is None or start > best[0]):
                    best = (start, [p for p in parts if p.startswith("N") and "=" in p])
        return " ".join(best[1]) if best else None
    except (OSError, ValueError):
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=4.0)
    ap.add_argument("--passes", type=int, default=3)
    args = ap.parse_args()

    import torch  # noqa: F401  (one HIP runtime: torch's)

    from netc_amd import mask as nm
    from netc_amd import synth

    total = int(args.gib * (1 << 30)) // 4096 * 4096
    n = total // 4096
    off = synth.uniform_offsets(n, 4096)
    keys = synth.random_keys(n, stream=900)
    A, B = nm.PinnedArray(total), nm.PinnedArray(total)
    out = {"gib": total / (1 << 30), "frames": n}
    try:
        synth.fill_payload(A.array)
        synth.fill_payload(B.array, stream=4)
        out["numa_A"] = numa_node(A.array.ctypes.data)
        out["numa_B"] = numa_node(B.array.ctypes.data)
        with nm.HostStream(0) as hs:
            for name, src, dst in (("A_to_B", A, B), ("B_to_A", B, A), ("A_in_place", A, A), ("B_in_place", B, B),
                                   ("A_to_B_again", A, B)):
                best = None
                for _ in range(args.passes):
                    t0 = time.perf_counter()
                    hs.mask(dst.array, src.array, off, keys)
                    dt = time.perf_counter() - t0
                    best = dt if best is None else min(best, dt)
                out[name + "_GiBps"] = round(total / best / (1 << 30), 2)
    finally:
        A.close()
        B.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
