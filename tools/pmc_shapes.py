"""HBM counter bytes of the mask kernel by buffer shape (is the frame assembly's
1.21x counter traffic real over-fetch, or the gfx950 FETCH_SIZE correction -- x2 for wide
coalesced 16-B reads, MI355X_MICROARCH.md -- misapplied to unaligned 16-B loads?).

The batch kernel (netc_gpu_mask_batch) on C2's frames, out of place over a 2 GiB rotation, with
the source at dst + SHIFT bytes: 0 (every load aligned), 3 and 8 (every 16-B load unaligned; the
assembly's loads at C2 are 8-B aligned, its frames moving the payload 8 bytes per frame).  The
algorithmic bytes are the same for every shape (read n + write n), so the counters' ratio to
them shows what the correction does with unaligned loads.  Run each shape under its own
rocprofv3 --pmc pass (FETCH_SIZE, then WRITE_SIZE):

    rocprofv3 --pmc FETCH_SIZE --kernel-include-regex mask_np_kernel -- python3 tools/pmc_shapes.py --shift 8
"""

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shift", type=int, default=0)
    ap.add_argument("--steps", type=int, default=20)
    args = ap.parse_args()
    import torch

    from netc_amd import mask as nm

    total, n, nb = 64 << 20, 65536, 32
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(7)
    bufs = [torch.randint(0, 256, (total,), dtype=torch.uint8, device=dev, generator=g) for _ in range(nb)]
    nbytes = total - args.shift
    off = torch.clamp(torch.arange(n + 1, dtype=torch.int64, device=dev) * 1024, max=nbytes)
    keys = torch.randint(-2**31, 2**31 - 1, (n,), dtype=torch.int32, device=dev, generator=g)
    lib = nm._lib.gpu()
    stream = torch.cuda.current_stream()

    def launch(i):
        src, dst = bufs[i % nb], bufs[(i + nb // 2) % nb]
        rc = lib.netc_gpu_mask_batch(0, dst.data_ptr(), src.data_ptr() + args.shift, nbytes, off.data_ptr(),
                                     keys.data_ptr(), n, stream.cuda_stream)
        assert rc == 0, rc

    for i in range(4):
        launch(i)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for i in range(args.steps):
        launch(4 + i)
    e1.record(stream)
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / args.steps * 1e3
    print(json.dumps({"shift": args.shift, "launches": 4 + args.steps, "us_per_launch": round(us, 3),
                      "algorithmic_bytes": 2 * nbytes, "GBps": round(2 * nbytes / us / 1e3, 1)}))


if __name__ == "__main__":
    main()
