#!/usr/bin/env python3
"""bench.py -- device-resident WebSocket payload XOR-mask throughput on MI355X.

Metric (BASELINE.json): GiB/s device-resident WS payload XOR-mask at 1/2/4/8 GPUs; % HBM roofline.

A "step" is one call of the hot path, netc_gpu_mask_batch (include/ws/mask.h), over
one batch of frames already resident in HBM -- by default BASELINE config 2:
65,536 frames x 1 KiB (64 MiB), an independent random 4-byte key per frame, unmasked
in place (the reference's receive direction, src/ws/common.c:317-323).  Each step
uses the next of R distinct batches (>= 1 GiB in total) so the 256 MiB Infinity
Cache cannot serve a batch from the previous touch.

Multi-GPU: one process per GPU (torchrun); every rank masks its own shard of
frames -- no data-path collective (frames are independent); the
only collectives are the timing barrier and the max-over-ranks of the elapsed time.

Prints ONE JSON line on rank 0.  Roofline: 2 x payload bytes per launch (read +
write) / mean kernel duration (HIP events on the launch stream) vs 8.0 TB/s.
cpu_baseline: the oracle's restatement of the reference loop on this host, rank 0,
N = 1 only, bounded sample (see --cpu-seconds).
"""

from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "GiB/s device-resident WS payload XOR-mask at 1/2/4/8 GPUs; % HBM roofline"
HBM_PEAK_GBPS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
GIB = float(1 << 30)

WORKLOADS = {
    "c2": "65,536 x 1 KiB frames (64 MiB) per GPU, independent random key per frame, in place",
    "c3": "1,024 x 1 MiB frames (1 GiB) per GPU, one random key per frame, in place",
    "c4": "1 GiB per GPU of mixed 256 B - 64 KiB frames packed back to back (unaligned), in place",
}


def parse_args():
    p = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--workload", choices=sorted(WORKLOADS), default="c2")
    p.add_argument("--rotation-bytes", type=int, default=2 << 30, help="distinct device bytes the steps rotate over")
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline budget (0 disables)")
    p.add_argument("--unroll", type=int, default=None)
    p.add_argument("--max-blocks", type=int, default=None)
    p.add_argument("--nt-flags", type=int, default=None)
    p.add_argument("--no-copy-ceiling", action="store_true")
    p.add_argument("--no-pipelined-probe", dest="pipelined_probe", action="store_false")
    return p.parse_args()


def dist_env():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return world, rank, local


def make_batches(torch, workload: str, rank: int, rotation_bytes: int, device):
    """R device batches of the workload shape (own seeds per rank / batch)."""
    from netc_amd import synth

    off, keys, total = synth.config(workload, shard=rank)
    nb = max(2, -(-rotation_bytes // total))
    batches = []
    gen = torch.Generator(device=device).manual_seed(1000 + rank)
    off_t = torch.from_numpy(off.view(np.int64)).to(device)
    for b in range(nb):
        payload = torch.randint(0, 256, (total,), dtype=torch.uint8, device=device, generator=gen)
        k = synth.random_keys(keys.size, stream=300 + 1000 * rank + b)
        batches.append((payload, off_t, torch.from_numpy(k.view(np.int32)).to(device)))
    return batches, total, keys.size


def traffic_per_launch(workload: str):
    """HBM bytes per launch of the masking kernel from the committed rocprofv3 PMC summary
    (profiles/pmc_traffic.json, written by tools/summarize_prof.py from separate --pmc
    FETCH_SIZE / WRITE_SIZE passes of this bench, gfx950 corrections applied), or None."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        rec = json.load(open(path))[workload]
        return rec["hbm_bytes_per_launch"]
    except (OSError, KeyError, ValueError):
        return None


def copy_ceiling(torch, device, nbytes=64 << 20, reps=64):
    """Practical roofline: device-to-device copy of rotating 64 MiB buffers (read + write bytes / time)."""
    nb = 16
    bufs = [torch.empty(nbytes, dtype=torch.uint8, device=device) for _ in range(nb + 1)]
    for i in range(8):
        bufs[(i + 1) % (nb + 1)].copy_(bufs[i % (nb + 1)])
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for i in range(reps):
        bufs[(i + 1) % (nb + 1)].copy_(bufs[i % (nb + 1)])
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / reps
    del bufs
    return 2 * nbytes / (ms * 1e-3) / 1e9


def cpu_baseline(workload: str, budget_s: float):
    """Oracle restatement of the reference loop timed on this host (rank 0, N = 1).

    Primary: liboracle.so (-O2), one thread, the exact per-byte expression of
    src/ws/common.c:321 over the workload's frames.  Variants: the reference's own
    flags (-O0, Makefile:3), all host cores (frames split by bytes over threads; ctypes
    releases the GIL), and -- when oracle/_ref was built -- the reference's compiled
    ws_parse_frame receiving the same frames over a socketpair.
    """
    from concurrent.futures import ThreadPoolExecutor

    from netc_amd import synth
    from oracle import oracle as orc

    off, keys, total = synth.config(workload)
    # bounded sample: the first frames of the workload, at most 256 MiB
    sample_bytes = min(total, 256 << 20)
    nf = int(np.searchsorted(off, sample_bytes, side="right")) - 1
    nf = max(1, nf)
    s_off = off[: nf + 1].copy()
    s_keys = keys[:nf].copy()
    s_total = int(s_off[-1])
    buf = synth.host_payload(s_total, stream=77)

    def timed(fn, share):
        reps, t = 0, 0.0
        t0 = time.perf_counter()
        while True:
            fn()
            reps += 1
            t = time.perf_counter() - t0
            if t >= share:
                break
        return reps * s_total / t / GIB, reps

    per = budget_s / 4.0
    o2 = orc.lib("O2")
    o0 = orc.lib("O0")
    bp = buf.ctypes.data
    po, pk = s_off.ctypes.data, s_keys.ctypes.data
    v_o2, r_o2 = timed(lambda: o2.oracle_mask_batch(bp, po, pk, nf), per)
    v_o0, r_o0 = timed(lambda: o0.oracle_mask_batch(bp, po, pk, nf), per)

    ncores = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    ncores = max(1, min(ncores, 64))
    from netc_amd.mask import shard_frames

    cuts = shard_frames(s_off, ncores)
    parts = []
    for i in range(ncores):
        a, b = int(cuts[i]), int(cuts[i + 1])
        if b > a:
            parts.append((a, b))
    pool = ThreadPoolExecutor(max_workers=len(parts))

    def all_cores():
        list(pool.map(lambda ab: o2.oracle_mask_batch(bp, s_off[ab[0]:].ctypes.data, s_keys[ab[0]:].ctypes.data,
                                                      ab[1] - ab[0]), parts))

    v_mt, r_mt = timed(all_cores, per)
    pool.shutdown()
    variants = {
        "port_O2_1thread_GiBps": round(v_o2, 4),
        "port_O0_reference_flags_1thread_GiBps": round(v_o0, 4),
        f"port_O2_{len(parts)}threads_GiBps": round(v_mt, 4),
    }
    if orc.ref_available():
        wire = build_wire(buf, s_off, s_keys, limit_frames=min(nf, 65536))
        got, secs = orc.ref_receive_timed(wire)
        variants["reference_ws_parse_frame_O0_1thread_GiBps"] = round(got / secs / GIB, 4)
    cpu = os.popen("lscpu 2>/dev/null | grep 'Model name' | head -1").read().split(":")[-1].strip() or platform.processor()
    return {
        "value": round(v_o2, 4),
        "unit": "GiB/s",
        "cores": 1,
        "kind": "port",
        "sample": f"first {nf} frames ({s_total / (1 << 20):.0f} MiB) of workload {workload}, host-resident, "
                  f"{r_o2} passes; oracle/ws_oracle.c -O2 (exact expression of src/ws/common.c:321)",
        "cpu_model": cpu,
        "host_cores_visible": ncores,
        "variants": variants,
    }


def build_wire(buf, off, keys, limit_frames):
    """Masked client frames (header + key + payload) for the first `limit_frames` frames."""
    from oracle import oracle as orc

    out = []
    for k in range(limit_frames):
        a, b = int(off[k]), int(off[k + 1])
        key = int(keys[k]).to_bytes(4, "little")
        out.append(orc.encode_frame(buf[a:b].tobytes(), 2, key))
    return np.frombuffer(b"".join(out), dtype=np.uint8)


def main():
    args = parse_args()
    world, rank, local = dist_env()
    import torch

    # NETC_BENCH_DEVICE / NETC_BENCH_BACKEND=gloo: rehearsal of the N-rank path on a
    # one-GPU box (every rank on one device, timing collectives on the CPU); the
    # real multi-GPU run uses one GPU per rank and RCCL ("nccl") for the barrier.
    local = int(os.environ.get("NETC_BENCH_DEVICE", local))
    backend = os.environ.get("NETC_BENCH_BACKEND", "nccl")
    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)
    coll_dev = device if backend == "nccl" else torch.device("cpu")

    from netc_amd import mask as nm

    if args.unroll or args.max_blocks or args.nt_flags is not None:
        nm.tune(args.unroll or 4, args.max_blocks or 0, -1 if args.nt_flags is None else args.nt_flags)
    nm.gpu_init(local)
    batches, total, nframes = make_batches(torch, args.workload, rank, args.rotation_bytes, device)
    stream = torch.cuda.Stream(device)            # a dedicated (non-NULL) HIP stream for the hot path
    torch.cuda.synchronize(device)                # batches were generated on the default stream
    for p, o, k in batches[:1]:
        nm.mask_batch(p, p, o, k, stream=stream)          # validated once through the Python mirror
    # hot loop: the C-ABI entry itself, with the argument words prepared once
    from netc_amd import _lib

    entry = _lib.gpu().netc_gpu_mask_batch
    prepared = [(p.data_ptr(), o.data_ptr(), k.data_ptr()) for p, o, k in batches]
    nb = len(prepared)

    def step(i, s_handle):
        p, o, k = prepared[i % nb]
        rc = entry(local, p, p, total, o, k, nframes, s_handle)
        if rc != 0:
            raise nm.NetcGpuError(rc, _lib.gpu().netc_gpu_strerror().decode())

    sh = stream.cuda_stream
    for i in range(args.warmup):
        step(i, sh)
    torch.cuda.synchronize(device)

    # Timed region: K back-to-back launches on one stream.  Two HIP events on that
    # stream bracket the launches: (end - start) / K is the average launch duration
    # on the GPU (kernel time plus the dependent-launch boundary, no host time).
    # Per-launch event pairs are NOT recorded inside the region: each event packet
    # breaks the back-to-back dispatch and cost 7-9 us per step on this path
    # (tools/launch_probe.py), which would be measuring the events, not the kernel.
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    ev0.record(stream)
    for i in range(args.steps):
        step(args.warmup + i, sh)
    ev1.record(stream)
    torch.cuda.synchronize(device)
    elapsed = time.perf_counter() - t0            # this rank's K steps, sync to sync
    if world > 1:
        torch.distributed.barrier()               # closing bracket; the max over ranks follows
    kern_ms = np.array([ev0.elapsed_time(ev1) / args.steps])

    # secondary figure: the same steps with two batches in flight on two HIP streams
    # (independent batches, as a serving loop would pipeline them); not the headline
    pipelined = None
    if args.pipelined_probe:
        s2 = [stream, torch.cuda.Stream(device)]
        for i in range(max(4, args.warmup)):      # first use of a stream pays a one-off set-up (~6 ms)
            step(i, s2[i % 2].cuda_stream)
        torch.cuda.synchronize(device)
        if world > 1:
            torch.distributed.barrier()
        t1 = time.perf_counter()
        for i in range(args.steps):
            step(i, s2[i % 2].cuda_stream)
        torch.cuda.synchronize(device)
        pipelined = time.perf_counter() - t1
        if world > 1:
            torch.distributed.barrier()

    if world > 1:
        t = torch.tensor([elapsed, kern_ms.mean(), pipelined or 0.0], dtype=torch.float64, device=coll_dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed, kern_mean, pipelined = float(t[0]), float(t[1]), (float(t[2]) or None)
    else:
        kern_mean = float(kern_ms.mean())

    ceiling = None
    if rank == 0 and not args.no_copy_ceiling:
        ceiling = copy_ceiling(torch, device)

    cpu = None
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        del batches
        torch.cuda.empty_cache()
        cpu = cpu_baseline(args.workload, args.cpu_seconds)

    if rank == 0:
        payload_all = float(total) * world * args.steps
        value = payload_all / elapsed / GIB
        achieved = 2.0 * total / (kern_mean * 1e-3) / 1e9
        line = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 5),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (seeded random payload bytes and keys, device-generated)",
            "config": {
                "workload": f"{args.workload}: {WORKLOADS[args.workload]}",
                "frames_per_gpu": nframes,
                "batch_bytes_per_gpu": total,
                "rotation_batches": args.rotation_bytes and max(2, -(-args.rotation_bytes // total)),
                "parallelism": f"shard{world} (independent frames, no collective)",
                "entry": "netc_gpu_mask_batch (include/ws/mask.h)",
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBPS, 4),
                "traffic": traffic_per_launch(args.workload),
                "kernel_ms_mean": round(kern_mean, 5),
                "kernel_timing": "HIP events on the launch stream around the K timed launches, / K",
                "algorithmic_bytes_per_launch": 2 * total,
                "copy_ceiling_GBps": round(ceiling, 1) if ceiling else None,
            },
            "cpu_baseline": cpu,
            "pipelined_2stream": None if not pipelined else {
                "value": round(float(total) * world * args.steps / pipelined / GIB, 3),
                "ms_per_step": round(pipelined / args.steps * 1e3, 5),
                "note": "same steps, two independent batches in flight on two HIP streams (not the headline)"},
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
