#!/usr/bin/env python3
"""bench.py -- device-resident WebSocket payload XOR-mask throughput on MI355X.

Metric (BASELINE.json): GiB/s device-resident WS payload XOR-mask at 1/2/4/8 GPUs; % HBM roofline.

A "step" is one call of the hot path, netc_gpu_mask_batch (include/ws/mask.h), over
one batch of frames already resident in HBM -- by default BASELINE config 2:
65,536 frames x 1 KiB (64 MiB), an independent random 4-byte key per frame, unmasked
in place (the reference's receive direction, src/ws/common.c:317-323).  Each step
uses the next of R distinct batches (>= 1 GiB in total) so the 256 MiB Infinity
Cache cannot serve a batch from the previous touch.

Multi-GPU: one process per GPU.  Under torchrun WORLD_SIZE must equal --gpus; a
plain `python bench.py --gpus N` (N > 1) starts torch.distributed.run as a child
process before anything touches the GPU and exits with its code, and exits 2 when
fewer than N GPUs are visible -- it never prints an n_gpus = 1 line for N > 1.
Every rank masks its own shard of frames -- no data-path collective (frames are
independent); the only collectives are the timing barrier and the
gather of every rank's elapsed time (the max is the job's; each rank's own rate is
reported as per_gpu).  At N > 1 a second leg (c4_shards) runs BASELINE config 4:
a 1 GiB mixed-frame shard per GPU, aggregate and per-GPU GiB/s.

Prints ONE JSON line on rank 0.  Roofline: 2 x payload bytes per launch (read +
write) / mean kernel duration (HIP events on the launch stream) vs 8.0 TB/s, next
to in-bench frame-free stream ceilings (hand-written kernels, same rotation) and the
same kernel out of place and with src misaligned against dst (roofline.shapes).
After the timed region: the timed entry is checked (involution + every frame's
keystream), BASELINE config 5's host-to-host rate is measured (rank 0, N = 1), and
cpu_baseline times the oracle's restatement of the reference loop on this host,
rank 0, N = 1 only, bounded sample (see --cpu-seconds).
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
    p.add_argument("--no-copy-ceiling", action="store_true", help="skip the in-bench HBM stream ceilings")
    p.add_argument("--c5-gib", type=float, default=16.0,
                   help="BASELINE config 5 leg: GiB of 4 KiB frames streamed host->device->host from a pinned "
                        "ring (rank 0, N = 1; 0 disables)")
    p.add_argument("--no-pipelined-probe", dest="pipelined_probe", action="store_false",
                   help="skip the secondary figure timed after the headline: the same steps with two independent "
                        "batches in flight on two streams (pipelined_2stream).  Profiling runs pass this: the "
                        "overlapping launches would mix into a rocprof average of the kernel")
    p.add_argument("--sync", choices=("auto", "spin"), default="auto",
                   help="how the host waits for the GPU (hipSetDeviceFlags before the context exists): the "
                        "runtime's heuristic, or spin-wait (the synchronize that closes the timed region returns "
                        "without a wake-up delay)")
    p.add_argument("--no-shard-leg", dest="shard_leg", action="store_false",
                   help="at N > 1, skip the BASELINE config 4 leg (8 x 1 GiB mixed-frame shards, c4_shards)")
    return p.parse_args()


def dist_env():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return world, rank, local


def synth_config(workload: str, rank: int):
    from netc_amd import synth

    return synth.config(workload, shard=rank)


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


# the sources the headline kernel is compiled from: a PMC traffic entry is valid only for the
# kernel it was measured on
KERNEL_SOURCES = ("netc_amd/csrc/ws_mask_gpu.hip", "netc_amd/csrc/ws_mask_gpu.h", "netc_amd/csrc/gpu_util.h")


def kernel_source_hash() -> str:
    """sha256 (first 16 hex digits) over the headline kernel's sources, in KERNEL_SOURCES order."""
    import hashlib

    h = hashlib.sha256()
    for rel in KERNEL_SOURCES:
        with open(os.path.join(ROOT, rel), "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def traffic_per_launch(workload: str):
    """HBM bytes per launch of the masking kernel from the committed rocprofv3 PMC summary
    (profiles/pmc_traffic.json, written by tools/summarize_round.py from separate --pmc
    FETCH_SIZE / WRITE_SIZE passes of this bench, gfx950 corrections applied), or None when
    there is no entry or the entry was measured on other kernel sources (its
    kernel_source_sha256 differs from this tree's): a stale figure is never published."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        rec = json.load(open(path))[workload]
        if rec.get("kernel_source_sha256") != kernel_source_hash():
            return None
        return rec["hbm_bytes_per_launch"]
    except (OSError, KeyError, ValueError):
        return None


def stream_ceilings(torch, batches, total, stream, steps):
    """Practical rooflines measured here, on the same rotation of batches and the same stream:
    hand-written gfx950 stream kernels with no frame logic (netc_amd/csrc/ceiling.hip), each
    walking the batch as the mask kernel does (one window of 2 x 1 KiB per wavefront, NT).
      xor_inplace_GBps : buf[i] ^= key, in place          -- the mask kernel minus its frames
      copy_GBps        : dst[i] = src[i], out of place    -- the guide's "float4 copy"
    (read + write bytes) / HIP-event time per launch, averaged over `steps` launches."""
    import ctypes

    lib = ctypes.CDLL(os.path.join(ROOT, "netc_amd", "lib", "libnetc_ceiling.so"))
    lib.netc_ceiling_walk.argtypes = [ctypes.c_int] * 8 + [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                                           ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]
    nb = len(batches)
    sink = torch.zeros(1024, dtype=torch.int32, device=batches[0][0].device)
    out = {}
    for name, mode in (("xor_inplace_GBps", 1), ("copy_GBps", 0)):
        def launch(i):
            src = batches[i % nb][0]
            dst = batches[(i + nb // 2) % nb][0] if mode == 0 else src   # a batch no recent step wrote
            rc = lib.netc_ceiling_walk(mode, 1, 1, 0, 2, 256, -1, 4, dst.data_ptr(), src.data_ptr(), total,
                                       0x5A5A5A5A, sink.data_ptr(), stream.cuda_stream)
            if rc != 0:
                raise RuntimeError(f"netc_ceiling_walk failed ({rc})")
        for i in range(4):
            launch(i)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record(stream)
        for i in range(steps):
            launch(4 + i)
        e1.record(stream)
        torch.cuda.synchronize()
        out[name] = round(2.0 * (total // 1024 * 1024) / (e0.elapsed_time(e1) / steps * 1e-3) / 1e9, 1)
    out["kernel"] = "netc_amd/csrc/ceiling.hip netc_ceiling_walk (NT, 2 x 1 KiB per wavefront, 256-thread workgroups)"
    return out


def shape_points(torch, entry, local, batches, total, nframes, stream, steps):
    """The same kernel on the same rotation, other buffer shapes (secondary figures, never
    `value`): out of place (dst a batch no recent step wrote, 16-B aligned like src) and
    out of place with src = dst + 3 (every 16-B load unaligned; frames clipped to the
    3 bytes shorter buffer).  (read + write bytes) / HIP-event time per launch, GB/s."""
    nb = len(batches)
    out = {}
    for name, shift in (("out_of_place_GBps", 0), ("src_misaligned_3_GBps", 3)):
        n_bytes = total - shift
        offs = [torch.clamp(o, max=n_bytes) for _, o, _ in batches[:1]][0] if shift else batches[0][1]

        def launch(i):
            src = batches[i % nb][0]
            dst = batches[(i + nb // 2) % nb][0]
            _, o, k = batches[i % nb]
            rc = entry(local, dst.data_ptr(), src.data_ptr() + shift, n_bytes, (offs if shift else o).data_ptr(),
                       k.data_ptr(), nframes, stream.cuda_stream)
            if rc != 0:
                raise RuntimeError(f"netc_gpu_mask_batch failed ({rc})")
        for i in range(4):
            launch(i)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record(stream)
        for i in range(steps):
            launch(4 + i)
        e1.record(stream)
        torch.cuda.synchronize()
        out[name] = round(2.0 * n_bytes / (e0.elapsed_time(e1) / steps * 1e-3) / 1e9, 1)
    return out


def verify_step(torch, nm, batch, total, nframes, off_h, keys_h, stream):
    """Checks what the timed loop ran, after the timed region, with the same C-ABI entry:
      * involution: masking a timed batch twice gives its bytes back, and once changes them;
      * keystream: masking a zero buffer yields, for EVERY frame, its 4 key bytes repeated
        from phase 0 (RFC 6455 §5.3; src/ws/common.c:321) -- checked with numpy here."""
    p, o, k = batch
    # clone / zeros run on torch's current stream, the masks on `stream`: synchronise
    # between them (a 1 GiB clone was still reading while the first mask ran)
    torch.cuda.synchronize()
    before = p.clone()
    torch.cuda.synchronize()
    nm.mask_batch(p, p, o, k, stream=stream)
    torch.cuda.synchronize()
    once_differs = not torch.equal(p, before)
    nm.mask_batch(p, p, o, k, stream=stream)
    torch.cuda.synchronize()
    involution = torch.equal(p, before)
    zero = torch.zeros(total, dtype=torch.uint8, device=p.device)
    torch.cuda.synchronize()
    nm.mask_batch(zero, zero, o, k, stream=stream)
    torch.cuda.synchronize()
    ks = zero.cpu().numpy()
    del zero
    keys_b = np.ascontiguousarray(keys_h, dtype=np.uint32).view(np.uint8).reshape(-1, 4)
    off64 = off_h.astype(np.int64)
    keystream = bool((ks[:off64[0]] == 0).all() and (ks[off64[-1]:] == 0).all())
    a = 0
    while keystream and a < nframes:   # frames in groups of ~32 MiB (bounded host memory)
        b = int(np.searchsorted(off64, off64[a] + (32 << 20), side="right"))
        b = min(max(b - 1, a + 1), nframes)
        sizes = np.diff(off64[a:b + 1])
        frame_of = np.repeat(np.arange(a, b), sizes)
        phase = np.arange(off64[a], off64[b], dtype=np.int64) - np.repeat(off64[a:b], sizes)
        keystream = bool(np.array_equal(ks[off64[a]:off64[b]], keys_b[frame_of, phase & 3]))
        a = b
    return {"involution": bool(involution and once_differs), "keystream_all_frames": keystream}


def c5_host_to_host(nm, gib: float):
    """BASELINE config 5: `gib` GiB of 4 KiB frames in a pinned host ring, streamed through the
    default persistent handle (2 x 512 MiB device slots, H2D / kernel / D2H overlapped) into a
    pinned output ring (the ring -> parser hand-off), and once more in place.  Host-to-host GiB/s,
    best of 2 passes each (the first pass also touches the slots); never `value`.

    Checked after the timing, through the oracle (the reference's expression, src/ws/common.c:321):
    the frames on both sides of every slot edge (where the pipeline cuts) and 256 random frames
    of the out-of-place output; and, since the ring was masked in place an even number of times,
    that the same frames of the ring are back to their original bytes."""
    from netc_amd import synth
    from oracle import oracle as orc

    total = int(gib * (1 << 30)) // 4096 * 4096
    nframes = total // 4096
    off = synth.uniform_offsets(nframes, 4096)
    keys = synth.random_keys(nframes, stream=900)
    ring, out = nm.PinnedArray(total), nm.PinnedArray(total)
    slot = 512 << 20
    edges = [e // 4096 + d for e in range(slot, total, slot) for d in (-1, 0)]
    picks = sorted(set(edges) | set(int(k) for k in synth.rng(901).choice(nframes, size=min(256, nframes),
                                                                         replace=False)))
    picks = [k for k in picks if 0 <= k < nframes]
    rates = {}
    try:
        synth.fill_payload(ring.array)
        orig = {k: ring.array[k * 4096:(k + 1) * 4096].copy() for k in picks}
        with nm.HostStream(0) as hs:
            for name, dst in (("out_of_place", out.array), ("in_place", ring.array)):
                best = None
                for _ in range(2):
                    t0 = time.perf_counter()
                    hs.mask(dst, ring.array, off, keys)
                    dt = time.perf_counter() - t0
                    best = dt if best is None else min(best, dt)
                rates[name] = round(total / best / GIB, 2)
        bad = 0
        for k in picks:
            exp = orc.mask_batch(orig[k], np.array([0, 4096], dtype=np.uint64), keys[k:k + 1])
            bad += int(not np.array_equal(out.array[k * 4096:(k + 1) * 4096], exp))
            bad += int(not np.array_equal(ring.array[k * 4096:(k + 1) * 4096], orig[k]))
    finally:
        ring.close()
        out.close()
    return {"value": rates["out_of_place"], "unit": "GiB/s host to host", "in_place": rates["in_place"],
            "bytes": total, "frames": nframes, "slots": "2 x 512 MiB (defaults)", "passes": 2,
            "verified": {"frames_checked": len(picks), "slot_edge_frames": len(edges), "mismatches": bad,
                         "ok": bad == 0},
            "note": "BASELINE config 5: pinned ring -> H2D -> mask -> D2H -> pinned output ring "
                    "(in_place: back into the ring); PCIe-bound"}


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


def free_port() -> int:
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args) -> int:
    """`--gpus N > 1` outside torchrun: one process per GPU.  This process never touches the
    GPU (device_count() does not initialise HIP on this image); it starts
    torch.distributed.run as a CHILD with the same arguments and returns the child's exit
    code, so the driver's `python bench.py --gpus N` yields an n_gpus = N line or fails."""
    import subprocess

    if "NETC_BENCH_DEVICE" not in os.environ:     # rehearsal (all ranks on one GPU) skips the count
        import torch

        have = torch.cuda.device_count()
        if have < args.gpus:
            print(f"bench.py: --gpus {args.gpus} but {have} GPU(s) visible", file=sys.stderr, flush=True)
            return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd).returncode


def set_spin_sync(device: int) -> None:
    """hipSetDeviceFlags(hipDeviceScheduleSpin) on `device` before its context exists: a
    synchronize then spin-waits on the GPU instead of yielding the thread (the runtime the
    flag goes to is torch's: same SONAME, already loaded by `import torch`)."""
    import ctypes

    hip = ctypes.CDLL("libamdhip64.so.7")
    if hip.hipSetDevice(device) != 0 or hip.hipSetDeviceFlags(1) != 0:   # hipDeviceScheduleSpin = 1
        print("bench.py: hipSetDeviceFlags(spin) failed; the runtime's default wait is used", file=sys.stderr)


def timed_steps(torch, step, steps: int, warmup: int, stream, device, world: int):
    """W untimed steps, then exactly K steps bracketed by barrier + synchronize on both sides.
    Returns (this rank's elapsed seconds, mean launch duration in ms from two HIP events on the
    launch stream).  Per-launch event pairs are NOT recorded inside the region: each event
    packet breaks the back-to-back dispatch and cost 7-9 us per step on this path
    (tools/launch_probe.py), which would be measuring the events, not the kernel."""
    sh = stream.cuda_stream
    for i in range(warmup):
        step(i, sh)
    torch.cuda.synchronize(device)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    ev0.record(stream)
    for i in range(steps):
        step(warmup + i, sh)
    ev1.record(stream)
    torch.cuda.synchronize(device)
    elapsed = time.perf_counter() - t0            # this rank's K steps, sync to sync
    if world > 1:
        torch.distributed.barrier()               # closing bracket; the max over ranks follows
    return elapsed, ev0.elapsed_time(ev1) / steps


def gather_max(torch, values, world: int, coll_dev):
    """all_gather one float64 vector per rank; returns the list of per-rank vectors."""
    if world == 1:
        return [list(values)]
    mine = torch.tensor(values, dtype=torch.float64, device=coll_dev)
    gathered = [torch.zeros_like(mine) for _ in range(world)]
    torch.distributed.all_gather(gathered, mine)
    return [[float(x) for x in g] for g in gathered]


def shard_leg(torch, nm, entry, local, rank, world, device, stream, coll_dev, args):
    """BASELINE config 4 at N GPUs: every rank masks its own 1 GiB shard of mixed 256 B - 64 KiB
    frames (own seed per rank), rotating over 2 such batches, K steps timed as the headline.
    Aggregate = all ranks' payload bytes / the slowest rank's time; per-GPU rates beside it;
    every rank's last batch checked (involution + every frame's keystream)."""
    batches, total, nframes = make_batches(torch, "c4", rank, 2 << 30, device)
    prepared = [(p.data_ptr(), o.data_ptr(), k.data_ptr()) for p, o, k in batches]

    def step(i, s_handle):
        p, o, k = prepared[i % len(prepared)]
        rc = entry(local, p, p, total, o, k, nframes, s_handle)
        if rc != 0:
            raise nm.NetcGpuError(rc, "c4 shard leg")

    steps = max(5, args.steps // 4)
    elapsed, kern = timed_steps(torch, step, steps, 2, stream, device, world)
    off_h, _, _ = synth_config("c4", rank)
    last = batches[(2 + steps - 1) % len(batches)]
    check = verify_step(torch, nm, last, total, nframes, off_h, last[2].cpu().numpy().view(np.uint32), stream)
    ok = int(check["involution"] and check["keystream_all_frames"])
    rows = gather_max(torch, [elapsed, kern, float(total), float(ok)], world, coll_dev)
    del batches, prepared
    torch.cuda.empty_cache()
    t_max = max(r[0] for r in rows)
    return {
        "workload": "c4: " + WORKLOADS["c4"],
        "value": round(sum(r[2] for r in rows) * steps / t_max / GIB, 3),
        "unit": "GiB/s aggregate",
        "steps": steps,
        "per_gpu": [round(r[2] * steps / r[0] / GIB, 3) for r in rows],
        "kernel_frac_of_hbm": [round(2.0 * r[2] / (r[1] * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4) for r in rows],
        "verified_all_ranks": all(r[3] == 1.0 for r in rows),
        "note": "BASELINE config 4 (8 x 1 GiB independent shards, no collective); secondary to the headline",
    }


def main():
    args = parse_args()
    if args.gpus < 1:
        print("bench.py: --gpus must be >= 1", file=sys.stderr)
        sys.exit(2)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args))
    world, rank, local = dist_env()
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr, flush=True)
        sys.exit(2)
    import torch

    # NETC_BENCH_DEVICE / NETC_BENCH_BACKEND=gloo: rehearsal of the N-rank path on a
    # one-GPU box (every rank on one device, timing collectives on the CPU); the
    # real multi-GPU run uses one GPU per rank and RCCL ("nccl") for the barrier.
    rehearsal = "NETC_BENCH_DEVICE" in os.environ
    local = int(os.environ.get("NETC_BENCH_DEVICE", local))
    backend = os.environ.get("NETC_BENCH_BACKEND", "nccl")
    if not rehearsal and torch.cuda.device_count() < world:
        print(f"bench.py: {world} ranks but {torch.cuda.device_count()} GPU(s) visible", file=sys.stderr, flush=True)
        sys.exit(2)
    if args.sync == "spin":
        set_spin_sync(local)
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

    # Timed region: K back-to-back launches on one stream (timed_steps).
    elapsed, kern_own = timed_steps(torch, step, args.steps, args.warmup, stream, device, world)

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

    rows = gather_max(torch, [elapsed, kern_own, pipelined or 0.0], world, coll_dev)
    per_rank_elapsed = [r[0] for r in rows]
    elapsed = max(per_rank_elapsed)
    kern_mean = max(r[1] for r in rows)
    pipelined = max(r[2] for r in rows) or None

    ceilings = None
    shapes = None
    if rank == 0 and not args.no_copy_ceiling:
        ceilings = stream_ceilings(torch, batches, total, stream, max(20, args.steps))
        shapes = shape_points(torch, entry, local, batches, total, nframes, stream, max(20, args.steps))

    off_h, _, _ = synth_config(args.workload, rank)
    last = batches[(args.warmup + args.steps - 1) % nb]
    keys_h = last[2].cpu().numpy().view(np.uint32)   # this batch's own keys
    check = verify_step(torch, nm, last, total, nframes, off_h, keys_h, stream)
    ok_rows = gather_max(torch, [float(check["involution"] and check["keystream_all_frames"])], world, coll_dev)
    check["ranks_verified"] = int(sum(r[0] for r in ok_rows))
    check["all_ranks_ok"] = check["ranks_verified"] == world

    shards = None
    if world > 1 and args.shard_leg:
        del batches, prepared
        torch.cuda.empty_cache()
        shards = shard_leg(torch, nm, entry, local, rank, world, device, stream, coll_dev, args)

    cpu = None
    c5 = None
    if rank == 0 and world == 1:
        del batches, prepared
        torch.cuda.empty_cache()
        if args.c5_gib > 0:
            c5 = c5_host_to_host(nm, args.c5_gib)
        if args.cpu_seconds > 0:
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
                "parallelism": f"shard{world} (independent frames, one process per GPU, no collective)",
                "entry": "netc_gpu_mask_batch (include/ws/mask.h)",
                "devices": "rehearsal: every rank on one GPU" if rehearsal else "one GPU per rank",
                "host_sync": args.sync,
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBPS, 4),
                "traffic": traffic_per_launch(args.workload),
                "traffic_source": "profiles/pmc_traffic.json entry for this workload whose kernel_source_sha256 "
                                  f"equals this tree's ({kernel_source_hash()}); null when none does",
                "kernel_ms_mean": round(kern_mean, 5),
                "kernel_timing": "HIP events on the launch stream around the K timed launches, / K "
                                 "(slowest rank)",
                "algorithmic_bytes_per_launch": 2 * total,
                "ceilings": ceilings,
                "frac_of_xor_stream": round(achieved / ceilings["xor_inplace_GBps"], 4) if ceilings else None,
                "shapes": shapes,
            },
            "per_gpu": [round(float(total) * args.steps / e / GIB, 3) for e in per_rank_elapsed],
            "verified": check,
            "c4_shards": shards,
            "c5_host_to_host": c5,
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
