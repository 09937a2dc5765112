"""N > 1 path on CPU: world_size-2 (and 3, 8: the driver's 8-GPU node, an odd split) gloo ranks each take a byte-balanced shard of one frame batch
(netc_shard_frames), rebase it exactly as a GPU shard is rebased (bench.py / netc_gpu_mask_batch_multi),
mask it with the host entry netc_ws_mask, and the gathered result must equal the oracle on the
whole batch.  No collective touches the data path except the final check's gather."""

import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def shard_view(off, keys, cuts, r):
    """Frames cuts[r]..cuts[r+1] rebased to their own payload start (what each GPU receives)."""
    a, b = int(cuts[r]), int(cuts[r + 1])
    base = int(off[a])
    return base, (off[a:b + 1] - np.uint64(base)).astype(np.uint64), keys[a:b]


def _worker(rank, world, port, result_q):
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from netc_amd import mask as nm
        from netc_amd import synth

        off = synth.mixed_offsets(3 << 20, 1, 40000, seed=77)
        keys = synth.random_keys(off.size - 1, 77)
        payload = synth.host_payload(int(off[-1]), 77)
        cuts = nm.shard_frames(off, world)
        base, soff, skeys = shard_view(off, keys, cuts, rank)
        end = int(off[cuts[rank + 1]])
        mine = payload[base:end].copy()
        for k in range(skeys.size):
            a, b = int(soff[k]), int(soff[k + 1])
            nm.mask_host(mine[a:b], int(skeys[k]).to_bytes(4, "little"), 0, out=mine[a:b])
        parts = [None] * world
        dist.all_gather_object(parts, (rank, base, mine.tobytes()))
        if rank == 0:
            from oracle import oracle as orc

            whole = b"".join(p[2] for p in sorted(parts))
            result_q.put(whole == orc.mask_batch(payload, off, keys).tobytes())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 8])
def test_gloo_sharded_batch_matches_oracle(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    ok = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert ok


def _hip_worker(rank, world, port, result_q):
    """As _worker, but each rank masks its shard with the HIP batch kernel (netc_gpu_mask_batch) on
    GPU rank % device_count -- one process per GPU as bench.py runs them; with one GPU the ranks
    share it, which is what this rehearses (the N-rank path had only ever
    masked with the host entry)."""
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import torch

        from netc_amd import mask as nm
        from netc_amd import synth

        dev = rank % torch.cuda.device_count()
        torch.cuda.set_device(dev)
        off = synth.mixed_offsets(24 << 20, 256, 65536, seed=91)
        keys = synth.random_keys(off.size - 1, 91)
        payload = synth.host_payload(int(off[-1]), 91)
        cuts = nm.shard_frames(off, world)
        base, soff, skeys = shard_view(off, keys, cuts, rank)
        end = int(off[cuts[rank + 1]])
        src = torch.from_numpy(payload[base:end].copy()).to(f"cuda:{dev}")
        dst = torch.empty_like(src)
        d_off = torch.from_numpy(soff.astype(np.int64)).to(f"cuda:{dev}")
        d_keys = torch.from_numpy(skeys.astype(np.int32)).to(f"cuda:{dev}")
        nm.mask_batch(dst, src, d_off, d_keys)
        torch.cuda.synchronize()
        parts = [None] * world
        dist.all_gather_object(parts, (rank, base, dst.cpu().numpy().tobytes()))
        if rank == 0:
            from oracle import oracle as orc

            whole = b"".join(p[2] for p in sorted(parts))
            result_q.put(whole == orc.mask_batch(payload, off, keys).tobytes())
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 4])
def test_gloo_sharded_batch_on_hip(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_hip_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    ok = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert ok
