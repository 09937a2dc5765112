"""GPU parity: netc_gpu_mask_batch (gfx950 kernel, through the C-ABI) vs the oracle.

The oracle (oracle/ws_oracle.c) is the reference's exact per-byte expression
(src/ws/common.c:321); the bar is bit-exact output for every byte of the
buffer, plus untouched guard bytes around it.
"""

import numpy as np
import pytest

from netc_amd import mask as nm
from netc_amd import synth
from oracle import oracle as orc

pytestmark = pytest.mark.gpu

GUARD = 64
SENTINEL = 0xA5


def _dev(torch, a: np.ndarray, device=None):
    """uint64 offsets / uint32 keys -> device int64 / int32 tensors with the same bits (on `device`, or cuda:0)."""
    a = np.ascontiguousarray(a)
    if a.dtype == np.uint64:
        a = a.view(np.int64)
    elif a.dtype == np.uint32:
        a = a.view(np.int32)
    t = torch.from_numpy(a)
    return t.to(device) if device is not None else t.cuda()


def run_case(torch, payload: np.ndarray, off: np.ndarray, keys: np.ndarray, dst_shift=0, src_shift=0, inplace=False):
    total = payload.size
    off = np.ascontiguousarray(off, dtype=np.uint64)
    keys = np.ascontiguousarray(keys, dtype=np.uint32)
    src_buf = torch.full((total + 2 * GUARD,), SENTINEL, dtype=torch.uint8, device="cuda")
    src = src_buf[GUARD + src_shift: GUARD + src_shift + total]
    src.copy_(torch.from_numpy(payload))
    if inplace:
        dst_buf, dst, dst_shift = src_buf, src, src_shift
    else:
        dst_buf = torch.full((total + 2 * GUARD,), SENTINEL, dtype=torch.uint8, device="cuda")
        dst = dst_buf[GUARD + dst_shift: GUARD + dst_shift + total]
    off_t = _dev(torch, off, None)
    keys_t = _dev(torch, keys, None)
    nm.mask_batch(dst, src, off_t, keys_t)
    torch.cuda.synchronize()
    expected = orc.mask_batch(payload, off, keys)
    whole = dst_buf.cpu().numpy()
    got = whole[GUARD + dst_shift: GUARD + dst_shift + total]
    if not np.array_equal(got, expected):
        bad = np.nonzero(got != expected)[0]
        raise AssertionError(f"{bad.size} bytes differ, first at {bad[:8].tolist()} "
                             f"(total={total}, frames={keys.size}, shifts={dst_shift},{src_shift}, inplace={inplace})")
    lo, hi = GUARD + dst_shift, GUARD + dst_shift + total
    assert (whole[:lo] == SENTINEL).all() and (whole[hi:] == SENTINEL).all(), "write outside the destination"


def frames_from_sizes(sizes, start=0):
    off = np.zeros(len(sizes) + 1, dtype=np.uint64)
    off[0] = start
    off[1:] = start + np.cumsum(np.asarray(sizes, dtype=np.uint64))
    return off


# ------------------------------------------------------------ known answers --

def test_rfc6455_known_answer(torch_cuda):
    # RFC 6455 §5.7: "Hello" masked with 37 fa 21 3d -> 7f 9f 4d 51 58
    key = np.frombuffer(bytes.fromhex("37fa213d"), dtype=np.uint8)
    masked = np.frombuffer(bytes.fromhex("7f9f4d5158"), dtype=np.uint8).copy()
    for shift in range(16):
        torch = torch_cuda
        buf = torch.zeros(64, dtype=torch.uint8, device="cuda")[shift: shift + 5]
        buf.copy_(torch.from_numpy(masked))
        off = torch.tensor([0, 5], dtype=torch.int64, device="cuda")
        k = torch.from_numpy(nm.pack_keys(key).view(np.int32)).cuda()
        nm.mask_batch(buf, buf, off, k)
        assert bytes(buf.cpu().numpy()) == b"Hello"


def test_reference_test_payloads(torch_cuda):
    # the payloads tests/ws/test001.c round-trips, with the keys ws_build_masking_key
    # yields on a fresh thread (src/ws/common.c:19-27)
    payloads = [bytes([0, 233, 5, 11, 65, 115, 112, 101, 99, 116, 108, 44, 108, 44, 107]),   # :233-246
                b"hello client masked",                                                      # :95-108
                b"hello server multiple frames masked",                                      # :253-266
                b"hello client multiple frames masked"]                                      # :149-162
    keys = np.frombuffer(orc.key_sequence(4), dtype=np.uint8).reshape(4, 4)
    buf = np.frombuffer(b"".join(payloads), dtype=np.uint8).copy()
    off = frames_from_sizes([len(p) for p in payloads])
    run_case(torch_cuda, buf, off, nm.pack_keys(keys))


# ------------------------------------------------------------- edge cases ---

@pytest.mark.parametrize("dst_shift,src_shift", [(0, 0), (1, 1), (7, 7), (15, 15), (3, 0), (0, 9), (5, 12)])
def test_ragged_frames_and_alignment(torch_cuda, dst_shift, src_shift):
    g = synth.rng(11, dst_shift * 16 + src_shift)
    sizes = list(range(0, 40)) + [63, 64, 65, 255, 256, 257, 1023, 1024, 1025, 4095, 4097, 70000, 3, 0, 0, 1]
    g.shuffle(sizes)
    off = frames_from_sizes(sizes)
    total = int(off[-1])
    payload = synth.host_payload(total, 11, 3)
    keys = synth.random_keys(len(sizes), 11, 4)
    run_case(torch_cuda, payload, off, keys, dst_shift, src_shift)


@pytest.mark.parametrize("taper", [1, 4096, 5000, 3 << 20, 1 << 40])
@pytest.mark.parametrize("shift,inplace", [(0, True), (5, True), (3, False)])
def test_tapered_end(torch_cuda, gpu_knob, taper, shift, inplace):
    # NETC_GPU_KNOB_MASK_TAPER: the batch's last bytes in one-step windows (the end of the launch);
    # 1 << 40 tapers the whole batch, 1 a single step; the batch ends in a partial vector
    gpu_knob("MASK_TAPER", taper)
    off = synth.mixed_offsets((6 << 20) + 11, 1, 70000, seed=13)
    keys = synth.random_keys(off.size - 1, 13)
    payload = synth.host_payload(int(off[-1]), 13)
    run_case(torch_cuda, payload, off, keys, shift, shift, inplace=inplace)
    sizes = [1024] * 4096                                       # config 2's shape, smaller
    off = frames_from_sizes(sizes)
    run_case(torch_cuda, synth.host_payload(4 << 20, 14), off, synth.random_keys(4096, 14), shift, shift,
             inplace=inplace)


@pytest.mark.parametrize("inplace", [False, True])
def test_in_place_and_out_of_place(torch_cuda, inplace):
    off = synth.mixed_offsets(3 << 20, 256, 65536, seed=5)
    keys = synth.random_keys(off.size - 1, 5)
    payload = synth.host_payload(int(off[-1]), 5)
    run_case(torch_cuda, payload, off, keys, 3, 3, inplace=inplace)


def test_dense_tiny_frames(torch_cuda):
    # > 63 frame boundaries inside one 1 KiB span: exercises the table walk
    g = synth.rng(7)
    sizes = g.integers(0, 4, size=20000)
    off = frames_from_sizes(sizes)
    payload = synth.host_payload(int(off[-1]), 7)
    run_case(torch_cuda, payload, off, synth.random_keys(sizes.size, 7), 0, 0)
    run_case(torch_cuda, payload, off, synth.random_keys(sizes.size, 8), 5, 5)


@pytest.mark.parametrize("shift", [0, 7])
def test_dense_spans_per_lane(torch_cuda, shift):
    # 3..63 frame starts per 1 KiB span (the per-lane keying path): frames under 16 B
    # (several starts inside one 16 B vector), empty frames, and some long ones between
    g = synth.rng(31 + shift)
    sizes = g.choice([0, 1, 2, 5, 9, 12, 15, 16, 17, 23, 31, 48, 64, 100, 200, 333], size=60000)
    sizes[g.choice(sizes.size, 30, replace=False)] = g.integers(1000, 9000, 30)
    off = frames_from_sizes(sizes)
    payload = synth.host_payload(int(off[-1]), 31)
    run_case(torch_cuda, payload, off, synth.random_keys(sizes.size, 31, 4), shift, shift)
    run_case(torch_cuda, payload, off, synth.random_keys(sizes.size, 32), shift, (shift + 3) % 16)


@pytest.mark.parametrize("shift,inplace", [(0, False), (9, False), (3, True)])
def test_dense_span_windows(torch_cuda, shift, inplace):
    # 64+ frame starts per 1 KiB span (frames of ~16 B and less): the per-lane path
    # walks the table in 63-entry windows.  Runs of uniform 16 / 15 / 8 B frames, a
    # mixed 0..24 B stretch, and a few long frames so spans switch between the
    # sparse, per-lane and windowed cases.
    g = synth.rng(57 + shift)
    parts = [np.full(9000, 16), np.full(7000, 15), g.choice([0, 1, 4, 7, 8, 13, 16, 24], size=12000),
             np.array([5000, 1, 3000]), np.full(6000, 8), g.integers(0, 3, size=3000), np.full(4000, 17)]
    sizes = np.concatenate(parts).astype(np.int64)
    off = frames_from_sizes(sizes, start=5)
    payload = synth.host_payload(int(off[-1]) + 11, 57)
    run_case(torch_cuda, payload, off, synth.random_keys(sizes.size, 57), shift, shift, inplace)
    run_case(torch_cuda, payload, off, synth.random_keys(sizes.size, 58), shift, (shift + 5) % 16)


def test_unframed_bytes_pass_through(torch_cuda):
    off = frames_from_sizes([100, 5000, 7, 0, 33333], start=123)
    total = int(off[-1]) + 77
    payload = synth.host_payload(total, 9)
    run_case(torch_cuda, payload, off, synth.random_keys(off.size - 1, 9), 2, 2)


def test_no_frames_is_a_copy(torch_cuda):
    payload = synth.host_payload(100003, 10)
    run_case(torch_cuda, payload, np.zeros(1, dtype=np.uint64), np.zeros(0, dtype=np.uint32), 1, 1)


def test_tiny_buffers(torch_cuda):
    for total in range(1, 40):
        for shift in (0, 1, 14, 15):
            payload = synth.host_payload(total, total, shift)
            off = frames_from_sizes([total // 3, total - total // 3])
            run_case(torch_cuda, payload, off, synth.random_keys(2, total, shift), shift, shift)


def test_empty_batch_is_noop(torch_cuda):
    torch = torch_cuda
    empty = torch.empty(0, dtype=torch.uint8, device="cuda")
    nm.mask_batch(empty, empty, torch.zeros(1, dtype=torch.int64, device="cuda"),
                  torch.zeros(0, dtype=torch.int32, device="cuda"))
    torch.cuda.synchronize()


def test_one_huge_frame(torch_cuda):
    total = (10 << 20) + 13
    payload = synth.host_payload(total, 12)
    run_case(torch_cuda, payload, frames_from_sizes([total]), np.array([0xDEADBEEF], dtype=np.uint32), 6, 6)


@pytest.mark.parametrize("unroll,max_blocks", [(1, 2048), (2, 64), (8, 0), (4, 1), (4, 100000), (2, 0)])
@pytest.mark.parametrize("flags", [-1, 0, 3, 7, 4, 11, 27, 43])
def test_launch_shapes(torch_cuda, unroll, max_blocks, flags):
    """Every kernel instantiation is bit-exact: U x cache-hint flags x walk (one window per
    wavefront, one or two steps, XCD order; or the persistent walk, flags & 4, with its grid cap)."""
    try:
        nm.tune(unroll, max_blocks, flags)
        off = synth.mixed_offsets(5 << 20, 1, 9000, seed=13)
        payload = synth.host_payload(int(off[-1]), 13)
        run_case(torch_cuda, payload, off, synth.random_keys(off.size - 1, 13), 4, 4)
        run_case(torch_cuda, payload, off, synth.random_keys(off.size - 1, 14), 4, 9)   # src misaligned vs dst
    finally:
        nm.tune()


@pytest.mark.parametrize("flags", [-1, 0, 7, 11, 43])
def test_near_uniform_frames(torch_cuda, flags):
    """Evenly sized frames with sparse irregular ones: the table-base guesses are exact
    until an irregular frame shifts every later frame start, then must recover
    (locate) — and dense 40-byte frames make the table slide inside a span."""
    try:
        nm.tune(4, 0, flags)
        rng = np.random.default_rng(21)
        sizes = np.full(40000, 1024, dtype=np.int64)
        irregular = rng.choice(sizes.size, 40, replace=False)
        sizes[irregular] = rng.integers(0, 20000, irregular.size)
        off = frames_from_sizes(sizes)
        payload = synth.host_payload(int(off[-1]), 21)
        run_case(torch_cuda, payload, off, synth.random_keys(sizes.size, 21))
        run_case(torch_cuda, payload, off, synth.random_keys(sizes.size, 22), 3, 3)
        # dense frames (many per chunk): the 16-entry table slides within a span
        sizes = np.full(30000, 40, dtype=np.int64)
        off = frames_from_sizes(sizes)
        payload = synth.host_payload(int(off[-1]), 23)
        run_case(torch_cuda, payload, off, synth.random_keys(sizes.size, 23))
    finally:
        nm.tune()


# ------------------------------------------------------------- full sizes ---

def test_c2_full_exact(torch_cuda):
    off, keys, total = synth.config("c2")
    payload = synth.host_payload(total, synth.SEED, 2)
    run_case(torch_cuda, payload, off, keys)


@pytest.mark.slow
def test_c4_shard_full_exact(torch_cuda):
    torch = torch_cuda
    off, keys, total = synth.config("c4", shard=3)
    g = torch.Generator(device="cuda").manual_seed(44)
    src = torch.randint(0, 256, (total,), dtype=torch.uint8, device="cuda", generator=g)
    host = src.cpu().numpy()
    nm.mask_batch(src, src, _dev(torch, off, None), _dev(torch, keys, None))
    torch.cuda.synchronize()
    orc.mask_batch_inplace(host, off, keys)
    assert np.array_equal(src.cpu().numpy(), host)


@pytest.mark.slow
@pytest.mark.parametrize("dst_shift,src_shift", [(0, 3), (5, 12), (0, 9)])
def test_misaligned_large_batch_exact(torch_cuda, dst_shift, src_shift):
    """src misaligned against dst at >= 256 MiB (the 4 x 1 KiB line-aligned source windows):
    320 MiB of C4's mixed frames, out of place, every byte and the guard bytes."""
    off, keys, _ = synth.config("c4", shard=1)
    n = int(np.searchsorted(off, 320 << 20, side="right")) - 1
    off, keys = off[:n + 1].copy(), keys[:n].copy()
    total = int(off[-1]) + 5                       # a ragged tail after the last frame
    payload = synth.host_payload(total, synth.SEED, 9)
    run_case(torch_cuda, payload, off, keys, dst_shift, src_shift)


@pytest.mark.slow
def test_c3_full_exact(torch_cuda):
    """1 GiB (BASELINE config 3): out of place, every byte against the oracle's in-place pass over
    a host copy (as C4 is checked); then involution and keystream linearity on the device."""
    torch = torch_cuda
    off, keys, total = synth.config("c3")
    off_t, keys_t = _dev(torch, off, None), _dev(torch, keys, None)
    g = torch.Generator(device="cuda").manual_seed(33)
    x = torch.randint(0, 256, (total,), dtype=torch.uint8, device="cuda", generator=g)
    y = torch.empty_like(x)
    nm.mask_batch(y, x, off_t, keys_t)
    torch.cuda.synchronize()
    host = x.cpu().numpy()
    orc.mask_batch_inplace(host, off, keys)         # the reference's expression, every frame
    assert np.array_equal(y.cpu().numpy(), host)
    del host
    z = torch.zeros_like(x)
    nm.mask_batch(z, z, off_t, keys_t)              # keystream = mask(0)
    assert torch.equal(torch.bitwise_xor(x, y), z)  # mask(x) ^ x == mask(0)
    nm.mask_batch(y, y, off_t, keys_t)              # involution
    assert torch.equal(y, x)


# ------------------------------------------------------- other entry points --

def test_multi_shard_entry(torch_cuda):
    torch = torch_cuda
    shards, expect = [], []
    for i in range(3):
        off = synth.mixed_offsets((1 << 20) + 7 * i, 1, 5000, seed=20 + i)
        keys = synth.random_keys(off.size - 1, 20 + i)
        payload = synth.host_payload(int(off[-1]), 20 + i)
        src = torch.from_numpy(payload).cuda()
        shards.append((torch.empty_like(src), src, _dev(torch, off, None), _dev(torch, keys, None)))
        expect.append(orc.mask_batch(payload, off, keys))
    nm.mask_batch_multi(shards, synchronize=True)
    for (dst, _, _, _), e in zip(shards, expect):
        assert np.array_equal(dst.cpu().numpy(), e)


def test_multi_shard_failing_shard(torch_cuda):
    # a failing shard must not leave earlier shards in flight.  Shard 1 is invalid
    # (null destination): shard 0 has completed and is exact when the call returns, shard 2
    # was never launched, and the error names shard 1.
    import ctypes

    from netc_amd import _lib

    torch = torch_cuda
    lib = _lib.gpu()
    off = synth.mixed_offsets(16 << 20, 1, 70000, seed=41)
    keys = synth.random_keys(off.size - 1, 41)
    payload = synth.host_payload(int(off[-1]), 41)
    src = torch.from_numpy(payload).cuda()
    dsts = [torch.zeros_like(src) for _ in range(3)]
    off_t, keys_t = _dev(torch, off, None), _dev(torch, keys, None)
    k = 3
    VP = ctypes.c_void_p * k
    devs = (ctypes.c_int * k)(0, 0, 0)
    dst_p = VP(dsts[0].data_ptr(), None, dsts[2].data_ptr())
    src_p = VP(*([src.data_ptr()] * k))
    totals = (ctypes.c_size_t * k)(*([int(off[-1])] * k))
    offs = VP(*([off_t.data_ptr()] * k))
    kp = VP(*([keys_t.data_ptr()] * k))
    ns = (ctypes.c_size_t * k)(*([keys.size] * k))
    s = torch.cuda.Stream()
    strs = VP(*([s.cuda_stream] * k))
    rc = lib.netc_gpu_mask_batch_multi(k, devs, dst_p, src_p, totals, offs, kp, ns, strs, 0)
    assert rc == nm.NETC_GPU_EINVAL
    assert b"shard 1" in lib.netc_gpu_strerror()
    # no synchronize here: the call itself waited for shard 0
    assert s.query(), "shard 0 still in flight after the failing call returned"
    assert np.array_equal(dsts[0].cpu().numpy(), orc.mask_batch(payload, off, keys))
    assert int(dsts[2].count_nonzero()) == 0


def test_multi_shard_distinct_devices(torch_cuda):
    # BASELINE config 4's single-process form: a byte-balanced batch cut into shards
    # (netc_shard_frames, offsets rebased per shard), one shard per device, launched
    # on all devices before any is waited on; every shard == the oracle
    torch = torch_cuda
    ndev = torch.cuda.device_count()
    if ndev < 2:
        pytest.skip("one device: the distinct-device path needs a multi-GPU box")
    off = synth.mixed_offsets(8 << 20, 256, 65536, seed=77)
    keys = synth.random_keys(off.size - 1, 77)
    payload = synth.host_payload(int(off[-1]), 77)
    cuts = nm.shard_frames(off, ndev)
    shards, expect, devs = [], [], []
    for d in range(ndev):
        f0, f1 = int(cuts[d]), int(cuts[d + 1])
        lo, hi = int(off[f0]), int(off[f1])
        o = (off[f0:f1 + 1] - np.uint64(lo)).astype(np.uint64)
        k = keys[f0:f1]
        dev = torch.device("cuda", d)
        src = torch.from_numpy(payload[lo:hi].copy()).to(dev)
        shards.append((torch.empty_like(src), src, _dev(torch, o, dev), _dev(torch, k, dev)))
        expect.append(orc.mask_batch(payload[lo:hi], o, k))
        devs.append(d)
    nm.mask_batch_multi(shards, synchronize=True)
    for (dst, _, _, _), e, d in zip(shards, expect, devs):
        assert dst.device.index == d
        assert np.array_equal(dst.cpu().numpy(), e)


@pytest.mark.parametrize("slot", [4096, 1 << 16, 3 << 20])
def test_stream_host_pipeline(torch_cuda, slot):
    off = synth.mixed_offsets(9 << 20, 1, 300000, seed=30)
    off = np.concatenate([[np.uint64(0)], off + np.uint64(5)]).astype(np.uint64)   # 5 unframed bytes first
    keys = synth.random_keys(off.size - 1, 30)
    total = int(off[-1]) + 3
    payload = synth.host_payload(total, 30)
    out = np.zeros_like(payload)
    nm.mask_stream_host(out, payload, off, keys, slot_bytes=slot, nslots=3)
    assert np.array_equal(out, orc.mask_batch(payload, off, keys))
    inplace = payload.copy()
    nm.mask_stream_host(inplace, inplace, off, keys, slot_bytes=slot, nslots=4)
    assert np.array_equal(inplace, out)


def test_errors_are_reported(torch_cuda):
    torch = torch_cuda
    from netc_amd import _lib

    lib = _lib.gpu()
    x = torch.zeros(100, dtype=torch.uint8, device="cuda")
    off = torch.tensor([0, 100], dtype=torch.int64, device="cuda")
    k = torch.zeros(1, dtype=torch.int32, device="cuda")
    assert lib.netc_gpu_mask_batch(0, None, x.data_ptr(), 100, off.data_ptr(), k.data_ptr(), 1, None) == nm.NETC_GPU_EINVAL
    assert b"null" in lib.netc_gpu_strerror()
    assert lib.netc_gpu_mask_batch(0, x.data_ptr(), x.data_ptr(), 100, None, k.data_ptr(), 1, None) == nm.NETC_GPU_EINVAL
    # partial overlap
    assert lib.netc_gpu_mask_batch(0, x.data_ptr() + 1, x.data_ptr(), 99, off.data_ptr(), k.data_ptr(), 1, None) \
        == nm.NETC_GPU_EINVAL
    assert lib.netc_gpu_mask_batch(1 << 20, x.data_ptr(), x.data_ptr(), 100, off.data_ptr(), k.data_ptr(), 1, None) \
        == nm.NETC_GPU_ENODEV
    with pytest.raises(nm.NetcGpuError) as ei:
        nm.tune(3, 10)
    assert ei.value.code == nm.NETC_GPU_EINVAL
    assert nm.device_count() >= 1
    nm.gpu_init(0)
