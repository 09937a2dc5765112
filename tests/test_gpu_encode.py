"""GPU parity: netc_gpu_encode_frames (send-side frame assembly, include/ws/frame.h) vs the oracle.

The oracle (oracle_encode_batch) concatenates the reference's single-frame send
(src/ws/common.c:53-125: header, extended length, key, payload masked with
:104-107), with the key kept on empty masked frames (defect B9).  The bar: the
wire bytes and wire offsets are bit-exact, and no byte past the wire length (or
before the wire start) is written.
"""

import numpy as np
import pytest

from netc_amd import mask as nm
from oracle import oracle as orc

pytestmark = pytest.mark.gpu

GUARD = 64
SENTINEL = 0xEE


def _dev(torch, a: np.ndarray):
    a = np.ascontiguousarray(a)
    if a.dtype == np.uint64:
        a = a.view(np.int64)
    elif a.dtype == np.uint32:
        a = a.view(np.int32)
    return torch.from_numpy(a).cuda()


def frames_from_sizes(sizes, start=0):
    off = np.zeros(len(sizes) + 1, dtype=np.uint64)
    off[0] = start
    off[1:] = start + np.cumsum(np.asarray(sizes, dtype=np.uint64))
    return off


def run_encode(torch, payload, off, keys, header0=None, masked=True, wire_shift=0, src_shift=0, check=True,
               length_class=None):
    total = payload.size
    n = off.size - 1
    src_buf = torch.full((total + 2 * GUARD,), 0x5A, dtype=torch.uint8, device="cuda")
    src = src_buf[GUARD + src_shift: GUARD + src_shift + total]
    src.copy_(torch.from_numpy(payload))
    cap = nm.wire_bound(total, n, masked)
    wire_buf = torch.full((cap + 2 * GUARD,), SENTINEL, dtype=torch.uint8, device="cuda")
    wire = wire_buf[GUARD + wire_shift: GUARD + wire_shift + cap]
    wo = torch.full((n + 1,), -1, dtype=torch.int64, device="cuda")
    keys_t = _dev(torch, np.asarray(keys, dtype=np.uint32)) if masked else None
    h_t = torch.from_numpy(np.ascontiguousarray(header0, dtype=np.uint8)).cuda() if header0 is not None else None
    nm.encode_frames(wire, wo, src, _dev(torch, off), keys_t, h_t, masked=masked, length_class=length_class)
    torch.cuda.synchronize()
    exp_wire, exp_wo = orc.encode_batch(payload, off, keys if masked else None, header0, masked)
    got_wo = wo.cpu().numpy().view(np.uint64)
    assert np.array_equal(got_wo, exp_wo), f"wire offsets differ (first at {np.nonzero(got_wo != exp_wo)[0][:4]})"
    assert int(exp_wo[-1]) == nm.wire_size(off, masked)
    whole = wire_buf.cpu().numpy()
    lo = GUARD + wire_shift
    got = whole[lo: lo + exp_wire.size]
    if check and not np.array_equal(got, exp_wire):
        bad = np.nonzero(got != exp_wire)[0]
        raise AssertionError(f"{bad.size} wire bytes differ, first at {bad[:8].tolist()} (n={n}, total={total}, "
                             f"masked={masked}, shifts={wire_shift},{src_shift})")
    assert (whole[:lo] == SENTINEL).all(), "write before the wire start"
    assert (whole[lo + exp_wire.size:] == SENTINEL).all(), "write past the wire length"
    return exp_wire


EDGE_SIZES = [0, 1, 2, 3, 4, 5, 15, 16, 17, 124, 125, 126, 127, 128, 1000, 1023, 1024, 1025, 4096, 65535, 65536,
              65537, 70000]


def _payload(rng, n):
    return rng.integers(0, 256, n, dtype=np.uint8)


# the assembly path: None = the default (wire-driven kernel; trailing blocks of the same launch
# compose the vectors holding header bytes), "fixscan" = those vectors by the wire-offsets scan
# (NETC_GPU_KNOB_ENC_FIX = 1), "src" = the source-driven walk writing headers in the same pass
# (NETC_GPU_KNOB_ENC_SRC = 1), "pf1" / "pf2" = the software-pipelined walk (NETC_GPU_KNOB_ENC_PF);
# all A/B paths
PATHS = [None, "fixscan", "fixtail", "src", "pf1", "pf2"]


def _set_path(gpu_knob, path):
    if path == "fixscan":
        gpu_knob("ENC_FIX", 1)
    elif path == "fixtail":
        gpu_knob("ENC_FIX", 2)
    elif path == "src":
        gpu_knob("ENC_SRC", 1)
    elif path in ("pf1", "pf2"):   # the software-pipelined walk (ENC_PF): 2 KiB / 4 KiB chunks
        gpu_knob("ENC_PF", int(path[2]))


@pytest.mark.parametrize("path", PATHS)
@pytest.mark.parametrize("masked", [True, False])
def test_every_length_class(torch_cuda, gpu_knob, masked, path):
    _set_path(gpu_knob, path)
    rng = np.random.default_rng(11)
    sizes = EDGE_SIZES + EDGE_SIZES[::-1]
    off = frames_from_sizes(sizes)
    payload = _payload(rng, int(off[-1]))
    keys = rng.integers(0, 2**32, len(sizes), dtype=np.uint64).astype(np.uint32)
    keys[:3] = [0, 0xFFFFFFFF, 0x00FF00FF]
    run_encode(torch_cuda, payload, off, keys, masked=masked)


@pytest.mark.parametrize("path", PATHS)
@pytest.mark.parametrize("wire_shift", [0, 1, 3, 7, 8, 13, 15])
@pytest.mark.parametrize("src_shift", [0, 5, 12])
def test_alignments(torch_cuda, gpu_knob, wire_shift, src_shift, path):
    _set_path(gpu_knob, path)
    rng = np.random.default_rng(100 + wire_shift * 16 + src_shift)
    sizes = rng.integers(0, 3000, 300)
    off = frames_from_sizes(sizes)
    payload = _payload(rng, int(off[-1]))
    keys = rng.integers(0, 2**32, len(sizes), dtype=np.uint64).astype(np.uint32)
    run_encode(torch_cuda, payload, off, keys, wire_shift=wire_shift, src_shift=src_shift)


def test_header_bytes_and_fragmented_message(torch_cuda):
    # one TEXT message in 4 fragments + a PING + a BINARY message: first-byte variants
    rng = np.random.default_rng(5)
    sizes = [300, 300, 300, 301, 0, 125, 70000]
    header0 = np.array([0x01, 0x00, 0x00, 0x80, 0x89, 0x8A, 0x82], dtype=np.uint8)
    off = frames_from_sizes(sizes)
    payload = _payload(rng, int(off[-1]))
    keys = rng.integers(0, 2**32, len(sizes), dtype=np.uint64).astype(np.uint32)
    wire = run_encode(torch_cuda, payload, off, keys, header0=header0)
    # the reference's receive path (oracle restatement of src/ws/common.c:146-347) decodes the message back
    used, msg, opcode = orc.decode_message(wire.tobytes())
    assert opcode == 1 and msg == payload[:1201].tobytes()


def test_tiny_frames_many_per_span(torch_cuda):
    # > 63 frame starts inside one 1 KiB span: the frame table slides mid-span
    rng = np.random.default_rng(9)
    sizes = rng.integers(0, 4, 5000)
    off = frames_from_sizes(sizes)
    payload = _payload(rng, int(off[-1]))
    keys = rng.integers(0, 2**32, len(sizes), dtype=np.uint64).astype(np.uint32)
    for masked in (True, False):
        run_encode(torch_cuda, payload, off, keys, masked=masked, wire_shift=3)


@pytest.mark.parametrize("path", PATHS)
def test_payload_with_unframed_prefix(torch_cuda, gpu_knob, path):
    # frames need not start at payload byte 0: off[0] > 0 (bytes before it are not sent)
    _set_path(gpu_knob, path)
    rng = np.random.default_rng(12)
    sizes = rng.integers(0, 2000, 50)
    off = frames_from_sizes(sizes, start=777)
    payload = _payload(rng, int(off[-1]) + 100)
    keys = rng.integers(0, 2**32, len(sizes), dtype=np.uint64).astype(np.uint32)
    run_encode(torch_cuda, payload, off, keys)


def test_single_frame_sizes(torch_cuda):
    rng = np.random.default_rng(13)
    for size in (0, 1, 17, 125, 126, 1024, 65535, 65536, 1 << 20):
        off = frames_from_sizes([size])
        payload = _payload(rng, size)
        keys = np.array([0x3D21FA37], dtype=np.uint32)
        run_encode(torch_cuda, payload, off, keys)
        run_encode(torch_cuda, payload, off, keys, wire_shift=7, src_shift=3)


@pytest.mark.parametrize("path", PATHS)
@pytest.mark.parametrize("src_shift", [0, 9])
def test_frame_starts_at_every_lane_byte(torch_cuda, gpu_knob, src_shift, path):
    # the source-driven lanes: a frame start at each byte j of a lane's 16 (one start per lane:
    # two overlapping 16-B stores + the header), two starts in one lane (frames of 1..15 B),
    # empty frames between long ones, and the batch ending on, inside and after a vector edge
    _set_path(gpu_knob, path)
    rng = np.random.default_rng(77 + src_shift)
    sizes = []
    for j in range(16):
        sizes += [1024 + j, 1000 - j, 17, 40 + j]
    sizes += [5, 9, 0, 0, 300, 0, 2048, 3, 15, 16, 1, 4000]
    for tail in (0, 1, 15, 16, 33):
        sz = sizes + [tail]
        off = frames_from_sizes(sz)
        payload = _payload(rng, int(off[-1]))
        keys = rng.integers(0, 2**32, len(sz), dtype=np.uint64).astype(np.uint32)
        h0 = rng.choice(np.array([0x81, 0x82, 0x01, 0x00, 0x80, 0x89], dtype=np.uint8), len(sz))
        for wire_shift in (0, 11):
            run_encode(torch_cuda, payload, off, keys, header0=h0, wire_shift=wire_shift, src_shift=src_shift)
        run_encode(torch_cuda, payload, off, keys, masked=False, src_shift=src_shift)


def test_rfc6455_hello(torch_cuda):
    # RFC 6455 §5.7: a single-frame masked text message "Hello" with key 37 fa 21 3d
    torch = torch_cuda
    payload = np.frombuffer(b"Hello", dtype=np.uint8).copy()
    off = frames_from_sizes([5])
    keys = nm.pack_keys(np.frombuffer(bytes.fromhex("37fa213d"), dtype=np.uint8))
    wire = run_encode(torch, payload, off, keys, header0=np.array([0x81], dtype=np.uint8))
    assert wire.tobytes() == bytes.fromhex("818537fa213d7f9f4d5158")
    # and unmasked: 0x81 0x05 "Hello"
    wire = run_encode(torch, payload, off, keys, header0=np.array([0x81], dtype=np.uint8), masked=False)
    assert wire.tobytes() == bytes.fromhex("810548656c6c6f")


def test_empty_batch(torch_cuda):
    torch = torch_cuda
    wo = torch.full((1,), -1, dtype=torch.int64, device="cuda")
    wire = torch.zeros(16, dtype=torch.uint8, device="cuda")
    src = torch.zeros(16, dtype=torch.uint8, device="cuda")
    off = torch.zeros(1, dtype=torch.int64, device="cuda")
    keys = torch.zeros(0, dtype=torch.int32, device="cuda")
    nm.encode_frames(wire, wo, src, off, keys)
    torch.cuda.synchronize()
    assert int(wo.cpu()[0]) == 0


@pytest.mark.parametrize("path", PATHS)
def test_c2_full_size(torch_cuda, gpu_knob, path):
    # config 2 shape: 65,536 x 1 KiB frames, independent keys
    _set_path(gpu_knob, path)
    rng = np.random.default_rng(0x6E657463)
    n = 65536
    off = frames_from_sizes(np.full(n, 1024))
    payload = _payload(rng, int(off[-1]))
    keys = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    run_encode(torch_cuda, payload, off, keys)


@pytest.mark.parametrize("path", PATHS)
def test_mixed_64mib(torch_cuda, gpu_knob, path):
    # config 4 shape (sizes uniform in [256, 65536], unaligned), 64 MiB
    _set_path(gpu_knob, path)
    rng = np.random.default_rng(44)
    sizes = rng.integers(256, 65537, 4096)
    off = frames_from_sizes(sizes)
    payload = _payload(rng, int(off[-1]))
    keys = rng.integers(0, 2**32, sizes.size, dtype=np.uint64).astype(np.uint32)
    run_encode(torch_cuda, payload, off, keys, wire_shift=5, src_shift=3)


def test_errors(torch_cuda):
    torch = torch_cuda
    src = torch.zeros(1000, dtype=torch.uint8, device="cuda")
    off = torch.tensor([0, 500, 1000], dtype=torch.int64, device="cuda")
    keys = torch.zeros(2, dtype=torch.int32, device="cuda")
    wo = torch.zeros(3, dtype=torch.int64, device="cuda")
    small = torch.zeros(1000 + 27, dtype=torch.uint8, device="cuda")   # bound is 1000 + 2 * 14
    with pytest.raises(nm.NetcGpuError) as e:
        nm.encode_frames(small, wo, src, off, keys)
    assert e.value.code == nm.NETC_GPU_EINVAL
    big = torch.zeros(4096, dtype=torch.uint8, device="cuda")
    with pytest.raises(nm.NetcGpuError) as e:   # wire overlapping the payload
        nm.encode_frames(big, wo, big[100:1100], off, keys)
    assert e.value.code == nm.NETC_GPU_EINVAL
    with pytest.raises(ValueError):
        nm.encode_frames(big, wo, src, off, None, masked=True)


@pytest.mark.parametrize("unroll,max_blocks", [(4, 0), (2, 1), (8, 3), (8, 0)])
def test_launch_shapes(torch_cuda, unroll, max_blocks):
    # both chunk sizes (unroll 8 selects 4 KiB), and grids far smaller than the work (long grid-stride walks)
    try:
        nm.tune(unroll, max_blocks)
        rng = np.random.default_rng(31 + unroll)
        sizes = np.concatenate([rng.integers(0, 3000, 400), rng.integers(0, 20, 400), np.full(300, 1024)])
        off = frames_from_sizes(sizes)
        payload = _payload(rng, int(off[-1]))
        keys = rng.integers(0, 2**32, sizes.size, dtype=np.uint64).astype(np.uint32)
        run_encode(torch_cuda, payload, off, keys, wire_shift=9, src_shift=2)
        run_encode(torch_cuda, payload, off, keys, masked=False)
    finally:
        nm.tune()


@pytest.mark.parametrize("path", PATHS)
@pytest.mark.parametrize("dense", ["0", "100000"])
@pytest.mark.parametrize("masked", [True, False])
def test_both_compose_paths(torch_cuda, gpu_knob, dense, masked, path):
    # the same batches through the vector path + header fixups (knob ENC_DENSE_BYTES = 0)
    # and through the dense per-lane compose of every span (threshold above any mean):
    # uniform 16 / 8 / 1 B frames, empty frames, 0..30 B mixes, and long frames between
    gpu_knob("ENC_DENSE_BYTES", dense)
    _set_path(gpu_knob, path)
    rng = np.random.default_rng(21)
    parts = [np.full(3000, 16), np.full(2000, 8), rng.integers(0, 31, 4000), np.full(1500, 1),
             np.array([126, 65536, 0, 0, 125, 3000]), np.zeros(700, dtype=np.int64), rng.integers(100, 300, 200)]
    sizes = np.concatenate(parts)
    off = frames_from_sizes(sizes, start=3)
    payload = _payload(rng, int(off[-1]) + 9)
    keys = rng.integers(0, 2**32, len(sizes), dtype=np.uint64).astype(np.uint32)
    h0 = rng.choice(np.array([0x81, 0x82, 0x01, 0x00, 0x80, 0x89], dtype=np.uint8), len(sizes))
    run_encode(torch_cuda, payload, off, keys, header0=h0, masked=masked, wire_shift=5, src_shift=11)
    run_encode(torch_cuda, payload, off, keys, masked=masked)


@pytest.mark.parametrize("wire_shift", [0, 1, 7, 15])
@pytest.mark.parametrize("src_shift", [0, 5])
@pytest.mark.parametrize("masked", [True, False])
def test_dense_compose_edges(torch_cuda, gpu_knob, wire_shift, src_shift, masked):
    # the dense per-lane compose forced on a batch of mostly short frames with long ones between
    # (spans walked over several 62-entry table windows), runs of empty frames, a long first and
    # last frame, at wire and source misalignments
    # (round 4 also tried a frame-driven form, one thread per frame composing the vectors that
    # start in it: 122 against 125 us at 64 MiB of 16-B frames, 122 against 91 us at 64-B frames)
    gpu_knob("ENC_DENSE_BYTES", "100000")
    rng = np.random.default_rng(300 + wire_shift * 8 + src_shift + masked)
    sizes = np.concatenate([[5000], rng.integers(100, 140, 400), np.zeros(50, dtype=np.int64),
                            rng.integers(0, 20, 500), [70000, 1, 65535, 126, 0], rng.integers(0, 300, 300), [4099]])
    off = frames_from_sizes(sizes)
    payload = _payload(rng, int(off[-1]))
    keys = rng.integers(0, 2**32, len(sizes), dtype=np.uint64).astype(np.uint32)
    run_encode(torch_cuda, payload, off, keys, masked=masked, wire_shift=wire_shift, src_shift=src_shift)


# ------------------------------------------------ one length class (netc_gpu_encode_frames_class) --
# Every frame in one header class: the wire offsets are affine in the payload offsets, the assembly
# launch computes and writes them (no scan launch).  Same bar as above: wire bytes and offsets
# bit-exact against oracle_encode_batch, nothing written outside the wire.

CLASS_SIZES = {
    nm.NETC_WS_CLASS_7BIT: (80, 126),          # mean >= 80 B: the vector path (below it, the dense path)
    nm.NETC_WS_CLASS_16BIT: (126, 65536),
    nm.NETC_WS_CLASS_64BIT: (65536, 200000),
}


@pytest.mark.parametrize("cls", sorted(CLASS_SIZES))
@pytest.mark.parametrize("masked", [True, False])
@pytest.mark.parametrize("shifts", [(0, 0), (5, 3), (15, 9)])
def test_one_class(torch_cuda, cls, masked, shifts):
    rng = np.random.default_rng(500 + cls * 8 + shifts[0] + masked)
    lo, hi = CLASS_SIZES[cls]
    n = {0: 3000, 2: 400, 8: 24}[cls]
    sizes = rng.integers(lo, hi, n)
    sizes[:2] = [lo, hi - 1]   # the class edges
    off = frames_from_sizes(sizes, start=int(rng.integers(0, 40)))
    assert nm.length_class(off) == cls
    payload = _payload(rng, int(off[-1]) + 7)
    keys = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    h0 = rng.choice(np.array([0x81, 0x82, 0x01, 0x00, 0x80], dtype=np.uint8), n)
    run_encode(torch_cuda, payload, off, keys, header0=h0, masked=masked, wire_shift=shifts[0], src_shift=shifts[1],
               length_class=cls)


@pytest.mark.parametrize("path", [None, "pf1", "pf2"])
def test_one_class_c2_full_size(torch_cuda, gpu_knob, path):
    # config 2: 65,536 x 1 KiB, every frame in the 16-bit class -- 256 fixup blocks share the counter
    _set_path(gpu_knob, path)
    rng = np.random.default_rng(0x6E657463)
    n = 65536
    off = frames_from_sizes(np.full(n, 1024))
    payload = _payload(rng, int(off[-1]))
    keys = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    run_encode(torch_cuda, payload, off, keys, length_class=nm.NETC_WS_CLASS_16BIT)


@pytest.mark.parametrize("path", ["fixscan", "fixtail", "src", "dense"])
def test_one_class_on_the_general_paths(torch_cuda, gpu_knob, path):
    # where the call takes another path (the knobs, or a batch averaging < 80 B) the scan runs
    # and the result is exact -- also when a frame breaks the promise
    if path == "dense":
        gpu_knob("ENC_DENSE_BYTES", "100000")
    else:
        _set_path(gpu_knob, path)
    rng = np.random.default_rng(61)
    sizes = rng.integers(126, 3000, 300)
    sizes[100] = 5   # outside the 16-bit class
    off = frames_from_sizes(sizes)
    payload = _payload(rng, int(off[-1]))
    keys = rng.integers(0, 2**32, sizes.size, dtype=np.uint64).astype(np.uint32)
    run_encode(torch_cuda, payload, off, keys, wire_shift=3, length_class=nm.NETC_WS_CLASS_16BIT)


def test_one_class_above_256_mib_takes_the_scan(torch_cuda):
    # a wire bound over 256 MiB: the scan runs (it costs less there than the one-launch form
    # saves), so the result is exact even with a frame outside the promised class
    rng = np.random.default_rng(71)
    n = 262144
    sizes = np.full(n, 1030)
    sizes[1000] = 99
    off = frames_from_sizes(sizes)
    assert nm.wire_bound(int(off[-1]), n, True) > (256 << 20)
    payload = _payload(rng, int(off[-1]))
    keys = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    run_encode(torch_cuda, payload, off, keys, length_class=nm.NETC_WS_CLASS_16BIT)


def _broken(torch, sizes, cls, masked=True, wire_shift=0):
    rng = np.random.default_rng(len(sizes) + cls)
    off = frames_from_sizes(sizes)
    total = int(off[-1])
    n = len(sizes)
    src = torch.from_numpy(_payload(rng, total)).cuda()
    cap = nm.wire_bound(total, n, masked)
    wire_buf = torch.full((cap + 2 * GUARD,), SENTINEL, dtype=torch.uint8, device="cuda")
    wire = wire_buf[GUARD + wire_shift: GUARD + wire_shift + cap]
    wo = torch.full((n + 1,), -1, dtype=torch.int64, device="cuda")
    keys = _dev(torch, rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)) if masked else None
    nm.encode_frames(wire, wo, src, _dev(torch, off), keys, masked=masked, length_class=cls)
    torch.cuda.synchronize()
    whole = wire_buf.cpu().numpy()
    assert (whole[:GUARD + wire_shift] == SENTINEL).all(), "write before the wire"
    assert (whole[GUARD + wire_shift + cap:] == SENTINEL).all(), "write past the wire bound"
    return wo.cpu().numpy().view(np.uint64)


@pytest.mark.parametrize("where", ["first", "middle", "last", "many"])
@pytest.mark.parametrize("masked", [True, False])
def test_one_class_broken_promise(torch_cuda, where, masked):
    # a frame outside the promised class: wire_offsets[n] = NETC_WS_WIRE_INVALID, no stray write
    sizes = np.full(20000, 1024)
    pick = {"first": [0], "middle": [9999], "last": [19999], "many": list(range(3, 20000, 997))}[where]
    for i, k in enumerate(pick):
        sizes[k] = [100, 70000, 0][i % 3]
    wo = _broken(torch_cuda, sizes, nm.NETC_WS_CLASS_16BIT, masked=masked, wire_shift=7)
    assert int(wo[-1]) == nm.NETC_WS_WIRE_INVALID


def test_one_class_counter_resets(torch_cuda):
    # the fixup blocks' counter is left zero by every call, broken or not: calls in a row on one
    # stream with grids of different sizes each give their own verdict
    torch = torch_cuda
    for n, bad in [(5000, False), (300, True), (70000, False), (64, True), (64, False), (30000, True), (1, False)]:
        sizes = np.full(n, 200)
        if bad:
            sizes[n // 2] = 7
        wo = _broken(torch, sizes, nm.NETC_WS_CLASS_16BIT)
        if bad:
            assert int(wo[-1]) == nm.NETC_WS_WIRE_INVALID
        else:
            assert int(wo[-1]) == nm.wire_size(frames_from_sizes(sizes), True)
    rng = np.random.default_rng(3)
    sizes = rng.integers(126, 5000, 2000)
    off = frames_from_sizes(sizes)
    run_encode(torch, _payload(rng, int(off[-1])), off, rng.integers(0, 2**32, 2000, dtype=np.uint64).astype(np.uint32),
               length_class=nm.NETC_WS_CLASS_16BIT)


def test_one_class_errors(torch_cuda):
    torch = torch_cuda
    src = torch.zeros(1000, dtype=torch.uint8, device="cuda")
    off = torch.tensor([0, 500, 1000], dtype=torch.int64, device="cuda")
    keys = torch.zeros(2, dtype=torch.int32, device="cuda")
    wo = torch.zeros(3, dtype=torch.int64, device="cuda")
    wire = torch.zeros(4096, dtype=torch.uint8, device="cuda")
    for bad in (-1, 1, 3, 4, 16):
        with pytest.raises(nm.NetcGpuError) as e:
            nm.encode_frames(wire, wo, src, off, keys, length_class=bad)
        assert e.value.code == nm.NETC_GPU_EINVAL
    nm.encode_frames(wire, wo, src, off, keys, length_class=nm.NETC_WS_CLASS_16BIT)
    torch.cuda.synchronize()
    assert int(wo.cpu()[-1]) == 1000 + 2 * 8
