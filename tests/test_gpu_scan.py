"""GPU parity: netc_gpu_scan_frames (device frame-boundary scan, include/ws/frame.h) vs the oracle.

The checker is oracle_scan_frames (the header decode of src/ws/common.c:146-296
walked over the stream; pinned in tests/test_scan_oracle.py by the reference's
golden wire and its compiled receiver).  The bar: identical header offsets, keys,
header bytes, frame count, consumed offset and error offset.
"""

import numpy as np
import pytest

from netc_amd import mask as nm
from oracle import oracle as orc

pytestmark = pytest.mark.gpu


def frames_from_sizes(sizes, start=0):
    off = np.zeros(len(sizes) + 1, dtype=np.uint64)
    off[0] = start
    off[1:] = start + np.cumsum(np.asarray(sizes, dtype=np.uint64))
    return off


def run_scan(torch, wire: np.ndarray, start=0, strict=True, max_frames=None, parallel=False):
    """parallel: also require that the scan did not fall back to the serial walk
    (netc_gpu_scan_diag == 0) -- results are identical either way, so only this sees it."""
    exp_hdr, exp_keys, exp_b0, exp_consumed, exp_err = orc.scan_frames(wire, start=start, strict=strict)
    n = exp_hdr.size
    cap = n if max_frames is None else max_frames
    w = torch.from_numpy(np.ascontiguousarray(wire)).cuda() if wire.size else torch.zeros(1, dtype=torch.uint8,
                                                                                          device="cuda")
    hdr = torch.full((cap + 1,), -7, dtype=torch.int64, device="cuda")
    keys = torch.zeros(max(cap, 1), dtype=torch.int32, device="cuda")
    b0 = torch.zeros(max(cap, 1), dtype=torch.uint8, device="cuda")
    res = torch.full((3,), -7, dtype=torch.int64, device="cuda")
    nm.scan_frames(w, hdr, keys, b0, res, start=start, strict=strict, length=wire.size)
    torch.cuda.synchronize()
    r = res.cpu().numpy().view(np.uint64)
    assert int(r[0]) == n, f"frames {int(r[0])} != {n}"
    assert int(r[1]) == exp_consumed, f"consumed {int(r[1])} != {exp_consumed}"
    assert (None if int(r[2]) == (1 << 64) - 1 else int(r[2])) == exp_err
    k = min(n, cap)
    got_hdr = hdr.cpu().numpy().view(np.uint64)
    assert np.array_equal(got_hdr[:k], exp_hdr[:k]), f"header offsets differ at {np.nonzero(got_hdr[:k] != exp_hdr[:k])[0][:4]}"
    assert np.array_equal(keys.cpu().numpy().view(np.uint32)[:k], exp_keys[:k])
    assert np.array_equal(b0.cpu().numpy()[:k], exp_b0[:k])
    if n <= cap:
        assert int(got_hdr[n]) == exp_consumed
    if parallel:
        why = nm.scan_diag()
        assert why == 0, f"serial fallback, reason {why:#x}"
    return n


def _stream(rng, sizes, masked=True, b0=None):
    off = frames_from_sizes(sizes)
    payload = rng.integers(0, 256, int(off[-1]), dtype=np.uint8)
    keys = rng.integers(0, 2**32, len(sizes), dtype=np.uint64).astype(np.uint32)
    wire, wo = orc.encode_batch(payload, off, keys, b0, masked)
    return wire, wo


@pytest.mark.parametrize("seed", range(3))
def test_mixed_sizes(torch_cuda, seed):
    rng = np.random.default_rng(seed)
    sizes = np.concatenate([rng.integers(0, 5000, 300), rng.integers(0, 130, 300), [65535, 65536, 200000]])
    rng.shuffle(sizes)
    wire, _ = _stream(rng, sizes)
    assert run_scan(torch_cuda, wire, parallel=True) == sizes.size


def test_c2_shape(torch_cuda):
    rng = np.random.default_rng(2)
    wire, _ = _stream(rng, np.full(65536, 1024))
    assert run_scan(torch_cuda, wire, parallel=True) == 65536


def test_c4_shape_64mib(torch_cuda):
    rng = np.random.default_rng(4)
    wire, _ = _stream(rng, rng.integers(256, 65537, 2000))
    assert run_scan(torch_cuda, wire, parallel=True) == 2000


def test_tiny_frames(torch_cuda):
    # 6-byte wire frames (empty masked payloads) and 1-3 byte payloads: long chains inside a chunk
    rng = np.random.default_rng(5)
    wire, _ = _stream(rng, rng.integers(0, 4, 20000))
    assert run_scan(torch_cuda, wire, parallel=True) == 20000


def test_truncated_streams(torch_cuda):
    rng = np.random.default_rng(6)
    wire, wo = _stream(rng, rng.integers(0, 9000, 200))
    for cut in [0, 1, 2, 5, int(wo[50]) - 1, int(wo[50]), int(wo[50]) + 1, int(wo[50]) + 3, int(wo[120]) + 7,
                wire.size - 1, wire.size]:
        run_scan(torch_cuda, wire[:cut], parallel=True)


def test_start_offset(torch_cuda):
    rng = np.random.default_rng(7)
    wire, wo = _stream(rng, rng.integers(0, 9000, 200))
    for s in (int(wo[1]), int(wo[77]), int(wo[199]), wire.size):
        run_scan(torch_cuda, wire, start=s, parallel=True)


def test_unmasked_and_non_strict(torch_cuda):
    rng = np.random.default_rng(8)
    wire, _ = _stream(rng, rng.integers(0, 3000, 300), masked=False)
    assert run_scan(torch_cuda, wire, strict=False, parallel=True) == 300   # the speculative pass covers it
    assert run_scan(torch_cuda, wire, strict=True) == 0   # the first unmasked header is rejected


@pytest.mark.parametrize("masked", [False, True])
def test_non_strict_many_chunks(torch_cuda, masked):
    # every position a K1 candidate: tiny, 7-bit, 16-bit and 64-bit lengths over ~1,000 chunks
    rng = np.random.default_rng(18 + masked)
    sizes = np.concatenate([rng.integers(0, 8, 3000), rng.integers(0, 126, 3000), rng.integers(126, 9000, 400),
                            [70000, 131072]])
    rng.shuffle(sizes)
    wire, _ = _stream(rng, sizes, masked=masked)
    assert run_scan(torch_cuda, wire, strict=False, parallel=True) == sizes.size


def test_strict_errors_mid_stream(torch_cuda):
    rng = np.random.default_rng(9)
    good, _ = _stream(rng, rng.integers(0, 6000, 100))
    for bad in (bytes.fromhex("8105") + b"Hello", bytes.fromhex("c185") + bytes(9), bytes.fromhex("0980") + bytes(4),
                bytes.fromhex("83850000000048656c6c6f")):
        wire = np.concatenate([good, np.frombuffer(bad, dtype=np.uint8), good])
        run_scan(torch_cuda, wire, strict=True)
        run_scan(torch_cuda, wire, strict=False)
        # the headers a client must not send but the reference accepts (RSV2/RSV3 set, a reserved
        # opcode, a fragmented control frame): the non-strict pass stops there and walks on
        # serially.  RSV1 (permessage-deflate) does not stop it.
        op = bad[0] & 0x0F
        stops = bool(bad[0] & 0x30) or 3 <= op <= 7 or op >= 11 or (op >= 8 and not bad[0] & 0x80)
        assert nm.scan_diag() == (0x10000 if stops else 0)


@pytest.mark.parametrize("b0, stops", [(0xC2, False), (0xC1, False), (0xA2, True), (0x92, True)])
def test_non_strict_rsv_headers(torch_cuda, b0, stops):
    # every frame with RSV1 set, as permessage-deflate sends them, stays on the
    # speculative parallel pass (diag 0); RSV2 / RSV3 still stop it at the first header and the
    # rest is walked serially (diag bit 16).  Results equal the oracle's either way; strict mode
    # rejects the first header.
    rng = np.random.default_rng(41)
    sizes = rng.integers(0, 5000, 3000)
    wire, _ = _stream(rng, sizes, b0=np.full(sizes.size, b0, dtype=np.uint8))
    assert run_scan(torch_cuda, wire, strict=False, parallel=not stops) == sizes.size
    assert nm.scan_diag() == (0x10000 if stops else 0)
    assert run_scan(torch_cuda, wire, strict=True) == 0


def test_header_byte_variants(torch_cuda):
    rng = np.random.default_rng(10)
    sizes = rng.integers(0, 125, 500)
    b0 = rng.choice(np.array([0x81, 0x82, 0x01, 0x00, 0x80, 0x89, 0x8A, 0x88], dtype=np.uint8), 500)
    wire, _ = _stream(rng, sizes, b0=b0)
    assert run_scan(torch_cuda, wire, parallel=True) == 500


def test_max_frames_cap(torch_cuda):
    rng = np.random.default_rng(11)
    wire, _ = _stream(rng, rng.integers(0, 2000, 400))
    run_scan(torch_cuda, wire, max_frames=100, parallel=True)
    run_scan(torch_cuda, wire, max_frames=0, parallel=True)


def test_scratch_left_clean_between_calls(torch_cuda):
    # every call leaves its counters, marks and flags zeroed for the next one on the
    # same stream (no clearing launch): alternate sizes, the serial fallback, the LDS
    # fallbacks (tiny frames), an error stop and non-strict mode, each checked
    rng = np.random.default_rng(21)
    rec = b"".join(bytes.fromhex("82fe") + (5000 + i % 997).to_bytes(2, "big") + bytes(4) for i in range(997))
    inner = np.tile(np.frombuffer(rec, dtype=np.uint8), 20)
    adv, _ = orc.encode_batch(inner, np.array([0, inner.size], dtype=np.uint64), np.array([0], dtype=np.uint32),
                              None, True)
    big, _ = _stream(rng, np.full(6000, 1024))
    small, _ = _stream(rng, rng.integers(0, 3000, 40))
    tiny, _ = _stream(rng, rng.integers(0, 4, 3000))
    bad = small.copy()
    bad[int(np.flatnonzero(bad)[0])] ^= 0x70   # RSV bits on the first header
    unmasked, _ = _stream(rng, rng.integers(0, 2000, 100), masked=False)
    for wire, strict in [(big, True), (small, True), (adv, True), (small, True), (tiny, True), (big, True),
                         (bad, True), (unmasked, False), (big, True), (tiny, True), (small, True)]:
        run_scan(torch_cuda, wire, strict=strict)


def test_adversarial_payload_falls_back(torch_cuda):
    # a big frame masked with the zero key whose payload is a run of valid-looking
    # 8-byte headers (16-bit lengths 5000..5996) that each jump to a different place:
    # hundreds of distinct exits per chunk (capacity overflow -> the serial walk)
    rng = np.random.default_rng(12)
    rec = b"".join(bytes.fromhex("82fe") + (5000 + i % 997).to_bytes(2, "big") + bytes(4) for i in range(997))
    inner = np.tile(np.frombuffer(rec, dtype=np.uint8), 40)
    off = np.array([0, inner.size, inner.size + 10], dtype=np.uint64)
    payload = np.concatenate([inner, rng.integers(0, 256, 10, dtype=np.uint8)])
    wire, _ = orc.encode_batch(payload, off, np.array([0, 0x01020304], dtype=np.uint32), None, True)
    assert run_scan(torch_cuda, wire) == 2


@pytest.mark.parametrize("strict", [True, False])
def test_periodic_payload_takes_full_check(torch_cuda, strict):
    # zero payloads under the key bytes 70 FE 11 22: every 4th wire byte is xFE, so K1's cheap
    # selection (second header byte xFE/xFF alone) finds ~1,000 positions per chunk; the chunk
    # takes the full quick check instead (the byte before each xFE has RSV bits set) and stays
    # on the parallel path.  Random frames between, so some chunks take each pass.
    rng = np.random.default_rng(31)
    sizes = np.concatenate([np.full(3000, 1024), rng.integers(0, 5000, 300)])
    off = frames_from_sizes(sizes)
    payload = np.zeros(int(off[-1]), dtype=np.uint8)
    rand = np.arange(sizes.size) >= 3000
    for k in np.flatnonzero(rand):
        payload[int(off[k]):int(off[k + 1])] = rng.integers(0, 256, int(sizes[k]), dtype=np.uint8)
    keys = np.where(rand, rng.integers(0, 2**32, sizes.size, dtype=np.uint64), 0x2211FE70).astype(np.uint32)
    order = rng.permutation(sizes.size)
    sizes, keys = sizes[order], keys[order]
    off2 = frames_from_sizes(sizes)
    payload2 = np.concatenate([payload[int(off[k]):int(off[k + 1])] for k in order])
    wire, _ = orc.encode_batch(payload2, off2, keys, None, True)
    assert run_scan(torch_cuda, wire, strict=strict, parallel=True) == sizes.size


def test_empty(torch_cuda):
    run_scan(torch_cuda, np.zeros(0, dtype=np.uint8))
    run_scan(torch_cuda, np.zeros(1, dtype=np.uint8))


@pytest.mark.parametrize("cut", [None, -3])
def test_scan_then_unmask_in_place(torch_cuda, cut):
    # the whole receive path on the device: scan -> unmask, no host round trip;
    # every payload byte equals the plaintext, every header byte (and the partial
    # frame at the end) is untouched
    torch = torch_cuda
    rng = np.random.default_rng(14)
    sizes = np.concatenate([rng.integers(0, 3000, 500), [0, 1, 125, 126, 65536]])
    off = frames_from_sizes(sizes)
    plain = rng.integers(0, 256, int(off[-1]), dtype=np.uint8)
    keys = rng.integers(0, 2**32, sizes.size, dtype=np.uint64).astype(np.uint32)
    wire, wo = orc.encode_batch(plain, off, keys, None, True)
    if cut is not None:
        wire = wire[:cut]
    n = sizes.size
    w = torch.from_numpy(wire.copy()).cuda()
    hdr = torch.zeros(n + 1, dtype=torch.int64, device="cuda")
    kk = torch.zeros(n, dtype=torch.int32, device="cuda")
    b0 = torch.zeros(n, dtype=torch.uint8, device="cuda")
    res = torch.zeros(3, dtype=torch.int64, device="cuda")
    nm.scan_frames(w, hdr, kk, b0, res)
    nm.unmask_frames(w, hdr, kk, res)
    torch.cuda.synchronize()
    got = w.cpu().numpy()
    found = int(res.cpu()[0])
    assert found == (n if cut is None else n - 1)
    expect = wire.copy()
    for k in range(found):   # payload region of frame k = its last len bytes before the next header
        lo, hi = int(off[k]), int(off[k + 1])
        p_end = int(wo[k + 1])
        expect[p_end - (hi - lo): p_end] = plain[lo:hi]
    assert np.array_equal(got, expect)


def test_repeat_calls_same_stream(torch_cuda):
    # the chained scan's status words are reused across calls (epochs)
    rng = np.random.default_rng(13)
    for i in range(5):
        wire, _ = _stream(rng, rng.integers(0, 4000, 300 + 50 * i))
        run_scan(torch_cuda, wire)


@pytest.mark.parametrize("emit", [None, "64"])
@pytest.mark.parametrize("slots", [None, "0", "3"])
@pytest.mark.parametrize("masked,strict", [(True, True), (False, False)])
def test_dense_chunks_parallel_walks(torch_cuda, gpu_knob, masked, strict, slots, emit):
    # chunks of 64+ frames (K2' and K4b': 16-hop links, anchored emit): uniform 16 / 8 B
    # payloads, empty frames (2-byte unmasked / 6-byte masked wire frames: up to 2,048
    # per chunk), mixes, and a long frame between; then truncations and start offsets
    # inside the dense stretch and a frame cap that ends inside an anchor's run.  slots:
    # K2' anchor slots (None: one per chunk, K4b' emits from them; "0": none, every
    # dense chunk goes through the LDS emit; "3": both paths in one call)
    gpu_knob("SCAN_ANCHOR_SLOTS", slots)
    gpu_knob("SCAN_BLOCK_CHUNKS", emit)   # "64": the link and emit blocks of streams over 128 MiB
    rng = np.random.default_rng(41 + masked)
    sizes = np.concatenate([np.full(3000, 16), np.full(2500, 8), np.zeros(3000, dtype=np.int64),
                            rng.integers(0, 20, 3000), [70000], np.full(1000, 1)])
    wire, wo = _stream(rng, sizes, masked=masked)
    assert run_scan(torch_cuda, wire, strict=strict, parallel=strict) == sizes.size
    for cut in (int(wo[3100]) + 1, int(wo[6000]), int(wo[9001]) + 3):
        run_scan(torch_cuda, wire[:cut], strict=strict, parallel=strict)
    for s in (int(wo[17]), int(wo[5600])):
        run_scan(torch_cuda, wire, start=s, strict=strict, parallel=strict)
    run_scan(torch_cuda, wire, strict=strict, max_frames=4123)


@pytest.mark.parametrize("fast", ["1", "0"])
def test_ranking_paths(torch_cuda, gpu_knob, fast):
    # K3a / K3b rank a tile's nodes (and the tiles' external nodes) with one barrier per
    # round when they fit (512 / 1,024 nodes), else with the generic loop; both on the
    # same streams (knob SCAN_FAST_RANK = 0 forces the generic loop)
    gpu_knob("SCAN_FAST_RANK", fast)
    rng = np.random.default_rng(31)
    wire, _ = _stream(rng, np.full(16384, 1024))   # 16 MiB: 16 full tiles of ~262 nodes
    assert run_scan(torch_cuda, wire, parallel=True) == 16384
    sizes = np.concatenate([rng.integers(0, 5000, 2000), rng.integers(0, 130, 2000), [65535, 65536, 300000]])
    rng.shuffle(sizes)
    wire, _ = _stream(rng, sizes)
    assert run_scan(torch_cuda, wire, parallel=True) == sizes.size
    assert run_scan(torch_cuda, wire, strict=False, parallel=True) == sizes.size


@pytest.mark.parametrize("strict", [True, False])
def test_far_exits(torch_cuda, strict):
    # frames of 64-bit lengths (exits more than a tile ahead) mixed with 7- and 16-bit ones, and
    # several big frames in a row (tiles entered only from far away)
    rng = np.random.default_rng(61 + strict)
    sizes = np.concatenate([rng.integers(70000, 1 << 21, 60), rng.integers(0, 5000, 600), [65535, 65536, 65537]])
    rng.shuffle(sizes)
    sizes = np.concatenate([sizes, np.full(8, 1 << 20)])
    wire, wo = _stream(rng, sizes)
    assert run_scan(torch_cuda, wire, strict=strict, parallel=True) == sizes.size
    run_scan(torch_cuda, wire, start=int(wo[300]), strict=strict, parallel=True)
    run_scan(torch_cuda, wire[:int(wo[-3]) + 100], strict=strict, parallel=True)


@pytest.mark.parametrize("onepass", ["0", "1"])
@pytest.mark.parametrize("fuse", ["1", "0", "2", "-1"])
def test_fused_and_separate_launches(torch_cuda, gpu_knob, fuse, onepass):
    # K2 + K3a + K3b as one launch (knob SCAN_FUSE = 1: arrival counters per tile and per
    # stream, the last arrival runs the next phase and re-zeroes its counter), as three
    # (SCAN_FUSE = 0, as for streams over 512 MiB), or the default, K3a + K3b as one launch
    # (the last tile block to arrive resolves; sc1 hand-off): the same results over
    # alternating stream sizes, the serial fallback, non-strict streams and truncations, one
    # call after another on one stream (a counter left non-zero would break the next call)
    # (with the one-pass path on, the K2 launch, whichever it is, reads its flag first)
    gpu_knob("SCAN_FUSE", fuse)
    gpu_knob("SCAN_ONEPASS", onepass)
    rng = np.random.default_rng(51)
    big, _ = _stream(rng, np.full(16384, 1024))                      # 16 tiles
    mixed_sizes = np.concatenate([rng.integers(0, 5000, 2000), rng.integers(0, 130, 2000), [65535, 300000]])
    rng.shuffle(mixed_sizes)
    mixed, wo = _stream(rng, mixed_sizes)
    tiny, _ = _stream(rng, rng.integers(0, 4, 5000))
    rec = b"".join(bytes.fromhex("82fe") + (5000 + i % 997).to_bytes(2, "big") + bytes(4) for i in range(997))
    inner = np.tile(np.frombuffer(rec, dtype=np.uint8), 20)
    adv, _ = orc.encode_batch(inner, np.array([0, inner.size], dtype=np.uint64), np.array([0], dtype=np.uint32),
                              None, True)
    for _ in range(2):
        assert run_scan(torch_cuda, big, parallel=True) == 16384
        assert run_scan(torch_cuda, mixed, parallel=True) == mixed_sizes.size
        assert run_scan(torch_cuda, mixed, strict=False, parallel=True) == mixed_sizes.size
        run_scan(torch_cuda, adv)   # capacity overflow: the serial walk, same results
        assert run_scan(torch_cuda, tiny, parallel=True) == 5000
        run_scan(torch_cuda, mixed[:int(wo[1500]) + 5], parallel=True)
        run_scan(torch_cuda, mixed, start=int(wo[2222]), parallel=True)
        run_scan(torch_cuda, big[:4096 * 300 + 7], parallel=True)     # a partial last tile


@pytest.mark.parametrize("emit", ["64", "32"])
def test_emit_block_sizes(torch_cuda, gpu_knob, emit):
    """K2 (scan_links) and K4 (scan_emit) take 32 chunks per block up to 128 MiB of stream and 64
    above (knob SCAN_BLOCK_CHUNKS forces either): the C2 and C4 shapes, tiny frames, mixed sizes with 64-bit
    lengths, non-strict streams, truncations, start offsets and the serial fallback, both ways"""
    gpu_knob("SCAN_BLOCK_CHUNKS", emit)
    rng = np.random.default_rng(77)
    wire, _ = _stream(rng, np.full(65536, 1024))
    assert run_scan(torch_cuda, wire, parallel=True) == 65536
    wire, _ = _stream(rng, rng.integers(256, 65537, 2000))
    assert run_scan(torch_cuda, wire, parallel=True) == 2000
    wire, _ = _stream(rng, rng.integers(0, 4, 20000))
    assert run_scan(torch_cuda, wire, parallel=True) == 20000
    sizes = np.concatenate([rng.integers(0, 5000, 300), rng.integers(0, 130, 300), [65535, 65536, 200000]])
    rng.shuffle(sizes)
    wire, wo = _stream(rng, sizes)
    assert run_scan(torch_cuda, wire, parallel=True) == sizes.size
    for cut in (1, int(wo[50]) + 1, int(wo[300]) + 3, wire.size - 1):
        run_scan(torch_cuda, wire[:cut], parallel=True)
    for st in (int(wo[1]), int(wo[477])):
        run_scan(torch_cuda, wire, start=st, parallel=True)
    wire, _ = _stream(rng, rng.integers(0, 126, 3000), masked=False)
    assert run_scan(torch_cuda, wire, strict=False, parallel=True) == 3000
    rec = b"".join(bytes.fromhex("82fe") + (5000 + i % 997).to_bytes(2, "big") + bytes(4) for i in range(997))
    inner = np.tile(np.frombuffer(rec, dtype=np.uint8), 40)
    off = np.array([0, inner.size, inner.size + 10], dtype=np.uint64)
    payload = np.concatenate([inner, rng.integers(0, 256, 10, dtype=np.uint8)])
    wire, _ = orc.encode_batch(payload, off, np.array([0, 0x01020304], dtype=np.uint32), None, True)
    assert run_scan(torch_cuda, wire) == 2   # capacity overflow: the serial walk in K4


@pytest.mark.parametrize("onepass,fuse", [("1", "-1"), ("1", "2"), ("0", "-1")])
def test_onepass_and_graph_paths(torch_cuda, gpu_knob, onepass, fuse):
    """the one-pass path (dense streams: K1 publishes each chunk's exit prediction; the next launch
    speculates every chunk's entry from its predecessors, walks and checks it, scans the counts and
    writes the frames; K2 + K3 and K4 only read a flag) and the graph path (knob SCAN_ONEPASS = 0)
    on the same streams: identical results; dense strict streams finish on the one-pass path
    (netc_gpu_scan_diag bit 32), streams with chunk-covering frames or chunks of more than 64
    frames on the graph kernels.  K2 + K3 are one gated launch by default, separate ones with
    SCAN_FUSE = 2."""
    gpu_knob("SCAN_ONEPASS", onepass)
    gpu_knob("SCAN_FUSE", fuse)
    rng = np.random.default_rng(97)
    want = onepass == "1"
    c2, _ = _stream(rng, np.full(65536, 1024))
    assert run_scan(torch_cuda, c2, parallel=True) == 65536
    assert nm.scan_onepass() == want
    dense, _ = _stream(rng, rng.integers(0, 3500, 20000))   # frames shorter than a chunk: every chunk visited
    assert run_scan(torch_cuda, dense, parallel=True) == 20000
    assert nm.scan_onepass() == want
    c4, _ = _stream(rng, rng.integers(256, 65537, 2000))   # frames that cover chunks: the graph kernels
    assert run_scan(torch_cuda, c4, parallel=True) == 2000
    assert not nm.scan_onepass()
    sizes = np.concatenate([rng.integers(0, 5000, 2000), rng.integers(0, 130, 2000), [65535, 65536, 300000]])
    rng.shuffle(sizes)
    mixed, wo = _stream(rng, sizes)
    assert run_scan(torch_cuda, mixed, parallel=True) == sizes.size
    # start offsets, truncations, a frame cap, an error mid-stream, non-strict, tiny frames,
    # unmasked non-strict, the adversarial overflow: parity whichever path finishes
    for s in (int(wo[1]), int(wo[3999]), mixed.size):
        run_scan(torch_cuda, mixed, start=s, parallel=True)
    for cut in (0, 1, 7, int(wo[2000]) + 3, int(wo[2000]), mixed.size - 1):
        run_scan(torch_cuda, mixed[:cut], parallel=True)
    run_scan(torch_cuda, mixed, max_frames=1234, parallel=True)
    bad = np.concatenate([mixed[:int(wo[1000])], np.frombuffer(bytes.fromhex("c185") + bytes(9), dtype=np.uint8),
                          mixed[int(wo[1000]):]])
    run_scan(torch_cuda, bad, strict=True)
    run_scan(torch_cuda, mixed, strict=False, parallel=True)
    tiny, _ = _stream(rng, rng.integers(0, 4, 20000))
    assert run_scan(torch_cuda, tiny, parallel=True) == 20000
    unm, _ = _stream(rng, rng.integers(0, 3000, 300), masked=False)
    assert run_scan(torch_cuda, unm, strict=False, parallel=True) == 300
    rec = b"".join(bytes.fromhex("82fe") + (5000 + i % 997).to_bytes(2, "big") + bytes(4) for i in range(997))
    inner = np.tile(np.frombuffer(rec, dtype=np.uint8), 20)
    adv, _ = orc.encode_batch(inner, np.array([0, inner.size], dtype=np.uint64), np.array([0], dtype=np.uint32),
                              None, True)
    run_scan(torch_cuda, adv)
    for _ in range(3):   # epochs: one call after another on the same scratch
        assert run_scan(torch_cuda, c2[:4096 * 300 + 11], parallel=True) > 0
        assert run_scan(torch_cuda, c4, parallel=True) == 2000
