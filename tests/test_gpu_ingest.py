"""GPU parity: the socket-ingest ring (include/ws/ingest.h) vs the oracle.

The checker is the oracle's stream walk (oracle_scan_frames: the header decode of
src/ws/common.c:146-296, pinned by the reference's golden wire and its compiled
receiver in tests/test_scan_oracle.py) plus the reference's unmask expression
(oracle_mask_batch, src/ws/common.c:321) on every payload.  The bar: the batches,
concatenated in order, hold exactly the oracle's frames -- header offsets (stream
coordinates), keys, header bytes, unmasked payload bytes, untouched header bytes --
and nothing else, whatever the slot size and however the bytes arrive.

The message-level reader (netc_ws_ingest_next_message) is checked against
libnetc's own ws_parse_frame on the same bytes (tests/wsutil.parse_stream) and against the
reference's golden fixtures (tests/golden/ws_golden.json, generated from the compiled
reference: fragmented, text_nul, rfc6455_kat).
"""

import json
import os
import socket
import threading

import numpy as np
import pytest

from netc_amd import ingest as ni
from netc_amd.mask import NetcGpuError
from oracle import oracle as orc
from tests.wsutil import parse_stream

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True, params=["auto", "gpu", "host"])
def scan_mode(request, monkeypatch):
    """Every ingest case runs with each way of finding a slot's frames (NETC_WS_INGEST_SCAN_*):
    the per-slot choice (default), always the GPU scan, always the host header walk."""
    init = ni.Ingest.__init__

    def with_mode(self, *args, **kwargs):
        kwargs.setdefault("scan", request.param)
        init(self, *args, **kwargs)

    monkeypatch.setattr(ni.Ingest, "__init__", with_mode)
    return request.param


def frames_from_sizes(sizes):
    off = np.zeros(len(sizes) + 1, dtype=np.uint64)
    off[1:] = np.cumsum(np.asarray(sizes, dtype=np.uint64))
    return off


def make_stream(rng, sizes, b0=None, masked=True):
    off = frames_from_sizes(sizes)
    plain = rng.integers(0, 256, int(off[-1]), dtype=np.uint8)
    keys = rng.integers(0, 2**32, len(sizes), dtype=np.uint64).astype(np.uint32)
    wire, wo = orc.encode_batch(plain, off, keys, b0, masked)
    return wire, wo, plain, off, keys


def expected(wire, strict=True):
    """(header offsets, keys, byte 0s, consumed, error, the stream with every complete frame unmasked)."""
    hdr, keys, b0, consumed, err = orc.scan_frames(wire, strict=strict)
    out = wire.copy()
    for k in range(hdr.size):
        end = int(hdr[k + 1]) if k + 1 < hdr.size else consumed
        second = int(wire[hdr[k] + 1])
        code = second & 0x7F
        hl = 2 + (2 if code == 126 else 8 if code == 127 else 0) + (4 if second & 0x80 else 0)
        ps = int(hdr[k]) + hl
        if second & 0x80:
            out[ps:end] = orc.mask_batch(wire[ps:end], np.array([0, end - ps], dtype=np.uint64), keys[k:k + 1])
    return hdr, keys, b0, consumed, err, out


class Collector:
    def __init__(self):
        self.batches = []

    def take(self, ing, wait=True):
        got = 0
        while True:
            b = ing.next(wait=wait)
            if b is None:
                return got
            self.batches.append((b.stream_offset, b.wire.copy(), b.hdr.copy(), b.keys.copy(), b.b0.copy(),
                                 [b.payload(k) for k in range(min(b.nframes, 3))]))
            b.release()
            got += 1

    def check(self, wire, strict=True):
        hdr, keys, b0, consumed, err, out = expected(wire, strict)
        pos, frames = 0, 0
        for off, w, h, k, b, pays in self.batches:
            assert off == pos, f"batch at stream offset {off}, expected {pos}"
            n = k.size
            assert h.size == n + 1 and int(h[-1]) == w.size
            assert np.array_equal(h[:n] + np.uint64(off), hdr[frames:frames + n]), "header offsets differ"
            assert np.array_equal(k, keys[frames:frames + n]), "keys differ"
            assert np.array_equal(b, b0[frames:frames + n]), "header bytes differ"
            assert np.array_equal(w, out[off:off + w.size]), "stream bytes differ"
            for j, (po, pl) in enumerate(pays):   # netc_ws_batch_payload agrees with the frame layout
                assert po + pl == int(h[j + 1]) and po > int(h[j])
            pos += w.size
            frames += n
        assert frames == hdr.size, f"{frames} frames delivered, oracle {hdr.size}"
        assert pos == consumed
        return frames


def feed(ing, col, wire, chunks, flush=True):
    """write() the stream in the given chunk sizes, draining batches whenever the ring is full."""
    i = 0
    for c in chunks:
        piece = wire[i:i + c]
        i += c
        while piece.size:
            r = ing.write(piece)
            if r == ni.NETC_WS_INGEST_FULL:
                assert col.take(ing, wait=True) > 0, "ring full but nothing in flight"
                continue
            piece = piece[r:]
    assert i >= wire.size
    if flush:
        ing.submit()
        col.take(ing, wait=True)


def random_chunks(rng, total, hi):
    out, s = [], 0
    while s < total:
        c = int(rng.integers(1, hi))
        out.append(c)
        s += c
    return out


@pytest.mark.parametrize("slot,nslots", [(4096, 2), (8192, 3), (65536, 4), (1 << 20, 4)])
def test_mixed_frames_any_slot_size(torch_cuda, slot, nslots):
    rng = np.random.default_rng(slot + nslots)
    sizes = np.concatenate([rng.integers(0, 3000, 400), rng.integers(0, 130, 300), [0, 125, 126, 65535, 65536]])
    rng.shuffle(sizes)
    wire, *_ = make_stream(rng, sizes)
    with ni.Ingest(0, slot_bytes=slot, nslots=nslots, max_frame_bytes=65536) as ing:
        col = Collector()
        feed(ing, col, wire, random_chunks(rng, wire.size, 20000))
        assert col.check(wire) == sizes.size


def test_scan_choice_follows_frame_size(torch_cuda, scan_mode):
    # 1 KiB frames, then ~60 KiB frames, then 1 KiB frames again, through 1 MiB slots, strict: by
    # default the ring frames the small-frame slots on the GPU and the large-frame slots on the host
    rng = np.random.default_rng(77)
    sizes = np.concatenate([np.full(3000, 1024), rng.integers(50000, 65536, 100), np.full(3000, 1024)])
    wire, *_ = make_stream(rng, sizes)
    with ni.Ingest(0, slot_bytes=1 << 20, nslots=3, strict=True) as ing:
        col = Collector()
        feed(ing, col, wire, [1 << 20] * (wire.size // (1 << 20) + 1))
        assert col.check(wire) == sizes.size
        gpu, host = ing.scan_counts()
        assert gpu + host == len(col.batches)
        if scan_mode == "gpu":
            assert host == 0
        elif scan_mode == "host":
            assert gpu == 0
        else:
            assert gpu >= 4 and host >= 4, (gpu, host)


def test_non_strict_scan_choice(torch_cuda, scan_mode):
    # non-strict: 1 KiB frames stay on the GPU by default until a slot holds RSV2 frames (the
    # GPU scan's parallel pass stops at them), after which the host walk takes the slots.  RSV1
    # frames (permessage-deflate) stay on the GPU (test_non_strict_rsv1_stays_on_gpu).
    rng = np.random.default_rng(78)
    b0 = np.full(6000, 0x82, dtype=np.uint8)
    b0[3000:] = 0xA2
    wire, *_ = make_stream(rng, np.full(6000, 1024), b0=b0)
    with ni.Ingest(0, slot_bytes=1 << 20, nslots=3, strict=False) as ing:
        col = Collector()
        feed(ing, col, wire, [1 << 20] * (wire.size // (1 << 20) + 1))
        assert col.check(wire, strict=False) == 6000
        gpu, host = ing.scan_counts()
        nb = len(col.batches)
        if scan_mode == "auto":
            assert gpu >= 3 and host >= 2, (gpu, host)
        else:
            assert (gpu, host) == ((nb, 0) if scan_mode == "gpu" else (0, nb))


def test_non_strict_choice_several_slots_one_write(torch_cuda, scan_mode):
    # one write() that fills several slots submits each slot right after the
    # previous one, while the previous slot's descriptor copy back is still queued.  The choice
    # must come from the scan's own diag word (copied with its result), not from those
    # descriptors: slot 0 (no history) is GPU-scanned and meets RSV2 headers, so with the
    # per-slot choice every later slot takes the host walk -- exactly, whatever the timing.
    rng = np.random.default_rng(79)
    n = 800
    wire, *_ = make_stream(rng, np.full(n, 1024), b0=np.full(n, 0xA2, dtype=np.uint8))
    with ni.Ingest(0, slot_bytes=256 << 10, nslots=4, strict=False) as ing:
        assert ing.write(wire) == wire.size   # ~806 KiB: four slots, all in one call
        ing.submit()
        col = Collector()
        col.take(ing, wait=True)
        assert col.check(wire, strict=False) == n
        gpu, host = ing.scan_counts()
        nb = len(col.batches)
        assert nb == 4
        if scan_mode == "auto":
            assert (gpu, host) == (1, nb - 1)
        else:
            assert (gpu, host) == ((nb, 0) if scan_mode == "gpu" else (0, nb))


def test_non_strict_rsv1_stays_on_gpu(torch_cuda, scan_mode):
    # permessage-deflate streams (RSV1 on every frame) are scanned by the GPU's parallel pass
    # in non-strict mode: in "auto" every slot stays on the GPU scan
    rng = np.random.default_rng(81)
    n = 3000
    wire, *_ = make_stream(rng, np.full(n, 1024), b0=np.full(n, 0xC2, dtype=np.uint8))
    with ni.Ingest(0, slot_bytes=1 << 20, nslots=3, strict=False) as ing:
        col = Collector()
        feed(ing, col, wire, [1 << 20] * (wire.size // (1 << 20) + 1))
        assert col.check(wire, strict=False) == n
        gpu, host = ing.scan_counts()
        nb = len(col.batches)
        assert (gpu, host) == ((0, nb) if scan_mode == "host" else (nb, 0))


def test_python_default_is_non_strict(torch_cuda):
    # the Python mirror follows the C default (flags 0: every header accepted, as the
    # reference's ws_parse_frame): an unmasked client frame is delivered, not rejected
    rng = np.random.default_rng(80)
    wire, *_ = make_stream(rng, np.full(10, 100), masked=False)
    with ni.Ingest(0, slot_bytes=4096, nslots=2) as ing:
        col = Collector()
        feed(ing, col, wire, [wire.size])
        assert col.check(wire, strict=False) == 10


def test_c5_shape_4k_frames(torch_cuda):
    # BASELINE config 5's frame shape: 4 KiB masked BINARY frames, 16 MiB through 1 MiB slots
    rng = np.random.default_rng(5)
    wire, *_ = make_stream(rng, np.full(4096, 4096))
    with ni.Ingest(0, slot_bytes=1 << 20, nslots=4) as ing:
        col = Collector()
        feed(ing, col, wire, [1 << 22] * 4 + [wire.size])
        assert col.check(wire) == 4096
        assert len(col.batches) >= 16


def test_byte_by_byte_and_tiny_frames(torch_cuda):
    rng = np.random.default_rng(6)
    wire, *_ = make_stream(rng, rng.integers(0, 6, 700))
    with ni.Ingest(0, slot_bytes=4096, nslots=2) as ing:
        col = Collector()
        feed(ing, col, wire, [1] * wire.size)
        assert col.check(wire) == 700


def test_truncated_stream_delivers_complete_frames(torch_cuda):
    rng = np.random.default_rng(7)
    wire, wo, *_ = make_stream(rng, rng.integers(0, 9000, 120))
    cut = wire[: int(wo[80]) + 5]
    with ni.Ingest(0, slot_bytes=16384, nslots=3) as ing:
        col = Collector()
        feed(ing, col, cut, [cut.size])
        assert col.check(cut) == 80


def test_header_byte_variants(torch_cuda):
    rng = np.random.default_rng(8)
    sizes = rng.integers(0, 125, 600)
    b0 = rng.choice(np.array([0x81, 0x82, 0x01, 0x00, 0x80, 0x89, 0x8A, 0x88], dtype=np.uint8), 600)
    wire, *_ = make_stream(rng, sizes, b0=b0)
    with ni.Ingest(0, slot_bytes=4096, nslots=4) as ing:
        col = Collector()
        feed(ing, col, wire, random_chunks(rng, wire.size, 3000))
        assert col.check(wire) == 600


def test_non_strict_unmasked_frames(torch_cuda):
    # a server -> client stream (no MASK): non-strict mode passes the payloads through
    rng = np.random.default_rng(9)
    wire, *_ = make_stream(rng, rng.integers(0, 4000, 300), masked=False)
    with ni.Ingest(0, slot_bytes=8192, nslots=2, strict=False) as ing:
        col = Collector()
        feed(ing, col, wire, random_chunks(rng, wire.size, 5000))
        assert col.check(wire, strict=False) == 300


def test_frame_over_the_limit(torch_cuda):
    rng = np.random.default_rng(10)
    wire, wo, *_ = make_stream(rng, [100, 200, 5000, 300])
    with ni.Ingest(0, slot_bytes=4096, nslots=3, max_frame_bytes=1000) as ing:
        col = Collector()
        with pytest.raises(NetcGpuError) as e:
            feed(ing, col, wire, [wire.size])
        assert e.value.code == ni.NETC_WS_INGEST_TOO_BIG
        # the two frames before the long one are delivered, then the error stands
        b = ing.next(wait=True)
        assert b.nframes == 2 and b.stream_offset == 0
        b.release()
        with pytest.raises(NetcGpuError) as e:
            ing.next(wait=True)
        assert e.value.code == ni.NETC_WS_INGEST_TOO_BIG


def test_strict_error_mid_stream(torch_cuda):
    rng = np.random.default_rng(11)
    good, *_ = make_stream(rng, rng.integers(0, 2000, 40))
    bad = np.frombuffer(bytes.fromhex("8105") + b"Hello", dtype=np.uint8)   # MASK clear: forbidden from a client
    wire = np.concatenate([good, bad, good])
    with ni.Ingest(0, slot_bytes=1 << 20, nslots=2, strict=True) as ing:
        col = Collector()
        ing.write(wire)
        ing.submit()
        b = ing.next(wait=True)
        assert b.nframes == 40 and b.stream_offset == 0
        b.release()
        with pytest.raises(NetcGpuError) as e:
            ing.next(wait=True)
        assert e.value.code == ni.NETC_WS_INGEST_PROTOCOL
        with pytest.raises(NetcGpuError):
            ing.write(good)


def test_full_ring_backpressure(torch_cuda):
    rng = np.random.default_rng(12)
    wire, *_ = make_stream(rng, np.full(64, 1000))
    with ni.Ingest(0, slot_bytes=4096, nslots=2) as ing:
        taken = ing.write(wire)
        # two slots submitted (filled), nothing released: the third slot cannot start
        assert taken == 2 * 4096
        assert ing.write(wire[taken:]) == ni.NETC_WS_INGEST_FULL
        b = ing.next(wait=True)
        assert b.stream_offset == 0
        b.release()
        assert ing.write(wire[taken:taken + 100]) == 100


def test_socketpair_with_writer_thread(torch_cuda):
    # the intended use: recv() straight into the slots while a peer writes the stream
    rng = np.random.default_rng(13)
    sizes = np.concatenate([rng.integers(0, 20000, 600), np.full(300, 4096)])
    rng.shuffle(sizes)
    wire, *_ = make_stream(rng, sizes)
    a, b = socket.socketpair()

    def writer():
        v = memoryview(wire.tobytes())
        i = 0
        for c in random_chunks(np.random.default_rng(1), len(v), 70000):
            a.sendall(v[i:i + c])
            i += c
        a.close()

    t = threading.Thread(target=writer)
    t.start()
    try:
        with ni.Ingest(0, slot_bytes=1 << 18, nslots=3) as ing:
            col = Collector()
            while True:
                r = ing.recv(b.fileno())
                if r == ni.NETC_WS_INGEST_FULL:
                    col.take(ing, wait=True)
                elif r == ni.NETC_WS_INGEST_CLOSED:
                    break
            col.take(ing, wait=True)
            assert col.check(wire) == sizes.size
    finally:
        t.join()
        b.close()


# ------------------------------------------------------- message contract ---

GOLDEN = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "ws_golden.json")))
TEXT, BINARY, CONT = 1, 2, 0


def gen(seed, n):
    return np.random.Generator(np.random.PCG64(seed)).integers(0, 256, n, dtype=np.uint8).tobytes()


def gpu_messages(wire: bytes, chunks=(), max_payload=(1 << 62), slot=4096, nslots=3, max_frame=65536):
    """Feed `wire` to an ingest ring in `chunks`, reading netc_ws_ingest_next_message after each
    piece (as an event loop would); returns (messages, last code) like wsutil.parse_stream."""
    w = np.frombuffer(wire, dtype=np.uint8)
    msgs, rc = [], 1
    with ni.Ingest(0, slot_bytes=slot, nslots=nslots, max_frame_bytes=max_frame) as ing:
        def drain(wait):
            nonlocal rc
            while True:
                rc, op, data = ing.next_message(max_payload, wait=wait)
                if rc != 0:
                    return rc
                msgs.append((op, data))
        sizes = [int(n) for n in chunks]
        if sum(sizes) < len(wire):
            sizes.append(len(wire) - sum(sizes))
        pos = 0
        for n in sizes:
            piece = w[pos:pos + n]
            pos += piece.size
            while piece.size:
                r = ing.write(piece)
                if r == ni.NETC_WS_INGEST_FULL:
                    if drain(True) < 0:
                        return msgs, rc
                    continue
                piece = piece[r:]
            if drain(False) < 0:
                return msgs, rc
        drain(True)   # submits what is left, waits for the GPU
        return msgs, rc


def test_message_fragmented_golden(torch_cuda):
    f = GOLDEN["fragmented"]
    wire = bytes.fromhex(f["wire"])
    for slot in (4096, 1 << 16):
        msgs, rc = gpu_messages(wire, f["chunks"], slot=slot)
        assert rc == 1 and msgs == [(f["opcode"], bytes.fromhex(f["message"]))]
    assert msgs == parse_stream(wire, f["chunks"])[0]


def test_message_text_nul_golden(torch_cuda):
    t = GOLDEN["text_nul"]
    msgs, rc = gpu_messages(bytes.fromhex(t["wire"]))
    assert msgs == [(TEXT, bytes.fromhex(t["delivered"]))] and len(msgs[0][1]) == t["payload_length"]


def test_message_rfc6455_kat_golden(torch_cuda):
    msgs, rc = gpu_messages(bytes.fromhex(GOLDEN["rfc6455_kat"]["wire"]))
    assert [[op, m.hex()] for op, m in msgs] == GOLDEN["rfc6455_kat"]["messages"]


def many_messages_stream():
    # the stream of tests/test_host_framing.py::test_many_messages_in_one_stream
    g = np.random.Generator(np.random.PCG64(9))
    wire, expect = b"", []
    for i in range(50):
        nfr = int(g.integers(1, 4))
        parts = [gen(100 * i + j, int(g.integers(0, 3000))) for j in range(nfr)]
        op = TEXT if i % 2 else BINARY
        for j, part in enumerate(parts):
            key = gen(7 * i + j, 4) if (i + j) % 3 else None
            if key is not None and not part:
                key = None
            wire += orc.encode_frame(part, op if j == 0 else CONT, key, fin=(j == nfr - 1))
        expect.append((op, b"".join(parts) + (b"\x00" if op == TEXT else b"")))
    cuts = np.sort(g.choice(np.arange(1, len(wire)), 200, replace=False))
    chunks = np.diff(np.concatenate([[0], cuts, [len(wire)]])).tolist()
    return wire, expect, chunks


@pytest.mark.parametrize("slot,nslots", [(4096, 2), (16384, 3), (1 << 20, 4)])
def test_message_many_in_one_stream(torch_cuda, slot, nslots):
    wire, expect, chunks = many_messages_stream()
    msgs, rc = gpu_messages(wire, chunks, slot=slot, nslots=nslots)
    assert msgs == expect
    assert msgs == parse_stream(wire, chunks)[0]   # the same sequence libnetc's ws_parse_frame gives


def test_message_control_frames_between_messages(torch_cuda):
    wire = (orc.encode_frame(b"ab", TEXT, b"1234", fin=False) + orc.encode_frame(b"cd", CONT, b"5678") +
            orc.encode_frame(b"hi", 0x9, b"abcd") + orc.encode_frame(b"", 0xA, None) +
            orc.encode_frame(gen(3, 900), BINARY, b"\x00\x00\x00\x00"))
    msgs, rc = gpu_messages(wire, [5, 9, 1, 30])
    assert msgs == parse_stream(wire, [5, 9, 1, 30])[0]
    assert [op for op, _ in msgs] == [TEXT, 0x9, 0xA, BINARY] and msgs[0][1] == b"abcd\x00"


def test_message_payload_too_big_accumulated(torch_cuda):
    # three 400-byte fragments: the third takes the message past 1000 bytes (src/ws/common.c:210,261)
    wire = orc.encode_frame(b"x" * 10, BINARY, b"kkkk")
    wire += b"".join(orc.encode_frame(gen(j, 400), BINARY if j == 0 else CONT, b"abcd", fin=(j == 2))
                     for j in range(3))
    msgs, rc = gpu_messages(wire, max_payload=1000)
    ref_msgs, ref_rc = parse_stream(wire, max_payload=1000)
    assert rc == ref_rc == -3 and msgs == ref_msgs == [(BINARY, b"x" * 10)]


def test_frame_over_the_limit_inside_one_slot(torch_cuda):
    # a frame longer than max_frame_bytes that fits in one slot is refused too
    rng = np.random.default_rng(14)
    wire, wo, *_ = make_stream(rng, [100, 5000, 300])
    with ni.Ingest(0, slot_bytes=1 << 20, nslots=2, max_frame_bytes=1000) as ing:
        ing.write(wire)
        ing.submit()
        b = ing.next(wait=True)
        assert b.nframes == 1 and int(b.hdr[1]) == int(wo[1])
        b.release()
        with pytest.raises(NetcGpuError) as e:
            ing.next(wait=True)
        assert e.value.code == ni.NETC_WS_INGEST_TOO_BIG
    msgs, rc = gpu_messages(wire.tobytes(), slot=1 << 20, max_frame=1000)
    assert rc == -3 and len(msgs) == 1


def test_message_socket_until_close(torch_cuda):
    wire, expect, chunks = many_messages_stream()
    a, b = socket.socketpair()

    def writer():
        v = memoryview(wire)
        i = 0
        for c in chunks:
            a.sendall(v[i:i + c])
            i += c
        a.close()

    t = threading.Thread(target=writer)
    t.start()
    msgs = []
    try:
        with ni.Ingest(0, slot_bytes=8192, nslots=3) as ing:
            while True:
                r = ing.recv(b.fileno())
                while True:
                    rc, op, data = ing.next_message(wait=r == ni.NETC_WS_INGEST_FULL)
                    if rc != 0:
                        break
                    msgs.append((op, data))
                if r == ni.NETC_WS_INGEST_CLOSED:
                    break
            while True:
                rc, op, data = ing.next_message(wait=True)
                if rc != 0:
                    break
                msgs.append((op, data))
            assert rc == -1   # the peer closed after the last complete message (recv() == 0)
    finally:
        t.join()
        b.close()
    assert msgs == expect


def test_create_destroy_does_not_leak_device_memory(torch_cuda):
    # the scan scratch is owned by each slot and freed with it (it was cached per
    # stream and leaked when an ingest destroyed its streams)
    torch = torch_cuda
    rng = np.random.default_rng(15)
    wire, *_ = make_stream(rng, rng.integers(0, 3000, 200))

    def one():
        with ni.Ingest(0, slot_bytes=1 << 20, nslots=4) as ing:
            ing.write(wire)
            ing.submit()
            while ing.next(wait=True) is not None:
                pass
    one()
    torch.cuda.synchronize()
    free0 = torch.cuda.mem_get_info()[0]
    for _ in range(12):
        one()
    torch.cuda.synchronize()
    free1 = torch.cuda.mem_get_info()[0]
    assert free0 - free1 < (16 << 20), f"{(free0 - free1) >> 20} MiB lost over 12 create/destroy cycles"
