"""GPU parity: the socket-ingest ring (include/ws/ingest.h) vs the oracle.

The checker is the oracle's stream walk (oracle_scan_frames: the header decode of
src/ws/common.c:146-296, pinned by the reference's golden wire and its compiled
receiver in tests/test_scan_oracle.py) plus the reference's unmask expression
(oracle_mask_batch, src/ws/common.c:321) on every payload.  The bar: the batches,
concatenated in order, hold exactly the oracle's frames -- header offsets (stream
coordinates), keys, header bytes, unmasked payload bytes, untouched header bytes --
and nothing else, whatever the slot size and however the bytes arrive.
"""

import socket
import threading

import numpy as np
import pytest

from netc_amd import ingest as ni
from netc_amd.mask import NetcGpuError
from oracle import oracle as orc

pytestmark = pytest.mark.gpu


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
    with ni.Ingest(0, slot_bytes=1 << 20, nslots=2) as ing:
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
