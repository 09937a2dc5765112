"""The frame-scan checker (oracle_scan_frames) is pinned before it is trusted (CPU).

* the golden fragmented wire the reference itself produced (tests/golden) scans
  into the frames whose payloads the reference delivered as one message;
* where oracle/_ref is built, random multi-message streams scan into exactly the
  messages the reference's compiled ws_parse_frame delivers;
* encode → scan round trips (frame offsets, keys, first bytes), truncation at every
  header / payload byte, and the strict-mode protocol errors.
"""

import json
import os

import numpy as np
import pytest

from oracle import oracle as orc

GOLDEN = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "ws_golden.json")))


def _frames(rng, n, max_len=3000):
    sizes = rng.integers(0, max_len, n)
    sizes[rng.random(n) < 0.1] = rng.choice([125, 126, 65535, 65536, 70000], int((rng.random(n) < 0.1).sum()) or 1)[0]
    off = np.zeros(n + 1, dtype=np.uint64)
    off[1:] = np.cumsum(sizes)
    return off


def payloads_of(wire: np.ndarray, hdr, keys, b0):
    """Unmasked payload of each scanned frame (byte 1 / extended length decoded here independently)."""
    out = []
    for k in range(len(hdr)):
        p = int(hdr[k])
        code = int(wire[p + 1]) & 0x7F
        masked = int(wire[p + 1]) >> 7
        ext = 2 if code == 126 else (8 if code == 127 else 0)
        plen = code if not ext else int.from_bytes(wire[p + 2: p + 2 + ext].tobytes(), "big")
        s = p + 2 + ext + (4 if masked else 0)
        key = int(keys[k]).to_bytes(4, "little")
        out.append(orc.unmask(wire[s: s + plen].tobytes(), key).tobytes() if masked else wire[s: s + plen].tobytes())
    return out


def test_golden_fragmented_wire():
    f = GOLDEN["fragmented"]
    wire = np.frombuffer(bytes.fromhex(f["wire"]), dtype=np.uint8)
    hdr, keys, b0, consumed, err = orc.scan_frames(wire, strict=False)
    assert consumed == wire.size and err is None
    assert (b0[-1] & 0x80) and not any(b & 0x80 for b in b0[:-1])   # FIN only on the last fragment
    assert b"".join(payloads_of(wire, hdr, keys, b0)).hex() == f["message"]


@pytest.mark.parametrize("masked", [True, False])
def test_encode_scan_round_trip(masked):
    rng = np.random.default_rng(3 + masked)
    off = _frames(rng, 400)
    payload = rng.integers(0, 256, int(off[-1]), dtype=np.uint8)
    keys = rng.integers(0, 2**32, 400, dtype=np.uint64).astype(np.uint32)
    b0 = rng.choice(np.array([0x82, 0x81, 0x01, 0x00, 0x80], dtype=np.uint8), 400)
    wire, wo = orc.encode_batch(payload, off, keys, b0, masked)
    hdr, k2, b2, consumed, err = orc.scan_frames(wire, strict=False)
    assert consumed == wire.size and err is None
    assert np.array_equal(hdr, wo[:-1]) and np.array_equal(b2, b0)
    assert np.array_equal(k2, keys if masked else np.zeros_like(keys))
    got = payloads_of(wire, hdr, k2, b2)
    assert all(got[i] == payload[int(off[i]): int(off[i + 1])].tobytes() for i in range(400))
    if masked:
        assert orc.scan_frames(wire, strict=True)[3] == wire.size


def test_truncation_at_every_byte():
    rng = np.random.default_rng(8)
    off = np.array([0, 5, 5, 130, 300, 70000 + 300, 70000 + 310], dtype=np.uint64)
    payload = rng.integers(0, 256, int(off[-1]), dtype=np.uint8)
    keys = rng.integers(0, 2**32, off.size - 1, dtype=np.uint64).astype(np.uint32)
    wire, wo = orc.encode_batch(payload, off, keys, None, True)
    cuts = sorted(set(list(range(0, 40)) + [int(w) + d for w in wo for d in (-1, 0, 1, 2, 3)]))
    for cut in cuts:
        if cut < 0 or cut > wire.size:
            continue
        hdr, _, _, consumed, err = orc.scan_frames(wire[:cut])
        complete = [k for k in range(off.size - 1) if wo[k + 1] <= cut]
        assert list(hdr) == [int(wo[k]) for k in complete] and err is None
        assert consumed == int(wo[len(complete)])


def test_strict_mode_errors():
    ok = bytes.fromhex("8185") + bytes(4) + b"Hello"   # masked final TEXT
    cases = {
        "unmasked": bytes.fromhex("8105") + b"Hello",
        "rsv1": bytes.fromhex("c185") + bytes(4) + b"Hello",
        "reserved opcode 3": bytes.fromhex("8385") + bytes(4) + b"Hello",
        "reserved opcode 0xb": bytes.fromhex("8b85") + bytes(4) + b"Hello",
        "fragmented ping": bytes.fromhex("0980") + bytes(4),
        "long close": bytes.fromhex("88fe007e") + bytes(4) + bytes(126),
        "64-bit length top bit": bytes.fromhex("82ff8000000000000000") + bytes(4),
    }
    for name, bad in cases.items():
        stream = np.frombuffer(ok + ok + bad + ok, dtype=np.uint8)
        hdr, _, _, consumed, err = orc.scan_frames(stream, strict=True)
        assert err == 2 * len(ok) and consumed == err and len(hdr) == 2, name
        # the reference accepts every one of them
        hdr, _, _, consumed, err = orc.scan_frames(stream, strict=False)
        assert err is None, name


@pytest.mark.skipif(not orc.ref_available(), reason="oracle/_ref (the compiled reference) not built")
@pytest.mark.parametrize("seed", range(4))
def test_scan_matches_reference_receiver(seed):
    # random client streams of several fragmented messages: grouping the scanned
    # frames by FIN gives exactly the messages the reference's ws_parse_frame delivers
    rng = np.random.default_rng(40 + seed)
    frames, msgs = [], []
    for m in range(6):
        op = int(rng.choice([1, 2]))
        parts = int(rng.integers(1, 4))
        body = b""
        for i in range(parts):
            piece = (rng.integers(1, 256, int(rng.integers(0, 700)), dtype=np.uint8)).tobytes()
            key = rng.integers(0, 256, 4, dtype=np.uint8).tobytes()
            if not piece:
                piece = b"x"
            first = (0x80 if i == parts - 1 else 0) | (op if i == 0 else 0)
            frames.append(orc.encode_frame(piece, first & 0x7F, key, fin=bool(first & 0x80)))
            body += piece
        msgs.append((op, body + (b"\x00" if op == 1 else b"")))
    wire = b"".join(frames)
    hdr, keys, b0, consumed, err = orc.scan_frames(np.frombuffer(wire, dtype=np.uint8))
    assert consumed == len(wire) and err is None and len(hdr) == len(frames)
    got, cur, op = [], b"", None
    for p, b in zip(payloads_of(np.frombuffer(wire, dtype=np.uint8), hdr, keys, b0), b0):
        op = b & 0x0F if b & 0x0F else op
        cur += p
        if b & 0x80:
            got.append((op, cur + (b"\x00" if op == 1 else b"")))
            cur = b""
    assert got == msgs
    assert orc.ref_parse(wire) == msgs
