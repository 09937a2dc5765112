"""netc_ws_scan_frames_host (libnetc.so, include/ws/frame.h) against the pinned scan oracle (CPU).

The host header walk is the ingest ring's scan for slots of large frames:
the same outputs as netc_gpu_scan_frames, so it is checked on the same streams the GPU scan
suite uses (tests/test_gpu_scan.py) -- mixed sizes, truncation at header and payload bytes,
start offsets, strict / non-strict, every strict-mode protocol error, the max_frames cap --
against oracle_scan_frames, itself pinned by the reference (tests/test_scan_oracle.py).
"""

import numpy as np
import pytest

from netc_amd import mask as nm
from oracle import oracle as orc

U64MAX = (1 << 64) - 1


def _stream(rng, sizes, masked=True, b0=None):
    off = np.zeros(len(sizes) + 1, dtype=np.uint64)
    off[1:] = np.cumsum(np.asarray(sizes, dtype=np.uint64))
    payload = rng.integers(0, 256, int(off[-1]), dtype=np.uint8)
    keys = rng.integers(0, 2**32, len(sizes), dtype=np.uint64).astype(np.uint32)
    return orc.encode_batch(payload, off, keys, b0, masked)


def check(wire, start=0, strict=True, max_frames=None):
    exp_hdr, exp_keys, exp_b0, exp_consumed, exp_err = orc.scan_frames(wire, start=start, strict=strict)
    n = exp_hdr.size
    cap = n if max_frames is None else max_frames
    hdr, keys, b0, res = nm.scan_frames_host(wire, cap, start=start, strict=strict)
    assert int(res[0]) == n
    assert int(res[1]) == exp_consumed
    assert (None if int(res[2]) == U64MAX else int(res[2])) == exp_err
    k = min(n, cap)
    assert np.array_equal(hdr[:k], exp_hdr[:k])
    assert np.array_equal(keys[:k], exp_keys[:k])
    assert np.array_equal(b0[:k], exp_b0[:k])
    if n <= cap:
        assert int(hdr[n]) == exp_consumed
    return n


@pytest.mark.parametrize("seed", range(3))
def test_mixed_sizes(seed):
    rng = np.random.default_rng(seed)
    sizes = np.concatenate([rng.integers(0, 5000, 300), rng.integers(0, 130, 300), [65535, 65536, 200000]])
    rng.shuffle(sizes)
    wire, _ = _stream(rng, sizes)
    assert check(wire) == sizes.size
    assert check(wire, strict=False) == sizes.size


def test_truncated_at_header_and_payload_bytes():
    rng = np.random.default_rng(6)
    wire, wo = _stream(rng, [3, 200, 70000, 5])
    edges = [int(x) for x in wo]
    cuts = set(range(0, edges[2] + 12))                        # every byte of the first two frames + a header
    for e in edges[2:]:
        cuts |= set(range(max(0, e - 3), min(wire.size, e + 14) + 1))   # around every later header
    cuts |= set(int(c) for c in rng.integers(0, wire.size, 64))        # and inside the 70,000-byte payload
    for cut in sorted(cuts):
        check(wire[:cut])


def test_start_offset():
    rng = np.random.default_rng(7)
    wire, wo = _stream(rng, rng.integers(0, 9000, 200))
    for s in (int(wo[1]), int(wo[77]), int(wo[199]), wire.size, wire.size + 5):
        check(wire, start=s)


def test_unmasked_and_strict_errors():
    rng = np.random.default_rng(9)
    wire, _ = _stream(rng, rng.integers(0, 3000, 50), masked=False)
    assert check(wire, strict=False) == 50
    assert check(wire, strict=True) == 0
    good, _ = _stream(rng, rng.integers(0, 6000, 20))
    for bad in (bytes.fromhex("8105") + b"Hello", bytes.fromhex("c185") + bytes(9), bytes.fromhex("0980") + bytes(4),
                bytes.fromhex("83850000000048656c6c6f"), bytes.fromhex("89fe007e") + bytes(130),
                bytes.fromhex("82ff8000000000000000") + bytes(8)):
        w = np.concatenate([good, np.frombuffer(bad, dtype=np.uint8), good])
        check(w, strict=True)
        check(w, strict=False)


def test_header_byte_variants_and_cap():
    rng = np.random.default_rng(10)
    sizes = rng.integers(0, 125, 500)
    b0 = rng.choice(np.array([0x81, 0x82, 0x01, 0x00, 0x80, 0x89, 0x8A, 0x88], dtype=np.uint8), 500)
    wire, _ = _stream(rng, sizes, b0=b0)
    assert check(wire) == 500
    check(wire, max_frames=100)
    check(wire, max_frames=0)


def test_empty_and_bad_arguments():
    check(np.zeros(0, np.uint8))
    lib = nm._lib.host()
    res = np.zeros(3, np.uint64)
    assert lib.netc_ws_scan_frames_host(None, 0, 0, 0, None, None, None, 0, None) == nm.NETC_GPU_EINVAL
    assert lib.netc_ws_scan_frames_host(None, 0, 0, 2, None, None, None, 0, res.ctypes.data) == nm.NETC_GPU_EINVAL
    assert lib.netc_ws_scan_frames_host(None, 0, 0, 0, None, None, None, 0, res.ctypes.data) == 0
    assert list(res) == [0, 0, U64MAX]
