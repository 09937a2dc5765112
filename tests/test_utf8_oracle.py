"""The UTF-8 checker (oracle_utf8_valid / oracle_validate_batch) is pinned before it is trusted (CPU).

The reference has no UTF-8 validation to compare with (src/ws/common.c:342 only
appends a NUL), so the checker is pinned by RFC 3629's own rules: known-answer
vectors at every boundary (shortest form, surrogates, U+10FFFF, truncation), and
randomized agreement with CPython's strict UTF-8 decoder (an independent
implementation of the same RFC) on mutated valid text.
"""

import numpy as np
import pytest

from oracle import oracle as orc

KAT = [
    (b"", True), (b"plain ascii {json: 1}", True), (b"\x00\x7f", True),
    (b"\xc2\x80", True), (b"\xdf\xbf", True), (b"\xc0\x80", False), (b"\xc1\xbf", False),
    (b"\xe0\xa0\x80", True), (b"\xe0\x9f\xbf", False), (b"\xed\x9f\xbf", True), (b"\xed\xa0\x80", False),
    (b"\xed\xbf\xbf", False), (b"\xee\x80\x80", True), (b"\xef\xbf\xbf", True),
    (b"\xf0\x90\x80\x80", True), (b"\xf0\x8f\xbf\xbf", False), (b"\xf4\x8f\xbf\xbf", True),
    (b"\xf4\x90\x80\x80", False), (b"\xf5\x80\x80\x80", False), (b"\xff", False), (b"\xfe", False),
    (b"\x80", False), (b"\xbf", False), (b"a\x80b", False),
    (b"\xc3", False), (b"\xe2\x82", False), (b"\xf0\x9f\x98", False), (b"\xe2\x82\xac", True),
    (b"\xf0\x9f\x98\x80", True), (b"\xc3\xa9\xc3", False), (b"\xe2\x28\xa1", False), (b"\xc3\x28", False),
]


@pytest.mark.parametrize("data,ok", KAT, ids=lambda x: x.hex() if isinstance(x, bytes) else str(x))
def test_known_answers(data, ok):
    assert orc.utf8_valid(data) == ok


def _py_valid(b: bytes) -> bool:
    try:
        b.decode("utf-8", errors="strict")
        return True
    except UnicodeDecodeError:
        return False


def random_text(rng, n_cp):
    # code points near every encoding boundary, plus ordinary ASCII
    pool = [0x24, 0x7F, 0x80, 0x7FF, 0x800, 0xD7FF, 0xE000, 0xFFFD, 0xFFFF, 0x10000, 0x1F600, 0x10FFFF]
    cps = [int(rng.choice(pool)) if rng.random() < 0.3 else int(rng.integers(0x20, 0x7F)) for _ in range(n_cp)]
    return "".join(chr(c) for c in cps).encode("utf-8")


@pytest.mark.parametrize("seed", range(6))
def test_agrees_with_cpython_decoder(seed):
    rng = np.random.default_rng(seed)
    agree = valid = 0
    for _ in range(400):
        b = bytearray(random_text(rng, int(rng.integers(0, 40))))
        for _ in range(int(rng.integers(0, 3))):   # mutate: flip, insert, truncate
            r = rng.random()
            if b and r < 0.4:
                b[int(rng.integers(0, len(b)))] = int(rng.integers(0, 256))
            elif r < 0.7:
                b.insert(int(rng.integers(0, len(b) + 1)), int(rng.integers(0x80, 0x100)))
            elif b:
                del b[int(rng.integers(0, len(b))):]
        b = bytes(b)
        assert orc.utf8_valid(b) == _py_valid(b), b.hex()
        agree += 1
        valid += _py_valid(b)
    assert 50 < valid < 390   # both outcomes exercised


def test_batch_verdicts_follow_messages():
    # TEXT "é" split inside the code point across two fragments with a PING between
    # them is valid; the same split with the continuation byte dropped is not
    frames = [(0x01, b"ab\xc3"), (0x89, b"\xff\xfe"), (0x80, b"\xa9cd"),      # valid, split code point
              (0x81, b"\xe2\x82"),                                          # truncated at message end
              (0x02, b"\xff"), (0x80, b"\xfe"),                             # BINARY: no verdict
              (0x01, b"ok"), (0x00, b"\x80"), (0x80, b"")]                  # orphan continuation byte
    payload = b"".join(p for _, p in frames)
    off = np.zeros(len(frames) + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(p) for _, p in frames])
    h = np.array([b for b, _ in frames], dtype=np.uint8)
    v = orc.validate_batch(payload, off, h)
    assert list(v) == [1, 1, 1, 0, 1, 1, 1, 1, 0]
