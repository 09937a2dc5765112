"""GPU parity: netc_gpu_unmask_validate (fused unmask + UTF-8 check of TEXT messages) vs the oracle.

Checkers: oracle_mask_batch (the reference's unmask expression, src/ws/common.c:321)
for the bytes, oracle_validate_batch (RFC 3629 decoder pinned by
tests/test_utf8_oracle.py) for the per-frame verdicts.  The bar: identical bytes,
identical verdicts.
"""

import numpy as np
import pytest

from netc_amd import mask as nm
from oracle import oracle as orc

pytestmark = pytest.mark.gpu

GUARD = 64


def _dev(torch, a):
    a = np.ascontiguousarray(a)
    if a.dtype == np.uint64:
        a = a.view(np.int64)
    elif a.dtype == np.uint32:
        a = a.view(np.int32)
    return torch.from_numpy(a).cuda()


def text_bytes(rng, n):
    """~n bytes of UTF-8 text: mostly ASCII, code points near every encoding boundary."""
    pool = [0x7F, 0x80, 0xE9, 0x7FF, 0x800, 0x20AC, 0xD7FF, 0xE000, 0xFFFD, 0xFFFF, 0x10000, 0x1F600, 0x10FFFF]
    out = bytearray()
    while len(out) < n:
        c = int(rng.choice(pool)) if rng.random() < 0.15 else int(rng.integers(0x20, 0x7F))
        out += chr(c).encode("utf-8")
    return bytes(out)


def corrupt(rng, b: bytes) -> bytes:
    b = bytearray(b)
    kind = rng.integers(0, 5)
    if not b:
        return bytes([0xC3])
    i = int(rng.integers(0, len(b)))
    if kind == 0:
        b[i] = 0xFF
    elif kind == 1:
        b.insert(i, 0x80)                    # stray continuation
    elif kind == 2:
        b[i:i] = b"\xed\xa0\x80"             # surrogate
    elif kind == 3:
        b[i:i] = b"\xe0\x80\xaf"             # overlong
    else:
        b += b"\xf0\x9f\x98"                 # truncated at the end
    return bytes(b)


def build_batch(rng, n_msgs, max_len, bad_frac=0.3, control_frac=0.1, binary_frac=0.1):
    """Frames (header byte, payload) of whole messages, fragments split at random byte offsets."""
    frames = []
    for _ in range(n_msgs):
        r = rng.random()
        if r < binary_frac:
            body = rng.integers(0, 256, int(rng.integers(0, max_len)), dtype=np.uint8).tobytes()
            op = 2
        else:
            body = text_bytes(rng, int(rng.integers(0, max_len)))
            if rng.random() < bad_frac:
                body = corrupt(rng, body)
            op = 1
        parts = int(rng.integers(1, 5))
        cuts = sorted(int(x) for x in rng.integers(0, len(body) + 1, parts - 1))
        pieces = [body[a:b] for a, b in zip([0] + cuts, cuts + [len(body)])]
        for i, piece in enumerate(pieces):
            frames.append(((0x80 if i == len(pieces) - 1 else 0) | (op if i == 0 else 0), piece))
            if rng.random() < control_frac:
                frames.append((0x89, rng.integers(0, 256, int(rng.integers(0, 20)), dtype=np.uint8).tobytes()))
    return frames


# where dst lies: in place; out of place 3 bytes off src's alignment (the SRC_ALIGNED = false
# kernels); out of place 16 bytes on, co-aligned with src (SRC_ALIGNED = true: with one-step
# windows each window checks its own first bytes from src -- seam_raw<true> -- ADVICE r3)
PLACES = {"inplace": None, "oop_misaligned": 3, "oop_coaligned": 16}


def run_validate(torch, frames, shift=0, inplace=True, dshift=3):
    payload = np.frombuffer(b"".join(p for _, p in frames), dtype=np.uint8)
    n = len(frames)
    off = np.zeros(n + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(p) for _, p in frames])
    h0 = np.array([h for h, _ in frames], dtype=np.uint8)
    rng = np.random.default_rng(n)
    keys = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    masked = orc.mask_batch(payload, off, keys)            # the wire payload (masking is an involution)
    total = masked.size
    buf = torch.zeros(total + 2 * GUARD, dtype=torch.uint8, device="cuda")
    src = buf[GUARD + shift: GUARD + shift + total]
    src.copy_(torch.from_numpy(masked))
    if inplace:
        dst = src
    else:
        dbuf = torch.zeros(total + 2 * GUARD, dtype=torch.uint8, device="cuda")
        dst = dbuf[GUARD + shift + dshift: GUARD + shift + dshift + total]
    valid = torch.full((n,), 7, dtype=torch.uint8, device="cuda")
    nm.unmask_validate(dst, src, _dev(torch, off), _dev(torch, keys), torch.from_numpy(h0).cuda(), valid)
    torch.cuda.synchronize()
    assert np.array_equal(dst.cpu().numpy(), payload), "unmasked bytes differ"
    exp = orc.validate_batch(payload, off, h0)
    got = valid.cpu().numpy()
    bad = np.nonzero(got != exp)[0]
    assert bad.size == 0, f"verdicts differ at frames {bad[:8].tolist()} (got {got[bad[:8]].tolist()})"
    return exp


@pytest.mark.parametrize("steps", [None, 1, 2, 4])
@pytest.mark.parametrize("seed", range(4))
def test_mixed_messages(torch_cuda, gpu_knob, seed, steps):
    gpu_knob("VAL_STEPS", steps)   # the 4 KiB window as 1, 2 or 4 steps (None: by batch size)
    rng = np.random.default_rng(seed)
    exp = run_validate(torch_cuda, build_batch(rng, 300, 3000))
    assert 0 < (exp == 0).sum()   # some messages are invalid


@pytest.mark.parametrize("shift", [1, 7, 13])
def test_alignments_and_out_of_place(torch_cuda, shift):
    rng = np.random.default_rng(40 + shift)
    run_validate(torch_cuda, build_batch(rng, 200, 2000), shift=shift)
    run_validate(torch_cuda, build_batch(rng, 200, 2000), shift=shift, inplace=False)


def test_tiny_fragments(torch_cuda):
    # fragments of 0-3 bytes: every code point split across frames
    rng = np.random.default_rng(50)
    frames = []
    for _ in range(200):
        body = text_bytes(rng, int(rng.integers(0, 40)))
        if rng.random() < 0.3:
            body = corrupt(rng, body)
        pieces, i = [], 0
        while i < len(body):
            k = int(rng.integers(0, 4))
            pieces.append(body[i:i + k])
            i += k
        pieces = pieces or [b""]
        for j, p in enumerate(pieces):
            frames.append(((0x80 if j == len(pieces) - 1 else 0) | (1 if j == 0 else 0), p))
    run_validate(torch_cuda, frames)


@pytest.mark.parametrize("place", sorted(PLACES))
@pytest.mark.parametrize("steps", [None, 1, 2, 4])
def test_errors_at_every_boundary(torch_cuda, gpu_knob, steps, place):
    # one long valid TEXT frame per case with an error at a vector / span / chunk edge
    gpu_knob("VAL_STEPS", steps)
    rng = np.random.default_rng(60)
    base = text_bytes(rng, 20000)
    base = base[: base.rfind(b" ") if b" " in base else len(base)]
    frames = []
    for pos in (0, 1, 2, 3, 15, 16, 17, 1023, 1024, 1025, 4093, 4094, 4095, 4096, 4097, 8191, 8192):
        for bad in (b"\x80", b"\xff", b"\xc3\x28", b"\xed\xa0\x80", b"\xe0\x80\xaf"):
            cut = base[:pos]
            while cut and (cut[-1] & 0xC0) == 0x80:   # keep the prefix itself valid
                cut = cut[:-1]
            if cut and cut[-1] >= 0xC0:
                cut = cut[:-1]
            frames.append((0x81, cut + bad + b"tail"))
    frames.append((0x81, base))   # and a valid one
    exp = run_validate(torch_cuda, frames, inplace=PLACES[place] is None, dshift=PLACES[place] or 0)
    assert (exp[:-1] == 0).all() and exp[-1] == 1


@pytest.mark.parametrize("place", sorted(PLACES))
@pytest.mark.parametrize("steps", [None, 1, 2, 4])
@pytest.mark.parametrize("shift", [0, 5])
def test_errors_at_chunk_seams(torch_cuda, gpu_knob, shift, steps, place):
    gpu_knob("VAL_STEPS", steps)
    # long frames (many 4 KiB chunks each) with one broken byte among the first 3 bytes
    # of a chunk -- the bytes phase B checks in place; out of place each window checks its
    # own first bytes (the 4 before it unmasked from src) -- or just before / after them
    rng = np.random.default_rng(70 + shift)
    flen, win, mis = 70000, 4096, shift & 15   # torch allocations are 256-B aligned
    frames, o = [], 0
    for i in range(30):
        body = bytearray(text_bytes(rng, flen)[:flen]) if i % 3 else bytearray(rng.integers(0x20, 0x7F, flen, dtype=np.uint8).tobytes())
        if i % 6 != 5:
            c = ((o + mis + 3 + win - 1) // win + int(rng.integers(0, 12))) * win   # a chunk start inside the frame
            p = c - mis - o + (-1, 0, 1, 2, 3)[i % 5]
            if 3 <= p < flen:
                body[p] = (0xFF, 0x80, 0xC0)[i % 3]
        frames.append((0x81, bytes(body)))
        o += flen
    run_validate(torch_cuda, frames, shift=shift, inplace=PLACES[place] is None, dshift=PLACES[place] or 0)


@pytest.mark.parametrize("inplace", [True, False])
@pytest.mark.parametrize("steps", [2, 4])
@pytest.mark.parametrize("shift", [0, 7])
def test_errors_at_step_starts_of_the_last_window(torch_cuda, gpu_knob, steps, shift, inplace):
    # a window of several steps that holds a partial vector (the batch's last) runs its steps
    # one by one; the first 3 bytes of each later step are checked with the carry from the
    # step before (they are no 4 KiB seam that phase B would check)
    gpu_knob("VAL_STEPS", steps)
    rng = np.random.default_rng(90 + steps + shift)
    win, mis = 4096, shift & 15
    total = 5 * win + 3000 - mis                     # the last window is partial
    last = (mis + total) // win * win                # its first byte (P coordinates)
    step = win // steps
    for k in range(1, steps):
        for d in range(3):
            # an overlong 2-byte sequence C0 80 whose second byte is byte d of the step: the
            # rule flags that byte and no other (ASCII around it)
            q = last + k * step + d - mis            # payload offset of the flagged byte
            if q + 6 >= total:
                continue
            body = bytearray(b"a" * 1000) + bytearray(text_bytes(rng, total)[:total - 1000])
            body[q - 5:q + 6] = b"a" * 11
            body[-4:] = b"tail"                      # no code point cut at the end
            body[q - 1], body[q] = 0xC0, 0x80
            frames = [(0x81, bytes(body[:1000])), (0x81, bytes(body[1000:]))]
            exp = run_validate(torch_cuda, frames, shift=shift, inplace=inplace)
            assert exp.tolist() == [1, 0]


def test_large_text_batch(torch_cuda):
    # ~64 MiB of 1 KiB TEXT frames (config 2 shape), 1 % corrupted
    rng = np.random.default_rng(70)
    chunk = text_bytes(rng, 1 << 20)
    frames = []
    pos = 0
    for i in range(65536):
        p = chunk[pos: pos + 1024]
        pos = (pos + 1024) % (len(chunk) - 1024)
        if i % 100 == 7:
            p = corrupt(rng, p)
        frames.append((0x81, p))
    exp = run_validate(torch_cuda, frames)
    assert (exp == 0).sum() > 300


def edge_text(rng, n, bad):
    """n bytes of text whose first and last 3 bytes are multi-byte sequences (or, bad: a stray
    continuation first / a truncated sequence last)"""
    if n < 8:
        return corrupt(rng, text_bytes(rng, n)) if bad else text_bytes(rng, n)
    head, tail = "\u20ac".encode(), "\U0001F600".encode()
    mid = bytearray(text_bytes(rng, max(0, n - 7)))
    body = head + bytes(mid) + tail
    if bad:
        body = (b"\x80" + body[1:]) if rng.random() < 0.5 else body[:-1]
    return body


@pytest.mark.parametrize("steps", [None, 1, 2, 4])
@pytest.mark.parametrize("place", sorted(PLACES))
def test_message_edges(torch_cuda, gpu_knob, steps, place):
    """single-frame TEXT messages starting and ending at every offset around span (1 KiB) and
    window (4 KiB) edges, with multi-byte first and last bytes, half of them broken at the start
    or end (the bytes the per-message launch checks), short ones among them"""
    gpu_knob("VAL_STEPS", steps)
    rng = np.random.default_rng(171)
    frames = []
    for _ in range(600):
        r = rng.random()
        n = int(rng.integers(0, 12)) if r < 0.2 else (int(rng.integers(1015, 1034)) if r < 0.7 else int(rng.integers(30, 3000)))
        bad = rng.random() < 0.5
        frames.append((0x81, edge_text(rng, n, bad)))
        if rng.random() < 0.05:
            frames.append((0x82, rng.integers(0, 256, int(rng.integers(0, 50)), dtype=np.uint8).tobytes()))
    shift = PLACES[place]
    exp = run_validate(torch_cuda, frames, shift=0 if shift is None else 0, inplace=shift is None,
                       dshift=shift or 3)
    assert 100 < (exp == 0).sum() < len(frames)
