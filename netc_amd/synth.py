"""Seeded synthetic frame batches of the BASELINE.json shapes.

A batch is (payload bytes, offsets[nframes + 1] uint64, keys[nframes] uint32
packed key32) exactly as include/ws/mask.h consumes it.  Frames are packed back
to back, unpadded.  Payload bytes are generated on the device for the large
configs (bench), on the host for parity tests.
"""

from __future__ import annotations

import numpy as np

SEED = 0x6E657463          # "netc"
EDGE_KEYS = np.array([0x00000000, 0xFFFFFFFF, 0x23C26100, 0x00FF00FF, 0x000000FF, 0xFF000000], dtype=np.uint32)
# 0x23C26100 is the reference's first ws_build_masking_key() output 00 61 c2 23 (src/ws/common.c:21-27)


def rng(seed: int = SEED, stream: int = 0) -> np.random.Generator:
    return np.random.Generator(np.random.PCG64([seed, stream]))


def uniform_offsets(nframes: int, frame_len: int, start: int = 0) -> np.ndarray:
    """C2 / C3 / C5: nframes frames of frame_len bytes at k * frame_len."""
    return (start + np.arange(nframes + 1, dtype=np.uint64) * np.uint64(frame_len)).astype(np.uint64)


def mixed_offsets(total: int, lo: int = 256, hi: int = 65536, seed: int = SEED, stream: int = 0) -> np.ndarray:
    """C4: frame sizes uniform-integer in [lo, hi], packed back to back, last frame truncated to hit total."""
    g = rng(seed, stream)
    est = total // ((lo + hi) // 2) + 64
    sizes = g.integers(lo, hi, size=est, endpoint=True, dtype=np.int64)
    while sizes.sum() < total:
        sizes = np.concatenate([sizes, g.integers(lo, hi, size=est, endpoint=True, dtype=np.int64)])
    csum = np.cumsum(sizes)
    n = int(np.searchsorted(csum, total)) + 1       # frames needed to reach total
    off = np.zeros(n + 1, dtype=np.uint64)
    off[1:] = np.minimum(csum[:n], total).astype(np.uint64)
    return off


def random_keys(nframes: int, seed: int = SEED, stream: int = 1, edge: bool = True) -> np.ndarray:
    """Independent random packed key per frame; the first frames get the edge keys."""
    k = rng(seed, stream).integers(0, 1 << 32, size=nframes, dtype=np.uint64).astype(np.uint32)
    if edge:
        m = min(nframes, EDGE_KEYS.size)
        k[:m] = EDGE_KEYS[:m]
    return k


def host_payload(total: int, seed: int = SEED, stream: int = 2) -> np.ndarray:
    return rng(seed, stream).integers(0, 256, size=total, dtype=np.uint8)


def config(name: str, shard: int = 0):
    """(offsets, keys, total) for a BASELINE.json config: 'c2', 'c3', 'c4', 'c5'."""
    name = name.lower()
    if name == "c2":
        off = uniform_offsets(65536, 1024)
    elif name == "c3":
        off = uniform_offsets(1024, 1 << 20)
    elif name == "c4":
        off = mixed_offsets(1 << 30, stream=100 + shard)
    elif name == "c5":
        off = uniform_offsets(4194304, 4096)
    else:
        raise ValueError(name)
    keys = random_keys(off.size - 1, stream=200 + shard)
    return off, keys, int(off[-1])


def fill_payload(out: np.ndarray, seed: int = SEED, stream: int = 3, block: int = 64 << 20) -> None:
    """Fill a large uint8 array (GiBs, e.g. a pinned host ring) with seeded bytes, fast: one
    random block, XORed with the block index for every block it is copied to."""
    base = rng(seed, stream).integers(0, 256, size=min(block, max(out.size, 1)), dtype=np.uint8)
    for i, lo in enumerate(range(0, out.size, base.size)):
        hi = min(out.size, lo + base.size)
        np.bitwise_xor(base[: hi - lo], np.uint8(i & 0xFF), out=out[lo:hi])
