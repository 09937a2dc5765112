"""GPU parity of BASELINE config 5 at its own shape: netc_gpu_stream_* / netc_gpu_mask_stream_host
(include/ws/mask.h) masking a pinned host ring of 4 KiB frames through the default 2 x 512 MiB
device slots, H2D / kernel / D2H overlapped.

The full config is 16 GiB (4,194,304 frames): test_c5_full_16gib runs it, or skips by name (with
the sizes in the reason) on a host without the memory for two pinned 16 GiB rings;
test_c5_2gib_past_2_31 always runs 2 GiB + 4 KiB (more than 4 slot rotations, offsets past 2^31).  Checks, byte for byte over the whole buffer:
  * out of place: dst = mask(src); in place: src := mask(src); the two results are equal;
  * the oracle (the reference's exact expression, src/ws/common.c:321) applied to dst gives
    back the original bytes (the mask is an involution, so this is dst == oracle(src)),
    compared through a 64-bit xxhash of the original taken before the runs.
The phase carry across slot edges (src/ws/common.c:301,321) is exercised by a frame size that
does not divide the slot (a second case with 4,100-byte frames).
"""

import os
import time

import numpy as np
import pytest

from netc_amd import mask as nm
from netc_amd import synth
from oracle import oracle as orc

pytestmark = pytest.mark.gpu
GIB = 1 << 30


def _xxh(a: np.ndarray) -> int:
    import xxhash

    h = xxhash.xxh64()
    step = 256 << 20
    for lo in range(0, a.size, step):
        h.update(memoryview(a[lo: lo + step]))
    return h.intdigest()


def _host_available():
    try:
        import psutil

        return psutil.virtual_memory().available
    except Exception:  # pragma: no cover
        return 0


def _run(torch_cuda, total, frame):
    nframes = total // frame
    off = synth.uniform_offsets(nframes, frame)
    keys = synth.random_keys(nframes, stream=500 + frame)
    src_p, dst_p = nm.PinnedArray(total), nm.PinnedArray(total)
    try:
        src, dst = src_p.array, dst_p.array
        synth.fill_payload(src)
        h0 = _xxh(src)
        with nm.HostStream(0) as hs:   # defaults: 2 slots x 512 MiB
            t0 = time.perf_counter()
            hs.mask(dst, src, off, keys)                 # out of place
            t1 = time.perf_counter()
            hs.mask(src, src, off, keys)                 # in place
            t2 = time.perf_counter()
        print(f"\nC5 {total / GIB:.2f} GiB of {frame}-B frames, pinned, 2 x 512 MiB slots: "
              f"out of place {total / GIB / (t1 - t0):.1f} GiB/s, in place {total / GIB / (t2 - t1):.1f} GiB/s "
              f"host to host")
        assert np.array_equal(src, dst), "in-place and out-of-place results differ"
        orc.mask_batch_inplace(dst, off, keys)           # oracle^-1: back to the original bytes
        assert _xxh(dst) == h0, "oracle(dst) != original: the stream output is not the reference's masking"
    finally:
        src_p.close()
        dst_p.close()


@pytest.mark.timeout(900)
def test_c5_full_16gib(torch_cuda):
    """BASELINE config 5 at its full size: 16 GiB = 4,194,304 frames of 4 KiB.  Two pinned
    16 GiB rings plus the hash pass need ~3 x 16 GiB of host memory; a host without it SKIPS
    this case by name (it never silently runs a smaller one)."""
    need = 3 * 16 * GIB + 8 * GIB
    avail = _host_available()
    if avail < need:
        pytest.skip(f"config 5 at 16 GiB needs {need / GIB:.0f} GiB of host memory, {avail / GIB:.0f} GiB available")
    _run(torch_cuda, 16 * GIB, 4096)


@pytest.mark.timeout(600)
def test_c5_2gib_past_2_31(torch_cuda):
    # the same shape at 2 GiB + 4 KiB on any host: > 4 slot rotations, offsets past 2^31
    _run(torch_cuda, 2 * GIB + 4096, 4096)


@pytest.mark.timeout(600)
def test_c5_frames_cut_by_slot_edges(torch_cuda):
    # 4,100-byte frames: slot edges (every 512 MiB) fall inside frames at every phase
    _run(torch_cuda, 2 * GIB + 4100 * 7, 4100)


def test_stream_handle_reuse_and_errors(torch_cuda):
    off = synth.mixed_offsets(3 << 20, 1, 70000, seed=5)
    keys = synth.random_keys(off.size - 1, 5)
    total = int(off[-1])
    payload = synth.host_payload(total, 5)
    exp = orc.mask_batch(payload, off, keys)
    with nm.HostStream(0, slot_bytes=1 << 20, nslots=3) as hs:
        for _ in range(3):                                # the handle is reused: same answer every call
            out = np.empty_like(payload)
            hs.mask(out, payload, off, keys)
            assert np.array_equal(out, exp)
        # a run with many more frames per slot than before grows the descriptor staging
        off2 = synth.uniform_offsets((2 << 20) // 8, 8)
        keys2 = synth.random_keys(off2.size - 1, 6)
        p2 = synth.host_payload(int(off2[-1]), 6)
        out2 = np.empty_like(p2)
        hs.mask(out2, p2, off2, keys2)
        assert np.array_equal(out2, orc.mask_batch(p2, off2, keys2))
        with pytest.raises(nm.NetcGpuError) as e:
            bad = off.copy()
            bad[-1] = total + 1                           # offsets[nframes] > total_bytes
            hs.mask(out, payload, bad, keys)
        assert e.value.code == nm.NETC_GPU_EINVAL
    with pytest.raises(nm.NetcGpuError) as e:
        nm.HostStream(0, slot_bytes=100)
    assert e.value.code == nm.NETC_GPU_EINVAL
