"""Scratch lifetime of the C-ABI entries that keep per-(device, stream) device scratch
(reentrant, thread-safe entries that leak nothing).

netc_gpu_scan_frames, netc_gpu_encode_frames and netc_gpu_unmask_validate each keep scratch
for the stream they run on; netc_gpu_stream_release(device, stream) frees all of it.  A loop
that creates a HIP stream, runs the three entries on it, releases and destroys it must keep
the device's free memory flat -- and every round's results must still equal the oracle's.
"""

import ctypes

import numpy as np
import pytest

from netc_amd import mask as nm
from oracle import oracle as orc

pytestmark = pytest.mark.gpu
MIB = 1 << 20


def _hip():
    lib = ctypes.CDLL("libamdhip64.so.7")   # the runtime torch already loaded (same SONAME)
    lib.hipStreamCreate.argtypes = [ctypes.POINTER(ctypes.c_void_p)]
    lib.hipStreamDestroy.argtypes = [ctypes.c_void_p]
    return lib


def test_stream_release_frees_scan_encode_validate_scratch(torch_cuda):
    torch = torch_cuda
    hip = _hip()
    rng = np.random.default_rng(7)
    n = 4096
    off = np.arange(n + 1, dtype=np.uint64) * np.uint64(1024)
    plain = rng.integers(0, 128, int(off[-1]), dtype=np.uint8)          # ASCII: valid TEXT
    keys = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    wire, _ = orc.encode_batch(plain, off, keys, None, True)
    masked = orc.mask_batch(plain, off, keys)                            # what a receiver holds
    exp_hdr, *_ = orc.scan_frames(wire, strict=True)

    dev = torch.device("cuda", 0)
    d_wire = torch.from_numpy(wire).to(dev)
    hdr = torch.zeros(n + 2, dtype=torch.int64, device=dev)
    sk = torch.zeros(n + 1, dtype=torch.int32, device=dev)
    sb = torch.zeros(n + 1, dtype=torch.uint8, device=dev)
    res = torch.zeros(3, dtype=torch.int64, device=dev)
    d_plain = torch.from_numpy(plain).to(dev)
    d_masked = torch.from_numpy(masked).to(dev)
    d_off = torch.from_numpy(off.view(np.int64)).to(dev)
    d_keys = torch.from_numpy(keys.view(np.int32)).to(dev)
    out_wire = torch.zeros(nm.wire_bound(plain.size, n, True), dtype=torch.uint8, device=dev)
    wo = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    h0 = torch.full((n,), 0x81, dtype=torch.uint8, device=dev)
    valid = torch.zeros(n, dtype=torch.uint8, device=dev)
    dst = torch.empty_like(d_plain)
    torch.cuda.synchronize()

    def one_round():
        s = ctypes.c_void_p(0)
        assert hip.hipStreamCreate(ctypes.byref(s)) == 0
        h = s.value
        nm.scan_frames(d_wire, hdr, sk, sb, res, stream=h)
        nm.encode_frames(out_wire, wo, d_plain, d_off, d_keys, masked=True, stream=h)
        nm.unmask_validate(dst, d_masked, d_off, d_keys, h0, valid, stream=h)
        nm.stream_release(stream=h)          # synchronises h, frees the three scratch sets
        assert hip.hipStreamDestroy(h) == 0
        assert int(res[0]) == n and np.array_equal(hdr[:n].cpu().numpy().view(np.uint64), exp_hdr)
        assert np.array_equal(out_wire[:wire.size].cpu().numpy(), wire)
        assert bool((valid == 1).all()) and torch.equal(dst, d_plain)

    one_round()
    torch.cuda.synchronize()
    free0 = torch.cuda.mem_get_info(dev)[0]
    for _ in range(24):
        one_round()
    torch.cuda.synchronize()
    free1 = torch.cuda.mem_get_info(dev)[0]
    # one round's scratch is several MiB (scan + assembly + flags); leaking it 24 times would
    # lose far more than this allowance for runtime noise
    assert free0 - free1 < 8 * MIB, f"device free memory fell by {(free0 - free1) / MIB:.1f} MiB over 24 rounds"
