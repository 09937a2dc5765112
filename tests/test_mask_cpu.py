"""Host CPU masking entry netc_ws_mask and the shard planner netc_shard_frames vs the oracle (CPU)."""

import numpy as np
import pytest

from netc_amd import mask as nm
from netc_amd import synth
from oracle import oracle as orc


@pytest.mark.parametrize("seed", range(6))
def test_mask_host_matches_oracle(seed):
    g = np.random.Generator(np.random.PCG64(seed))
    for _ in range(60):
        n = int(g.integers(0, 300))
        base = g.integers(0, 256, n + 32, dtype=np.uint8)
        so, do = int(g.integers(0, 16)), int(g.integers(0, 16))
        src = base[so:so + n]
        key = bytes(g.integers(0, 256, 4, dtype=np.uint8))
        phase = int(g.integers(0, 1 << 40))
        out_buf = np.zeros(n + 32, dtype=np.uint8)
        out = out_buf[do:do + n]
        nm.mask_host(src, key, phase, out=out)
        assert np.array_equal(out, orc.unmask(src, key, phase))
        assert not out_buf[:do].any() and not out_buf[do + n:].any()


def test_mask_host_in_place_and_involution():
    g = np.random.Generator(np.random.PCG64(99))
    x = g.integers(0, 256, 100001, dtype=np.uint8)
    y = x.copy()
    nm.mask_host(y, b"\x9a\xbc\xde\xf0", 3, out=y)
    assert np.array_equal(y, orc.unmask(x, b"\x9a\xbc\xde\xf0", 3))
    nm.mask_host(y, b"\x9a\xbc\xde\xf0", 3, out=y)
    assert np.array_equal(y, x)


def test_pack_keys_little_endian():
    assert nm.pack_keys([[0x00, 0x61, 0xC2, 0x23]])[0] == 0x23C26100


@pytest.mark.parametrize("nshards", [1, 2, 3, 8, 13])
def test_shard_frames_balanced(nshards):
    off = synth.mixed_offsets(64 << 20, 256, 65536, seed=nshards)
    cuts = nm.shard_frames(off, nshards)
    assert cuts[0] == 0 and cuts[-1] == off.size - 1 and np.all(np.diff(cuts) >= 0)
    sizes = np.diff(off[cuts].astype(np.int64))
    ideal = (int(off[-1]) - int(off[0])) / nshards
    assert np.all(np.abs(sizes - ideal) <= 65536)     # within one frame of ideal


def test_shard_frames_edge_cases():
    assert list(nm.shard_frames(np.array([0], dtype=np.uint64), 4)) == [0, 0, 0, 0, 0]
    off = np.array([0, 10, 10, 10, 1000], dtype=np.uint64)
    cuts = nm.shard_frames(off, 2)
    assert list(cuts) == [0, 3, 4] or list(cuts) == [0, 4, 4] or cuts[1] in (1, 2, 3, 4)
    with pytest.raises(nm.NetcGpuError):
        nm.shard_frames(np.array([0, 5, 3], dtype=np.uint64), 2)     # decreasing
    with pytest.raises(nm.NetcGpuError):
        nm.shard_frames(off, 0)


def test_synth_shapes():
    off, keys, total = synth.config("c2")
    assert off.size == 65537 and total == 64 << 20 and keys.size == 65536
    off4, keys4, total4 = synth.config("c4", shard=5)
    sizes = np.diff(off4.astype(np.int64))
    assert total4 == 1 << 30 and sizes[:-1].min() >= 256 and sizes.max() <= 65536
    assert keys4[0] == 0 and keys4[1] == 0xFFFFFFFF


def test_sanitized_build_is_the_one_loaded():
    """Under `make asan` the suites run against the ASan + UBSan builds (NETC_HOST_LIB /
    NETC_ORACLE_LIB); this checks that the instrumented libraries are the ones in use."""
    import os
    import subprocess

    from netc_amd import _lib
    from oracle import oracle as orc

    host = os.environ.get("NETC_HOST_LIB")
    if not host:
        pytest.skip("not a `make asan` run")
    _lib.host()
    orc.lib()
    for path in (os.path.abspath(host), os.path.abspath(os.environ["NETC_ORACLE_LIB"])):
        syms = subprocess.run(["nm", "-D", path], capture_output=True, text=True, check=True).stdout
        assert "__asan_report" in syms and "__ubsan_handle" in syms, path
        maps = open("/proc/self/maps").read()
        assert path in maps, f"{path} is not mapped in this process"
