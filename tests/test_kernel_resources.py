"""The hot kernels of the built gfx950 library do not spill to scratch (CPU test, no GPU).

A kernel whose registers spill to scratch memory runs its loop through per-lane scratch loads
and stores: round 5 measured a frame-assembly build whose fixup loop made the compiler spill
86 VGPRs at 89-92 us per config-2 step against 35-38 us without
(profiles/r05_kernels/encode_class.json).  The library's code objects carry the compiler's
count per kernel (AMDGPU metadata notes: .vgpr_spill_count, .private_segment_fixed_size), so
this test reads them from netc_amd/lib/libnetc_ws_gpu.so and holds every kernel on a default
path at zero.  Kernels only a measurement knob or netc_gpu_tune reaches are listed apart and
reported, not held.
"""

import os
import re
import struct
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "netc_amd", "lib", "libnetc_ws_gpu.so")
READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"

# kernels a default call reaches (demangled name prefixes)
HOT = [
    "void netc_gpu::mask_np_kernel<1, 2, true, true, false, netc_gpu::Args>",   # the headline (config 2)
    "void netc_gpu::mask_np_kernel<",
    "void netc_gpu::encode_frames_kernel<4, true, 5, false>",
    "void netc_gpu::encode_frames_kernel<4, false, 5, false>",
    "void netc_gpu::encode_frames_kernel<4, true, 4, true>",    # pipelined, above 256 MiB of wire
    "void netc_gpu::encode_frames_kernel<4, false, 4, true>",
    "void netc_gpu::wire_offsets_chained<4, false>",
    "void netc_gpu::wire_offsets_chained<16, false>",
    "void netc_gpu::scan_links<",
    "netc_gpu::scan_links_fused(",              # the one-pass path's gated launch
    "netc_gpu::scan_tiles_resolve(",
    "netc_gpu::scan_tiles(",
    "netc_gpu::scan_resolve(",
    "void netc_gpu::scan_emit<",
    "void netc_gpu::scan_exits<",
    "netc_gpu::utf8_messages(",
]
# reached only through netc_gpu_tune or NETC_GPU_KNOB_* (A/B paths), not held at zero
KNOB_ONLY = [
    "void netc_gpu::mask_frames_kernel<",      # round-1 walk (NETC_GPU_TUNE_PERSISTENT)
    "void netc_gpu::encode_frames_kernel<2,",  # 2 KiB chunks (netc_gpu_tune unroll 2 / 4; ENC_PF = 1)
    "void netc_gpu::wire_offsets_chained<16, true>",   # fixups in the scan (ENC_FIX = 1)
    "void netc_gpu::wire_offsets_chained<1, true>",
]


def _code_objects(path):
    """The gfx950 ELF code objects of the library's .hip_fatbin clang offload bundles."""
    out = subprocess.run([READELF, "-S", "-W", path], capture_output=True, text=True, check=True).stdout
    m = re.search(r"\.hip_fatbin\s+PROGBITS\s+[0-9a-f]+\s+([0-9a-f]+)\s+([0-9a-f]+)", out)
    assert m, "no .hip_fatbin section"
    off, size = int(m.group(1), 16), int(m.group(2), 16)
    with open(path, "rb") as f:
        f.seek(off)
        sec = f.read(size)
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    objs = []
    i = sec.find(magic)
    while i >= 0:
        n = struct.unpack_from("<Q", sec, i + len(magic))[0]
        p = i + len(magic) + 8
        for _ in range(n):
            eo, es, tl = struct.unpack_from("<QQQ", sec, p)
            p += 24
            triple = sec[p:p + tl].decode()
            p += tl
            if "gfx950" in triple and es:
                objs.append(sec[i + eo:i + eo + es])
        i = sec.find(magic, i + 1)
    return objs


def kernel_resources(path=LIB, lds_out=None):
    """{demangled kernel name: (vgpr_count, vgpr_spill_count, private_segment_fixed_size)};
    lds_out, if given, receives {demangled name: group_segment_fixed_size}"""
    res, lds = {}, {}
    for obj in _code_objects(path):
        with tempfile.NamedTemporaryFile(suffix=".co") as f:
            f.write(obj)
            f.flush()
            notes = subprocess.run([READELF, "--notes", f.name], capture_output=True, text=True, check=True).stdout
        for blk in re.split(r"\n\s+- \.agpr_count", notes)[1:]:
            name = re.search(r"\.name:\s+(\S+)", blk).group(1)

            def field(k):
                return int(re.search(rf"\.{k}:\s+(\d+)", blk).group(1))

            res[name] = (field("vgpr_count"), field("vgpr_spill_count"), field("private_segment_fixed_size"))
            lds[name] = field("group_segment_fixed_size")
    names = list(res)
    dem = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True, check=True).stdout.split("\n")
    if lds_out is not None:
        lds_out.update({d: lds[m] for m, d in zip(names, dem)})
    return {d: res[m] for m, d in zip(names, dem)}


@pytest.fixture(scope="module")
def resources():
    if not os.path.exists(LIB):
        pytest.skip("libnetc_ws_gpu.so not built (make)")
    if not os.path.exists(READELF):
        pytest.skip("llvm-readelf not found")
    return kernel_resources()


def test_every_hot_kernel_is_found(resources):
    for prefix in HOT:
        assert any(k.startswith(prefix) for k in resources), f"no kernel {prefix}* in the library"


# kernels allowed a small private segment (no spills): bytes per lane, and why
SCRATCH_OK = {
    # K2 + K3a + K3b in one launch: on the default path only as the one-pass path's gate (a flag
    # read, then return); its graph body runs when the one-pass path fails over (or with SCAN_FUSE=1)
    "netc_gpu::scan_links_fused(": 64,
}


def test_hot_kernels_do_not_spill(resources):
    bad = []
    for k, (vgprs, spills, scratch) in sorted(resources.items()):
        if any(k.startswith(p) for p in KNOB_ONLY):
            continue
        if not spills and any(k.startswith(p) and scratch <= lim for p, lim in SCRATCH_OK.items()):
            continue
        if any(k.startswith(p) for p in HOT) and (spills or scratch):
            bad.append(f"{k}: {vgprs} VGPRs, {spills} spilled, {scratch} B scratch per lane")
    assert not bad, "kernels on a default path spill:\n" + "\n".join(bad)


def test_scan_k1_fits_eight_blocks_per_cu():
    """K1 (scan_exits) at 20,480 B of LDS per 4-wave block: 8 blocks, the SIMDs' 32 waves, fit a
    CU's 160 KiB (C4 scan 81.2 -> 80.1 us against the 20,608-B layout; DESIGN_ROUNDS.md §15.5)"""
    if not os.path.exists(LIB) or not os.path.exists(READELF):
        pytest.skip("libnetc_ws_gpu.so or llvm-readelf missing")
    lds = {}
    kernel_resources(lds_out=lds)
    k1 = {k: v for k, v in lds.items() if k.startswith("void netc_gpu::scan_exits<")}
    assert len(k1) == 4, k1   # NT x one-pass
    for k, v in k1.items():
        assert 0 < v <= 20480, f"{k}: {v} B of LDS"
