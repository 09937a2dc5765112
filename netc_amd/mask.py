"""Python mirror of the masking C-ABI (include/ws/mask.h).

Same names, argument meaning and error behaviour as the C entry points; device
buffers are torch tensors (uint8 payload, int64 offsets, int32 packed keys) and
host buffers numpy arrays.  Every call goes straight to the in-tree shared
libraries; a failing call raises :class:`NetcGpuError` carrying the negative
NETC_GPU_E* code and the library's message.  There is no CPU fallback for the
GPU entries.
"""

from __future__ import annotations

import contextlib

import ctypes
from typing import Optional, Sequence, Tuple

import numpy as np

from . import _lib

NETC_GPU_OK = 0
NETC_GPU_EINVAL = -101
NETC_GPU_ENODEV = -102
NETC_GPU_ELAUNCH = -103
NETC_GPU_ERUNTIME = -104
NETC_GPU_ENOMEM = -105
NETC_REASON_GPU = 18


class NetcGpuError(RuntimeError):
    def __init__(self, code: int, message: str):
        super().__init__(f"netc_gpu error {code}: {message}")
        self.code = code
        self.message = message


def _check(rc: int) -> None:
    if rc != 0:
        msg = _lib.gpu().netc_gpu_strerror()
        raise NetcGpuError(rc, msg.decode(errors="replace") if msg else "")


def _ptr(a) -> int:
    """Address of a torch tensor / numpy array / bytearray."""
    if hasattr(a, "data_ptr"):
        return a.data_ptr()
    if isinstance(a, np.ndarray):
        return a.ctypes.data
    if isinstance(a, bytearray):
        return ctypes.addressof((ctypes.c_char * len(a)).from_buffer(a))
    raise TypeError(f"unsupported buffer type {type(a)!r}")


# ------------------------------------------------------------------ host ---

def pack_keys(keys) -> np.ndarray:
    """(n, 4) wire key bytes -> n packed key32 = k0 | k1<<8 | k2<<16 | k3<<24 (uint32)."""
    k = np.ascontiguousarray(np.asarray(keys, dtype=np.uint8).reshape(-1, 4))
    return k.view("<u4").reshape(-1).astype(np.uint32)


def mask_host(src, key: bytes, phase: int = 0, out: Optional[np.ndarray] = None) -> np.ndarray:
    """netc_ws_mask: out[i] = src[i] ^ key[(phase + i) & 3] (host CPU entry)."""
    s = np.ascontiguousarray(np.frombuffer(bytes(src), dtype=np.uint8) if isinstance(src, (bytes, bytearray)) else src)
    if s.dtype != np.uint8:
        raise TypeError("src must be uint8")
    if out is None:
        out = np.empty_like(s)
    kb = (ctypes.c_uint8 * 4)(*bytes(key)[:4])
    _lib.host().netc_ws_mask(_ptr(out), _ptr(s), s.size, kb, phase)
    return out


def shard_frames(offsets: np.ndarray, nshards: int) -> np.ndarray:
    """netc_shard_frames: byte-balanced contiguous frame ranges, nshards + 1 cut indices."""
    off = np.ascontiguousarray(offsets, dtype=np.uint64)
    cuts = np.zeros(nshards + 1, dtype=np.uintp)
    rc = _lib.host().netc_shard_frames(_ptr(off), off.size - 1, nshards, _ptr(cuts))
    if rc != 0:
        raise NetcGpuError(rc, "netc_shard_frames: invalid offsets or shard count")
    return cuts.astype(np.int64)


# ------------------------------------------------------------------- gpu ---

def device_count() -> int:
    return int(_lib.gpu().netc_gpu_device_count())


def gpu_init(device: int = 0) -> None:
    _check(_lib.gpu().netc_gpu_init(device))


NETC_GPU_TUNE_NT_LOADS = 1
NETC_GPU_TUNE_NT_STORES = 2
NETC_GPU_TUNE_PERSISTENT = 4
NETC_GPU_TUNE_TWO_STEPS = 8
NETC_GPU_TUNE_XCD_ORDER = 16
NETC_GPU_TUNE_XCD_GROUPS = 32


NETC_GPU_TUNE_AUTO = -1


def tune(unroll: int = 1, max_blocks: int = 0, flags: int = NETC_GPU_TUNE_AUTO) -> None:
    """netc_gpu_tune: process-wide launch shape (KiB a wavefront loads at once, workgroup cap of the
    persistent walk, cache / walk flags); the defaults are the C library's."""
    _check(_lib.gpu().netc_gpu_tune(unroll, max_blocks, flags))


KNOBS = {"ENC_DENSE_BYTES": 1, "ENC_SCAN_PER": 2, "SCAN_FAST_RANK": 3, "SCAN_ANCHOR_SLOTS": 4, "VAL_STEPS": 5, "SCAN_FUSE": 6,
         "MASK_TAPER": 7, "ENC_SRC": 8, "ENC_FIX": 9, "INJECT_FAULT": 10,
         "ENC_PROBE": 11, "ENC_PF": 12, "SCAN_BLOCK_CHUNKS": 13, "SCAN_ONEPASS": 14}


def set_knob(name: str, value: int) -> None:
    """netc_gpu_knob: a measurement / test knob of the frame assembly or scan (value < 0 = default)."""
    _check(_lib.gpu().netc_gpu_knob(KNOBS[name], int(value)))


@contextlib.contextmanager
def knob(name: str, value):
    """Sets a knob for the duration of a `with` block (None: leave the default), then restores it."""
    if value is None:
        yield
        return
    set_knob(name, value)
    try:
        yield
    finally:
        set_knob(name, -1)


def stream_release(stream=None, device: int = 0) -> None:
    """netc_gpu_stream_release: synchronise `stream`, then free every scratch array the library
    keeps for it (scan, frame assembly, UTF-8 flags)."""
    _check(_lib.gpu().netc_gpu_stream_release(device, _stream_handle(stream)))


def _stream_handle(stream) -> int:
    import torch

    if stream is None:
        return torch.cuda.current_stream().cuda_stream
    if isinstance(stream, int):
        return stream
    return stream.cuda_stream


def _check_batch(dst, src, offsets, keys) -> Tuple[int, int]:
    import torch

    for name, t in (("dst", dst), ("src", src), ("offsets", offsets), ("keys", keys)):
        if not isinstance(t, torch.Tensor):
            raise TypeError(f"{name} must be a torch tensor")
        if not t.is_cuda:
            raise ValueError(f"{name} must be a device tensor")
        if not t.is_contiguous():
            raise ValueError(f"{name} must be contiguous")
    if src.dtype != torch.uint8 or dst.dtype != torch.uint8:
        raise TypeError("payload tensors must be uint8")
    if offsets.dtype not in (torch.int64, torch.uint64):
        raise TypeError("offsets must be int64 (uint64 bit pattern)")
    if keys.dtype not in (torch.int32, torch.uint32):
        raise TypeError("keys must be int32 (packed key32 bit pattern)")
    if dst.numel() != src.numel():
        raise ValueError("dst and src sizes differ")
    n = keys.numel()
    if offsets.numel() != n + 1:
        raise ValueError(f"offsets must have nframes + 1 = {n + 1} entries, got {offsets.numel()}")
    return src.numel(), n


def mask_batch(dst, src, offsets, keys, stream=None, device: Optional[int] = None) -> None:
    """netc_gpu_mask_batch on the tensors' device, queued on `stream` (default: torch's current stream)."""
    total, n = _check_batch(dst, src, offsets, keys)
    dev = src.device.index if device is None else device
    _check(_lib.gpu().netc_gpu_mask_batch(dev, dst.data_ptr(), src.data_ptr(), total, offsets.data_ptr(),
                                          keys.data_ptr(), n, _stream_handle(stream)))


def unmask_validate(dst, src, offsets, keys, header0, valid, stream=None, device: Optional[int] = None) -> None:
    """netc_gpu_unmask_validate: mask_batch plus per-frame UTF-8 verdicts of the TEXT messages (valid: uint8, n)."""
    import torch

    total, n = _check_batch(dst, src, offsets, keys)
    for name, t in (("header0", header0), ("valid", valid)):
        if not isinstance(t, torch.Tensor) or not t.is_cuda or t.dtype != torch.uint8 or t.numel() != n:
            raise ValueError(f"{name} must be a device uint8 tensor of nframes entries")
    dev = src.device.index if device is None else device
    _check(_lib.gpu().netc_gpu_unmask_validate(dev, dst.data_ptr(), src.data_ptr(), total, offsets.data_ptr(),
                                               keys.data_ptr(), header0.data_ptr(), n, valid.data_ptr(),
                                               _stream_handle(stream)))


def mask_batch_multi(shards: Sequence[Tuple], streams: Optional[Sequence] = None, synchronize: bool = True) -> None:
    """netc_gpu_mask_batch_multi: shards = [(dst, src, offsets, keys), ...], each on its own device."""
    k = len(shards)
    devs = (ctypes.c_int * k)()
    dsts = (ctypes.c_void_p * k)()
    srcs = (ctypes.c_void_p * k)()
    totals = (ctypes.c_size_t * k)()
    offs = (ctypes.c_void_p * k)()
    keys = (ctypes.c_void_p * k)()
    ns = (ctypes.c_size_t * k)()
    strs = (ctypes.c_void_p * k)()
    for i, (d, s, o, kk) in enumerate(shards):
        total, n = _check_batch(d, s, o, kk)
        devs[i] = s.device.index
        dsts[i], srcs[i], offs[i], keys[i] = d.data_ptr(), s.data_ptr(), o.data_ptr(), kk.data_ptr()
        totals[i], ns[i] = total, n
        strs[i] = streams[i].cuda_stream if streams else None
    _check(_lib.gpu().netc_gpu_mask_batch_multi(k, devs, dsts, srcs, totals, offs, keys, ns,
                                                strs if streams else None, 1 if synchronize else 0))


def wire_bound(total: int, nframes: int, masked: bool) -> int:
    """NETC_WS_WIRE_BOUND: capacity netc_gpu_encode_frames needs for the wire buffer."""
    return int(total) + int(nframes) * (14 if masked else 10)


def wire_size(offsets: np.ndarray, masked: bool) -> int:
    """netc_ws_wire_size: exact wire bytes of the frames described by host offsets."""
    off = np.ascontiguousarray(offsets, dtype=np.uint64)
    return int(_lib.host().netc_ws_wire_size(_ptr(off), off.size - 1, 1 if masked else 0))


# include/ws/frame.h: length classes of netc_gpu_encode_frames_class (extended-length bytes)
NETC_WS_CLASS_7BIT, NETC_WS_CLASS_16BIT, NETC_WS_CLASS_64BIT = 0, 2, 8
NETC_WS_WIRE_INVALID = (1 << 64) - 1


def length_class(offsets: np.ndarray) -> Optional[int]:
    """The one NETC_WS_CLASS_* every frame of host offsets lies in, or None when they are mixed."""
    ln = np.diff(np.asarray(offsets, dtype=np.uint64))
    if ln.size == 0:
        return None
    cls = np.where(ln <= 125, 0, np.where(ln <= 0xFFFF, 2, 8))
    return int(cls[0]) if (cls == cls[0]).all() else None


def encode_frames(wire, wire_offsets, src, offsets, keys=None, header0=None, masked: bool = True, stream=None,
                  device: Optional[int] = None, length_class: Optional[int] = None) -> None:
    """netc_gpu_encode_frames: headers + keys + masked payloads of every frame into `wire` (device tensors).

    wire: uint8, >= wire_bound(src.numel(), n, masked) bytes; wire_offsets: int64, n + 1 (output);
    header0: uint8 per frame (FIN | RSV | opcode) or None for 0x82; keys: packed key32 (masked only).
    length_class: a NETC_WS_CLASS_* every frame lies in, as the caller promises
    (netc_gpu_encode_frames_class: one launch; wire_offsets[n] reads NETC_WS_WIRE_INVALID after
    the call when a frame breaks it), or None.
    """
    import torch

    n = offsets.numel() - 1
    for name, t in (("wire", wire), ("wire_offsets", wire_offsets), ("src", src), ("offsets", offsets)):
        if not isinstance(t, torch.Tensor) or not t.is_cuda or not t.is_contiguous():
            raise ValueError(f"{name} must be a contiguous device tensor")
    if wire.dtype != torch.uint8 or src.dtype != torch.uint8:
        raise TypeError("wire and src must be uint8")
    if offsets.dtype not in (torch.int64, torch.uint64) or wire_offsets.dtype not in (torch.int64, torch.uint64):
        raise TypeError("offsets and wire_offsets must be int64")
    if wire_offsets.numel() != n + 1:
        raise ValueError("wire_offsets must have nframes + 1 entries")
    kp = 0
    if masked:
        if keys is None or keys.numel() != n or keys.dtype not in (torch.int32, torch.uint32):
            raise ValueError("masked frames need nframes int32 keys")
        kp = keys.data_ptr()
    hp = 0
    if header0 is not None:
        if header0.numel() != n or header0.dtype != torch.uint8:
            raise ValueError("header0 must be nframes uint8")
        hp = header0.data_ptr()
    dev = src.device.index if device is None else device
    if length_class is None:
        _check(_lib.gpu().netc_gpu_encode_frames(dev, wire.data_ptr(), wire.numel(), wire_offsets.data_ptr(),
                                                 src.data_ptr(), src.numel(), offsets.data_ptr(), kp, hp, n,
                                                 1 if masked else 0, _stream_handle(stream)))
    else:
        _check(_lib.gpu().netc_gpu_encode_frames_class(dev, wire.data_ptr(), wire.numel(), wire_offsets.data_ptr(),
                                                       src.data_ptr(), src.numel(), offsets.data_ptr(), kp, hp, n,
                                                       1 if masked else 0, int(length_class),
                                                       _stream_handle(stream)))


NETC_WS_SCAN_STRICT = 1


def scan_frames(wire, hdr, keys, b0, result, start: int = 0, strict: bool = True, length: Optional[int] = None,
                stream=None, device: Optional[int] = None) -> None:
    """netc_gpu_scan_frames: frame boundaries of the device stream `wire` (uint8 tensor).

    hdr: int64 (max_frames + 1), keys: int32 (max_frames), b0: uint8 (max_frames), result: int64 (3)
    receives [frames, consumed, error offset or -1 (UINT64_MAX)].  Asynchronous on `stream`.
    """
    n = wire.numel() if length is None else int(length)
    max_frames = hdr.numel() - 1
    if keys.numel() < max_frames or b0.numel() < max_frames or result.numel() < 3:
        raise ValueError("output tensors too small")
    dev = wire.device.index if device is None else device
    _check(_lib.gpu().netc_gpu_scan_frames(dev, wire.data_ptr(), n, start, NETC_WS_SCAN_STRICT if strict else 0,
                                           hdr.data_ptr(), keys.data_ptr(), b0.data_ptr(), max_frames,
                                           result.data_ptr(), _stream_handle(stream)))


def scan_frames_host(wire: np.ndarray, max_frames: int, start: int = 0, strict: bool = True,
                     length: Optional[int] = None):
    """netc_ws_scan_frames_host (libnetc.so): the same scan over a host uint8 array, on this thread.

    Returns (hdr uint64 [max_frames + 1], keys uint32 [max_frames], b0 uint8 [max_frames],
    result uint64 [3] = frames, consumed, error offset or UINT64_MAX).
    """
    w = np.ascontiguousarray(wire, dtype=np.uint8)
    n = w.size if length is None else int(length)
    if n > w.size:
        raise ValueError("length past the array")
    hdr = np.zeros(max_frames + 1, np.uint64)
    keys = np.zeros(max(max_frames, 1), np.uint32)
    b0 = np.zeros(max(max_frames, 1), np.uint8)
    res = np.zeros(3, np.uint64)
    _check(_lib.host().netc_ws_scan_frames_host(w.ctypes.data, n, start, NETC_WS_SCAN_STRICT if strict else 0,
                                                hdr.ctypes.data, keys.ctypes.data, b0.ctypes.data, max_frames,
                                                res.ctypes.data))
    return hdr, keys[:max_frames], b0[:max_frames], res


def scan_diag(stream=None, device: int = 0) -> int:
    """netc_gpu_scan_diag: why the last scan on `stream` took the serial walk (0: it did not; -1: no scan)."""
    r = int(_lib.gpu().netc_gpu_scan_diag(device, _stream_handle(stream)))
    if r < -1:
        _check(r)
    return r if r < 0 else r & 0xFFFFFFFF


def scan_onepass(stream=None, device: int = 0) -> bool:
    """bit 32 of netc_gpu_scan_diag: the last scan on `stream` finished on its one-pass path"""
    r = int(_lib.gpu().netc_gpu_scan_diag(device, _stream_handle(stream)))
    if r < -1:
        _check(r)
    return r >= 0 and bool((r >> 32) & 1)


def unmask_frames(wire, hdr, keys, result, length: Optional[int] = None, stream=None,
                  device: Optional[int] = None) -> None:
    """netc_gpu_unmask_frames: unmask in place the payloads scan_frames found (outputs read on the device)."""
    n = wire.numel() if length is None else int(length)
    dev = wire.device.index if device is None else device
    _check(_lib.gpu().netc_gpu_unmask_frames(dev, wire.data_ptr(), n, hdr.data_ptr(), keys.data_ptr(),
                                             hdr.numel() - 1, result.data_ptr(), _stream_handle(stream)))


def mask_stream_host(dst: np.ndarray, src: np.ndarray, offsets: np.ndarray, keys: np.ndarray,
                     slot_bytes: int = 512 << 20, nslots: int = 2, device: int = 0) -> None:
    """netc_gpu_mask_stream_host: host buffers through device slots on overlapped streams."""
    off, kk = _host_frames(dst, src, offsets, keys)
    _check(_lib.gpu().netc_gpu_mask_stream_host(device, _ptr(dst), _ptr(src), src.size, _ptr(off), _ptr(kk),
                                                kk.size, slot_bytes, nslots))


def _host_frames(dst, src, offsets, keys):
    off = np.ascontiguousarray(offsets, dtype=np.uint64)
    kk = np.ascontiguousarray(keys, dtype=np.uint32)
    if src.dtype != np.uint8 or dst.dtype != np.uint8 or dst.size != src.size:
        raise ValueError("dst/src must be uint8 arrays of equal size")
    if off.size != kk.size + 1:
        raise ValueError("offsets must have nframes + 1 entries")
    return off, kk


class HostStream:
    """netc_gpu_stream_*: the config-5 pipeline with its slots kept across calls (include/ws/mask.h)."""

    def __init__(self, device: int = 0, slot_bytes: int = 0, nslots: int = 0):
        h = ctypes.c_void_p()
        _check(_lib.gpu().netc_gpu_stream_create(ctypes.byref(h), device, slot_bytes, nslots))
        self._h = h

    def mask(self, dst: np.ndarray, src: np.ndarray, offsets: np.ndarray, keys: np.ndarray) -> None:
        if self._h is None:
            raise ValueError("stream handle destroyed")
        off, kk = _host_frames(dst, src, offsets, keys)
        _check(_lib.gpu().netc_gpu_stream_mask(self._h, _ptr(dst), _ptr(src), src.size, _ptr(off), _ptr(kk),
                                               kk.size))

    def close(self) -> None:
        if self._h is not None:
            _lib.gpu().netc_gpu_stream_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class PinnedArray:
    """A uint8 numpy view of netc_gpu_host_alloc memory (page-locked); freed by close()."""

    def __init__(self, nbytes: int):
        p = _lib.gpu().netc_gpu_host_alloc(nbytes)
        if not p:
            raise NetcGpuError(NETC_GPU_ENOMEM, _lib.gpu().netc_gpu_strerror().decode())
        self._p = p
        self.array = np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(p)) if nbytes else \
            np.zeros(0, dtype=np.uint8)

    def close(self) -> None:
        if self._p:
            self.array = None
            _lib.gpu().netc_gpu_host_free(self._p)
            self._p = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
