"""Python mirror of the socket-ingest C-ABI (include/ws/ingest.h).

Same names, argument meaning and error behaviour as the C entry points: an
:class:`Ingest` owns one ring (netc_ws_ingest_create), ``recv`` / ``write`` /
``submit`` feed it, ``next`` hands out :class:`Batch` objects whose arrays are
views into the ring's pinned memory (valid until ``release``).  Failing calls
raise :class:`netc_amd.mask.NetcGpuError` with the negative code; the stream
conditions CLOSED / FULL come back as return values, as in C.
"""

from __future__ import annotations

import ctypes
from typing import Optional, Tuple

import numpy as np

from . import _lib
from .mask import NetcGpuError

NETC_WS_INGEST_STRICT = 1
NETC_WS_INGEST_SCAN_GPU = 2
NETC_WS_INGEST_SCAN_HOST = 4
_SCAN_FLAGS = {"auto": 0, "gpu": NETC_WS_INGEST_SCAN_GPU, "host": NETC_WS_INGEST_SCAN_HOST}
NETC_WS_INGEST_CLOSED = -20
NETC_WS_INGEST_FULL = -21
NETC_WS_INGEST_TOO_BIG = -22
NETC_WS_INGEST_PROTOCOL = -23
NETC_WS_INGEST_ERECV = -24


class WsMessage(ctypes.Structure):
    """struct ws_message (include/ws/common.h): opcode, buffer (malloc'd, caller frees), payload_length."""
    _fields_ = [("opcode", ctypes.c_uint8), ("buffer", ctypes.c_void_p), ("payload_length", ctypes.c_size_t)]


WS_FRAME_PARSE_ERROR_RECV = -1
WS_FRAME_PARSE_ERROR_INVALID_FRAME_LENGTH = -2
WS_FRAME_PARSE_ERROR_PAYLOAD_TOO_BIG = -3
_libc = ctypes.CDLL(None)
_libc.free.argtypes = [ctypes.c_void_p]
_libc.free.restype = None


class _RawBatch(ctypes.Structure):
    _fields_ = [("wire", ctypes.c_void_p), ("len", ctypes.c_uint64), ("hdr", ctypes.c_void_p),
                ("keys", ctypes.c_void_p), ("b0", ctypes.c_void_p), ("nframes", ctypes.c_uint64),
                ("stream_offset", ctypes.c_uint64), ("slot", ctypes.c_int32)]


def _bind(lib):
    if getattr(lib, "_ingest_bound", False):
        return lib
    vp, sz = ctypes.c_void_p, ctypes.c_size_t
    lib.netc_ws_ingest_create.argtypes = [ctypes.POINTER(vp), ctypes.c_int, sz, ctypes.c_int, sz, ctypes.c_int]
    lib.netc_ws_ingest_create.restype = ctypes.c_int
    lib.netc_ws_ingest_destroy.argtypes = [vp]
    lib.netc_ws_ingest_destroy.restype = None
    lib.netc_ws_ingest_recv.argtypes = [vp, ctypes.c_int]
    lib.netc_ws_ingest_recv.restype = ctypes.c_long
    lib.netc_ws_ingest_write.argtypes = [vp, vp, sz]
    lib.netc_ws_ingest_write.restype = ctypes.c_long
    lib.netc_ws_ingest_submit.argtypes = [vp]
    lib.netc_ws_ingest_submit.restype = ctypes.c_int
    lib.netc_ws_ingest_next.argtypes = [vp, ctypes.POINTER(_RawBatch), ctypes.c_int]
    lib.netc_ws_ingest_next.restype = ctypes.c_int
    lib.netc_ws_ingest_release.argtypes = [vp, ctypes.POINTER(_RawBatch)]
    lib.netc_ws_ingest_release.restype = ctypes.c_int
    lib.netc_ws_batch_payload.argtypes = [ctypes.POINTER(_RawBatch), ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64),
                                          ctypes.POINTER(ctypes.c_uint64)]
    lib.netc_ws_batch_payload.restype = ctypes.c_int
    lib.netc_ws_ingest_next_message.argtypes = [vp, ctypes.POINTER(WsMessage), sz, ctypes.c_int]
    lib.netc_ws_ingest_next_message.restype = ctypes.c_int
    lib.netc_ws_ingest_scan_counts.argtypes = [vp, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]
    lib.netc_ws_ingest_scan_counts.restype = ctypes.c_int
    lib.netc_ws_gpu_attach.argtypes = [ctypes.c_int, vp]
    lib.netc_ws_gpu_attach.restype = ctypes.c_int
    lib.netc_ws_gpu_detach.argtypes = [ctypes.c_int]
    lib.netc_ws_gpu_detach.restype = ctypes.c_int
    lib._ingest_bound = True
    return lib


def _raise(rc: int, lib=None):
    lib = lib if lib is not None else _lib.gpu()
    lib.netc_gpu_strerror.restype = ctypes.c_char_p
    msg = lib.netc_gpu_strerror()
    raise NetcGpuError(rc, msg.decode(errors="replace") if msg else "")


def _view(ptr: int, n: int, dtype) -> np.ndarray:
    dt = np.dtype(dtype)
    if n == 0 or not ptr:
        return np.zeros(0, dtype=dt)
    return np.frombuffer((ctypes.c_char * (n * dt.itemsize)).from_address(ptr), dtype=dt)


class Batch:
    """A delivered batch: ``wire`` (payloads unmasked), ``hdr`` (nframes + 1), ``keys``, ``b0``,
    ``stream_offset`` -- numpy views into pinned memory, valid until :meth:`release`."""

    def __init__(self, owner: "Ingest", raw: _RawBatch):
        self._owner, self._raw = owner, raw
        self.nframes = int(raw.nframes)
        self.stream_offset = int(raw.stream_offset)
        self.wire = _view(raw.wire, int(raw.len), np.uint8)
        self.hdr = _view(raw.hdr, self.nframes + 1, np.uint64)
        self.keys = _view(raw.keys, self.nframes, np.uint32)
        self.b0 = _view(raw.b0, self.nframes, np.uint8)

    def payload(self, k: int) -> Tuple[int, int]:
        """netc_ws_batch_payload: (offset into wire, length) of frame k's payload."""
        o, n = ctypes.c_uint64(0), ctypes.c_uint64(0)
        rc = self._owner._lib.netc_ws_batch_payload(ctypes.byref(self._raw), k, ctypes.byref(o), ctypes.byref(n))
        if rc:
            raise NetcGpuError(rc, f"frame {k} not in the batch")
        return int(o.value), int(n.value)

    def release(self) -> None:
        if self._raw is not None:
            rc = self._owner._lib.netc_ws_ingest_release(self._owner._h, ctypes.byref(self._raw))
            self._raw = None
            if rc:
                _raise(rc, self._owner._lib)


class Ingest:
    """netc_ws_ingest_*: one connection's byte stream -> pinned slots -> GPU scan + unmask -> batches."""

    def __init__(self, device: int = 0, slot_bytes: int = 16 << 20, nslots: int = 4, max_frame_bytes: int = 65536,
                 strict: bool = False, scan: str = "auto", lib=None):
        """scan: "auto" (per slot by frame size, the C default), "gpu" or "host" (NETC_WS_INGEST_SCAN_*).
        lib: the library holding the ring (default libnetc_ws_gpu.so; the CPU tests pass the ring's host
        code built over a mock HIP runtime, tests/mockhip)."""
        if scan not in _SCAN_FLAGS:
            raise ValueError(f"scan must be one of {sorted(_SCAN_FLAGS)}")
        lib = _bind(lib if lib is not None else _lib.gpu())
        h = ctypes.c_void_p(0)
        rc = lib.netc_ws_ingest_create(ctypes.byref(h), device, slot_bytes, nslots, max_frame_bytes,
                                       (NETC_WS_INGEST_STRICT if strict else 0) | _SCAN_FLAGS[scan])
        if rc:
            _raise(rc, lib)
        self._lib, self._h = lib, h

    def scan_counts(self) -> Tuple[int, int]:
        """netc_ws_ingest_scan_counts: (slots the GPU scan framed, slots the host walk framed)."""
        g, h = ctypes.c_uint64(0), ctypes.c_uint64(0)
        rc = self._lib.netc_ws_ingest_scan_counts(self._h, ctypes.byref(g), ctypes.byref(h))
        if rc:
            _raise(rc, self._lib)
        return int(g.value), int(h.value)

    def recv(self, fd: int) -> int:
        """netc_ws_ingest_recv: bytes read (> 0), 0 (would block), CLOSED or FULL; raises on other errors."""
        r = self._lib.netc_ws_ingest_recv(self._h, fd)
        if r < 0 and r not in (NETC_WS_INGEST_CLOSED, NETC_WS_INGEST_FULL):
            _raise(int(r), self._lib)
        return int(r)

    def write(self, data) -> int:
        """netc_ws_ingest_write: bytes taken (fewer than given when the ring is full), or FULL."""
        buf = np.ascontiguousarray(np.frombuffer(data, dtype=np.uint8) if isinstance(data, (bytes, bytearray))
                                   else data, dtype=np.uint8)
        r = self._lib.netc_ws_ingest_write(self._h, buf.ctypes.data if buf.size else None, buf.size)
        if r < 0 and r != NETC_WS_INGEST_FULL:
            _raise(int(r), self._lib)
        return int(r)

    def submit(self) -> None:
        rc = self._lib.netc_ws_ingest_submit(self._h)
        if rc:
            _raise(rc, self._lib)

    def next(self, wait: bool = True) -> Optional[Batch]:
        """netc_ws_ingest_next: the oldest finished batch, or None; raises a stream error once it is due."""
        raw = _RawBatch()
        rc = self._lib.netc_ws_ingest_next(self._h, ctypes.byref(raw), 1 if wait else 0)
        if rc < 0:
            _raise(rc, self._lib)
        return Batch(self, raw) if rc == 1 else None

    def next_message(self, max_payload_length: int = (1 << 64) - 1, wait: bool = True):
        """netc_ws_ingest_next_message: (0, opcode, payload bytes) for a complete message (the C
        buffer is copied and freed here; a TEXT payload ends with the NUL the contract appends),
        (1, None, None) when more data is needed, or (code, None, None) for a
        WS_FRAME_PARSE_ERROR_* code -- the same 0 / 1 / < 0 contract as ws_parse_frame.
        Device / runtime failures (NETC_GPU_E*) raise."""
        m = WsMessage()
        rc = self._lib.netc_ws_ingest_next_message(self._h, ctypes.byref(m), max_payload_length, 1 if wait else 0)
        if rc == 0:
            data = ctypes.string_at(m.buffer, m.payload_length) if m.payload_length else b""
            _libc.free(m.buffer)
            return 0, int(m.opcode), data
        if rc in (1, WS_FRAME_PARSE_ERROR_RECV, WS_FRAME_PARSE_ERROR_INVALID_FRAME_LENGTH,
                  WS_FRAME_PARSE_ERROR_PAYLOAD_TOO_BIG):
            return rc, None, None
        _raise(rc, self._lib)

    def attach(self, sockfd: int) -> None:
        """netc_ws_gpu_attach: libnetc's ws_parse_frame on sockfd is served from this ring (one
        ring, one connection; a ring that has carried a stream cannot be attached)."""
        rc = self._lib.netc_ws_gpu_attach(sockfd, self._h)
        if rc:
            _raise(rc, self._lib)

    def detach(self, sockfd: int) -> None:
        rc = self._lib.netc_ws_gpu_detach(sockfd)
        if rc:
            _raise(rc, self._lib)

    def close(self) -> None:
        if self._h:
            self._lib.netc_ws_ingest_destroy(self._h)
            self._h = ctypes.c_void_p(0)

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
