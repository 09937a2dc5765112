"""Python mirror of the send-side egress C-ABI (include/ws/egress.h).

Same names, argument meaning and error behaviour as the C entry points: an
:class:`Egress` owns one ring (netc_ws_egress_create); ``queue`` appends a
message (split into frames as ws_send_message splits them), ``submit`` sends the
current slot to the GPU, ``next`` hands out :class:`Wire` objects whose bytes are
a view into the ring's pinned memory (valid until ``release``), ``send`` /
``flush`` put finished slots on a socket.  Failing calls raise
:class:`netc_amd.mask.NetcGpuError` with the negative code; FULL comes back as a
return value, as in C.
"""

from __future__ import annotations

import ctypes
from typing import Optional

import numpy as np

from . import _lib
from .mask import NetcGpuError

NETC_WS_EGRESS_DEFER = 1
NETC_WS_EGRESS_FULL = -30
NETC_WS_EGRESS_TOO_BIG = -31
NETC_WS_EGRESS_ESEND = -32


class _RawWire(ctypes.Structure):
    _fields_ = [("wire", ctypes.c_void_p), ("len", ctypes.c_uint64), ("nframes", ctypes.c_uint64),
                ("nmessages", ctypes.c_uint64), ("slot", ctypes.c_int32)]


def _bind(lib):
    if getattr(lib, "_egress_bound", False):
        return lib
    vp, sz = ctypes.c_void_p, ctypes.c_size_t
    lib.netc_ws_egress_create.argtypes = [ctypes.POINTER(vp), ctypes.c_int, sz, ctypes.c_int, sz, ctypes.c_int]
    lib.netc_ws_egress_create.restype = ctypes.c_int
    lib.netc_ws_egress_destroy.argtypes = [vp]
    lib.netc_ws_egress_destroy.restype = None
    lib.netc_ws_egress_queue.argtypes = [vp, vp, sz, ctypes.c_uint8, vp, sz]
    lib.netc_ws_egress_queue.restype = ctypes.c_int
    lib.netc_ws_egress_submit.argtypes = [vp]
    lib.netc_ws_egress_submit.restype = ctypes.c_int
    lib.netc_ws_egress_next.argtypes = [vp, ctypes.POINTER(_RawWire), ctypes.c_int]
    lib.netc_ws_egress_next.restype = ctypes.c_int
    lib.netc_ws_egress_release.argtypes = [vp, ctypes.POINTER(_RawWire)]
    lib.netc_ws_egress_release.restype = ctypes.c_int
    lib.netc_ws_egress_send.argtypes = [vp, ctypes.c_int, ctypes.c_int]
    lib.netc_ws_egress_send.restype = ctypes.c_long
    lib.netc_ws_egress_flush.argtypes = [vp, ctypes.c_int]
    lib.netc_ws_egress_flush.restype = ctypes.c_long
    lib.netc_ws_gpu_attach_send.argtypes = [ctypes.c_int, vp]
    lib.netc_ws_gpu_attach_send.restype = ctypes.c_int
    lib.netc_ws_gpu_detach_send.argtypes = [ctypes.c_int]
    lib.netc_ws_gpu_detach_send.restype = ctypes.c_int
    lib._egress_bound = True
    return lib


def _raise(rc: int):
    msg = _lib.gpu().netc_gpu_strerror()
    raise NetcGpuError(rc, msg.decode(errors="replace") if msg else "")


class Wire:
    """A finished slot: ``wire`` (numpy view of the wire bytes in pinned memory, valid until
    :meth:`release`), ``nframes``, ``nmessages``."""

    def __init__(self, owner: "Egress", raw: _RawWire):
        self._owner, self._raw = owner, raw
        self.nframes = int(raw.nframes)
        self.nmessages = int(raw.nmessages)
        n = int(raw.len)
        self.wire = (np.frombuffer((ctypes.c_char * n).from_address(raw.wire), dtype=np.uint8) if n
                     else np.zeros(0, dtype=np.uint8))

    def release(self) -> None:
        if self._raw is not None:
            rc = _lib.gpu().netc_ws_egress_release(self._owner._h, ctypes.byref(self._raw))
            self._raw = None
            if rc:
                _raise(rc)


class Egress:
    """netc_ws_egress_*: messages -> pinned payload slots -> GPU frame assembly -> pinned wire slots."""

    def __init__(self, device: int = 0, slot_bytes: int = 16 << 20, nslots: int = 4, max_frames: int = 0,
                 defer: bool = False):
        lib = _bind(_lib.gpu())
        h = ctypes.c_void_p(0)
        rc = lib.netc_ws_egress_create(ctypes.byref(h), device, slot_bytes, nslots, max_frames,
                                       NETC_WS_EGRESS_DEFER if defer else 0)
        if rc:
            _raise(rc)
        self._lib, self._h = lib, h

    def queue(self, payload, opcode: int = 2, key: Optional[bytes] = None, num_frames: int = 1) -> int:
        """netc_ws_egress_queue: 0, or FULL (nothing queued); raises on other errors (TOO_BIG ...)."""
        buf = np.ascontiguousarray(np.frombuffer(bytes(payload), dtype=np.uint8)
                                   if isinstance(payload, (bytes, bytearray, memoryview)) else payload,
                                   dtype=np.uint8)
        kb = (ctypes.c_uint8 * 4)(*key) if key is not None else None
        rc = self._lib.netc_ws_egress_queue(self._h, buf.ctypes.data if buf.size else None, buf.size, opcode,
                                            ctypes.cast(kb, ctypes.c_void_p) if kb is not None else None,
                                            num_frames)
        if rc and rc != NETC_WS_EGRESS_FULL:
            _raise(rc)
        return rc

    def submit(self) -> None:
        rc = self._lib.netc_ws_egress_submit(self._h)
        if rc:
            _raise(rc)

    def next(self, wait: bool = True) -> Optional[Wire]:
        raw = _RawWire()
        rc = self._lib.netc_ws_egress_next(self._h, ctypes.byref(raw), 1 if wait else 0)
        if rc < 0:
            _raise(rc)
        return Wire(self, raw) if rc == 1 else None

    def send(self, fd: int, wait: bool = True) -> int:
        r = self._lib.netc_ws_egress_send(self._h, fd, 1 if wait else 0)
        if r < 0:
            _raise(int(r))
        return int(r)

    def flush(self, fd: int) -> int:
        r = self._lib.netc_ws_egress_flush(self._h, fd)
        if r < 0:
            _raise(int(r))
        return int(r)

    def attach(self, sockfd: int) -> None:
        """netc_ws_gpu_attach_send: libnetc's ws_send_message on sockfd goes through this ring."""
        rc = self._lib.netc_ws_gpu_attach_send(sockfd, self._h)
        if rc:
            _raise(rc)

    def detach(self, sockfd: int) -> None:
        rc = self._lib.netc_ws_gpu_detach_send(sockfd)
        if rc:
            _raise(rc)

    def close(self) -> None:
        if self._h:
            self._lib.netc_ws_egress_destroy(self._h)
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
