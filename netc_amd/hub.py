"""Python mirror of the shared rings' C-ABI: receive (include/ws/hub.h) and send (include/ws/egress_hub.h).

A :class:`Hub` owns one hub (netc_ws_hub_create); ``attach`` / ``detach`` put a socket's
ws_parse_frame behind it (netc_ws_gpu_attach_hub / _detach_hub); ``stats`` reads its counters.
Failing calls raise :class:`netc_amd.mask.NetcGpuError` with the negative code, as in C.
"""

from __future__ import annotations

import ctypes

from . import _lib
from .mask import NetcGpuError

NETC_WS_INGEST_STRICT = 1


class HubStats(ctypes.Structure):
    _fields_ = [("launches", ctypes.c_uint64), ("frames", ctypes.c_uint64), ("bytes", ctypes.c_uint64),
                ("max_connections", ctypes.c_uint64), ("connection_slots", ctypes.c_uint64),
                ("connections", ctypes.c_uint64)]


def _bind(lib):
    if getattr(lib, "_hub_bound", False):
        return lib
    vp, sz = ctypes.c_void_p, ctypes.c_size_t
    lib.netc_ws_hub_create.argtypes = [ctypes.POINTER(vp), ctypes.c_int, sz, ctypes.c_int, sz, ctypes.c_int]
    lib.netc_ws_hub_create.restype = ctypes.c_int
    lib.netc_ws_hub_destroy.argtypes = [vp]
    lib.netc_ws_hub_destroy.restype = None
    lib.netc_ws_gpu_attach_hub.argtypes = [ctypes.c_int, vp]
    lib.netc_ws_gpu_attach_hub.restype = ctypes.c_int
    lib.netc_ws_gpu_detach_hub.argtypes = [ctypes.c_int]
    lib.netc_ws_gpu_detach_hub.restype = ctypes.c_int
    lib.netc_ws_hub_stats.argtypes = [vp, ctypes.POINTER(HubStats)]
    lib.netc_ws_hub_stats.restype = ctypes.c_int
    lib.netc_gpu_strerror.restype = ctypes.c_char_p
    lib._hub_bound = True
    return lib


class Hub:
    """netc_ws_hub_*: one GPU receive ring serving many connections' ws_parse_frame."""

    def __init__(self, device: int = 0, slot_bytes: int = 16 << 20, nslots: int = 8, max_frame_bytes: int = 65536,
                 strict: bool = False, lib=None):
        """lib: the library holding the hub (default libnetc_ws_gpu.so; the CPU tests pass the host
        code built over a mock HIP runtime, tests/mockhip)."""
        lib = _bind(lib if lib is not None else _lib.gpu())
        h = ctypes.c_void_p(0)
        rc = lib.netc_ws_hub_create(ctypes.byref(h), device, slot_bytes, nslots, max_frame_bytes,
                                    NETC_WS_INGEST_STRICT if strict else 0)
        if rc:
            self._raise(rc, lib)
        self._lib, self._h = lib, h

    @staticmethod
    def _raise(rc, lib):
        msg = lib.netc_gpu_strerror()
        raise NetcGpuError(rc, msg.decode(errors="replace") if msg else "")

    def attach(self, sockfd: int) -> None:
        rc = self._lib.netc_ws_gpu_attach_hub(sockfd, self._h)
        if rc:
            self._raise(rc, self._lib)

    def detach(self, sockfd: int) -> None:
        rc = self._lib.netc_ws_gpu_detach_hub(sockfd)
        if rc:
            self._raise(rc, self._lib)

    def stats(self) -> dict:
        st = HubStats()
        rc = self._lib.netc_ws_hub_stats(self._h, ctypes.byref(st))
        if rc:
            self._raise(rc, self._lib)
        return {name: int(getattr(st, name)) for name, _ in HubStats._fields_}

    def close(self) -> None:
        if self._h:
            self._lib.netc_ws_hub_destroy(self._h)
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


# ------------------------------------------------------------------ the send side --
# include/ws/egress_hub.h: one GPU send ring serving many connections' ws_send_message.

class EgressHubStats(ctypes.Structure):
    _fields_ = [("launches", ctypes.c_uint64), ("messages", ctypes.c_uint64), ("frames", ctypes.c_uint64),
                ("wire_bytes", ctypes.c_uint64), ("max_connections", ctypes.c_uint64),
                ("connection_slots", ctypes.c_uint64), ("sendmsg_calls", ctypes.c_uint64),
                ("send_errors", ctypes.c_uint64), ("connections", ctypes.c_uint64),
                ("deferred_sends", ctypes.c_uint64), ("pending_bytes", ctypes.c_uint64)]


def _bind_send(lib):
    if getattr(lib, "_egress_hub_bound", False):
        return lib
    vp, sz = ctypes.c_void_p, ctypes.c_size_t
    lib.netc_ws_egress_hub_create.argtypes = [ctypes.POINTER(vp), ctypes.c_int, sz, ctypes.c_int, sz]
    lib.netc_ws_egress_hub_create.restype = ctypes.c_int
    lib.netc_ws_egress_hub_destroy.argtypes = [vp]
    lib.netc_ws_egress_hub_destroy.restype = None
    lib.netc_ws_gpu_attach_send_hub.argtypes = [ctypes.c_int, vp]
    lib.netc_ws_gpu_attach_send_hub.restype = ctypes.c_int
    lib.netc_ws_gpu_detach_send_hub.argtypes = [ctypes.c_int]
    lib.netc_ws_gpu_detach_send_hub.restype = ctypes.c_int
    lib.netc_ws_egress_hub_flush.argtypes = [vp]
    lib.netc_ws_egress_hub_flush.restype = ctypes.c_long
    lib.netc_ws_egress_hub_stats.argtypes = [vp, ctypes.POINTER(EgressHubStats)]
    lib.netc_ws_egress_hub_stats.restype = ctypes.c_int
    lib.netc_ws_egress_hub_pending.argtypes = [vp]
    lib.netc_ws_egress_hub_pending.restype = ctypes.c_long
    lib.netc_gpu_strerror.restype = ctypes.c_char_p
    lib._egress_hub_bound = True
    return lib


class EgressHub:
    """netc_ws_egress_hub_*: ws_send_message of many connections queued into shared slots, one
    frame-assembly launch per slot, sent at ``flush`` (include/ws/egress_hub.h)."""

    def __init__(self, device: int = 0, slot_bytes: int = 16 << 20, nslots: int = 4, max_frames: int = 0, lib=None):
        lib = _bind_send(lib if lib is not None else _lib.gpu())
        h = ctypes.c_void_p(0)
        rc = lib.netc_ws_egress_hub_create(ctypes.byref(h), device, slot_bytes, nslots, max_frames)
        if rc:
            Hub._raise(rc, lib)
        self._lib, self._h = lib, h

    def attach(self, sockfd: int) -> None:
        rc = self._lib.netc_ws_gpu_attach_send_hub(sockfd, self._h)
        if rc:
            Hub._raise(rc, self._lib)

    def detach(self, sockfd: int) -> None:
        rc = self._lib.netc_ws_gpu_detach_send_hub(sockfd)
        if rc:
            Hub._raise(rc, self._lib)

    def flush(self) -> int:
        r = self._lib.netc_ws_egress_hub_flush(self._h)
        if r < 0:
            Hub._raise(int(r), self._lib)
        return int(r)

    def pending(self) -> int:
        """bytes the hub's connections hold in their send backlogs (sockets that were full)"""
        return int(self._lib.netc_ws_egress_hub_pending(self._h))

    def drain(self, timeout: float = 30.0) -> int:
        """flush, then keep flushing until every backlog is on its socket (the peers must be reading);
        bytes flushed by the first call"""
        import time
        sent = self.flush()
        deadline = time.monotonic() + timeout
        while self.pending() > 0:
            if time.monotonic() > deadline:
                raise TimeoutError(f"egress hub: {self.pending()} bytes still held after {timeout} s")
            time.sleep(0.001)
            self.flush()
        return sent

    def stats(self) -> dict:
        st = EgressHubStats()
        rc = self._lib.netc_ws_egress_hub_stats(self._h, ctypes.byref(st))
        if rc:
            Hub._raise(rc, self._lib)
        return {name: int(getattr(st, name)) for name, _ in EgressHubStats._fields_}

    def close(self) -> None:
        if self._h:
            self._lib.netc_ws_egress_hub_destroy(self._h)
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
