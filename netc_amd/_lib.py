"""Loads the in-tree C-ABI libraries and declares their signatures (include/ws/mask.h).

Fails loudly: a missing or unloadable library raises ImportError-like
``RuntimeError`` with the path and the reason -- there is no fallback path.
"""

from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIBDIR = os.path.join(_HERE, "lib")
HOST_LIB = os.path.join(LIBDIR, "libnetc.so")
GPU_LIB = os.path.join(LIBDIR, "libnetc_ws_gpu.so")
# instrumented builds of the same libraries: NETC_HOST_LIB (`make asan`: ASan + UBSan),
# NETC_GPU_LIB (tools/: stamps, checks)
if os.environ.get("NETC_HOST_LIB"):
    HOST_LIB = os.path.abspath(os.environ["NETC_HOST_LIB"])
if os.environ.get("NETC_GPU_LIB"):
    GPU_LIB = os.path.abspath(os.environ["NETC_GPU_LIB"])

_lock = threading.Lock()
_host = None
_gpu = None

c_u8p = ctypes.POINTER(ctypes.c_uint8)
c_u64p = ctypes.POINTER(ctypes.c_uint64)
c_u32p = ctypes.POINTER(ctypes.c_uint32)
c_sizep = ctypes.POINTER(ctypes.c_size_t)


def _load(path: str) -> ctypes.CDLL:
    if not os.path.exists(path):
        raise RuntimeError(f"netc_amd: {path} is missing -- run `make` (or __graft_entry__.build()) first")
    try:
        return ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
    except OSError as e:  # pragma: no cover - message passthrough
        raise RuntimeError(f"netc_amd: cannot load {path}: {e}") from e


def host() -> ctypes.CDLL:
    """libnetc.so: framing API + CPU mask + shard planner."""
    global _host
    with _lock:
        if _host is None:
            lib = _load(HOST_LIB)
            lib.netc_ws_mask.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t]
            lib.netc_ws_mask.restype = None
            lib.netc_shard_frames.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_void_p]
            lib.netc_shard_frames.restype = ctypes.c_int
            lib.netc_ws_wire_size.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
            lib.netc_ws_wire_size.restype = ctypes.c_uint64
            lib.ws_build_masking_key.argtypes = [ctypes.c_void_p]
            lib.ws_build_masking_key.restype = None
            lib.ws_build_message.argtypes = [ctypes.c_void_p, ctypes.c_uint8, ctypes.c_uint64, ctypes.c_void_p]
            lib.ws_build_message.restype = None
            lib.ws_send_message.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
            lib.ws_send_message.restype = ctypes.c_int
            lib.ws_parse_frame.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
            lib.ws_parse_frame.restype = ctypes.c_int
            lib.netc_ws_scan_frames_host.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_int,
                                                     ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                                     ctypes.c_void_p]
            lib.netc_ws_scan_frames_host.restype = ctypes.c_int
            _host = lib
        return _host


def gpu() -> ctypes.CDLL:
    """libnetc_ws_gpu.so: the gfx950 batch entries.

    torch is imported first so that the HIP runtime torch ships (same SONAME,
    libamdhip64.so.7) is the one this library binds to -- one runtime per process.
    """
    global _gpu
    import torch  # noqa: F401  (see docstring)

    host()
    with _lock:
        if _gpu is None:
            lib = _load(GPU_LIB)
            vp = ctypes.c_void_p
            lib.netc_gpu_device_count.argtypes = []
            lib.netc_gpu_device_count.restype = ctypes.c_int
            lib.netc_gpu_init.argtypes = [ctypes.c_int]
            lib.netc_gpu_init.restype = ctypes.c_int
            lib.netc_gpu_strerror.argtypes = []
            lib.netc_gpu_strerror.restype = ctypes.c_char_p
            lib.netc_gpu_tune.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int]
            lib.netc_gpu_tune.restype = ctypes.c_int
            lib.netc_gpu_mask_batch.argtypes = [ctypes.c_int, vp, vp, ctypes.c_size_t, vp, vp, ctypes.c_size_t, vp]
            lib.netc_gpu_mask_batch.restype = ctypes.c_int
            lib.netc_gpu_mask_batch_multi.argtypes = [ctypes.c_int, vp, vp, vp, vp, vp, vp, vp, vp, ctypes.c_int]
            lib.netc_gpu_mask_batch_multi.restype = ctypes.c_int
            lib.netc_gpu_mask_stream_host.argtypes = [ctypes.c_int, vp, vp, ctypes.c_size_t, vp, vp, ctypes.c_size_t,
                                                      ctypes.c_size_t, ctypes.c_int]
            lib.netc_gpu_mask_stream_host.restype = ctypes.c_int
            lib.netc_gpu_stream_create.argtypes = [vp, ctypes.c_int, ctypes.c_size_t, ctypes.c_int]
            lib.netc_gpu_stream_create.restype = ctypes.c_int
            lib.netc_gpu_stream_mask.argtypes = [vp, vp, vp, ctypes.c_size_t, vp, vp, ctypes.c_size_t]
            lib.netc_gpu_stream_mask.restype = ctypes.c_int
            lib.netc_gpu_stream_destroy.argtypes = [vp]
            lib.netc_gpu_stream_destroy.restype = None
            lib.netc_gpu_host_alloc.argtypes = [ctypes.c_size_t]
            lib.netc_gpu_host_alloc.restype = vp
            lib.netc_gpu_host_free.argtypes = [vp]
            lib.netc_gpu_host_free.restype = None
            lib.netc_gpu_encode_frames.argtypes = [ctypes.c_int, vp, ctypes.c_size_t, vp, vp, ctypes.c_size_t, vp, vp,
                                                   vp, ctypes.c_size_t, ctypes.c_int, vp]
            lib.netc_gpu_encode_frames.restype = ctypes.c_int
            lib.netc_gpu_encode_frames_class.argtypes = [ctypes.c_int, vp, ctypes.c_size_t, vp, vp, ctypes.c_size_t,
                                                         vp, vp, vp, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, vp]
            lib.netc_gpu_encode_frames_class.restype = ctypes.c_int
            lib.netc_gpu_scan_frames.argtypes = [ctypes.c_int, vp, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_int, vp,
                                                 vp, vp, ctypes.c_size_t, vp, vp]
            lib.netc_gpu_scan_frames.restype = ctypes.c_int
            lib.netc_gpu_scan_release.argtypes = [ctypes.c_int, vp]
            lib.netc_gpu_scan_release.restype = ctypes.c_int
            lib.netc_gpu_stream_release.argtypes = [ctypes.c_int, vp]
            lib.netc_gpu_stream_release.restype = ctypes.c_int
            lib.netc_gpu_knob.argtypes = [ctypes.c_int, ctypes.c_int64]
            lib.netc_gpu_knob.restype = ctypes.c_int
            lib.netc_gpu_scan_diag.argtypes = [ctypes.c_int, vp]
            lib.netc_gpu_scan_diag.restype = ctypes.c_int64
            lib.netc_gpu_unmask_frames.argtypes = [ctypes.c_int, vp, ctypes.c_size_t, vp, vp, ctypes.c_size_t, vp, vp]
            lib.netc_gpu_unmask_frames.restype = ctypes.c_int
            lib.netc_gpu_unmask_validate.argtypes = [ctypes.c_int, vp, vp, ctypes.c_size_t, vp, vp, vp,
                                                     ctypes.c_size_t, vp, vp]
            lib.netc_gpu_unmask_validate.restype = ctypes.c_int
            _gpu = lib
        return _gpu
