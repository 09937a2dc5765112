"""ORACLE -- TEST INFRASTRUCTURE ONLY.

ctypes bindings for
  * liboracle.so / liboracle_O0.so -- the plain-C restatement of the reference's
    masking path (ws_oracle.c, every function cites src/ws/common.c lines);
  * _ref/libref_ws.so -- the reference's own src/ws/common.c compiled from
    /root/reference (oracle/Makefile) and driven over a socketpair
    (ref_harness.c).  Present only where it was built; ``ref_available()``.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this
module, as the checker / baseline -- never as the thing measured or shipped.
"""

from __future__ import annotations

import ctypes
import os
from typing import List, Optional, Sequence, Tuple

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_libs = {}

vp = ctypes.c_void_p
sz = ctypes.c_size_t


def _load(name: str) -> ctypes.CDLL:
    if name not in _libs:
        path = os.path.join(_HERE, name)
        if name == "liboracle.so" and os.environ.get("NETC_ORACLE_LIB"):   # `make asan`: instrumented build
            path = os.path.abspath(os.environ["NETC_ORACLE_LIB"])
        if not os.path.exists(path):
            raise RuntimeError(f"oracle: {path} not built (run `make -C oracle`)")
        lib = ctypes.CDLL(path)
        if name.startswith("liboracle"):
            lib.oracle_unmask.argtypes = [vp, sz, vp, ctypes.c_uint64]
            lib.oracle_mask.argtypes = [vp, ctypes.c_uint64, vp]
            lib.oracle_mask_batch.argtypes = [vp, vp, vp, sz]
            lib.oracle_build_masking_key.argtypes = [vp, vp]
            lib.oracle_encode_frame.argtypes = [vp, ctypes.c_int, ctypes.c_uint8, vp, ctypes.c_uint64, vp]
            lib.oracle_encode_frame.restype = sz
            lib.oracle_encode_batch.argtypes = [vp, vp, vp, vp, vp, vp, sz, ctypes.c_int]
            lib.oracle_encode_batch.restype = sz
            lib.oracle_scan_frames.argtypes = [vp, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int, vp, vp, vp, sz,
                                               vp, vp]
            lib.oracle_scan_frames.restype = sz
            lib.oracle_utf8_valid.argtypes = [vp, sz]
            lib.oracle_utf8_valid.restype = ctypes.c_int
            lib.oracle_validate_batch.argtypes = [vp, vp, vp, sz, vp]
            lib.oracle_validate_batch.restype = None
            lib.oracle_decode_message.argtypes = [vp, sz, vp, sz, vp, vp]
            lib.oracle_decode_message.restype = sz
        else:
            lib.ref_parse.argtypes = [vp, sz, vp, sz, sz, vp, sz, vp, vp, sz]
            lib.ref_parse.restype = ctypes.c_long
            lib.ref_send.argtypes = [ctypes.c_uint8, vp, sz, vp, sz, vp, sz]
            lib.ref_send.restype = ctypes.c_long
            lib.ref_key_sequence.argtypes = [sz, vp]
            lib.ref_key_sequence.restype = ctypes.c_int
            lib.ref_receive_timed.argtypes = [vp, sz, sz, ctypes.POINTER(ctypes.c_double)]
            lib.ref_receive_timed.restype = ctypes.c_long
        _libs[name] = lib
    return _libs[name]


def lib(opt: str = "O2") -> ctypes.CDLL:
    return _load("liboracle.so" if opt == "O2" else "liboracle_O0.so")


def _p(a: np.ndarray) -> int:
    return a.ctypes.data


def _u8(x) -> np.ndarray:
    if isinstance(x, (bytes, bytearray, memoryview)):
        return np.frombuffer(bytes(x), dtype=np.uint8).copy()
    return np.ascontiguousarray(x, dtype=np.uint8).copy()


def unmask(buf, key: bytes, phase: int = 0, opt: str = "O2") -> np.ndarray:
    """src/ws/common.c:319-322 on a copy of buf."""
    b = _u8(buf)
    k = np.frombuffer(bytes(key), dtype=np.uint8).copy()
    lib(opt).oracle_unmask(_p(b), b.size, _p(k), phase)
    return b


def mask_batch(buf, offsets: np.ndarray, keys32: np.ndarray, opt: str = "O2") -> np.ndarray:
    """Every frame [off[k], off[k+1]) unmasked from phase 0 with its packed key (copy)."""
    b = _u8(buf)
    off = np.ascontiguousarray(offsets, dtype=np.uint64)
    kk = np.ascontiguousarray(keys32, dtype=np.uint32)
    assert off.size == kk.size + 1
    lib(opt).oracle_mask_batch(_p(b), _p(off), _p(kk), kk.size)
    return b


def mask_batch_inplace(b: np.ndarray, offsets: np.ndarray, keys32: np.ndarray, opt: str = "O2") -> None:
    off = np.ascontiguousarray(offsets, dtype=np.uint64)
    kk = np.ascontiguousarray(keys32, dtype=np.uint32)
    lib(opt).oracle_mask_batch(_p(b), _p(off), _p(kk), kk.size)


def key_sequence(n: int) -> bytes:
    """src/ws/common.c:19-27 from a fresh seed."""
    seed = ctypes.c_int(0)
    out = np.zeros(4 * n, dtype=np.uint8)
    for i in range(n):
        lib().oracle_build_masking_key(out.ctypes.data + 4 * i, ctypes.addressof(seed))
    return out.tobytes()


def encode_frame(payload: bytes, opcode: int, key: Optional[bytes], fin: bool = True) -> bytes:
    p = _u8(payload)
    out = np.zeros(p.size + 14, dtype=np.uint8)
    k = np.frombuffer(bytes(key), dtype=np.uint8).copy() if key is not None else None
    n = lib().oracle_encode_frame(_p(out), 1 if fin else 0, opcode, _p(p), p.size, _p(k) if k is not None else None)
    return out[:n].tobytes()


def encode_batch(payload, offsets: np.ndarray, keys32: Optional[np.ndarray], header0: Optional[np.ndarray] = None,
                 masked: bool = True, opt: str = "O2") -> Tuple[np.ndarray, np.ndarray]:
    """oracle_encode_batch: (wire bytes, n + 1 wire offsets) of a frame batch (include/ws/frame.h)."""
    p = _u8(payload)
    off = np.ascontiguousarray(offsets, dtype=np.uint64)
    n = off.size - 1
    k = np.ascontiguousarray(keys32, dtype=np.uint32) if masked else None
    h = np.ascontiguousarray(header0, dtype=np.uint8) if header0 is not None else None
    out = np.zeros(p.size + 14 * n + 1, dtype=np.uint8)
    wo = np.zeros(n + 1, dtype=np.uint64)
    w = lib(opt).oracle_encode_batch(_p(out), _p(wo), _p(p), _p(off), _p(k) if k is not None else None,
                                     _p(h) if h is not None else None, n, 1 if masked else 0)
    return out[:w], wo


def scan_frames(wire, start: int = 0, strict: bool = True, opt: str = "O2", cap: Optional[int] = None):
    """oracle_scan_frames: (header offsets, packed keys, byte 0s, consumed, error or None) of a byte stream."""
    w = _u8(wire)
    cap = max(1, w.size // 2 + 1) if cap is None else max(1, cap)
    hdr = np.zeros(cap, dtype=np.uint64)
    keys = np.zeros(cap, dtype=np.uint32)
    b0 = np.zeros(cap, dtype=np.uint8)
    consumed = ctypes.c_uint64(0)
    error = ctypes.c_uint64(0)
    n = lib(opt).oracle_scan_frames(_p(w), w.size, start, 1 if strict else 0, _p(hdr), _p(keys), _p(b0), cap,
                                    ctypes.addressof(consumed), ctypes.addressof(error))
    err = None if error.value == (1 << 64) - 1 else int(error.value)
    return hdr[:n], keys[:n], b0[:n], int(consumed.value), err


def utf8_valid(data) -> bool:
    """oracle_utf8_valid: RFC 3629 validity of a byte string."""
    b = _u8(data)
    return bool(lib().oracle_utf8_valid(_p(b) if b.size else None, b.size))


def validate_batch(payload, offsets: np.ndarray, header0: np.ndarray) -> np.ndarray:
    """oracle_validate_batch: per-frame TEXT-message verdicts (0 on the last frame of an invalid message)."""
    p = _u8(payload)
    off = np.ascontiguousarray(offsets, dtype=np.uint64)
    h = np.ascontiguousarray(header0, dtype=np.uint8)
    out = np.zeros(max(1, off.size - 1), dtype=np.uint8)
    lib().oracle_validate_batch(_p(p) if p.size else None, _p(off), _p(h), off.size - 1, _p(out))
    return out[: off.size - 1]


def decode_message(wire: bytes, cap: Optional[int] = None) -> Tuple[int, bytes, int]:
    w = _u8(wire)
    cap = cap if cap is not None else max(1, w.size)
    out = np.zeros(cap, dtype=np.uint8)
    n = ctypes.c_size_t(0)
    op = ctypes.c_uint8(0)
    used = lib().oracle_decode_message(_p(w), w.size, _p(out), cap, ctypes.addressof(n), ctypes.addressof(op))
    return int(used), out[: n.value].tobytes(), int(op.value)


# ---------------------------------------------------- compiled reference ---

def ref_available() -> bool:
    return os.path.exists(os.path.join(_HERE, "_ref", "libref_ws.so"))


def _ref() -> ctypes.CDLL:
    return _load(os.path.join("_ref", "libref_ws.so"))


def ref_parse(wire: bytes, chunks: Sequence[int] = (), max_payload: int = (1 << 62)) -> List[Tuple[int, bytes]]:
    """Messages the reference's ws_parse_frame delivers for `wire` fed in `chunks`.

    Each message is (opcode, buffer as the reference reports it -- TEXT messages
    include the NUL the reference appends, src/ws/common.c:342-343)."""
    w = _u8(wire)
    ch = np.ascontiguousarray(np.asarray(list(chunks), dtype=np.uintp))
    cap = w.size + 4096
    out = np.zeros(cap, dtype=np.uint8)
    lens = np.zeros(1024, dtype=np.uintp)
    ops = np.zeros(1024, dtype=np.uint8)
    r = _ref().ref_parse(_p(w), w.size, _p(ch) if ch.size else None, ch.size, max_payload, _p(out), cap, _p(lens),
                         _p(ops), lens.size)
    if r < 0:
        raise RuntimeError(f"reference ws_parse_frame returned {r}")
    msgs, pos = [], 0
    for i in range(r):
        n = int(lens[i])
        msgs.append((int(ops[i]), out[pos:pos + n].tobytes()))
        pos += n
    return msgs


def ref_send(payload: bytes, opcode: int, key: Optional[bytes], num_frames: int = 1) -> bytes:
    """Wire bytes of the reference's ws_send_message (defined-behaviour inputs only)."""
    p = _u8(payload)
    out = np.zeros(p.size + 64 * max(1, num_frames) + 64, dtype=np.uint8)
    k = np.frombuffer(bytes(key), dtype=np.uint8).copy() if key is not None else None
    r = _ref().ref_send(opcode, _p(p), p.size, _p(k) if k is not None else None, num_frames, _p(out), out.size)
    if r < 0:
        raise RuntimeError("reference ws_send_message failed")
    return out[:r].tobytes()


def ref_key_sequence(n: int) -> bytes:
    out = np.zeros(4 * n, dtype=np.uint8)
    if _ref().ref_key_sequence(n, _p(out)) != 0:
        raise RuntimeError("ref_key_sequence failed")
    return out.tobytes()


def ref_receive_timed(wire: np.ndarray, max_payload: int = (1 << 62)) -> Tuple[int, float]:
    w = np.ascontiguousarray(wire, dtype=np.uint8)
    secs = ctypes.c_double(0.0)
    r = _ref().ref_receive_timed(_p(w), w.size, max_payload, ctypes.byref(secs))
    if r < 0:
        raise RuntimeError("reference receive failed")
    return int(r), float(secs.value)
