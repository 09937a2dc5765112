"""Sends never wait for a peer: libnetc's ws_send_message and the connection's send backlog
(include/ws/route.h, round 6).

The reference sends each frame with one send() and returns its result (src/tcp/server.c:219-225):
on a non-blocking socket whose buffer is full that is -1 (EAGAIN), and a short send is counted as
sent (defect B5: the rest of the frame is lost and the stream is corrupt).  Neither waits.  Here
what a non-blocking socket does not take is kept per connection and written ahead of the
connection's later bytes, without waiting, by the next ws_send_message / ws_parse_frame /
netc_ws_send_flush on it; past a bound the connection fails alone.  Checked:

  * a peer that stops reading: every ws_send_message returns 1 at once (no call waits), the
    backlog grows, and once the peer reads, the bytes it gets are exactly the frames sent, in
    order (the wire rendering pinned by tests/test_host_framing.py against the reference);
  * the bound: that connection fails with -1 / ENOBUFS / BADSEND and stays failed; another
    connection is unaffected;
  * a blocking socket keeps the reference's blocking send;
  * ws_parse_frame on a readable connection writes its backlog first;
  * in this process close() is libc's (ctypes), so lookups keep the identity check.
"""

import ctypes
import socket
import threading
import time

import numpy as np

from netc_amd import _lib
from tests import test_gpu_route as G
from tests.wsutil import Endpoint, ParseState, WsMessage, libc, pair


def lib():
    h = _lib.host()
    if not getattr(h, "_backlog_bound", False):
        h.netc_ws_send_flush.argtypes = [ctypes.c_int]
        h.netc_ws_send_flush.restype = ctypes.c_long
        h.netc_ws_send_pending.argtypes = [ctypes.c_int]
        h.netc_ws_send_pending.restype = ctypes.c_long
        h.netc_ws_send_backlog_limit.argtypes = [ctypes.c_size_t]
        h.netc_ws_send_backlog_limit.restype = ctypes.c_size_t
        h.netc_ws_route_close_tracked.restype = ctypes.c_int
        h._backlog_bound = True
    return h


def send(h, ep, op, payload, key, nf=1):
    buf = ctypes.create_string_buffer(bytes(payload), len(payload) + 1)
    m = WsMessage()
    h.ws_build_message(ctypes.byref(m), op, len(payload), buf)
    kb = (ctypes.c_uint8 * 4)(*key) if key is not None else None
    return h.ws_send_message(ctypes.byref(ep.client), ctypes.byref(m), kb, nf)


def wire(msgs):
    out = b""
    for op, p, nf, key in msgs:
        one = [(op, p, nf, [key] * nf)]
        out += G.wire_of(one) if key is not None else G.wire_of_unmasked(one)
    return out


def read_all(sock, n, timeout=30):
    out = bytearray()
    sock.settimeout(timeout)
    while len(out) < n:
        d = sock.recv(1 << 20)
        if not d:
            break
        out.extend(d)
    return bytes(out)


def small_pair():
    a, b = socket.socketpair(socket.AF_UNIX, socket.SOCK_STREAM)
    for s in (a, b):
        s.setsockopt(socket.SOL_SOCKET, socket.SO_SNDBUF, 1 << 16)
        s.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 1 << 16)
    a.setblocking(False)
    return a, b


def test_close_is_libc_here_so_lookups_check_identity():
    assert lib().netc_ws_route_close_tracked() == 0


def test_peer_not_reading_never_blocks_then_gets_every_byte():
    h = lib()
    rng = np.random.default_rng(61)
    a, b = small_pair()
    ep = Endpoint(a)
    sent = []
    worst = 0.0
    for i in range(400):   # about 1.6 MB against a ~128 KiB socket: most of it waits in the backlog
        op = G.BINARY if i % 2 else G.TEXT
        p = rng.integers(0, 256, int(rng.integers(0, 8000)), dtype=np.uint8).tobytes()
        nf = 1 + i % 3
        key = bytes(rng.integers(0, 256, 4, dtype=np.uint8)) if i % 4 else None
        t0 = time.perf_counter()
        assert send(h, ep, op, p, key, nf) == 1
        worst = max(worst, time.perf_counter() - t0)
        sent.append((op, p, nf, key))
    held = h.netc_ws_send_pending(a.fileno())
    want = wire(sent)
    assert 0 < held < len(want)
    assert worst < 0.05, f"a send waited {worst * 1e3:.1f} ms"
    got = bytearray()

    def reader():
        got.extend(read_all(b, len(want)))

    th = threading.Thread(target=reader)
    th.start()
    deadline = time.monotonic() + 30
    while h.netc_ws_send_flush(a.fileno()) > 0:
        assert time.monotonic() < deadline
        time.sleep(0.001)
    th.join()
    assert h.netc_ws_send_pending(a.fileno()) == 0
    assert bytes(got) == want
    a.close()
    b.close()


def test_backlog_bound_fails_only_that_connection():
    h = lib()
    old = h.netc_ws_send_backlog_limit(256 << 10)
    try:
        a, b = small_pair()        # its peer never reads
        c, d = small_pair()        # this one does
        ea, ec = Endpoint(a), Endpoint(c)
        key = bytes([1, 2, 3, 4])
        rc = 1
        n = 0
        while rc == 1 and n < 1000:
            rc = send(h, ea, G.BINARY, bytes(4000), key)
            n += 1
        assert rc == -1 and n > 10
        assert h.netc_ws_send_pending(a.fileno()) == -1
        assert send(h, ea, G.BINARY, b"after", key) == -1          # stays failed
        kept = [(G.TEXT, b"other connection", 1, key)]
        assert send(h, ec, G.TEXT, b"other connection", key) == 1
        assert read_all(d, len(wire(kept))) == wire(kept)
        for s in (a, b, c, d):
            s.close()
    finally:
        h.netc_ws_send_backlog_limit(old)


def test_blocking_socket_keeps_the_blocking_send():
    h = lib()
    a, b = pair()
    a.setblocking(True)
    ep = Endpoint(a)
    rng = np.random.default_rng(3)
    msgs = [(G.BINARY, rng.integers(0, 256, 200000, dtype=np.uint8).tobytes(), 2, bytes([9, 8, 7, 6]))
            for _ in range(30)]
    want = wire(msgs)
    got = bytearray()
    th = threading.Thread(target=lambda: got.extend(read_all(b, len(want))))
    th.start()
    for op, p, nf, key in msgs:
        assert send(h, ep, op, p, key, nf) == 1
    assert h.netc_ws_send_pending(a.fileno()) == 0   # the kernel took everything (it waited)
    th.join()
    assert bytes(got) == want
    a.close()
    b.close()


def test_parse_frame_writes_the_backlog_first():
    h = lib()
    a, b = small_pair()
    ep = Endpoint(a)
    key = bytes([5, 5, 5, 5])
    msgs = [(G.BINARY, bytes([i % 256]) * 3000, 1, key) for i in range(100)]
    for op, p, nf, k in msgs:
        assert send(h, ep, op, p, k, nf) == 1
    assert h.netc_ws_send_pending(a.fileno()) > 0
    want = wire(msgs)
    got = bytearray()
    th = threading.Thread(target=lambda: got.extend(read_all(b, len(want))))
    th.start()
    # the peer now sends one frame; each ws_parse_frame on the readable socket moves the backlog on
    b.sendall(G.wire_of([(G.TEXT, b"ping", 1, [key])]))
    st = ParseState()
    deadline = time.monotonic() + 30
    delivered = False
    while h.netc_ws_send_pending(a.fileno()) > 0 or not delivered:
        assert time.monotonic() < deadline
        rc = h.ws_parse_frame(ctypes.byref(ep.client), ctypes.byref(st), 1 << 20)
        if rc == 0:
            assert ctypes.string_at(st.message.buffer, st.message.payload_length) == b"ping\0"
            libc.free(st.message.buffer)
            ctypes.memset(ctypes.byref(st), 0, ctypes.sizeof(st))
            delivered = True
        time.sleep(0.0005)
    th.join()
    assert bytes(got) == want
    a.close()
    b.close()
