"""The GPU receive route behind netc's own ws_parse_frame, under the reference caller's contract
(VERDICT r4 "next" #1).

netc's server calls ws_parse_frame ONCE per EPOLLIN and goes back to epoll_wait
(reference src/tcp/server.c:72-75 -> src/web/server.c:86-98; src/web/client.c:25 likewise).  A
ring attached with netc_ws_gpu_attach reads ahead of the message it returns, so these tests
drive it exactly that way -- one ws_parse_frame per readiness of the socket -- and check that

  * every message the peer sent is delivered, and the socket stays readable while a complete
    message waits in the ring: nothing is stranded when the peer goes quiet after a burst
    (the driver fails the moment the socket is not readable with messages still owed);
  * the messages equal, in order, the oracle's: the wire is built with oracle_encode_batch
    (the reference's send path, src/ws/common.c:53-125, pinned by the golden send vectors in
    tests/test_oracle.py) from known plaintexts, and each delivered message must be that
    plaintext (with the NUL the reference appends to TEXT, src/ws/common.c:340-344);
  * a device failure reaches the caller as NETC_GPU_ELAUNCH (-103), never as one of
    WS_FRAME_PARSE_ERROR_RECV / INVALID_FRAME_LENGTH / PAYLOAD_TOO_BIG (-1..-3), which
    netc's web layer would read as a malformed frame from the peer;
  * one ring serves one connection, and a route left behind by a connection closed without a
    detach does not serve the next socket that gets its descriptor number.
"""

import ctypes
import os
import select
import socket
import threading
import time

import numpy as np
import pytest

from netc_amd import _lib
from netc_amd import ingest as ni
from netc_amd import mask as nm
from netc_amd.mask import NetcGpuError
from oracle import oracle as orc
from tests.wsutil import Endpoint, ParseState, libc, pair, send_wire

pytestmark = pytest.mark.gpu

TEXT, BINARY, PING = 1, 2, 9


def tcp_pair():
    ls = socket.socket()
    ls.bind(("127.0.0.1", 0))
    ls.listen(1)
    c = socket.create_connection(ls.getsockname())
    s, _ = ls.accept()
    ls.close()
    c.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
    return c, s


def script(rng, n, big=False):
    """n messages: (opcode, plaintext, fragments, key per fragment), sizes from empty to 70 KB
    (16- and 64-bit lengths) and, with big, one of 3 MiB in 48 frames; a PING between messages"""
    sizes = [0, 1, 5, 125, 126, 1000, 1024, 4096, 20000, 65535, 70000]
    msgs = []
    for i in range(n):
        op = PING if i % 17 == 5 else int(rng.choice([TEXT, BINARY]))
        ln = int(rng.integers(0, 126)) if op == PING else int(rng.choice(sizes))
        nf = 1 if op == PING else int(rng.choice([1, 1, 2, 3]))
        msgs.append((op, rng.integers(0, 256, ln, dtype=np.uint8).tobytes(), nf))
    if big:
        msgs.insert(n // 2, (BINARY, rng.integers(0, 256, 3 << 20, dtype=np.uint8).tobytes(), 48))
    out = []
    for op, p, nf in msgs:
        keys = [rng.integers(0, 256, 4, dtype=np.uint8).tobytes() for _ in range(nf)]
        keys[0] = b"\x00\x61\xc2\x23" if len(out) == 0 else keys[0]   # the reference's first key
        out.append((op, p, nf, keys))
    return out


def wire_of(msgs):
    """the oracle's frames of every message (a fragment per key, the reference's split) --
    oracle_encode_batch, which gives a masked empty frame its key (RFC 6455 §5.2; the
    reference's single-frame send omits it, defect B9, so its wire would not parse)"""
    w = bytearray()
    for op, p, nf, keys in msgs:
        split, rem = divmod(len(p), nf)
        off = [0]
        for i in range(nf):
            off.append(off[-1] + split + (rem if i + 1 == nf else 0))
        h0 = [(0x80 if i + 1 == nf else 0) | (op if i == 0 else 0) for i in range(nf)]
        k32 = [int.from_bytes(k, "little") for k in keys]
        wire, _ = orc.encode_batch(np.frombuffer(p, dtype=np.uint8), np.array(off, dtype=np.uint64),
                                   np.array(k32, dtype=np.uint32), np.array(h0, dtype=np.uint8), True)
        w += wire.tobytes()
    return bytes(w)


def wire_of_unmasked(msgs):
    """the same frames unmasked, as netc's server sends them to its clients (ws_send_message with
    no key, src/ws/common.c:40; src/web/client.c:25 parses them)"""
    w = bytearray()
    for op, p, nf, _ in msgs:
        split, rem = divmod(len(p), nf)
        off = [0]
        for i in range(nf):
            off.append(off[-1] + split + (rem if i + 1 == nf else 0))
        h0 = [(0x80 if i + 1 == nf else 0) | (op if i == 0 else 0) for i in range(nf)]
        wire, _ = orc.encode_batch(np.frombuffer(p, dtype=np.uint8), np.array(off, dtype=np.uint64), None,
                                   np.array(h0, dtype=np.uint8), False)
        w += wire.tobytes()
    return bytes(w)


def expected(msgs):
    return [(op, p + (b"\0" if op == TEXT else b"")) for op, p, _, _ in msgs]


def ring_state(ing):
    lib = ing._lib
    out = (ctypes.c_uint64 * 8)()
    lib.netc_ws_ingest_debug_state.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    lib.netc_ws_ingest_debug_state(ing._h, out)
    names = ["in_pos", "sock_pos", "end_pos", "batches", "cur_fill", "msg_size", "err", "scanned_to"]
    return dict(zip(names, list(out)))


def once_per_event(sock, ep, lib, n, limit, timeout=10.0, ing=None, sent=None):
    """netc's server loop: wait for readability, ONE ws_parse_frame, dispatch, repeat"""
    st = ParseState()
    got = []
    while len(got) < n:
        r, _, _ = select.select([sock], [], [], timeout)
        assert r, (f"stranded: {len(got)} of {n} messages delivered and the socket is not readable; "
                   f"ring {ring_state(ing) if ing else None}, sent {sent}")
        rc = lib.ws_parse_frame(ctypes.byref(ep.client), ctypes.byref(st), limit)
        if rc == 0:
            m = st.message
            got.append((int(m.opcode), ctypes.string_at(m.buffer, m.payload_length)))
            libc.free(m.buffer)                                      # src/web/server.c:139
            ctypes.memset(ctypes.byref(st), 0, ctypes.sizeof(st))    # src/web/server.c:140
        else:
            assert rc == 1, f"ws_parse_frame returned {rc}"
    return got


@pytest.mark.timeout(300)
@pytest.mark.parametrize("kind", ["tcp", "unix"])
@pytest.mark.parametrize("slot_bytes,scan", [(1 << 16, "gpu"), (1 << 20, "auto"), (1 << 20, "host")])
def test_once_per_event_delivers_everything(kind, slot_bytes, scan):
    """a burst sent without waiting, then silence: every message comes out of one ws_parse_frame
    per readiness event, equal to the oracle's, and the socket is drained at the end"""
    lib = _lib.host()
    rng = np.random.default_rng(slot_bytes + len(kind) + len(scan))
    msgs = script(rng, 300, big=slot_bytes > 1 << 16)
    wire = wire_of(msgs)
    c, s = tcp_pair() if kind == "tcp" else pair()
    s.setblocking(False)
    ep = Endpoint(s)
    sent = [0, len(wire)]

    def send_all():
        for i in range(0, len(wire), 1 << 16):
            c.sendall(wire[i:i + (1 << 16)])
            sent[0] = i + len(wire[i:i + (1 << 16)])

    sender = threading.Thread(target=send_all)
    with ni.Ingest(slot_bytes=slot_bytes, nslots=4, max_frame_bytes=4 << 20, scan=scan) as ing:
        ing.attach(s.fileno())
        try:
            sender.start()
            got = once_per_event(s, ep, lib, len(msgs), 64 << 20, ing=ing, sent=sent)
            sender.join()
            # everything delivered: the ring took every byte out of the socket
            assert not select.select([s], [], [], 0.2)[0]
            st = ParseState()
            assert lib.ws_parse_frame(ctypes.byref(ep.client), ctypes.byref(st), 64 << 20) == 1
        finally:
            ing.detach(s.fileno())
    c.close()
    s.close()
    assert len(got) == len(msgs)
    for j, (g, e) in enumerate(zip(got, expected(msgs))):
        assert g[0] == e[0] and g[1] == e[1], f"message {j}: opcode {g[0]}/{e[0]}, {len(g[1])}/{len(e[1])} bytes"


@pytest.mark.timeout(120)
def test_trickle_one_byte_at_a_time_then_close():
    """bytes arrive in pieces of 1..7 bytes with the peer pausing in between, then it closes:
    every message, then WS_FRAME_PARSE_ERROR_RECV (the reference's recv() == 0, src/ws/common.c:151-154)"""
    lib = _lib.host()
    rng = np.random.default_rng(7)
    msgs = script(rng, 12)
    wire = wire_of(msgs)
    c, s = tcp_pair()
    s.setblocking(False)
    ep = Endpoint(s)

    def trickle():
        pos = 0
        while pos < len(wire):
            n = int(rng.integers(1, 8)) if pos < 400 else 30000
            c.sendall(wire[pos:pos + n])
            pos += n
            if pos < 400:
                time.sleep(0.002)   # the peer pauses: the server sees partial headers
        c.shutdown(socket.SHUT_WR)

    with ni.Ingest(slot_bytes=1 << 16, nslots=3, max_frame_bytes=1 << 17) as ing:
        ing.attach(s.fileno())
        try:
            th = threading.Thread(target=trickle)
            th.start()
            got = once_per_event(s, ep, lib, len(msgs), 1 << 20)
            th.join()
            st = ParseState()
            rc = 1
            for _ in range(100):
                select.select([s], [], [], 5)
                rc = lib.ws_parse_frame(ctypes.byref(ep.client), ctypes.byref(st), 1 << 20)
                if rc != 1:
                    break
            assert rc == ni.WS_FRAME_PARSE_ERROR_RECV
        finally:
            ing.detach(s.fileno())
    c.close()
    s.close()
    assert got == expected(msgs)


def flood_of_empty_frames(make_ctx, n=30000):
    """a flood of empty masked frames (6 B each) with one large message between: far more frames
    per read than a small slot's frame table holds -- every message arrives, in order, under
    netc's once-per-event loop"""
    lib = _lib.host()
    c, s = tcp_pair()
    s.setblocking(False)
    ep = Endpoint(s)
    msgs = [(BINARY if i % 3 else TEXT, b"", 1, [bytes([i & 0xFF, 1, 2, 3])]) for i in range(n)]
    msgs[n // 4] = (BINARY, bytes(range(256)) * 200, 2, [b"\x11\x22\x33\x44"] * 2)
    wire = wire_of(msgs)
    ctx = make_ctx()
    ctx.attach(s.fileno())
    try:
        th = threading.Thread(target=lambda: c.sendall(wire))
        th.start()
        got = once_per_event(s, ep, lib, len(msgs), 1 << 20)
        th.join()
    finally:
        ctx.detach(s.fileno())
        c.close()
        s.close()
    assert got == expected(msgs)
    return ctx


@pytest.mark.timeout(120)
def test_flood_of_empty_frames():
    with ni.Ingest(slot_bytes=1 << 16, nslots=3, max_frame_bytes=65536) as ing:
        flood_of_empty_frames(lambda: ing)


def client_side_case(make_ctx):
    """netc's client side (src/web/client.c:25): a non-strict ring or hub on the client's socket
    receives the server's UNMASKED frames; every message arrives as sent"""
    lib = _lib.host()
    rng = np.random.default_rng(23)
    msgs = script(rng, 120)
    wire = wire_of_unmasked(msgs)
    c, s = tcp_pair()
    s.setblocking(False)
    ep = Endpoint(s)
    ctx = make_ctx()
    ctx.attach(s.fileno())
    try:
        th = threading.Thread(target=lambda: c.sendall(wire))
        th.start()
        got = once_per_event(s, ep, lib, len(msgs), 1 << 20)
        th.join()
    finally:
        ctx.detach(s.fileno())
        c.close()
        s.close()
    assert got == expected(msgs)


@pytest.mark.timeout(120)
def test_client_side_unmasked_frames():
    with ni.Ingest(slot_bytes=1 << 20, nslots=3, max_frame_bytes=1 << 17, strict=False) as ing:
        client_side_case(lambda: ing)


def blocking_socket_case(attach, detach):
    """A socket left BLOCKING (netc makes its sockets non-blocking, but a caller may not): a call
    that finds only part of a frame must return 1 at once -- the route releases its hostage and
    peeks again, and that peek must not wait for the peer -- and the message comes whole once
    the rest arrives.  A timer sends the rest after 3 s, so a call that blocks ends then and
    fails the timing check instead of hanging the test."""
    lib = _lib.host()
    msgs = [(BINARY, bytes(range(256)) * 40, 1, [b"\x01\x02\x03\x04"]), (TEXT, b"after", 1, [b"\x05\x06\x07\x08"])]
    wire = wire_of(msgs)
    c, s = tcp_pair()   # s stays blocking
    ep = Endpoint(s)
    attach(s.fileno())
    rest = threading.Timer(3.0, lambda: c.sendall(wire[3000:]))
    try:
        c.sendall(wire[:3000])
        assert select.select([s], [], [], 5)[0]
        st = ParseState()
        rest.start()
        t0 = time.monotonic()
        rc = lib.ws_parse_frame(ctypes.byref(ep.client), ctypes.byref(st), 1 << 20)
        took = time.monotonic() - t0
        assert rc == 1 and took < 1.0, f"rc {rc} after {took:.2f} s: the call waited for the peer"
        rest.join()
        got = once_per_event(s, ep, lib, len(msgs), 1 << 20)
        assert got == expected(msgs)
    finally:
        rest.cancel()
        detach(s.fileno())
        c.close()
        s.close()


@pytest.mark.timeout(60)
def test_blocking_socket_never_stalls_the_loop():
    with ni.Ingest(slot_bytes=1 << 16, nslots=2) as ing:
        blocking_socket_case(ing.attach, ing.detach)


@pytest.mark.timeout(60)
def test_device_failure_is_not_a_parse_error():
    """an injected launch failure (NETC_GPU_KNOB_INJECT_FAULT) reaches ws_parse_frame's caller
    as NETC_GPU_ELAUNCH, distinct from every WS_FRAME_PARSE_ERROR_*, and stays (the ring's
    stream is over, as after any error of the reference parser)"""
    lib = _lib.host()
    assert {nm.NETC_GPU_EINVAL, nm.NETC_GPU_ENODEV, nm.NETC_GPU_ELAUNCH, nm.NETC_GPU_ERUNTIME,
            nm.NETC_GPU_ENOMEM}.isdisjoint({-1, -2, -3})
    c, s = tcp_pair()
    s.setblocking(False)
    ep = Endpoint(s)
    with ni.Ingest(slot_bytes=1 << 16, nslots=2) as ing:
        ing.attach(s.fileno())
        try:
            with nm.knob("INJECT_FAULT", 0):
                c.sendall(orc.encode_frame(b"hello", TEXT, b"\x37\xfa\x21\x3d", fin=True))
                assert select.select([s], [], [], 5)[0]
                st = ParseState()
                rc = lib.ws_parse_frame(ctypes.byref(ep.client), ctypes.byref(st), 1 << 20)
            assert rc == nm.NETC_GPU_ELAUNCH, rc
            assert b"injected fault" in nm._lib.gpu().netc_gpu_strerror()
            assert lib.ws_parse_frame(ctypes.byref(ep.client), ctypes.byref(st), 1 << 20) == nm.NETC_GPU_ELAUNCH
        finally:
            ing.detach(s.fileno())
    # the knob disarmed itself: a fresh ring works
    with ni.Ingest(slot_bytes=1 << 16, nslots=2) as ing:
        ing.write(orc.encode_frame(b"hello", TEXT, b"\x37\xfa\x21\x3d", fin=True))
        assert ing.next_message() == (0, TEXT, b"hello\0")
    c.close()
    s.close()


def test_one_ring_one_connection():
    """a second ring on a socket, or a ring on a second socket, is refused; re-attaching the same
    pair is a no-op; an attached ring cannot also be fed by hand"""
    a, b = tcp_pair()
    c, d = tcp_pair()
    with ni.Ingest(slot_bytes=1 << 16, nslots=2) as r1, ni.Ingest(slot_bytes=1 << 16, nslots=2) as r2:
        r1.attach(b.fileno())
        try:
            r1.attach(b.fileno())
            with pytest.raises(NetcGpuError) as e:
                r2.attach(b.fileno())
            assert e.value.code == nm.NETC_GPU_EINVAL
            with pytest.raises(NetcGpuError) as e:
                r1.attach(d.fileno())
            assert e.value.code == nm.NETC_GPU_EINVAL and "one ring, one connection" in e.value.message
            with pytest.raises(NetcGpuError):
                r1.recv(b.fileno())
            with pytest.raises(NetcGpuError):
                r1.write(b"\x81\x00")
            with pytest.raises(NetcGpuError):
                r2.attach(1 << 29)   # not an open socket
        finally:
            r1.detach(b.fileno())
        r2.attach(d.fileno())   # r2 never carried a stream
        r2.detach(d.fileno())
    for x in (a, b, c, d):
        x.close()


def test_route_does_not_outlive_its_connection():
    """a connection closed without a detach leaves its route behind; the descriptor number, reused
    by the next socket, gets the CPU parser -- not the old ring -- and a fresh ring can attach"""
    lib = _lib.host()
    a, b = tcp_pair()
    fd = b.fileno()
    with ni.Ingest(slot_bytes=1 << 16, nslots=2) as old, ni.Ingest(slot_bytes=1 << 16, nslots=2) as new:
        old.attach(fd)
        a.close()
        b.close()                      # closed without netc_ws_gpu_detach
        c, d = pair()
        if d.fileno() != fd:           # the number now names another connection
            os.dup2(d.fileno(), fd)
        try:
            rc, w = send_wire(b"after reuse", BINARY, b"\x01\x02\x03\x04", 1)
            c.sendall(w)
            ep = Endpoint(d)
            ep.tcp.sockfd = fd
            st = ParseState()
            while (r := lib.ws_parse_frame(ctypes.byref(ep.client), ctypes.byref(st), 1 << 20)) == 1:
                pass
            assert r == 0 and ctypes.string_at(st.message.buffer, st.message.payload_length) == b"after reuse"
            libc.free(st.message.buffer)
            new.attach(fd)             # the stale route does not block a fresh ring
            new.detach(fd)
            old.detach(fd)             # nothing of old's is left there: a no-op
        finally:
            if d.fileno() != fd:
                os.close(fd)
            c.close()
            d.close()


@pytest.mark.timeout(60)
def test_route_errors_after_the_messages_before_them():
    """a strict ring: the messages before an unmasked client frame first, then
    WS_FRAME_PARSE_ERROR_INVALID_FRAME_LENGTH, sticky; a frame over the ring's limit likewise
    ends in PAYLOAD_TOO_BIG -- all with one call per readiness (the socket stays readable until
    the error is reported)"""
    lib = _lib.host()
    good = [(TEXT, b"first", 1, [b"\x01\x02\x03\x04"]), (BINARY, bytes(range(200)), 2, [b"\x05\x06\x07\x08"] * 2)]
    for tail, want_rc, kw in ((bytes([0x81, 0x03]) + b"abc", -2, dict(strict=True)),
                              (wire_of([(BINARY, bytes(5000), 1, [b"\x09\x09\x09\x09"])]), -3,
                               dict(max_frame_bytes=4096))):
        c, s = tcp_pair()
        s.setblocking(False)
        ep = Endpoint(s)
        with ni.Ingest(slot_bytes=1 << 16, nslots=2, **kw) as ing:
            ing.attach(s.fileno())
            try:
                c.sendall(wire_of(good) + tail)
                got = once_per_event(s, ep, lib, len(good), 1 << 20)
                assert got == expected(good)
                st = ParseState()
                assert select.select([s], [], [], 5)[0], "the error's bytes must keep the socket readable"
                assert lib.ws_parse_frame(ctypes.byref(ep.client), ctypes.byref(st), 1 << 20) == want_rc
                assert lib.ws_parse_frame(ctypes.byref(ep.client), ctypes.byref(st), 1 << 20) == want_rc
            finally:
                ing.detach(s.fileno())
        c.close()
        s.close()
