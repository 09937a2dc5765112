"""GPU parity: the send-side egress ring (include/ws/egress.h; VERDICT r3 "missing" #3, SURVEY.md
§8(f) row 2 from host buffers) vs the oracle and libnetc's own ws_send_message.

The checker is oracle_encode_batch (the reference's single-frame send, src/ws/common.c:53-125,
pinned by the reference's golden send vectors in tests/test_oracle.py) over the frame table of
ws_send_message's split (:42-49: equal parts, the remainder on the last frame, opcode on the
first, FIN on the last, the same key on every frame).  The bar: the wire batches, concatenated
in order, are byte-identical to the oracle's frames of the queued messages -- and to what
libnetc's CPU ws_send_message puts on a socket for the same messages -- whatever the slot size,
masked or not, with the ring's slots filling, rolling over and refilling.

The route test drives libnetc's ws_send_message on a socket attached to the ring
(netc_ws_gpu_attach_send) and compares the bytes that arrive with the CPU route's.
"""

import ctypes
import os
import socket
import threading

import numpy as np
import pytest

from netc_amd import _lib
from netc_amd import egress as ne
from netc_amd.mask import NETC_GPU_EINVAL, NetcGpuError
from oracle import oracle as orc
from tests.wsutil import Endpoint, WsMessage, pair, send_wire

pytestmark = pytest.mark.gpu


def table(messages):
    """(payload, offsets, keys32, header0, masked) of ws_send_message's frames of `messages`
    [(payload bytes, opcode, key or None, num_frames)] -- one mask mode."""
    pay, off, keys, h0 = [], [0], [], []
    pos = 0
    masked = None
    for p, op, key, nf in messages:
        nf = nf or 1
        m = key is not None
        assert masked in (None, m)
        masked = m
        k32 = int.from_bytes(bytes(key), "little") if m else 0
        split, rem = divmod(len(p), nf)
        for i in range(nf):
            last = i + 1 == nf
            flen = split + (rem if last else 0)
            pos += flen
            off.append(pos)
            keys.append(k32)
            h0.append((0x80 if last else 0) | (op & 0x0F if i == 0 else 0))
        pay.append(bytes(p))
    return (np.frombuffer(b"".join(pay), dtype=np.uint8), np.array(off, dtype=np.uint64),
            np.array(keys, dtype=np.uint32), np.array(h0, dtype=np.uint8), bool(masked))


def oracle_wire(messages):
    out = []
    run = []
    for m in messages:   # the oracle batch holds one mask mode: split where it changes
        if run and (run[-1][2] is None) != (m[2] is None):
            out.append(run)
            run = []
        run.append(m)
    if run:
        out.append(run)
    wire = b""
    for r in out:
        p, off, keys, h0, masked = table(r)
        w, _ = orc.encode_batch(p, off, keys, h0, masked)
        wire += w.tobytes()
    return wire


def drain(eg, wait=True):
    """every finished wire batch, released; (bytes, frames, messages)"""
    got, nf, nm = [], 0, 0
    while True:
        w = eg.next(wait)
        if w is None:
            break
        got.append(w.wire.tobytes())
        nf += w.nframes
        nm += w.nmessages
        w.release()
    return b"".join(got), nf, nm


def run_ring(messages, **kw):
    """queue every message (draining when the ring is full), submit, drain: the wire bytes"""
    out = []
    with ne.Egress(**kw) as eg:
        for p, op, key, nf in messages:
            rc = eg.queue(p, op, key, nf)
            if rc == ne.NETC_WS_EGRESS_FULL:
                out.append(drain(eg)[0])
                assert eg.queue(p, op, key, nf) == 0
        eg.submit()
        out.append(drain(eg)[0])
    return b"".join(out)


def random_messages(rng, n, masked, sizes=None, frames=(1, 1, 1, 2, 3, 7)):
    sizes = sizes or [0, 1, 2, 3, 17, 125, 126, 127, 1000, 4096, 65535, 65536, 65537, 200_000]
    msgs = []
    for _ in range(n):
        ln = int(rng.choice(sizes))
        op = int(rng.choice([1, 2, 2, 9, 10]))
        key = bytes(rng.integers(0, 256, 4, dtype=np.uint8)) if masked else None
        msgs.append((rng.integers(0, 256, ln, dtype=np.uint8).tobytes(), op, key, int(rng.choice(frames))))
    return msgs


@pytest.mark.parametrize("masked", [True, False])
def test_messages_match_oracle(masked):
    rng = np.random.default_rng(11 + masked)
    msgs = random_messages(rng, 120, masked)
    assert run_ring(msgs) == oracle_wire(msgs)


@pytest.mark.parametrize("masked", [True, False])
def test_matches_host_ws_send_message(masked):
    """the same messages through libnetc's CPU ws_send_message, one at a time"""
    rng = np.random.default_rng(21 + masked)
    msgs = random_messages(rng, 24, masked)
    host = b""
    for p, op, key, nf in msgs:
        rc, w = send_wire(p, op, key, nf)
        assert rc == 1
        host += w
    assert run_ring(msgs) == host


def test_every_length_class_and_split():
    """header forms at their edges, splits with empty frames (num_frames > length), masked empty frames"""
    msgs = []
    for ln in (0, 1, 124, 125, 126, 127, 128, 65534, 65535, 65536, 65537):
        for nf in (1, 2, 5, 130):
            msgs.append((bytes((i * 7 + ln) & 0xFF for i in range(ln)), 2, b"\x01\x80\xfe\x7f", nf))
    assert run_ring(msgs) == oracle_wire(msgs)


def test_rollover_small_slots():
    """64 KiB slots, 3 of them: many slots, FULL handled by draining, order kept"""
    rng = np.random.default_rng(5)
    msgs = random_messages(rng, 300, True, sizes=[0, 5, 125, 126, 3000, 20000, 65536], frames=(1, 2, 4))
    assert run_ring(msgs, slot_bytes=65536, nslots=3) == oracle_wire(msgs)


def test_frame_table_limit_rolls_over():
    """max_frames = 64: a slot ends when its frame table is full"""
    msgs = [(bytes([i & 0xFF] * (i % 40)), 2, bytes([i & 0xFF, 1, 2, 3]), 1 + i % 9) for i in range(400)]
    assert run_ring(msgs, slot_bytes=1 << 20, nslots=2, max_frames=64) == oracle_wire(msgs)


def test_mask_mode_switch_submits():
    """masked and unmasked messages alternate: each switch ends the slot; the wire is in queue order"""
    rng = np.random.default_rng(9)
    msgs = []
    for i in range(60):
        m = random_messages(rng, 1, i % 3 != 0, sizes=[0, 10, 126, 70000])[0]
        msgs.append(m)
    assert run_ring(msgs) == oracle_wire(msgs)


def test_c2_shape():
    """65,536 x 1 KiB masked messages (BASELINE config 2's frames) through the default ring"""
    rng = np.random.default_rng(2)
    n = 65536
    data = rng.integers(0, 256, n * 1024, dtype=np.uint8)
    keys = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    out = []
    with ne.Egress() as eg:
        for i in range(n):
            k = int(keys[i]).to_bytes(4, "little")
            rc = eg.queue(data[i * 1024:(i + 1) * 1024], 2, k, 1)
            if rc == ne.NETC_WS_EGRESS_FULL:
                out.append(drain(eg)[0])
                assert eg.queue(data[i * 1024:(i + 1) * 1024], 2, k, 1) == 0
        eg.submit()
        out.append(drain(eg)[0])
    off = np.arange(n + 1, dtype=np.uint64) * 1024
    want, _ = orc.encode_batch(data, off, keys, np.full(n, 0x82, dtype=np.uint8), True)
    assert b"".join(out) == want.tobytes()


def test_limits_and_errors():
    with ne.Egress(slot_bytes=4096, nslots=2, max_frames=16) as eg:
        with pytest.raises(NetcGpuError) as e:
            eg.queue(bytes(4097), 2, None, 1)
        assert e.value.code == ne.NETC_WS_EGRESS_TOO_BIG
        with pytest.raises(NetcGpuError) as e:
            eg.queue(bytes(10), 2, None, 17)
        assert e.value.code == ne.NETC_WS_EGRESS_TOO_BIG
        # two full slots queued and not taken: the third message finds no slot, nothing is queued
        assert eg.queue(bytes(4096), 2, None, 1) == 0
        assert eg.queue(bytes(4096), 2, None, 1) == 0
        assert eg.queue(bytes(1), 2, None, 1) == ne.NETC_WS_EGRESS_FULL
        w = eg.next()
        assert w.nframes == 1 and w.nmessages == 1 and len(w.wire) == 4096 + 4   # 16-bit length form
        w.release()
        assert eg.queue(bytes(1), 2, None, 1) == 0
        eg.submit()
        w, nf, nm = drain(eg)
        assert nf == 2 and nm == 2
    with pytest.raises(NetcGpuError):
        ne.Egress(slot_bytes=100)


def test_send_to_closed_peer_reports_esend():
    """send() failing (peer closed: EPIPE; MSG_NOSIGNAL, so no SIGPIPE) -> ESEND; the failed slot is
    released and the ring keeps working"""
    a, b = socket.socketpair()
    b.close()
    try:
        with ne.Egress(slot_bytes=1 << 16, nslots=2) as eg:
            assert eg.queue(bytes(1000), 2, b"\x01\x02\x03\x04", 1) == 0
            with pytest.raises(NetcGpuError) as e:
                eg.flush(a.fileno())
            assert e.value.code == ne.NETC_WS_EGRESS_ESEND
            msgs = [(bytes([7] * 300), 1, b"\x05\x06\x07\x08", 2)]
            assert eg.queue(*msgs[0]) == 0
            eg.submit()
            assert drain(eg)[0] == oracle_wire(msgs)
    finally:
        a.close()


def test_release_out_of_order_and_twice():
    """wire batches released out of order; a second release of one is refused; slots refill in ring
    order (a free slot behind a taken one waits for it)"""
    lib = ne._bind(_lib.gpu())
    msgs = [(bytes([i + 1] * 4000), 2, None, 1) for i in range(3)]
    with ne.Egress(slot_bytes=4096, nslots=3) as eg:
        for m in msgs:   # 4000 B each: every message after the first submits the slot before it
            assert eg.queue(*m) == 0
        eg.submit()
        ws = [eg.next(), eg.next(), eg.next()]
        assert b"".join(w.wire.tobytes() for w in ws) == oracle_wire(msgs)
        raw1 = ws[1]._raw
        ws[1].release()
        assert lib.netc_ws_egress_release(eg._h, ctypes.byref(raw1)) < 0   # already released
        extra = (bytes(10), 2, None, 1)
        assert eg.queue(*extra) == ne.NETC_WS_EGRESS_FULL   # the next slot in ring order (0) is still taken
        ws[0].release()
        assert eg.queue(*extra) == 0
        ws[2].release()
        eg.submit()
        assert drain(eg)[0] == oracle_wire([extra])


class Reader:
    def __init__(self, sock):
        self.sock, self.out = sock, bytearray()
        self.th = threading.Thread(target=self.run)
        self.th.start()

    def run(self):
        while True:
            d = self.sock.recv(1 << 20)
            if not d:
                break
            self.out.extend(d)

    def join(self):
        self.th.join()
        return bytes(self.out)


def send_through(lib, ep, msgs):
    for p, op, key, nf in msgs:
        buf = ctypes.create_string_buffer(bytes(p), len(p) + 1)
        m = WsMessage()
        lib.ws_build_message(ctypes.byref(m), op, len(p), buf)
        kb = (ctypes.c_uint8 * 4)(*key) if key is not None else None
        assert lib.ws_send_message(ctypes.byref(ep.client), ctypes.byref(m), kb, nf) == 1


@pytest.mark.parametrize("defer", [False, True])
def test_ws_send_message_route(defer):
    """libnetc's ws_send_message on an attached socket: the GPU ring's bytes equal the CPU route's"""
    lib = _lib.host()
    rng = np.random.default_rng(31 + defer)
    msgs = random_messages(rng, 40, True) + random_messages(rng, 10, False)
    cpu = b""
    for p, op, key, nf in msgs:
        cpu += send_wire(p, op, key, nf)[1]
    a, b = pair()
    rd = Reader(b)
    ep = Endpoint(a)
    with ne.Egress(slot_bytes=1 << 20, nslots=3, defer=defer) as eg:
        eg.attach(a.fileno())
        try:
            send_through(lib, ep, msgs)
            if defer:
                eg.flush(a.fileno())
        finally:
            eg.detach(a.fileno())
        # detached: the CPU path again on the same socket
        send_through(lib, ep, msgs[:3])
    a.shutdown(socket.SHUT_WR)
    got = rd.join()
    a.close()
    b.close()
    tail = b"".join(send_wire(p, op, key, nf)[1] for p, op, key, nf in msgs[:3])
    assert got == cpu + tail


def test_send_ring_serves_one_connection():
    """one ring, one connection: a ring already serving an open socket is
    refused for a second one (and a second ring for the same socket); re-attaching the same pair
    is a no-op; once its socket closed without a detach, the ring may serve a new socket, and the
    reused descriptor number no longer routes to it"""
    lib = _lib.host()
    a, b = pair()
    c, d = pair()
    with ne.Egress(slot_bytes=1 << 16, nslots=2) as eg, ne.Egress(slot_bytes=1 << 16, nslots=2) as eg2:
        eg.attach(a.fileno())
        try:
            eg.attach(a.fileno())
            with pytest.raises(NetcGpuError) as e:
                eg.attach(c.fileno())
            assert e.value.code == NETC_GPU_EINVAL and "one ring, one connection" in e.value.message
            with pytest.raises(NetcGpuError):
                eg2.attach(a.fileno())
            # c keeps the CPU path
            rd = Reader(d)
            send_through(lib, Endpoint(c), [(b"cpu", 2, None, 1)])
            c.shutdown(socket.SHUT_WR)
            assert rd.join() == b"\x82\x03cpu"
        finally:
            eg.detach(a.fileno())
        # closed without a detach: the number, reused, is another connection
        eg.attach(a.fileno())
        fd = a.fileno()
        a.close()
        b.close()
        x, y = pair()
        if x.fileno() != fd:   # (the kernel usually hands out the same number by itself)
            os.dup2(x.fileno(), fd)
        try:
            rd = Reader(y)
            send_through(lib, Endpoint(x), [(b"new", 2, None, 1)])   # CPU path, not the ring
            ep = Endpoint(x)
            ep.tcp.sockfd = fd
            send_through(lib, ep, [(b"dup", 2, None, 1)])
            if x.fileno() != fd:
                os.close(fd)
            x.shutdown(socket.SHUT_WR)
            assert rd.join() == b"\x82\x03new\x82\x03dup"
            eg.attach(y.fileno())   # the ring's old connection is gone: it may serve a new one
            eg.detach(y.fileno())
        finally:
            x.close()
            y.close()
            c.close()
            d.close()


def test_detach_flushes_deferred_messages():
    """a DEFER ring's ws_send_message returns 1 once queued; netc_ws_gpu_detach_send puts every
    queued message on the socket before the route goes (no silent loss)"""
    lib = _lib.host()
    rng = np.random.default_rng(41)
    msgs = random_messages(rng, 30, True, sizes=[0, 5, 126, 3000, 70000])
    cpu = b"".join(send_wire(p, op, key, nf)[1] for p, op, key, nf in msgs)
    a, b = pair()
    rd = Reader(b)
    ep = Endpoint(a)
    with ne.Egress(slot_bytes=1 << 20, nslots=3, defer=True) as eg:
        eg.attach(a.fileno())
        send_through(lib, ep, msgs)     # queued; most of it still in the ring
        eg.detach(a.fileno())           # flushes
    a.shutdown(socket.SHUT_WR)
    got = rd.join()
    a.close()
    b.close()
    assert got == cpu


def test_send_route_refuses_a_message_over_the_slot():
    """ws_send_message on an attached socket with a message larger than the ring's slot: -1 and
    NETC_WS_EGRESS_TOO_BIG in the error text, nothing of it on the socket, and the next messages
    go out as before (include/ws/egress.h: size the slots for the largest message)"""
    from netc_amd import mask as nm
    lib = _lib.host()
    a, b = pair()
    rd = Reader(b)
    ep = Endpoint(a)
    small = [(b"before", 1, b"\x01\x02\x03\x04", 1)]
    after = [(b"after" * 100, 2, b"\x05\x06\x07\x08", 2)]
    big = bytes(100000)
    with ne.Egress(slot_bytes=1 << 16, nslots=2) as eg:
        eg.attach(a.fileno())
        try:
            send_through(lib, ep, small)
            buf = ctypes.create_string_buffer(big, len(big) + 1)
            m = WsMessage()
            lib.ws_build_message(ctypes.byref(m), 2, len(big), buf)
            kb = (ctypes.c_uint8 * 4)(9, 9, 9, 9)
            assert lib.ws_send_message(ctypes.byref(ep.client), ctypes.byref(m), kb, 1) == -1
            assert b"exceeds a slot" in nm._lib.gpu().netc_gpu_strerror()
            send_through(lib, ep, after)
        finally:
            eg.detach(a.fileno())
    a.shutdown(socket.SHUT_WR)
    got = rd.join()
    a.close()
    b.close()
    assert got == b"".join(send_wire(p, op, key, nf)[1] for p, op, key, nf in small + after)


def test_egress_injected_fault_reports_and_recovers():
    """a failing submission (NETC_GPU_KNOB_INJECT_FAULT) is reported as NETC_GPU_ELAUNCH and leaves
    the slot's queued messages intact: the retried submission sends exactly the oracle's wire
    (the table is packed into its own buffer, so a failure cannot corrupt it)"""
    from netc_amd import mask as nm
    msgs = [(bytes([i] * (100 + 37 * i)), 2, bytes([i, 1, 2, 3]), 1 + i % 3) for i in range(50)]
    with ne.Egress(slot_bytes=1 << 20, nslots=2, max_frames=120) as eg:
        for m in msgs:
            assert eg.queue(*m) == 0
        with nm.knob("INJECT_FAULT", 0):
            with pytest.raises(NetcGpuError) as e:
                eg.submit()
        assert e.value.code == nm.NETC_GPU_ELAUNCH
        eg.submit()
        assert drain(eg)[0] == oracle_wire(msgs)
