"""One GPU send ring shared by many connections (include/ws/egress_hub.h): the send side of the hub.

netc's server answers its clients from one event loop; each ws_send_message (reference
src/ws/common.c:36-131) frames, masks and send()s one message.  With every socket attached to an
egress hub, the messages of all connections share the hub's slots: one frame-assembly launch per
slot, then one sendmsg() per connection per slot.  Checked here:

  * per connection, the bytes that arrive are exactly the frames of what it sent, in order --
    the oracle's wire (oracle_encode_batch: the reference's send path with B1/B2 fixed, pinned by
    the golden send vectors in tests/test_oracle.py; tests/test_gpu_egress.py pins libnetc's CPU
    ws_send_message to the same bytes), masked and unmasked connections mixed, 1-3 fragments,
    sizes across the 7-, 16- and 64-bit length forms;
  * launches span messages of many connections (the hub's counters);
  * detach sends what was queued, and the socket then takes the CPU path;
  * a peer that went away fails only its own connection: its next ws_send_message returns -1;
  * a message larger than a slot is refused, and nothing of it is sent.

tests/test_route_mock.py runs these on the CPU, over the mock HIP runtime.
"""

import ctypes
import json
import os
import socket
import subprocess
import threading

import numpy as np
import pytest

from netc_amd import _lib
from netc_amd import egress as ne
from netc_amd import hub as nh
from netc_amd.mask import NETC_GPU_EINVAL, NetcGpuError
from tests import test_gpu_route as G
from tests.wsutil import Endpoint, WsMessage, pair, settle

pytestmark = pytest.mark.gpu
HUB_LIB = None   # the library holding the hub (None: libnetc_ws_gpu.so; the CPU tests set the mock)


def make(**kw):
    return nh.EgressHub(lib=HUB_LIB, **kw)


class Reader:
    def __init__(self, sock):
        self.sock, self.out = sock, bytearray()
        self.th = threading.Thread(target=self.run)
        self.th.start()

    def run(self):
        while True:
            try:
                d = self.sock.recv(1 << 20)
            except OSError:
                break
            if not d:
                break
            self.out.extend(d)

    def join(self):
        self.th.join()
        return bytes(self.out)


def send(lib, ep, op, payload, key, nf):
    buf = ctypes.create_string_buffer(bytes(payload), len(payload) + 1)
    m = WsMessage()
    lib.ws_build_message(ctypes.byref(m), op, len(payload), buf)
    kb = (ctypes.c_uint8 * 4)(*key) if key is not None else None
    return lib.ws_send_message(ctypes.byref(ep.client), ctypes.byref(m), kb, nf)


def wire(msgs):
    """the frames of (op, payload, frames, key or None) messages, as ws_send_message sends them"""
    out = b""
    for op, p, nf, key in msgs:
        one = [(op, p, nf, [key] * nf)]
        out += G.wire_of(one) if key is not None else G.wire_of_unmasked(one)
    return out


def message(rng, big=False):
    sizes = [0, 1, 17, 125, 126, 700, 1024, 3000] + ([65535, 70000] if big else [])
    op = int(rng.choice([G.TEXT, G.BINARY]))
    ln = int(rng.choice(sizes))
    nf = int(rng.choice([1, 1, 2, 3]))
    return op, rng.integers(0, 256, ln, dtype=np.uint8).tobytes(), nf


@pytest.mark.timeout(300)
@pytest.mark.parametrize("nconn,rounds,slot", [(64, 30, 1 << 20), (16, 40, 64 << 10), (256, 6, 1 << 20)])
def test_many_connections_interleaved(nconn, rounds, slot):
    lib = _lib.host()
    rng = np.random.default_rng(nconn * 100 + rounds)
    pairs = [pair() for _ in range(nconn)]
    readers = [Reader(b) for _, b in pairs]
    eps = [Endpoint(a) for a, _ in pairs]
    sent = [[] for _ in range(nconn)]
    with make(slot_bytes=slot, nslots=3) as hub:
        for a, _ in pairs:
            hub.attach(a.fileno())
        try:
            for r in range(rounds):
                for c in rng.permutation(nconn)[: max(1, nconn // 2)]:
                    op, p, nf = message(rng, big=slot > (64 << 10))
                    key = rng.integers(0, 256, 4, dtype=np.uint8).tobytes() if c % 3 else None   # a third unmasked
                    assert send(lib, eps[c], op, p, key, nf) == 1
                    sent[c].append((op, p, nf, key))
                if r % 5 == 4:   # the server's loop flushes once per iteration
                    hub.flush()
            hub.drain()
            st = hub.stats()
        finally:
            for a, _ in pairs:
                hub.detach(a.fileno())
    for a, _ in pairs:
        a.shutdown(socket.SHUT_WR)
    got = [rd.join() for rd in readers]
    for a, b in pairs:
        a.close()
        b.close()
    for c in range(nconn):
        assert got[c] == wire(sent[c]), f"connection {c}: {len(got[c])} bytes against {len(wire(sent[c]))}"
    total = sum(len(m) for m in sent)
    assert st["messages"] == total and st["launches"] < total, st
    assert st["max_connections"] > 1, st
    assert st["send_errors"] == 0 and st["connections"] == nconn


@pytest.mark.timeout(60)
def test_detach_sends_what_was_queued_then_cpu_path():
    lib = _lib.host()
    rng = np.random.default_rng(5)
    (a, b), (c, d) = pair(), pair()
    ra, rc = Reader(b), Reader(d)
    ea, ec = Endpoint(a), Endpoint(c)
    msgs_a = [message(rng) + (bytes([1, 2, 3, 4]),) for _ in range(20)]
    msgs_c = [message(rng) + (bytes([5, 6, 7, 8]),) for _ in range(20)]
    with make(slot_bytes=1 << 20, nslots=2) as hub:
        hub.attach(a.fileno())
        hub.attach(c.fileno())
        for (op, p, nf, key), (op2, p2, nf2, key2) in zip(msgs_a, msgs_c):
            assert send(lib, ea, op, p, key, nf) == 1
            assert send(lib, ec, op2, p2, key2, nf2) == 1
        hub.detach(a.fileno())   # everything queued goes out first (both connections' bytes)
        tail = [(G.BINARY, b"cpu path", 1, bytes([9, 9, 9, 9]))]
        assert send(lib, ea, *[tail[0][i] for i in (0, 1, 3, 2)]) == 1   # not routed any more
        assert hub.stats()["connections"] == 1
        hub.detach(c.fileno())
    settle(a, c)
    a.shutdown(socket.SHUT_WR)
    c.shutdown(socket.SHUT_WR)
    got_a, got_c = ra.join(), rc.join()
    for s in (a, b, c, d):
        s.close()
    assert got_a == wire([(op, p, nf, key) for op, p, nf, key in msgs_a] + tail)
    assert got_c == wire([(op, p, nf, key) for op, p, nf, key in msgs_c])


@pytest.mark.timeout(60)
def test_a_peer_gone_fails_only_its_connection():
    lib = _lib.host()
    (a, b), (c, d) = pair(), pair()
    rc = Reader(d)
    ea, ec = Endpoint(a), Endpoint(c)
    b.close()   # a's peer is gone
    key = bytes([1, 2, 3, 4])
    with make(slot_bytes=1 << 20, nslots=2) as hub:
        hub.attach(a.fileno())
        hub.attach(c.fileno())
        try:
            assert send(lib, ea, G.BINARY, b"lost" * 100, key, 1) == 1   # queued: the failure comes at the flush
            assert send(lib, ec, G.BINARY, b"kept" * 100, key, 1) == 1
            hub.flush()
            st = hub.stats()
            assert st["send_errors"] == 1, st
            assert send(lib, ea, G.BINARY, b"again", key, 1) == -1       # its send() failed
            assert send(lib, ec, G.TEXT, b"still fine", key, 2) == 1
            hub.flush()
        finally:
            hub.detach(a.fileno())
            hub.detach(c.fileno())
    c.shutdown(socket.SHUT_WR)
    got = rc.join()
    a.close()
    c.close()
    d.close()
    assert got == wire([(G.BINARY, b"kept" * 100, 1, key), (G.TEXT, b"still fine", 2, key)])


@pytest.mark.timeout(60)
def test_rules_and_limits():
    """one send route per socket (a socket an egress ring serves is refused; re-attaching to the
    same hub is a no-op); a message over the slot is refused with nothing sent"""
    from netc_amd import mask as nm
    lib = _lib.host()
    a, b = pair()
    rd = Reader(b)
    ep = Endpoint(a)
    key = bytes([7, 7, 7, 7])
    with make(slot_bytes=64 << 10, nslots=2) as hub:
        if HUB_LIB is None:   # (the egress ring lives in the GPU library only)
            with ne.Egress(slot_bytes=1 << 16, nslots=2) as eg:
                eg.attach(a.fileno())
                with pytest.raises(NetcGpuError) as e:
                    hub.attach(a.fileno())
                assert e.value.code == NETC_GPU_EINVAL
                eg.detach(a.fileno())
        hub.attach(a.fileno())
        hub.attach(a.fileno())
        try:
            assert send(lib, ep, G.BINARY, b"small", key, 1) == 1
            assert send(lib, ep, G.BINARY, bytes(100000), key, 1) == -1
            assert b"exceeds a slot" in hub._lib.netc_gpu_strerror()
            assert send(lib, ep, G.BINARY, b"after", key, 1) == 1
        finally:
            hub.detach(a.fileno())
    with pytest.raises(NetcGpuError):
        make(slot_bytes=1024)
    a.shutdown(socket.SHUT_WR)
    got = rd.join()
    a.close()
    b.close()
    assert got == wire([(G.BINARY, b"small", 1, key), (G.BINARY, b"after", 1, key)])


@pytest.mark.timeout(300)
@pytest.mark.parametrize("masked", ["0", "1"])
def test_egress_hub_server_256_connections(masked):
    """tests/drivers/ws_egress_hub_server.c: 256 TCP connections answered 60 times each from one
    loop through the egress hub (flushed per iteration); every connection's bytes hashed by its
    client equal the frames the server expects (the same rendering that libnetc's CPU leg and
    the reference's own ws_send_message leg match)"""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(root, "tests", "bin", "ws_egress_hub_server")
    assert os.path.exists(exe), "tests/bin/ws_egress_hub_server missing: run make"
    for leg in ("hub", "cpu"):
        r = subprocess.run([exe, leg, "256", "60", "1024", masked], capture_output=True, text=True, timeout=240,
                           cwd=root)
        assert r.returncode == 0, f"{leg}: rc {r.returncode}\n{r.stdout[-2000:]}\n{r.stderr[-3000:]}"
        d = json.loads(r.stdout.strip().splitlines()[-1])
        assert d["mismatched"] == 0 and d["messages"] == 256 * 60, d
        if leg == "hub":
            assert d["launches"] >= 1 and d["max_conns_per_launch"] >= 64 and d["send_errors"] == 0, d


@pytest.mark.timeout(120)
def test_slots_run_out_between_flushes():
    """two small slots and no flush for a long while: with no slot free the oldest is sent from
    inside ws_send_message, over and over; every connection's bytes still come in order"""
    lib = _lib.host()
    rng = np.random.default_rng(77)
    nconn = 32
    pairs = [pair() for _ in range(nconn)]
    readers = [Reader(b) for _, b in pairs]
    eps = [Endpoint(a) for a, _ in pairs]
    sent = [[] for _ in range(nconn)]
    with make(slot_bytes=8192, nslots=2, max_frames=64) as hub:
        for a, _ in pairs:
            hub.attach(a.fileno())
        try:
            for _ in range(600):
                c = int(rng.integers(0, nconn))
                op, p, nf = message(rng)
                key = bytes(rng.integers(0, 256, 4, dtype=np.uint8)) if c % 2 else None
                assert send(lib, eps[c], op, p, key, nf) == 1
                sent[c].append((op, p, nf, key))
            hub.drain()
            st = hub.stats()
        finally:
            for a, _ in pairs:
                hub.detach(a.fileno())
    for a, _ in pairs:
        a.shutdown(socket.SHUT_WR)
    got = [rd.join() for rd in readers]
    for a, b in pairs:
        a.close()
        b.close()
    for c in range(nconn):
        assert got[c] == wire(sent[c]), c
    assert st["launches"] > 20, st


@pytest.mark.timeout(60)
def test_descriptor_reused_after_a_close_without_detach():
    """a connection closed without a detach leaves its queued messages behind; the next socket
    given the same descriptor number is a new connection: attaching it drops the old one's bytes
    (nowhere to go), and only the new connection's messages reach the new peer"""
    import os as _os
    lib = _lib.host()
    key = bytes([3, 1, 4, 1])
    with make(slot_bytes=1 << 20, nslots=2) as hub:
        a, b = pair()
        hub.attach(a.fileno())
        assert send(lib, Endpoint(a), G.BINARY, b"old connection", key, 1) == 1   # queued
        fd = a.fileno()
        a.close()
        b.close()
        x, y = pair()
        if x.fileno() != fd:   # (the kernel usually hands out the same number by itself)
            _os.dup2(x.fileno(), fd)
            x.close()
            x = socket.socket(fileno=fd)
        rd = Reader(y)
        try:
            hub.attach(x.fileno())
            assert send(lib, Endpoint(x), G.TEXT, b"new connection", key, 2) == 1
            hub.drain()
        finally:
            hub.detach(x.fileno())
        x.shutdown(socket.SHUT_WR)
        got = rd.join()
        x.close()
        y.close()
    assert got == wire([(G.TEXT, b"new connection", 2, key)])


def fault_then_recover(arm, disarm):
    """a failing submission (injected) fails the flush with NETC_GPU_ELAUNCH and leaves the queued
    messages in their slot: the next flush sends them once each, in order -- nothing lost, nothing
    twice"""
    from netc_amd import mask as nm
    lib = _lib.host()
    a, b = pair()
    rd = Reader(b)
    ep = Endpoint(a)
    rng = np.random.default_rng(8)
    msgs = [message(rng) + (bytes([i, 2, 3, 4]),) for i in range(12)]
    with make(slot_bytes=1 << 20, nslots=2) as hub:
        hub.attach(a.fileno())
        try:
            for op, p, nf, key in msgs[:6]:
                assert send(lib, ep, op, p, key, nf) == 1
            arm()
            try:
                with pytest.raises(NetcGpuError) as e:
                    hub.flush()
                assert e.value.code == nm.NETC_GPU_ELAUNCH
            finally:
                disarm()
            for op, p, nf, key in msgs[6:]:
                assert send(lib, ep, op, p, key, nf) == 1
            hub.drain()
        finally:
            hub.detach(a.fileno())
    a.shutdown(socket.SHUT_WR)
    got = rd.join()
    a.close()
    b.close()
    assert got == wire(msgs)


def bad_wire_fails_only_its_slot(arm, disarm):
    """a slot whose wire the device does not vouch for (wire length mismatch) fails its own
    connections as a failed send would -- their next ws_send_message returns -1 -- and the flush
    reports it after sending the later slots; a connection with nothing in that slot, and the
    hub, go on"""
    from netc_amd import mask as nm
    lib = _lib.host()
    (a, b), (c, d) = pair(), pair()
    ra, rc = Reader(b), Reader(d)
    ea, ec = Endpoint(a), Endpoint(c)
    rng = np.random.default_rng(12)
    first = [message(rng) + (bytes([9, 8, 7, i]),) for i in range(4)]
    later = [message(rng) + (bytes([1, 2, 3, i]),) for i in range(6)]
    with make(slot_bytes=1 << 20, nslots=2) as hub:
        hub.attach(a.fileno())
        hub.attach(c.fileno())
        try:
            for op, p, nf, key in first:   # connection a only: the slot that goes bad
                assert send(lib, ea, op, p, key, nf) == 1
            arm()
            try:
                with pytest.raises(NetcGpuError) as e:
                    hub.flush()
                assert e.value.code == nm.NETC_GPU_ERUNTIME
            finally:
                disarm()
            op, p, nf, key = later[0]
            assert send(lib, ea, op, p, key, nf) == -1   # its bytes are gone: the connection failed
            for op, p, nf, key in later:
                assert send(lib, ec, op, p, key, nf) == 1
            assert hub.drain() > 0
            st = hub.stats()
        finally:
            hub.detach(a.fileno())
            hub.detach(c.fileno())
    for s in (a, c):
        s.shutdown(socket.SHUT_WR)
    got_a, got_c = ra.join(), rc.join()
    for s in (a, b, c, d):
        s.close()
    assert got_a == b""
    assert got_c == wire(later)
    assert st["send_errors"] == 1, st


@pytest.mark.timeout(60)
def test_injected_fault_then_recovery():
    from netc_amd import mask as nm
    _lib.gpu().netc_gpu_knob.restype = ctypes.c_int
    fault_then_recover(lambda: _lib.gpu().netc_gpu_knob(nm.KNOBS["INJECT_FAULT"], 0),
                       lambda: _lib.gpu().netc_gpu_knob(nm.KNOBS["INJECT_FAULT"], -1))


@pytest.mark.timeout(180)
def test_echo_server_both_hubs():
    """netc's server loop with both hubs: every client's masked messages come in through the
    receive hub (one ws_parse_frame per readable socket per iteration) and go back out through
    the egress hub (ws_send_message, unmasked as a server sends, one flush per iteration); each
    client gets back exactly the frames of what it sent"""
    import select
    from tests.wsutil import ParseState, libc
    lib = _lib.host()
    rng = np.random.default_rng(99)
    nconn, nmsg = 32, 25
    pairs = [G.tcp_pair() for _ in range(nconn)]
    msgs = [[message(rng) for _ in range(nmsg)] for _ in range(nconn)]
    keys = [[bytes(rng.integers(0, 256, 4, dtype=np.uint8)) for _ in range(nmsg)] for _ in range(nconn)]
    readers = [Reader(c) for c, _ in pairs]

    def client():
        for i in range(nmsg):
            for c in range(nconn):
                op, p, nf = msgs[c][i]
                pairs[c][0].sendall(G.wire_of([(op, p, nf, [keys[c][i]] * nf)]))

    socks = [s for _, s in pairs]
    with nh.Hub(lib=HUB_LIB, slot_bytes=1 << 20, nslots=4) as rx, make(slot_bytes=1 << 20, nslots=3) as tx:
        for s in socks:
            s.setblocking(False)
            rx.attach(s.fileno())
            tx.attach(s.fileno())
        eps = [Endpoint(s) for s in socks]
        sts = [ParseState() for _ in socks]
        index = {s.fileno(): c for c, s in enumerate(socks)}
        th = threading.Thread(target=client)
        th.start()
        try:
            left = nconn * nmsg
            while left:
                ready, _, _ = select.select(socks, [], [], 10)
                assert ready, f"stranded: {nconn * nmsg - left} of {nconn * nmsg}"
                for s in ready:
                    c = index[s.fileno()]
                    rc = lib.ws_parse_frame(ctypes.byref(eps[c].client), ctypes.byref(sts[c]), 1 << 20)
                    if rc == 0:
                        m = sts[c].message
                        n = m.payload_length - (1 if m.opcode == G.TEXT else 0)   # (the NUL the reference appends)
                        echo = WsMessage()
                        lib.ws_build_message(ctypes.byref(echo), m.opcode, n, m.buffer)
                        assert lib.ws_send_message(ctypes.byref(eps[c].client), ctypes.byref(echo), None, 1) == 1
                        libc.free(m.buffer)
                        ctypes.memset(ctypes.byref(sts[c]), 0, ctypes.sizeof(sts[c]))
                        left -= 1
                    else:
                        assert rc == 1, rc
                tx.flush()   # once per loop iteration
            th.join()
            tx.drain()
            st = tx.stats()
        finally:
            for s in socks:
                rx.detach(s.fileno())
                tx.detach(s.fileno())
    for c, s in pairs:
        s.shutdown(socket.SHUT_WR)
    got = [rd.join() for rd in readers]
    for c, s in pairs:
        c.close()
        s.close()
    for c in range(nconn):
        want = wire([(op, p, 1, None) for op, p, _ in msgs[c]])
        assert got[c] == want, c
    assert st["messages"] == nconn * nmsg and st["max_connections"] > 1, st


@pytest.mark.timeout(300)
@pytest.mark.parametrize("chunk", ["0", "65536"])
def test_echo_server_driver(chunk):
    """tests/drivers/ws_echo_server.c: 256 TCP connections, 40 masked requests each, echoed by a
    netc-shaped loop through the receive hub and the egress hub; every connection's reply bytes
    hashed against the expected frames, beside libnetc's CPU leg"""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(root, "tests", "bin", "ws_echo_server")
    assert os.path.exists(exe), "tests/bin/ws_echo_server missing: run make"
    for leg in ("hub", "cpu"):
        r = subprocess.run([exe, leg, "256", "40", "1024", chunk], capture_output=True, text=True, timeout=240,
                           cwd=root)
        assert r.returncode == 0, f"{leg}: rc {r.returncode}\n{r.stdout[-2000:]}\n{r.stderr[-3000:]}"
        d = json.loads(r.stdout.strip().splitlines()[-1])
        assert d["mismatched"] == 0 and d["messages"] == 256 * 40, d
        if leg == "hub":
            assert d["rx_launches"] >= 1 and d["tx_launches"] >= 1 and d["tx_max_conns_per_launch"] > 1, d


def small_buffers(*socks, size=1 << 16):
    for s in socks:
        s.setsockopt(socket.SOL_SOCKET, socket.SO_SNDBUF, size)
        s.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, size)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("bounded", [False, True])
def test_one_stalled_reader_of_256(bounded):
    """one of 256 connections stops reading until its socket is full: no flush waits for it (each
    returns within ~10 ms), every other connection gets all its messages meanwhile, and the stalled
    one gets every byte once it reads -- or, with the backlog bounded, fails alone with -1 (BADSEND)
    while the others go on.  The reference's send never waits either (src/tcp/server.c:219-225)."""
    import time
    lib = _lib.host()
    lib.netc_ws_send_backlog_limit.argtypes = [ctypes.c_size_t]
    lib.netc_ws_send_backlog_limit.restype = ctypes.c_size_t
    rng = np.random.default_rng(256 + bounded)
    nconn, rounds = 256, 40
    pairs = [pair() for _ in range(nconn)]
    small_buffers(*pairs[0])
    readers = [None] + [Reader(b) for _, b in pairs[1:]]   # connection 0's peer does not read yet
    eps = [Endpoint(a) for a, _ in pairs]
    sent = [[] for _ in range(nconn)]
    bound = 0.010 if HUB_LIB is None else 0.100   # (the mock frames on the CPU, inside the flush)
    old = lib.netc_ws_send_backlog_limit((192 << 10) if bounded else (64 << 20))
    worst, failed_at = 0.0, None
    try:
        with make(slot_bytes=1 << 20, nslots=3) as hub:
            for a, _ in pairs:
                hub.attach(a.fileno())
            try:
                for r in range(rounds):
                    for c in range(nconn):
                        op, p, nf = message(rng)
                        key = bytes(rng.integers(0, 256, 4, dtype=np.uint8)) if c % 2 else None
                        if c == 0:
                            p = rng.integers(0, 256, 16000, dtype=np.uint8).tobytes()
                        rc = send(lib, eps[c], op, p, key, nf)
                        if c == 0 and failed_at is not None:
                            assert rc == -1
                            continue
                        if c == 0 and rc == -1:
                            failed_at = r
                            continue
                        assert rc == 1, (r, c)
                        sent[c].append((op, p, nf, key))
                    t0 = time.perf_counter()
                    hub.flush()
                    worst = max(worst, time.perf_counter() - t0)
                st = hub.stats()
                assert worst < bound, f"a flush took {worst * 1e3:.1f} ms"
                assert st["deferred_sends"] >= 1, st
                settle(*[a for a, _ in pairs[1:]])
                for a, _ in pairs[1:]:
                    a.shutdown(socket.SHUT_WR)
                got = [rd.join() for rd in readers[1:]]
                for c in range(1, nconn):   # everyone else: all of it, while connection 0 was stuck
                    assert got[c - 1] == wire(sent[c]), c
                if bounded:
                    assert failed_at is not None and st["send_errors"] == 1, (failed_at, st)
                else:
                    assert failed_at is None and hub.pending() > 0, st
                    stalled = Reader(pairs[0][1])   # it reads now: every byte, in order
                    hub.drain()
                    settle(pairs[0][0])
                    pairs[0][0].shutdown(socket.SHUT_WR)
                    assert stalled.join() == wire(sent[0])
            finally:
                for a, _ in pairs:
                    hub.detach(a.fileno())
    finally:
        lib.netc_ws_send_backlog_limit(old)
        for a, b in pairs:
            a.close()
            b.close()


@pytest.mark.timeout(60)
def test_reused_descriptor_not_attached_gets_nothing():
    """a connection closed without a detach (a close() the hub never saw), its descriptor number
    reused by a socket that is NOT attached: the flush must not send the old connection's frames to
    the new peer (its identity differs); the old connection fails alone"""
    import os as _os
    lib = _lib.host()
    key = bytes([3, 1, 4, 1])
    with make(slot_bytes=1 << 20, nslots=2) as hub:
        a, b = pair()
        (c, d) = pair()
        rd_other = Reader(d)
        hub.attach(a.fileno())
        hub.attach(c.fileno())
        assert send(lib, Endpoint(a), G.BINARY, b"old connection" * 50, key, 1) == 1   # queued
        assert send(lib, Endpoint(c), G.BINARY, b"still here", key, 1) == 1
        fd = a.fileno()
        a.close()
        b.close()
        x, y = pair()
        if x.fileno() != fd:
            _os.dup2(x.fileno(), fd)
            x.close()
            x = socket.socket(fileno=fd)
        rd = Reader(y)
        try:
            hub.drain()
            st = hub.stats()
        finally:
            hub.detach(c.fileno())
            hub.detach(fd)
        settle(c)
        x.shutdown(socket.SHUT_WR)
        c.shutdown(socket.SHUT_WR)
        assert rd.join() == b""
        assert rd_other.join() == wire([(G.BINARY, b"still here", 1, key)])
        assert st["send_errors"] == 1, st
        for s in (x, y, c, d):
            s.close()


@pytest.mark.timeout(60)
def test_close_frame_goes_out_with_what_was_queued_before_it():
    """netc's ws_server_close_client sends a CLOSE frame and closes the socket at once
    (src/ws/server.c:108-125): a CLOSE on a hub connection flushes immediately, so the peer has the
    replies queued before it and the close frame, in order, without any flush by the loop"""
    lib = _lib.host()
    rng = np.random.default_rng(42)
    (a, b), (c, d) = pair(), pair()
    rc_other = Reader(d)
    msgs = [message(rng) + (None,) for _ in range(6)]
    with make(slot_bytes=1 << 20, nslots=2) as hub:
        hub.attach(a.fileno())
        hub.attach(c.fileno())
        try:
            assert send(lib, Endpoint(c), G.TEXT, b"queued elsewhere", None, 1) == 1
            for op, p, nf, key in msgs:
                assert send(lib, Endpoint(a), op, p, key, nf) == 1
            close_payload = bytes([0x03, 0xEA]) + b"Malformed frame."   # 1002, as src/web/server.c:94
            assert send(lib, Endpoint(a), 8, close_payload, None, 1) == 1
            want = wire(msgs + [(8, close_payload, 1, None)])
            b.settimeout(10)
            got = bytearray()
            while len(got) < len(want):   # no flush from us: the CLOSE did it
                chunk = b.recv(1 << 20)
                assert chunk
                got.extend(chunk)
            assert bytes(got) == want
        finally:
            hub.detach(a.fileno())
            hub.detach(c.fileno())
    settle(c)
    c.shutdown(socket.SHUT_WR)
    assert rc_other.join() == wire([(G.TEXT, b"queued elsewhere", 1, None)])
    for s in (a, b, c, d):
        s.close()
