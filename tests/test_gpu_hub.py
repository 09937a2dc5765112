"""One GPU receive ring shared by many connections (include/ws/hub.h; VERDICT r4 "next" #7).

netc's server serves every client from one event loop (reference src/tcp/server.c:30-75) and
calls ws_parse_frame once per readable client (src/web/server.c:69-98).  With every socket
attached to one hub, the frames of all connections share the hub's slots, so one unmask launch
covers frames from many sockets -- the C2 shape from real sockets.

Checked here, with the server driven exactly as netc drives it (one ws_parse_frame per
readable socket per loop iteration):
  * per connection, the delivered messages are exactly what its client sent, in order -- each
    compared with the plaintext (the wire is oracle_encode_batch's: the reference's send path
    pinned by the golden vectors in tests/test_oracle.py), a TEXT message with the NUL the
    reference appends (src/ws/common.c:340-344);
  * launches span frames of many connections (the hub's counters);
  * the same per-connection results through libnetc's CPU ws_parse_frame
    (tests/drivers/ws_hub_server.c: 256 connections, its per-connection hashes equal for the
    hub, the CPU parser and the reference's own parser).

tests/test_route_mock.py runs the Python cases on the CPU, over the mock HIP runtime.
"""

import ctypes
import json
import os
import select
import socket
import subprocess
import threading
import time

import numpy as np
import pytest

from netc_amd import _lib
from netc_amd import hub as nh
from netc_amd.mask import NETC_GPU_EINVAL, NetcGpuError
from tests import test_gpu_route as G
from tests.wsutil import Endpoint, ParseState, libc

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "bin", "ws_hub_server")
HUB_LIB = None   # the library holding the hub (None: libnetc_ws_gpu.so; the CPU tests set the mock)


def make_hub(**kw):
    return nh.Hub(lib=HUB_LIB, **kw)


def serve(nconn, nmsg, rng, slot_bytes=1 << 20, sizes=(0, 1, 17, 125, 126, 700, 1024, 3000), kind="tcp",
          timeout=10.0):
    """nconn client sockets sending nmsg messages each (round robin, no waiting); the server loop
    calls ws_parse_frame once per readable socket.  Returns (per-connection delivered, expected, stats)."""
    lib = _lib.host()
    pairs = [G.tcp_pair() if kind == "tcp" else G.pair() for _ in range(nconn)]
    msgs = []
    for c in range(nconn):
        m = []
        for i in range(nmsg):
            op = G.PING if i % 13 == 12 else int(rng.choice([G.TEXT, G.BINARY]))
            ln = int(rng.integers(0, 126)) if op == G.PING else int(rng.choice(sizes))
            nf = 1 if op == G.PING else int(rng.choice([1, 1, 2, 3]))
            m.append((op, rng.integers(0, 256, ln, dtype=np.uint8).tobytes(), nf,
                      [rng.integers(0, 256, 4, dtype=np.uint8).tobytes() for _ in range(nf)]))
        msgs.append(m)
    wires = [[G.wire_of([x]) for x in m] for m in msgs]

    def client():
        for i in range(nmsg):
            for c in range(nconn):
                pairs[c][0].sendall(wires[c][i])

    got = [[] for _ in range(nconn)]
    with make_hub(slot_bytes=slot_bytes, nslots=8, max_frame_bytes=65536) as hub:
        socks = [s for _, s in pairs]
        for s in socks:
            s.setblocking(False)
            hub.attach(s.fileno())
        eps = [Endpoint(s) for s in socks]
        sts = [ParseState() for _ in socks]
        index = {s.fileno(): c for c, s in enumerate(socks)}
        th = threading.Thread(target=client)
        th.start()
        try:
            left = nconn * nmsg
            while left:
                ready, _, _ = select.select(socks, [], [], timeout)
                assert ready, f"stranded: {nconn * nmsg - left} of {nconn * nmsg} delivered, stats {hub.stats()}"
                for s in ready:   # netc: on_data once per readable client
                    c = index[s.fileno()]
                    rc = lib.ws_parse_frame(ctypes.byref(eps[c].client), ctypes.byref(sts[c]), 1 << 20)
                    if rc == 0:
                        m = sts[c].message
                        got[c].append((int(m.opcode), ctypes.string_at(m.buffer, m.payload_length)))
                        libc.free(m.buffer)
                        ctypes.memset(ctypes.byref(sts[c]), 0, ctypes.sizeof(sts[c]))
                        left -= 1
                    else:
                        assert rc == 1, f"connection {c}: ws_parse_frame returned {rc}"
            th.join()
            stats = hub.stats()
        finally:
            for s in socks:
                hub.detach(s.fileno())
    for a, b in pairs:
        a.close()
        b.close()
    return got, [G.expected(m) for m in msgs], stats


@pytest.mark.timeout(300)
@pytest.mark.parametrize("nconn,nmsg,slot", [(64, 40, 1 << 20), (256, 12, 1 << 20), (16, 60, 128 << 10)])
def test_hub_many_connections(nconn, nmsg, slot):
    rng = np.random.default_rng(nconn * 1000 + nmsg)
    got, want, stats = serve(nconn, nmsg, rng, slot_bytes=slot)
    for c in range(nconn):
        assert got[c] == want[c], f"connection {c}: {len(got[c])} vs {len(want[c])} messages"
    assert stats["connections"] == nconn
    assert stats["max_connections"] > 1, stats   # launches spanned frames of several sockets
    assert stats["frames"] >= nconn * nmsg


@pytest.mark.timeout(120)
def test_hub_unix_sockets_and_big_frames():
    rng = np.random.default_rng(3)
    got, want, stats = serve(8, 20, rng, sizes=(0, 5000, 65535, 40000), kind="unix")
    assert got == want


def test_hub_attach_rules():
    a, b = G.tcp_pair()
    with make_hub(slot_bytes=1 << 20, nslots=2) as h1, make_hub(slot_bytes=1 << 20, nslots=2) as h2:
        h1.attach(b.fileno())
        h1.attach(b.fileno())   # the same connection again: a no-op
        with pytest.raises(NetcGpuError) as e:
            h2.attach(b.fileno())   # another route serves it
        assert e.value.code == NETC_GPU_EINVAL
        with pytest.raises(NetcGpuError):
            h1.attach(1 << 29)
        h1.detach(b.fileno())
        h2.attach(b.fileno())
        h2.detach(b.fileno())
        with pytest.raises(NetcGpuError):
            nh.Hub(lib=HUB_LIB, slot_bytes=4096, max_frame_bytes=65536)   # a slot must hold a frame
    a.close()
    b.close()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("chunk", ["0", "65536"])
def test_hub_server_256_connections_equals_cpu_parser(chunk):
    """tests/drivers/ws_hub_server.c: 256 TCP connections, 200 messages each (0-1024 B, 1-3
    fragments, PINGs), netc's loop; every message regenerated and compared; the per-connection
    results of the hub equal those of libnetc's CPU ws_parse_frame and of the reference's own
    parser (when oracle/_ref is present).  chunk 65536: the clients' frames rendered in memory
    beforehand and sent 64 KiB per send() (many messages per read on the server side)"""
    assert os.path.exists(EXE), "tests/bin/ws_hub_server missing: run make"
    out = {}
    legs = ["hub", "cpu"] + (["ref"] if os.path.exists(os.path.join(ROOT, "oracle", "_ref", "libref_ws.so")) else [])
    for leg in legs:
        r = subprocess.run([EXE, leg, "256", "200", "1024", "0", "1", "-", chunk], capture_output=True, text=True,
                           timeout=240, cwd=ROOT)
        assert r.returncode == 0, f"{leg}: rc {r.returncode}\n{r.stdout[-2000:]}\n{r.stderr[-3000:]}"
        out[leg] = json.loads(r.stdout.strip().splitlines()[-1])
        assert out[leg]["bad"] == 0 and out[leg]["mismatched"] == 0 and out[leg]["verified"] == 1
    for leg in legs[1:]:
        assert out[leg]["conn_hash"] == out["hub"]["conn_hash"]
    hub = out["hub"]
    assert hub["frames"] >= 256 * 200 and hub["max_conns_per_launch"] >= 16, hub


def _call(lib, ep, st, limit=1 << 20, tries=200):
    """ws_parse_frame once per readiness until it returns something other than 1 (or tries run out)"""
    rc = 1
    for _ in range(tries):
        if not select.select([ep.sock], [], [], 2)[0]:
            return 1
        rc = lib.ws_parse_frame(ctypes.byref(ep.client), ctypes.byref(st), limit)
        if rc != 1:
            return rc
    return rc


def _take(st):
    m = st.message
    out = (int(m.opcode), ctypes.string_at(m.buffer, m.payload_length))
    libc.free(m.buffer)
    ctypes.memset(ctypes.byref(st), 0, ctypes.sizeof(st))
    return out


@pytest.mark.timeout(60)
def test_hub_stream_errors_after_the_messages_before_them():
    """per connection, as the reference's parser and the single-connection ring: every complete
    message before a bad frame is delivered first, then the error, and it stays; other
    connections of the hub go on (strict: an unmasked client frame; a frame over the hub's
    limit; a message over the caller's limit; the peer closing)"""
    lib = _lib.host()
    good = [(G.TEXT, b"first", 1, [b"\x01\x02\x03\x04"]), (G.BINARY, bytes(range(200)), 2, [b"\x05\x06\x07\x08"] * 2)]
    unmasked = bytes([0x81, 0x03]) + b"abc"
    big = G.wire_of([(G.BINARY, bytes(5000), 1, [b"\x09\x09\x09\x09"])])
    pairs = [G.tcp_pair() for _ in range(4)]
    with make_hub(slot_bytes=64 << 10, nslots=4, max_frame_bytes=4096, strict=True) as hub:
        eps, sts = [], []
        for c, s in pairs:
            s.setblocking(False)
            hub.attach(s.fileno())
            eps.append(Endpoint(s))
            sts.append(ParseState())
        try:
            pairs[0][0].sendall(G.wire_of(good) + unmasked)          # strict: MASK clear
            pairs[1][0].sendall(G.wire_of(good) + big)               # 5,000 B > the hub's 4,096
            pairs[2][0].sendall(G.wire_of(good))                     # fine, then closes
            pairs[2][0].shutdown(socket.SHUT_WR)
            pairs[3][0].sendall(G.wire_of(good))                     # fine, stays open
            want = G.expected(good)
            for c in range(4):
                for m in want:
                    assert _call(lib, eps[c], sts[c], limit=1 << 20) == 0, c
                    assert _take(sts[c]) == m
            assert _call(lib, eps[0], sts[0]) == ni_codes.INVALID
            assert _call(lib, eps[0], sts[0]) == ni_codes.INVALID   # sticky
            assert _call(lib, eps[1], sts[1]) == ni_codes.TOO_BIG
            assert _call(lib, eps[2], sts[2]) == ni_codes.RECV
            assert _call(lib, eps[3], sts[3], tries=3) == 1          # nothing more, still open
            # a message over the caller's limit (src/ws/common.c:210-211)
            pairs[3][0].sendall(G.wire_of([(G.BINARY, bytes(3000), 1, [b"\x0a\x0b\x0c\x0d"])]))
            assert _call(lib, eps[3], sts[3], limit=2000) == ni_codes.TOO_BIG
        finally:
            for _, s in pairs:
                hub.detach(s.fileno())
    for a, b in pairs:
        a.close()
        b.close()


@pytest.mark.timeout(60)
def test_hub_detach_with_frames_pending():
    """a connection detached while its frames sit in the shared slots: the other connections'
    messages still arrive, the slots return to the pool (many more messages pass through 2 slots)"""
    lib = _lib.host()
    rng = np.random.default_rng(12)
    pairs = [G.tcp_pair() for _ in range(3)]
    with make_hub(slot_bytes=32 << 10, nslots=2, max_frame_bytes=8192) as hub:
        eps, sts = [], []
        for c, s in pairs:
            s.setblocking(False)
            hub.attach(s.fileno())
            eps.append(Endpoint(s))
            sts.append(ParseState())
        try:
            msgs = [(G.BINARY, rng.integers(0, 256, 700, dtype=np.uint8).tobytes(), 1,
                     [bytes(rng.integers(0, 256, 4, dtype=np.uint8))]) for _ in range(60)]
            for c, _ in pairs:
                c.sendall(G.wire_of(msgs[:5]))
            # connection 0 reads its frames into the hub, then is dropped with them undelivered
            assert _call(lib, eps[0], sts[0], tries=1) in (0, 1)
            hub.detach(pairs[0][1].fileno())
            got = {1: [], 2: []}
            for i in range(5, 60):
                for c in (1, 2):
                    pairs[c][0].sendall(G.wire_of([msgs[i]]))
            for c in (1, 2):
                while len(got[c]) < 60:
                    rc = _call(lib, eps[c], sts[c])
                    assert rc == 0, (c, len(got[c]), rc)
                    got[c].append(_take(sts[c]))
            assert got[1] == got[2] == G.expected(msgs)
            assert hub.stats()["connections"] == 2
        finally:
            for _, s in pairs[1:]:
                hub.detach(s.fileno())
    for a, b in pairs:
        a.close()
        b.close()


@pytest.mark.timeout(120)
def test_hub_table_fills_before_the_bytes():
    """the flood of empty frames (test_gpu_route.flood_of_empty_frames) on a hub with the smallest
    slot: one peek holds far more frames than a slot's frame table, so each take records what
    fits and carries the rest -- complete frames included -- walking them before new bytes and
    keeping the hostage meanwhile (round 5: without that, the carried frames were stranded)"""
    with make_hub(slot_bytes=65536 + 14 + 4096, nslots=2, max_frame_bytes=65536) as hub:
        G.flood_of_empty_frames(lambda: hub)
        st = hub.stats()
    assert st["frames"] >= 30000 and st["launches"] > 10, st


@pytest.mark.timeout(120)
def test_hub_many_connections_trickle_then_close():
    """8 connections whose peers send 1-7 bytes at a time with pauses (headers, keys and payloads
    cut anywhere, the pieces of different connections interleaved), then close: per connection
    every message in order, then WS_FRAME_PARSE_ERROR_RECV (src/ws/common.c:151-154)"""
    lib = _lib.host()
    rng = np.random.default_rng(29)
    nconn = 8
    pairs = [G.tcp_pair() for _ in range(nconn)]
    msgs = [G.script(rng, 10) for _ in range(nconn)]
    wires = [G.wire_of(m) for m in msgs]

    def trickle():
        pos = [0] * nconn
        while any(pos[c] < len(wires[c]) for c in range(nconn)):
            for c in range(nconn):
                if pos[c] >= len(wires[c]):
                    continue
                n = int(rng.integers(1, 8)) if pos[c] < 300 else 40000
                pairs[c][0].sendall(wires[c][pos[c]:pos[c] + n])
                pos[c] += n
                if pos[c] >= len(wires[c]):
                    pairs[c][0].shutdown(socket.SHUT_WR)
            time.sleep(0.001)

    got = [[] for _ in range(nconn)]
    codes = [None] * nconn
    with make_hub(slot_bytes=1 << 20, nslots=4, max_frame_bytes=1 << 17) as hub:
        socks = [s for _, s in pairs]
        eps, sts = [], []
        for s in socks:
            s.setblocking(False)
            hub.attach(s.fileno())
            eps.append(Endpoint(s))
            sts.append(ParseState())
        index = {s.fileno(): c for c, s in enumerate(socks)}
        th = threading.Thread(target=trickle)
        th.start()
        try:
            while any(x is None for x in codes):
                live = [s for c, s in enumerate(socks) if codes[c] is None]
                ready, _, _ = select.select(live, [], [], 10)
                assert ready, f"stranded: {[len(g) for g in got]} delivered, codes {codes}"
                for s in ready:
                    c = index[s.fileno()]
                    rc = lib.ws_parse_frame(ctypes.byref(eps[c].client), ctypes.byref(sts[c]), 1 << 20)
                    if rc == 0:
                        got[c].append(_take(sts[c]))
                    elif rc != 1:
                        codes[c] = rc
            th.join()
        finally:
            for s in socks:
                hub.detach(s.fileno())
    for a, b in pairs:
        a.close()
        b.close()
    for c in range(nconn):
        assert got[c] == G.expected(msgs[c]), c
        assert codes[c] == ni_codes.RECV, codes


@pytest.mark.timeout(120)
def test_hub_client_side_unmasked_frames():
    with make_hub(slot_bytes=1 << 20, nslots=3, max_frame_bytes=1 << 17) as hub:
        G.client_side_case(lambda: hub)


@pytest.mark.timeout(60)
def test_hub_blocking_socket_never_stalls_the_loop():
    with make_hub(slot_bytes=1 << 20, nslots=2) as hub:
        G.blocking_socket_case(hub.attach, hub.detach)


class ni_codes:
    RECV, INVALID, TOO_BIG = -1, -2, -3
