"""The GPU receive route under netc's caller contract over a real TCP connection
(VERDICT r2 "missing" #2; SURVEY.md §3 call stack A, §8(b)).

tests/bin/ws_gpu_epoll (tests/drivers/ws_gpu_epoll.c, built by `make`) is a C program: an
epoll server on 127.0.0.1 that, on every EPOLLIN, calls netc_ws_ingest_recv +
netc_ws_ingest_next_message (the GPU ingest ring: pinned slots, GPU scan or host walk, GPU
unmask) and dispatches each message as netc's web layer dispatches ws_parse_frame's
(reference src/web/server.c:86-140: ping -> pong echo, close -> close reply, message ->
callback, free); and a client that sends through libnetc.so's ws_send_message -- test001's
script (reference tests/ws/test001.c:192-273), a ping, one 16 MiB message in 256 frames, a
burst of 2,000 fragmented messages -- checking every reply with ws_parse_frame.

Route "parse" runs the same server with ONLY netc's ws_parse_frame on its side: the socket is
attached to the ring (netc_ws_gpu_attach), so libnetc.so's ws_parse_frame receives into the ring
and returns the GPU-unmasked messages with the reference's 0 / 1 / < 0 contract.  Route "parse1"
is netc's own loop exactly: ONE ws_parse_frame per EPOLLIN, then back to epoll_wait
(reference src/tcp/server.c:72-75, src/web/server.c:86-98) -- the burst of 2,000 messages sent
without waiting is then delivered only if the ring leaves every undelivered message's bytes in
the socket; a stranded message shows up as the server's 20 s epoll timeout.

Checked here, per scan mode of the ring and route:
  * the program's own checks (replies, pong payload, close echo, 16 MiB and burst hashes);
  * every message the GPU route delivered equals, in order, what libnetc's ws_parse_frame
    delivers from the same bytes -- rebuilt from the client's log of (opcode, key, frames,
    payload) with libnetc's ws_send_message -- control frames included;
  * the keys are the reference's fresh-thread sequence and test001's two masked frames have
    the reference's golden wire bytes (tests/golden/ws_golden.json, made by the compiled
    reference).
"""

import json
import os
import struct
import subprocess

import pytest

from tests.wsutil import parse_stream, send_wire

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "bin", "ws_gpu_epoll")
GOLDEN = json.load(open(os.path.join(ROOT, "tests", "golden", "ws_golden.json")))


def read_server_log(path):
    out = []
    with open(path, "rb") as f:
        data = f.read()
    i = 0
    while i < len(data):
        kind, op = data[i], data[i + 1]
        (n,) = struct.unpack_from("<Q", data, i + 2)
        i += 10
        out.append((chr(kind), op, data[i:i + n]))
        i += n
    return out


def read_client_log(path):
    out = []
    with open(path, "rb") as f:
        data = f.read()
    i = 0
    while i < len(data):
        op, masked = data[i], data[i + 1]
        key = data[i + 2:i + 6]
        frames, n = struct.unpack_from("<QQ", data, i + 6)
        i += 22
        out.append((op, bool(masked), key, frames, data[i:i + n]))
        i += n
    return out


@pytest.mark.timeout(600)
@pytest.mark.parametrize("mode,route", [("auto", "ingest"), ("gpu", "ingest"), ("host", "ingest"),
                                        ("auto", "parse"), ("gpu", "parse"), ("auto", "parse1"), ("gpu", "parse1"),
                                        ("host", "parse1")])
def test_epoll_server_on_gpu_ingest(tmp_path, mode, route):
    # route "parse": the server calls only netc's ws_parse_frame on a socket attached to the ring
    # (netc_ws_gpu_attach) -- the kept C API reaching the GPU
    assert os.path.exists(EXE), "tests/bin/ws_gpu_epoll missing: run make"
    slog, clog = str(tmp_path / "server.log"), str(tmp_path / "client.log")
    r = subprocess.run([EXE, slog, clog, mode, str(1 << 20), route], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, f"rc {r.returncode}\nstdout: {r.stdout}\nstderr: {r.stderr[-3000:]}"
    summary = json.loads(r.stdout.strip().splitlines()[-1])
    assert summary["server_rc"] == 0 and summary["client_ok"] == 1
    assert summary["route"] == route
    if route == "parse1":   # one call per wake-up: at least one wake-up per message
        assert summary["events"] >= summary["delivered"]
    gpu_slots, host_slots = summary["gpu_slots"], summary["host_slots"]
    if mode == "gpu":
        assert host_slots == 0 and gpu_slots > 0
    elif mode == "host":
        assert gpu_slots == 0 and host_slots > 0

    sent = read_client_log(clog)
    got = read_server_log(slog)
    # the keys: the reference's fresh-thread sequence (src/ws/common.c:19-27)
    seq = bytes.fromhex(GOLDEN["key_sequence_fresh_thread"])
    keys = [k for _, masked, k, _, _ in sent if masked]
    assert keys[0] == seq[0:4] and keys[1] == seq[4:8] and keys[2] == seq[8:12]

    # rebuild the wire with libnetc's ws_send_message, and parse it with libnetc's ws_parse_frame
    wire = bytearray()
    golden = {g["name"]: g for g in GOLDEN["send_single_frame"]}
    for i, (op, masked, key, frames, payload) in enumerate(sent):
        rc, w = send_wire(payload, op, key if masked else None, frames)
        assert rc == 1
        if i == 0:   # test001.c:192-202: client -> server TEXT, unmasked
            assert w.hex() == golden["client->server TEXT unmasked (tests/ws/test001.c:192-202)"]["wire"]["hex"]
        if i == 2:   # test001.c:233-246: client -> server BINARY 15 B, key 00 61 c2 23
            assert w.hex() == golden["client->server BINARY 15 B (tests/ws/test001.c:233-246)"]["wire"]["hex"]
        if i == 3:   # test001.c:253-266: client -> server TEXT 35 B, key 84 e5 46 a7
            name = [n for n in golden if n.startswith("client->server TEXT 35 B")][0]
            assert w.hex() == golden[name]["wire"]["hex"]
        wire.extend(w)
    step = 1 << 20   # the socketpair holds a few MiB: feed the parser 1 MiB at a time
    chunks = [step] * (len(wire) // step) + ([len(wire) % step] if len(wire) % step else [])
    msgs, rc = parse_stream(bytes(wire), chunks=chunks)
    assert rc == 0
    assert len(got) == len(msgs) == len(sent) == summary["delivered"]
    for j, ((kind, op, payload), (eop, epayload)) in enumerate(zip(got, msgs)):
        assert op == eop, f"message {j}: opcode {op} vs {eop}"
        assert payload == epayload, f"message {j} ({len(payload)} vs {len(epayload)} bytes) differs"
    kinds = [k for k, _, _ in got]
    assert kinds.count("P") == 1 and kinds[-1] == "C"
    big = [p for _, op, p in got if op == 2 and len(p) == 16 << 20]
    assert len(big) == 1
