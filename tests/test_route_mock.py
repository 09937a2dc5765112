"""The ingest ring's host code and the ws_parse_frame route, on the CPU (no GPU needed).

tests/bin/libnetc_ingest_mock.so is netc_amd/csrc/ws_ingest.hip -- the ring's stream accounting,
slot carries, message reassembly, the peek-and-consume route of netc_ws_gpu_attach and its
one-ring-one-connection rules -- compiled by g++ over a host-memory mock of the HIP runtime
(tests/mockhip: "device" memory is host memory, streams run their work when queued, the frame
scan is libnetc's host header walk and the unmask the reference's scalar loop).  The same test
bodies as tests/test_gpu_route.py (which runs them on the real ring, on the GPU) run here, so
the route's contract with netc's once-per-EPOLLIN caller (reference src/tcp/server.c:72-75 ->
src/web/server.c:86-98) is checked in the CPU suite too.  The mock is test infrastructure
only: the product library is libnetc_ws_gpu.so, built by hipcc, and has no CPU fallback.
"""

import ctypes
import os
import select
import socket
import threading

import numpy as np
import pytest

from netc_amd import _lib
from netc_amd import ingest as ni
from netc_amd.mask import NETC_GPU_ELAUNCH, NetcGpuError
from tests import test_gpu_route as G
from tests.wsutil import Endpoint, ParseState

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MOCK = os.path.join(ROOT, "tests", "bin", "libnetc_ingest_mock.so")


@pytest.fixture
def mock(monkeypatch):
    assert os.path.exists(MOCK), "tests/bin/libnetc_ingest_mock.so missing: run make"
    lib = ctypes.CDLL(MOCK)
    init = ni.Ingest.__init__

    def with_lib(self, *args, **kwargs):
        kwargs.setdefault("lib", lib)
        init(self, *args, **kwargs)

    monkeypatch.setattr(ni.Ingest, "__init__", with_lib)
    return lib


@pytest.mark.timeout(120)
@pytest.mark.parametrize("kind", ["tcp", "unix"])
@pytest.mark.parametrize("slot_bytes,scan", [(1 << 16, "gpu"), (1 << 20, "auto"), (1 << 20, "host")])
def test_once_per_event_delivers_everything(mock, kind, slot_bytes, scan):
    G.test_once_per_event_delivers_everything(kind, slot_bytes, scan)


@pytest.mark.timeout(60)
def test_trickle_one_byte_at_a_time_then_close(mock):
    G.test_trickle_one_byte_at_a_time_then_close()


def test_one_ring_one_connection(mock):
    G.test_one_ring_one_connection()


def test_route_does_not_outlive_its_connection(mock):
    G.test_route_does_not_outlive_its_connection()


def test_device_failure_is_not_a_parse_error(mock):
    """a failing submission reaches ws_parse_frame's caller as NETC_GPU_ELAUNCH (-103), never as a
    WS_FRAME_PARSE_ERROR_* (-1..-3), and stays"""
    lib = _lib.host()
    c, s = G.tcp_pair()
    s.setblocking(False)
    ep = Endpoint(s)
    with ni.Ingest(slot_bytes=1 << 16, nslots=2) as ing:
        ing.attach(s.fileno())
        try:
            mock.netc_mock_inject_fault(0)
            c.sendall(G.wire_of([(1, b"hello", 1, [b"\x37\xfa\x21\x3d"])]))
            assert select.select([s], [], [], 5)[0]
            st = ParseState()
            assert lib.ws_parse_frame(ctypes.byref(ep.client), ctypes.byref(st), 1 << 20) == NETC_GPU_ELAUNCH
            assert lib.ws_parse_frame(ctypes.byref(ep.client), ctypes.byref(st), 1 << 20) == NETC_GPU_ELAUNCH
        finally:
            mock.netc_mock_inject_fault(-1)
            ing.detach(s.fileno())
    c.close()
    s.close()


@pytest.mark.timeout(120)
@pytest.mark.parametrize("msg_bytes", [16, 1024, 70000])
def test_peer_waits_for_each_reply(mock, msg_bytes):
    """request / reply: the peer sends a message and waits for the server to have delivered it
    before sending the next -- the case a read-ahead that strands bytes would deadlock"""
    lib = _lib.host()
    rng = np.random.default_rng(msg_bytes)
    c, s = G.tcp_pair()
    s.setblocking(False)
    ep = Endpoint(s)
    delivered = threading.Semaphore(0)
    msgs = [(2, rng.integers(0, 256, msg_bytes, dtype=np.uint8).tobytes(), 1, [bytes(rng.integers(0, 256, 4, dtype=np.uint8))])
            for _ in range(50)]

    def peer():
        for m in msgs:
            c.sendall(G.wire_of([m]))
            assert delivered.acquire(timeout=10)

    th = threading.Thread(target=peer)
    with ni.Ingest(slot_bytes=1 << 20, nslots=2, max_frame_bytes=1 << 17) as ing:
        ing.attach(s.fileno())
        try:
            th.start()
            st = ParseState()
            got = []
            while len(got) < len(msgs):
                assert select.select([s], [], [], 10)[0], f"stranded after {len(got)}"
                rc = lib.ws_parse_frame(ctypes.byref(ep.client), ctypes.byref(st), 1 << 20)
                if rc == 0:
                    got.append((st.message.opcode, ctypes.string_at(st.message.buffer, st.message.payload_length)))
                    G.libc.free(st.message.buffer)
                    ctypes.memset(ctypes.byref(st), 0, ctypes.sizeof(st))
                    delivered.release()
                else:
                    assert rc == 1
            th.join()
        finally:
            ing.detach(s.fileno())
    c.close()
    s.close()
    assert got == [(op, p) for op, p, _, _ in msgs]


# ---------------------------------------------------------------- the shared ring (hub) --

@pytest.fixture
def hub_mock(mock, monkeypatch):
    from tests import test_gpu_hub as H
    monkeypatch.setattr(H, "HUB_LIB", mock)
    return H


@pytest.mark.timeout(120)
@pytest.mark.parametrize("nconn,nmsg,slot", [(64, 40, 1 << 20), (16, 60, 128 << 10)])
def test_hub_many_connections(hub_mock, nconn, nmsg, slot):
    hub_mock.test_hub_many_connections(nconn, nmsg, slot)


@pytest.mark.timeout(60)
def test_hub_unix_sockets_and_big_frames(hub_mock):
    hub_mock.test_hub_unix_sockets_and_big_frames()


def test_hub_attach_rules(hub_mock):
    hub_mock.test_hub_attach_rules()


def test_hub_stream_errors_after_the_messages_before_them(hub_mock):
    hub_mock.test_hub_stream_errors_after_the_messages_before_them()


def test_hub_detach_with_frames_pending(hub_mock):
    hub_mock.test_hub_detach_with_frames_pending()


def test_blocking_socket_never_stalls_the_loop(mock):
    G.test_blocking_socket_never_stalls_the_loop()


def test_flood_of_empty_frames(mock):
    G.test_flood_of_empty_frames()


def test_client_side_unmasked_frames(mock):
    G.test_client_side_unmasked_frames()


def test_hub_client_side_unmasked_frames(hub_mock):
    hub_mock.test_hub_client_side_unmasked_frames()


def test_hub_many_connections_trickle_then_close(hub_mock):
    hub_mock.test_hub_many_connections_trickle_then_close()


def test_hub_table_fills_before_the_bytes(hub_mock):
    hub_mock.test_hub_table_fills_before_the_bytes()


def test_hub_blocking_socket_never_stalls_the_loop(hub_mock):
    hub_mock.test_hub_blocking_socket_never_stalls_the_loop()


def test_route_errors_after_the_messages_before_them(mock):
    G.test_route_errors_after_the_messages_before_them()


# ---------------------------------------------------------- the shared send ring (egress hub) --

@pytest.fixture
def egress_hub_mock(mock, monkeypatch):
    from tests import test_gpu_egress_hub as E
    monkeypatch.setattr(E, "HUB_LIB", mock)
    return E


@pytest.mark.timeout(120)
@pytest.mark.parametrize("nconn,rounds,slot", [(64, 30, 1 << 20), (16, 40, 64 << 10)])
def test_egress_hub_many_connections_interleaved(egress_hub_mock, nconn, rounds, slot):
    egress_hub_mock.test_many_connections_interleaved(nconn, rounds, slot)


def test_egress_hub_detach_sends_what_was_queued_then_cpu_path(egress_hub_mock):
    egress_hub_mock.test_detach_sends_what_was_queued_then_cpu_path()


def test_egress_hub_a_peer_gone_fails_only_its_connection(egress_hub_mock):
    egress_hub_mock.test_a_peer_gone_fails_only_its_connection()


def test_egress_hub_rules_and_limits(egress_hub_mock):
    egress_hub_mock.test_rules_and_limits()


def test_egress_hub_slots_run_out_between_flushes(egress_hub_mock):
    egress_hub_mock.test_slots_run_out_between_flushes()


def test_egress_hub_descriptor_reused_after_a_close_without_detach(egress_hub_mock):
    egress_hub_mock.test_descriptor_reused_after_a_close_without_detach()


def test_egress_hub_injected_fault_then_recovery(egress_hub_mock, mock):
    egress_hub_mock.fault_then_recover(lambda: mock.netc_mock_inject_fault(0), lambda: mock.netc_mock_inject_fault(-1))


def test_egress_hub_echo_server_both_hubs(egress_hub_mock):
    egress_hub_mock.test_echo_server_both_hubs()


def test_egress_hub_bad_wire_fails_only_its_slot(egress_hub_mock, mock):
    egress_hub_mock.bad_wire_fails_only_its_slot(lambda: mock.netc_mock_bad_wire(0), lambda: mock.netc_mock_bad_wire(-1))


@pytest.mark.timeout(300)
@pytest.mark.parametrize("bounded", [False, True])
def test_egress_hub_one_stalled_reader_of_256(egress_hub_mock, bounded):
    egress_hub_mock.test_one_stalled_reader_of_256(bounded)


def test_egress_hub_reused_descriptor_not_attached_gets_nothing(egress_hub_mock):
    egress_hub_mock.test_reused_descriptor_not_attached_gets_nothing()


def test_egress_hub_close_frame_goes_out_with_what_was_queued_before_it(egress_hub_mock):
    egress_hub_mock.test_close_frame_goes_out_with_what_was_queued_before_it()
