"""close() on routed sockets (include/ws/route.h "close tracking").

tests/drivers/ws_close_track.c runs in a process linked the way netc links libnetc.so, so its
close() -- like netc's own at src/tcp/server.c:267 and src/ws/server.c:124 -- reaches libnetc.so's
close(): queued egress-hub bytes go out before the descriptor closes, a receive hub releases the
slots a closed connection held, and nothing of a closed connection (route, send backlog) is left
for the next socket to get its number.  MODE raw closes with syscall(SYS_close), which the hooks
never see: the egress hub's per-send identity check still keeps the old connection's frames from a
new, unattached socket with the same number, and a full receive hub finds and drops the closed
holders.  NETC_WS_ROUTE_VERIFY=1 forces the per-call identity checks (close() not "tracked").

The CPU suite runs the driver linked against the mock build of the same host code
(tests/bin/ws_close_track_mock); the GPU suite against libnetc_ws_gpu.so.
"""

import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(exe, mode, verify=False):
    path = os.path.join(ROOT, "tests", "bin", exe)
    assert os.path.exists(path), f"tests/bin/{exe} missing: run make"
    env = dict(os.environ)
    env.pop("NETC_WS_ROUTE_VERIFY", None)
    if verify:
        env["NETC_WS_ROUTE_VERIFY"] = "1"
    r = subprocess.run([path, mode], capture_output=True, text=True, timeout=100, env=env, cwd=ROOT)
    assert r.returncode == 0, f"{exe} {mode}: rc {r.returncode}\n{r.stdout}\n{r.stderr}"
    assert r.stdout.startswith(f"ok {mode} tracked={0 if verify else 1}"), r.stdout


@pytest.mark.timeout(120)
@pytest.mark.parametrize("mode,verify", [("close", False), ("raw", False), ("close", True)])
def test_close_tracking_mock(mode, verify):
    run("ws_close_track_mock", mode, verify)


@pytest.mark.gpu
@pytest.mark.timeout(120)
@pytest.mark.parametrize("mode,verify", [("close", False), ("raw", False), ("close", True)])
def test_close_tracking_gpu(mode, verify):
    run("ws_close_track", mode, verify)


@pytest.mark.parametrize("verify", [False, True])
def test_route_lookup_identity(verify):
    """tests/drivers/ws_route_lookup.c: the lookups of every ws_parse_frame / ws_send_message call on
    an attached socket resolve; close-tracked (netc's link) unless NETC_WS_ROUTE_VERIFY forces the
    per-call fstat.  (The timing it prints is DESIGN.md §16.1's; not asserted here.)"""
    import json
    exe = os.path.join(ROOT, "tests", "bin", "ws_route_lookup")
    env = dict(os.environ)
    env.pop("NETC_WS_ROUTE_VERIFY", None)
    if verify:
        env["NETC_WS_ROUTE_VERIFY"] = "1"
    r = subprocess.run([exe, "20000"], capture_output=True, text=True, env=env, timeout=60)
    assert r.returncode == 0, r.stderr
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["ok"] is True
    assert d["tracked"] == (0 if verify else 1)
