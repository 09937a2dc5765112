"""The drop-in, proven with netc's own caller (CPU, build container only).

oracle/Makefile `dropin` compiles the reference's WS integration test (tests/ws/test001.c, run
alone by oracle/dropin_main.c as the reference's main.c:11,40 runs it) with the reference's own
callers -- src/web, src/http, src/tcp, src/ws/{server,client}.c, src/utils, src/socket.c --
from /root/reference where they lie (only SURVEY.md §4's one-token fix of src/http/common.c:132,
on a copy), twice:
  * with the reference's own src/ws/common.c (the baseline the reference passes 12/12 with);
  * with libnetc.so of this repo INSTEAD of src/ws/common.c.
Both must pass all 12 checks of test001.c:353-461.  The libnetc build must bind the WS path
(ws_parse_frame, ws_send_message, ws_build_masking_key) to libnetc.so; the utilities libnetc.so
also exports under netc's names (vector_*, tcp_server_send, netc_errno_reason) are interposed
by the program's own copies, so they must behave as the reference's: oracle/vector_probe.c runs
the same vector_* sequence against both implementations and must print the same.

Skipped where /root/reference is absent (the GPU box): nothing here reads it at run time there.
"""

import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
ORACLE = os.path.join(ROOT, "oracle")
DROPIN_DIR = "/tmp/netc_dropin"   # oracle/Makefile DROPIN_DIR: outside the repository
LIBNETC = os.path.join(ROOT, "netc_amd", "lib", "libnetc.so")

pytestmark = pytest.mark.skipif(not os.path.isfile(os.path.join(REF, "tests", "ws", "test001.c")),
                                reason="needs the reference sources (build container only)")

CHECKS = ["on_connect_server", "send_basic_server", "send_multiple_frames_server", "send_masked_server",
          "send_multiple_frames_masked_server", "send_close_server", "on_open_client", "send_basic_client",
          "send_multiple_frames_client", "send_masked_client", "send_multiple_frames_masked_client",
          "send_close_client"]


@pytest.fixture(scope="module")
def built():
    subprocess.run(["make", "-C", ORACLE, "dropin"], check=True, capture_output=True, text=True)
    return {k: os.path.join(DROPIN_DIR, f"ws_test001_{k}") for k in ("reference", "libnetc")}


def run(exe, env=None):
    # the test binds 127.0.0.1:8923 (test001.c:42-43); both runs are sequential
    p = subprocess.run([exe], capture_output=True, text=True, timeout=120, env=env)
    return p.returncode, re.sub(r"\x1b\[[0-9;]*m", "", p.stdout), p.stderr


def passed_checks(out):
    return [c for c in CHECKS if f"[WS TEST CASE 001] {c} passed" in out]


def test_reference_baseline_passes(built):
    rc, out, err = run(built["reference"])
    assert rc == 0 and passed_checks(out) == CHECKS, out[-2000:] + err[-2000:]


def test_reference_callers_pass_with_libnetc(built):
    rc, out, err = run(built["libnetc"])
    assert rc == 0, out[-2000:] + err[-2000:]
    assert passed_checks(out) == CHECKS, out[-2000:]
    binds = dict(re.findall(r"^bind (\S+) (\S+)$", out, flags=re.M))
    libnetc = os.path.realpath(LIBNETC)
    for sym in ("ws_parse_frame", "ws_send_message", "ws_build_masking_key", "dlsym:netc_ws_mask"):
        assert os.path.realpath(binds[sym]) == libnetc, (sym, binds[sym])
    for sym in ("vector_init", "vector_get_buffer", "tcp_server_send", "dlsym:vector_resize"):
        assert binds[sym].endswith("ws_test001_libnetc"), (sym, binds[sym])   # the program's own copies


def test_libnetc_utilities_bind_to_the_program(built):
    """What the dynamic linker binds libnetc.so's own references to: the program's copies."""
    env = dict(os.environ, LD_DEBUG="bindings")
    rc, out, err = run(built["libnetc"], env=env)
    assert rc == 0
    lines = [ln for ln in err.splitlines() if "binding file" in ln and "libnetc.so" in ln.split(" to ")[0]]
    to_prog = {m.group(1) for ln in lines if " to ./" in ln or "ws_test001_libnetc [" in ln
               for m in [re.search(r"symbol `([^']+)'", ln)] if m}
    # the reference's vector / error side channel, not libnetc's copies, serve libnetc's calls
    assert {"vector_init", "netc_errno_reason"} <= to_prog, sorted(to_prog)


def test_vector_semantics_match_the_reference(tmp_path):
    outs = []
    for impl, header in ((os.path.join(REF, "src", "utils", "vector.c"), os.path.join(REF, "include", "utils",
                                                                                       "vector.h")),
                         (os.path.join(ROOT, "netc_amd", "csrc", "host", "vector.c"),
                          os.path.join(ROOT, "include", "utils", "vector.h"))):
        exe = tmp_path / ("vp_" + str(len(outs)))
        subprocess.run(["gcc", "-w", "-O0", f'-DVECTOR_HEADER="{header}"', "-o", str(exe),
                        os.path.join(ORACLE, "vector_probe.c"), impl], check=True)
        outs.append(subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout)
    assert outs[0] == outs[1]
    assert "get_buffer off=24" in outs[0] and "set5 size=6" in outs[0]
