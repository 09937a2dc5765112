"""The C-ABI boundary (CPU): libraries load, export every function include/*.h declares,
and the netc structs keep the reference's layout."""

import json
import os
import re
import subprocess
import tempfile

import pytest

from netc_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INCLUDE = os.path.join(ROOT, "include")


def declared_functions():
    names = set()
    for dirpath, _, files in os.walk(INCLUDE):
        for f in files:
            if not f.endswith(".h"):
                continue
            text = open(os.path.join(dirpath, f)).read()
            text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
            text = re.sub(r"//[^\n]*", "", text)
            text = re.sub(r"#[^\n]*", "", text)
            for m in re.finditer(r"([A-Za-z_][A-Za-z0-9_]*)\s*\([^;{)]*\)\s*;", text):
                name = m.group(1)
                if name not in ("if", "while", "for", "return", "sizeof"):
                    names.add(name)
    return names


def exported(path):
    out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True, check=True).stdout
    return {line.split()[-1] for line in out.splitlines() if line.strip()}


# Declared by the kept C API (include/socket.h, include/utils/string.h, include/ws/server.h,
# include/ws/client.h) but implemented by netc's own sources, which a netc program links next
# to libnetc.so (out of scope; tests/test_dropin.py).
PROVIDED_BY_NETC = {
    "socket_recv_until_dynamic", "socket_recv_until_fixed", "socket_set_non_blocking",
    "sso_string_init", "sso_string_set", "sso_string_get", "sso_string_concat", "sso_string_concat_buffer",
    "sso_string_concat_char", "sso_string_backspace", "sso_string_copy", "sso_string_copy_buffer",
    "sso_string_compare", "sso_string_ensure_null_terminated", "sso_string_free",
    "ws_server_upgrade_connection", "ws_server_close_client", "ws_client_connect",
}


def test_every_declared_symbol_is_exported():
    decl = declared_functions()
    assert {"netc_ws_mask", "netc_gpu_mask_batch", "ws_parse_frame", "ws_send_message", "netc_gpu_encode_frames",
            "netc_ws_wire_size", "netc_gpu_stream_create", "ws_server_upgrade_connection"} <= decl
    assert PROVIDED_BY_NETC <= decl
    have = exported(_lib.HOST_LIB) | exported(_lib.GPU_LIB)
    missing = sorted(decl - PROVIDED_BY_NETC - have)
    assert not missing, f"declared but not exported: {missing}"
    # ... and the libraries do not carry their own copies of netc's out-of-scope code
    assert not (PROVIDED_BY_NETC & have), sorted(PROVIDED_BY_NETC & have)


def test_libraries_load_without_gpu():
    _lib.host()
    _lib.gpu()
    from netc_amd import mask as nm

    assert nm.device_count() >= 0


def test_length_class_and_wire_size_helpers():
    """host helpers around netc_gpu_encode_frames_class: the one length class of a batch (or None)
    and the exact wire size it implies -- affine in the offsets when the class is one"""
    import numpy as np
    from netc_amd import mask as nm

    def offs(sizes, start=0):
        return np.concatenate([[start], start + np.cumsum(sizes)]).astype(np.uint64)

    assert nm.length_class(offs([0, 5, 125])) == nm.NETC_WS_CLASS_7BIT
    assert nm.length_class(offs([126, 1024, 65535])) == nm.NETC_WS_CLASS_16BIT
    assert nm.length_class(offs([65536, 1 << 20])) == nm.NETC_WS_CLASS_64BIT
    assert nm.length_class(offs([125, 126])) is None
    assert nm.length_class(offs([65535, 65536])) is None
    assert nm.length_class(offs([])) is None
    for sizes, cls in (([7] * 9, 0), ([1024] * 65, 2), ([70000, 65536], 8)):
        for masked in (True, False):
            o = offs(sizes, start=13)
            n = len(sizes)
            affine = int(o[-1] - o[0]) + n * (2 + cls + (4 if masked else 0))
            assert nm.wire_size(o, masked) == affine


LAYOUT_C = r"""
#include <stdio.h>
#include <stddef.h>
#include "ws/common.h"
#define F(t, m) printf("\"%s.%s\": [%zu, %zu],\n", #t, #m, offsetof(struct t, m), sizeof(((struct t *)0)->m))
int main(void) {
    printf("{\n");
    F(ws_frame, mask); F(ws_frame, masking_key); F(ws_frame, payload_length);
    F(ws_message, opcode); F(ws_message, buffer); F(ws_message, payload_length);
    F(ws_frame_parsing_state, parsing_state); F(ws_frame_parsing_state, frame); F(ws_frame_parsing_state, message);
    F(ws_frame_parsing_state, real_payload_length); F(ws_frame_parsing_state, payload_data);
    F(ws_frame_parsing_state, received_length);
    F(vector, size); F(vector, capacity); F(vector, element_size); F(vector, elements);
    printf("\"sizeof\": [%zu, %zu, %zu, %zu, %zu]\n}\n", sizeof(struct ws_header), sizeof(struct ws_frame),
           sizeof(struct ws_message), sizeof(struct ws_frame_parsing_state), sizeof(struct vector));
    return 0;
}
"""


def layout(include_dir):
    with tempfile.TemporaryDirectory() as d:
        src, exe = os.path.join(d, "l.c"), os.path.join(d, "l")
        open(src, "w").write(LAYOUT_C)
        subprocess.run(["gcc", "-w", "-I", include_dir, src, "-o", exe], check=True)
        return json.loads(subprocess.run([exe], capture_output=True, text=True, check=True).stdout)


def test_every_knob_is_accepted_and_no_other():
    """netc_gpu_knob (include/ws/mask.h): each NETC_GPU_KNOB_* the header declares, and the Python
    mirror's names, is accepted (set, then restored to its default); 0 and the next index are not"""
    from netc_amd import mask as nm
    hdr = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "ws",
                            "mask.h")).read()
    declared = {m.group(1): int(m.group(2)) for m in re.finditer(r"#define NETC_GPU_KNOB_(\w+)\s+(\d+)", hdr)}
    assert declared == nm.KNOBS
    g = _lib.gpu()
    for k in declared.values():
        assert g.netc_gpu_knob(k, -1) == 0, k
    assert g.netc_gpu_knob(0, -1) != 0
    assert g.netc_gpu_knob(max(declared.values()) + 1, -1) != 0


def test_struct_layout_is_the_reference_layout():
    mine = layout(INCLUDE)
    golden = json.load(open(os.path.join(ROOT, "tests", "golden", "ws_layout.json")))
    assert mine == golden
    ref = "/root/reference/include"
    if os.path.isdir(ref):
        assert layout(ref) == golden


def test_ingest_without_gpu_fails_loudly():
    """No device here: creating an ingest ring reports NETC_GPU_ENODEV (there is no CPU fallback)."""
    import torch

    from netc_amd import ingest as ni
    from netc_amd.mask import NETC_GPU_ENODEV, NetcGpuError

    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    with pytest.raises(NetcGpuError) as e:
        ni.Ingest(0)
    assert e.value.code == NETC_GPU_ENODEV
