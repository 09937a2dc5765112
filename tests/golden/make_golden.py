#!/usr/bin/env python3
"""Regenerate tests/golden/ws_golden.json from the REFERENCE itself.

Runs Altanis/netc's own src/ws/common.c (ws_send_message, ws_parse_frame,
ws_build_masking_key), compiled from /root/reference into oracle/_ref/libref_ws.so
by oracle/Makefile, and records inputs and the reference's outputs as data.
Needs /root/reference (this build container only); the committed JSON is what
the tests read everywhere else.

    make -C oracle && python tests/golden/make_golden.py
"""

import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import oracle as orc  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "ws_golden.json")
TEXT, BINARY, CONT = 1, 2, 0


def gen_bytes(seed: int, n: int) -> bytes:
    """Seeded payload generator shared with tests/test_oracle.py (PCG64)."""
    return np.random.Generator(np.random.PCG64(seed)).integers(0, 256, size=n, dtype=np.uint8).tobytes()


def payload_field(p: bytes, seed=None):
    if len(p) <= 4096:
        return {"hex": p.hex()}
    return {"gen_seed": seed, "len": len(p), "sha256": hashlib.sha256(p).hexdigest()}


def wire_field(w: bytes):
    if len(w) <= 8192:
        return {"hex": w.hex()}
    return {"len": len(w), "sha256": hashlib.sha256(w).hexdigest()}


def main():
    if not orc.ref_available():
        sys.exit("oracle/_ref/libref_ws.so missing: build it with `make -C oracle` where /root/reference exists")
    g = {"generator": "tests/golden/make_golden.py (reference src/ws/common.c compiled by oracle/Makefile)",
         "key_sequence_fresh_thread": orc.ref_key_sequence(6).hex()}

    # 1. the exact frames tests/ws/test001.c exchanges, with the keys its threads draw
    keys = orc.ref_key_sequence(2)
    k0, k1 = keys[:4], keys[4:]
    t001 = [
        ("client->server BINARY 15 B (tests/ws/test001.c:233-246)", BINARY,
         bytes([0, 233, 5, 11, 65, 115, 112, 101, 99, 116, 108, 44, 108, 44, 107]), k0),
        ("client->server TEXT 35 B (tests/ws/test001.c:253-266)", TEXT, b"hello server multiple frames masked", k1),
        ("server->client TEXT 19 B (tests/ws/test001.c:95-108)", TEXT, b"hello client masked", k0),
        ("server->client TEXT 35 B (tests/ws/test001.c:149-162)", TEXT, b"hello client multiple frames masked", k1),
        ("client->server TEXT unmasked (tests/ws/test001.c:192-202)", TEXT, b"hello server basic", None),
    ]
    g["send_single_frame"] = []
    for name, op, p, k in t001:
        w = orc.ref_send(p, op, k, 1)
        g["send_single_frame"].append({"name": name, "opcode": op, "payload": payload_field(p),
                                       "key": k.hex() if k else None, "wire": wire_field(w)})

    # more defined-behaviour sends: TEXT of every length class, BINARY <= 254 B
    for n, op, seed in [(0, TEXT, 1), (1, TEXT, 2), (125, TEXT, 3), (126, TEXT, 4), (254, BINARY, 5),
                        (65535, TEXT, 6), (65536, TEXT, 7), (70000, TEXT, 8)]:
        p = bytes(b % 255 + 1 for b in gen_bytes(seed, n)) if op == TEXT else gen_bytes(seed, n)   # no NUL in TEXT (B3)
        k = gen_bytes(seed + 100, 4)
        if op == TEXT and n == 0:
            k = None                     # masked empty payload: reference omits the key (documented divergence)
        w = orc.ref_send(p, op, k, 1)
        g["send_single_frame"].append({"name": f"{'TEXT' if op == TEXT else 'BINARY'} {n} B", "opcode": op,
                                       "payload": payload_field(p, seed) if op == BINARY or n <= 4096 else
                                       {"text_gen_seed": seed, "len": n, "sha256": hashlib.sha256(p).hexdigest()},
                                       "key": k.hex() if k else None, "wire": wire_field(w)})

    # 2. RFC 6455 §5.7 known answer, through the reference parser
    kat = bytes.fromhex("818537fa213d7f9f4d5158")
    msgs = orc.ref_parse(kat)
    g["rfc6455_kat"] = {"wire": kat.hex(), "messages": [[op, m.hex()] for op, m in msgs]}

    # 3. receive-path differential vectors (payload, key, masked wire, reference-unmasked result)
    g["receive"] = []
    for n, key_hex, seed in [(5, None, 10), (1024, None, 11), (4096, None, 12), (4096, "0061c223", 13),
                             (70000, None, 14), (1 << 20, None, 15), (3, "00000000", 16), (7, "ffffffff", 17)]:
        p = gen_bytes(seed, n)
        k = bytes.fromhex(key_hex) if key_hex else gen_bytes(seed + 1000, 4)
        wire = orc.encode_frame(p, BINARY, k)
        got = orc.ref_parse(wire, chunks=[], max_payload=1 << 40)
        assert len(got) == 1 and got[0][1] == p, n
        # the same wire delivered in uneven pieces inside the payload (phase continuity, src/ws/common.c:321)
        hdr = len(wire) - n
        chunks = [hdr + 1] + ([3, 1, 2, 97, 500] if n > 700 else [1])
        got2 = orc.ref_parse(wire, chunks=chunks, max_payload=1 << 40)
        assert len(got2) == 1 and got2[0][1] == p, n
        g["receive"].append({"payload": payload_field(p, seed), "key": k.hex(), "wire": wire_field(wire),
                             "chunks": chunks, "opcode": BINARY})

    # 4. a fragmented message: BINARY + CONT + CONT with distinct keys, chunked delivery
    parts = [gen_bytes(20, 1000), gen_bytes(21, 777), gen_bytes(22, 333)]
    fk = [gen_bytes(23, 4), gen_bytes(24, 4), gen_bytes(25, 4)]
    wire = b"".join(orc.encode_frame(parts[i], BINARY if i == 0 else CONT, fk[i], fin=(i == 2)) for i in range(3))
    chunks = [13, 7, 301, 1, 2, 3, 499, 97]
    msgs = orc.ref_parse(wire, chunks=chunks)
    assert len(msgs) == 1 and msgs[0][1] == b"".join(parts)
    g["fragmented"] = {"wire": wire.hex(), "chunks": chunks, "message": msgs[0][1].hex(), "opcode": msgs[0][0]}

    # 5. TEXT delivery: the reference appends a NUL and counts it in payload_length (src/ws/common.c:342-343)
    wire = orc.encode_frame(b"hello server basic", TEXT, bytes.fromhex("84e546a7"))
    msgs = orc.ref_parse(wire)
    g["text_nul"] = {"wire": wire.hex(), "delivered": msgs[0][1].hex(), "payload_length": len(msgs[0][1])}

    # (Reference defect B2 -- a multi-frame masked send -- is not recorded: it reads
    #  uninitialised heap (malloc of the header byte, src/ws/common.c:100, then memcpy
    #  at :123 past the bytes copied at :101), so its wire bytes are not reproducible.)

    with open(OUT, "w") as f:
        json.dump(g, f, indent=1, sort_keys=True)
        f.write("\n")
    print(f"wrote {OUT}")


if __name__ == "__main__":
    main()
