"""The oracle is pinned before it is trusted (CPU).

* against the golden vectors the REFERENCE produced (tests/golden/ws_golden.json,
  from its own compiled src/ws/common.c via oracle/_ref);
* against the RFC 6455 §5.7 known answer and the reference's test payloads;
* where oracle/_ref is built (this container), against the reference directly on
  randomized frames and chunkings.
"""

import hashlib
import json
import os

import numpy as np
import pytest

from oracle import oracle as orc

GOLDEN = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "ws_golden.json")))


def gen_bytes(seed: int, n: int) -> bytes:
    return np.random.Generator(np.random.PCG64(seed)).integers(0, 256, size=n, dtype=np.uint8).tobytes()


def payload_of(field) -> bytes:
    if "hex" in field:
        return bytes.fromhex(field["hex"])
    if "text_gen_seed" in field:
        p = bytes(b % 255 + 1 for b in gen_bytes(field["text_gen_seed"], field["len"]))
    else:
        p = gen_bytes(field["gen_seed"], field["len"])
    assert hashlib.sha256(p).hexdigest() == field["sha256"]
    return p


def wire_matches(field, w: bytes) -> bool:
    if "hex" in field:
        return w.hex() == field["hex"]
    return len(w) == field["len"] and hashlib.sha256(w).hexdigest() == field["sha256"]


def test_rfc6455_known_answer():
    assert orc.unmask(bytes.fromhex("7f9f4d5158"), bytes.fromhex("37fa213d")).tobytes() == b"Hello"
    used, msg, op = orc.decode_message(bytes.fromhex(GOLDEN["rfc6455_kat"]["wire"]))
    assert (used, msg, op) == (11, b"Hello", 1)
    # the reference delivers it with its TEXT NUL appended
    assert GOLDEN["rfc6455_kat"]["messages"] == [[1, b"Hello\x00".hex()]]


def test_key_sequence_matches_reference():
    assert orc.key_sequence(6).hex() == GOLDEN["key_sequence_fresh_thread"]
    assert GOLDEN["key_sequence_fresh_thread"][:16] == "0061c22384e546a7"


@pytest.mark.parametrize("case", GOLDEN["send_single_frame"], ids=lambda c: c["name"])
def test_encoder_matches_reference_sender(case):
    p = payload_of(case["payload"])
    key = bytes.fromhex(case["key"]) if case["key"] else None
    assert wire_matches(case["wire"], orc.encode_frame(p, case["opcode"], key))


@pytest.mark.parametrize("masked", [True, False])
def test_batch_encoder_matches_reference_sender(masked):
    # oracle_encode_batch (the checker of netc_gpu_encode_frames) over every golden
    # single-frame send of one kind, concatenated: each frame's slice of the batch
    # wire equals the reference's wire for that frame (B9: an empty masked frame
    # additionally carries its key, which the reference omits)
    cases = [c for c in GOLDEN["send_single_frame"] if bool(c["key"]) == masked]
    assert cases
    payloads = [payload_of(c["payload"]) for c in cases]
    off = np.zeros(len(cases) + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(p) for p in payloads])
    keys = np.array([int.from_bytes(bytes.fromhex(c["key"]), "little") if c["key"] else 0 for c in cases],
                    dtype=np.uint32)
    header0 = np.array([0x80 | c["opcode"] for c in cases], dtype=np.uint8)
    wire, wo = orc.encode_batch(b"".join(payloads), off, keys, header0, masked)
    for k, c in enumerate(cases):
        w = wire[int(wo[k]): int(wo[k + 1])].tobytes()
        if masked and not payloads[k]:
            assert w[2:] == bytes.fromhex(c["key"])
            w = w[:2]
        assert wire_matches(c["wire"], w), c["name"]


@pytest.mark.parametrize("case", GOLDEN["receive"], ids=lambda c: f"{len(payload_of(c['payload']))}B-{c['key']}")
def test_decoder_matches_reference_receiver(case):
    p = payload_of(case["payload"])
    wire = orc.encode_frame(p, case["opcode"], bytes.fromhex(case["key"]))
    assert wire_matches(case["wire"], wire)
    used, msg, op = orc.decode_message(wire)
    assert used == len(wire) and msg == p and op == case["opcode"]


def test_fragmented_message():
    f = GOLDEN["fragmented"]
    used, msg, op = orc.decode_message(bytes.fromhex(f["wire"]))
    assert msg.hex() == f["message"] and op == f["opcode"] == 2


def test_unmask_phase_continuity():
    # unmasking in arbitrary pieces with phase = bytes already received equals one pass (src/ws/common.c:321)
    g = np.random.Generator(np.random.PCG64(1))
    p = g.integers(0, 256, 5000, dtype=np.uint8)
    key = bytes(g.integers(0, 256, 4, dtype=np.uint8))
    whole = orc.unmask(p, key, 0)
    cuts = np.sort(g.choice(np.arange(1, 5000), 40, replace=False))
    pieces, prev = [], 0
    for c in list(cuts) + [5000]:
        pieces.append(orc.unmask(p[prev:c], key, prev))
        prev = c
    assert np.array_equal(np.concatenate(pieces), whole)


def test_o0_and_o2_builds_agree():
    g = np.random.Generator(np.random.PCG64(2))
    sizes = g.integers(0, 3000, 200)
    off = np.zeros(201, dtype=np.uint64)
    off[1:] = np.cumsum(sizes)
    keys = g.integers(0, 1 << 32, 200, dtype=np.uint64).astype(np.uint32)
    buf = g.integers(0, 256, int(off[-1]), dtype=np.uint8)
    assert np.array_equal(orc.mask_batch(buf, off, keys, "O2"), orc.mask_batch(buf, off, keys, "O0"))


@pytest.mark.skipif(not orc.ref_available(), reason="oracle/_ref (compiled reference) not built here")
@pytest.mark.parametrize("seed", range(12))
def test_oracle_vs_compiled_reference_random(seed):
    g = np.random.Generator(np.random.PCG64(100 + seed))
    nframes = int(g.integers(1, 6))
    parts = [gen_bytes(1000 * seed + i, int(g.choice([1, 5, 125, 126, 300, 4096, 65535, 65536, 70001])))
             for i in range(nframes)]
    keys = [bytes(g.integers(0, 256, 4, dtype=np.uint8)) for _ in range(nframes)]
    if seed % 3 == 0:
        keys[0] = b"\x00\x61\xc2\x23"
    wire = b"".join(orc.encode_frame(parts[i], 2 if i == 0 else 0, keys[i], fin=(i == nframes - 1))
                    for i in range(nframes))
    # chunk boundaries only inside payloads (the reference mis-resumes elsewhere: defects B6-B8)
    chunks, pos = [], 0
    for i in range(nframes):
        hdr = len(orc.encode_frame(parts[i], 2, keys[i])) - len(parts[i])
        body = len(parts[i])
        if body > 2:
            cut = int(g.integers(1, body))
            chunks += [hdr + cut, body - cut]
        else:
            chunks += [hdr + body]
    msgs = orc.ref_parse(wire, chunks)
    used, msg, op = orc.decode_message(wire, cap=len(wire) + 16)
    assert len(msgs) == 1 and msgs[0][1] == msg == b"".join(parts)
