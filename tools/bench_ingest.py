#!/usr/bin/env python3
"""Socket ingest (include/ws/ingest.h) end to end, one GPU.

A writer thread sends a stream of masked client frames (BASELINE config 5's shape:
4 KiB BINARY frames, a random key each) over an AF_UNIX socketpair; the reader
recv()s it straight into the ingest ring's pinned slots, each slot goes H2D ->
frame scan -> unmask -> D2H, and the batches come back with their frame
descriptors.  Reported (host to host, PCIe-inclusive -- never bench.py's value):

  socket_only       the socketpair drained by plain recv_into, no processing: the socket's ceiling
  socket_ingest     recv -> GPU -> batches, GiB/s of wire (and of payload)
  memory_ingest     the same ring fed from memory (write()), no socket: the ring's own rate
  reference_parse   the reference's own ws_parse_frame (oracle/_ref, -O0 as it ships) over a socketpair
  oracle_walk       the serial CPU restatement: oracle scan + unmask of the same stream (-O2, 1 thread)

Delivered frames are checked: count, stream offsets, and 8 frames of every 4th
batch against the plaintext (inside the timed loop, so kept small).
"""
import argparse
import json
import os
import socket
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
GIB = float(1 << 30)


def build_base(frame, nframes, seed=5):
    from oracle import oracle as orc

    rng = np.random.default_rng(seed)
    off = (np.arange(nframes + 1, dtype=np.uint64) * np.uint64(frame)).astype(np.uint64)
    plain = rng.integers(0, 256, int(off[-1]), dtype=np.uint8)
    keys = rng.integers(0, 2**32, nframes, dtype=np.uint64).astype(np.uint32)
    wire, wo = orc.encode_batch(plain, off, keys, None, True)
    return wire, wo, plain, off


def writer_thread(sock, base, total, piece):
    v = memoryview(base)
    sent = 0
    try:
        while sent < total:
            i = sent % len(v)
            n = min(piece, len(v) - i, total - sent)
            sock.sendall(v[i:i + n])
            sent += n
    finally:
        sock.shutdown(socket.SHUT_WR)


def socketpair(sz=8 << 20):
    a, b = socket.socketpair()
    for s in (a, b):
        for opt in (socket.SO_SNDBUF, socket.SO_RCVBUF):
            try:
                s.setsockopt(socket.SOL_SOCKET, opt, sz)
            except OSError:
                pass
    return a, b


class Checker:
    """Counts delivered frames and checks sampled batches frame by frame against the plaintext."""

    def __init__(self, wire_base, wo, plain, off, sample_every):
        self.base_len = wire_base.size
        self.wo, self.plain, self.off = wo, plain, off
        self.frames = self.bytes = self.pos = self.batches = self.bad = self.checked = 0
        self.sample_every = sample_every
        self.per_batch = 8   # frames checked per sampled batch (the check runs inside the timed loop)

    def batch(self, b):
        if b.stream_offset != self.pos:
            self.bad += 1
        self.pos = b.stream_offset + b.wire.size
        self.frames += b.nframes
        self.bytes += b.wire.size
        if self.batches % self.sample_every == 0 and b.nframes:
            for k in np.unique(np.linspace(0, b.nframes - 1, self.per_batch).astype(np.int64)):
                k = int(k)
                g = (b.stream_offset + int(b.hdr[k])) % self.base_len
                j = int(np.searchsorted(self.wo, g))
                if j >= self.wo.size - 1 or int(self.wo[j]) != g:
                    self.bad += 1
                    continue
                po, pl = b.payload(k)
                exp = self.plain[int(self.off[j]):int(self.off[j + 1])]
                if pl != exp.size or not np.array_equal(b.wire[po:po + pl], exp):
                    self.bad += 1
                self.checked += 1
        self.batches += 1


def drain(ing, chk, wait):
    n = 0
    while True:
        b = ing.next(wait=wait)
        if b is None:
            return n
        chk.batch(b)
        b.release()
        n += 1


def run_socket_ingest(args, base, wo, plain, off, total):
    from netc_amd import ingest as ni

    a, b = socketpair()
    chk = Checker(base, wo, plain, off, args.sample_every)
    with ni.Ingest(0, slot_bytes=args.slot_mib << 20, nslots=args.slots, scan=args.scan, strict=args.strict) as ing:
        t = threading.Thread(target=writer_thread, args=(a, base, total, args.piece_kib << 10))
        t0 = time.perf_counter()
        t.start()
        fd = b.fileno()
        while True:
            r = ing.recv(fd)
            if r == ni.NETC_WS_INGEST_FULL:
                drain(ing, chk, True)
            elif r == ni.NETC_WS_INGEST_CLOSED:
                break
            elif r > 0:
                drain(ing, chk, False)
        drain(ing, chk, True)
        secs = time.perf_counter() - t0
        chk.scan_counts = ing.scan_counts()
        t.join()
    a.close()
    b.close()
    return secs, chk


def run_memory_ingest(args, base, wo, plain, off, total):
    from netc_amd import ingest as ni

    chk = Checker(base, wo, plain, off, args.sample_every)
    with ni.Ingest(0, slot_bytes=args.slot_mib << 20, nslots=args.slots, scan=args.scan, strict=args.strict) as ing:
        t0 = time.perf_counter()
        sent = 0
        while sent < total:
            i = sent % base.size
            r = ing.write(base[i:i + min(base.size - i, total - sent)])
            if r == ni.NETC_WS_INGEST_FULL:
                drain(ing, chk, True)
                continue
            sent += r
            drain(ing, chk, False)
        ing.submit()
        drain(ing, chk, True)
        secs = time.perf_counter() - t0
        chk.scan_counts = ing.scan_counts()
    return secs, chk


def run_socket_only(args, base, total):
    a, b = socketpair()
    t = threading.Thread(target=writer_thread, args=(a, base, total, args.piece_kib << 10))
    mv = memoryview(bytearray(args.slot_mib << 20))
    got = 0
    t0 = time.perf_counter()
    t.start()
    while True:
        r = b.recv_into(mv)
        if r == 0:
            break
        got += r
    secs = time.perf_counter() - t0
    t.join()
    a.close()
    b.close()
    return secs, got


def oracle_walk(sample, cap):
    """The serial CPU restatement on the same stream: header walk + per-frame unmask (-O2, 1 thread)."""
    from oracle import oracle as orc

    t0 = time.perf_counter()
    hdr, keys, b0, consumed, err = orc.scan_frames(sample, strict=True, cap=cap)
    second = sample[hdr.astype(np.int64) + 1]
    code = second & 0x7F
    hl = (2 + np.where(code == 126, 2, np.where(code == 127, 8, 0)) + 4).astype(np.uint64)
    voff = np.empty(2 * hdr.size + 1, dtype=np.uint64)   # header (key 0) / payload (frame key) alternate
    voff[0:-1:2] = hdr
    voff[1::2] = hdr + hl
    voff[-1] = consumed
    vkeys = np.zeros(2 * hdr.size, dtype=np.uint32)
    vkeys[1::2] = keys
    buf = sample.copy()
    t1 = time.perf_counter()
    orc.mask_batch_inplace(buf, voff, vkeys)
    t2 = time.perf_counter()
    return sample.size / (t2 - t0) / GIB, hdr.size


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=4.0, help="stream bytes sent per measurement")
    ap.add_argument("--frame", type=int, default=4096)
    ap.add_argument("--base-mib", type=int, default=256, help="distinct stream bytes (repeated to --gib)")
    ap.add_argument("--slot-mib", type=int, default=16)
    ap.add_argument("--scan", default="auto", choices=["auto", "gpu", "host"], help="NETC_WS_INGEST_SCAN_*")
    ap.add_argument("--skip-cpu", action="store_true", help="no reference / oracle CPU legs")
    ap.add_argument("--strict", action="store_true", help="NETC_WS_INGEST_STRICT (RFC 6455 client checks)")
    ap.add_argument("--slots", type=int, default=4)
    ap.add_argument("--piece-kib", type=int, default=4096, help="writer's sendall size")
    ap.add_argument("--sample-every", type=int, default=4, help="check 8 frames of every n-th batch")
    ap.add_argument("--ref-mib", type=int, default=256, help="sample for the reference / oracle CPU legs")
    args = ap.parse_args()

    import torch

    from netc_amd import mask as nm
    from oracle import oracle as orc

    assert torch.cuda.is_available()
    nm.gpu_init(0)
    nframes = (args.base_mib << 20) // args.frame
    base, wo, plain, off = build_base(args.frame, nframes)
    reps = max(1, int(args.gib * GIB) // base.size)
    total = reps * base.size
    frames_total = nframes * reps
    payload_total = frames_total * args.frame
    out = {"config": f"c5 frame shape: {args.frame} B masked BINARY frames, {total / GIB:.2f} GiB of wire "
                     f"({frames_total} frames) over an AF_UNIX socketpair",
           "slot_MiB": args.slot_mib, "slots": args.slots, "wire_bytes": total, "payload_bytes": payload_total}

    secs, got = run_socket_only(args, base, total)
    out["socket_only_GiBps"] = round(got / secs / GIB, 3)

    for name, fn in (("socket_ingest", run_socket_ingest), ("memory_ingest", run_memory_ingest)):
        secs, chk = fn(args, base, wo, plain, off, total)
        out[name] = {"wire_GiBps": round(total / secs / GIB, 3), "payload_GiBps": round(payload_total / secs / GIB, 3),
                     "seconds": round(secs, 3), "batches": chk.batches, "frames": chk.frames,
                     "frames_checked": chk.checked, "frames_wrong": chk.bad,
                     "slots_gpu_scan_host_walk": list(chk.scan_counts),
                     "ok": chk.frames == frames_total and chk.bytes == total and chk.bad == 0}
    out["scan"] = args.scan
    out["strict"] = args.strict
    if args.skip_cpu:
        print(json.dumps(out), flush=True)
        return

    # CPU legs on a bounded sample of the same stream
    nref = int(np.searchsorted(wo, min(base.size, args.ref_mib << 20), side="right")) - 1
    sample = base[: int(wo[nref])]
    if orc.ref_available():
        got, rsecs = orc.ref_receive_timed(sample)
        out["reference_parse_payload_GiBps"] = round(got / rsecs / GIB, 3)
        out["reference_parse_note"] = (f"the reference's ws_parse_frame (src/ws/common.c:134-348, -O0 as its Makefile "
                                       f"builds it) receiving {sample.size / (1 << 20):.0f} MiB of the same frames over "
                                       f"a socketpair, 1 thread")
    rate, nf = oracle_walk(sample, nref + 1)
    out["oracle_walk_wire_GiBps"] = round(rate, 3)
    out["oracle_walk_note"] = f"oracle_scan_frames + oracle_mask_batch (-O2, 1 thread), {nf} frames, no socket"
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
