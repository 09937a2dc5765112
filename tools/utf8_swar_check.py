#!/usr/bin/env python3
"""Design-time check of the UTF-8 validator in ws_mask_gpu.hip (utf8_err_word, utf8_rule).  CPU only.

The kernel's rule is the three-lookup validator (Keiser & Lemire, "Validating UTF-8 in less than
one instruction per byte", 2021): for each byte, the AND of three 16-entry lookups -- the
previous byte's high nibble, its low nibble, the byte's own high nibble -- flags every error a
two-byte window shows; bit 7 (TWO_CONTS) is XORed with "a lead two or three bytes back asks for
a continuation here".  The kernel runs it four bytes at a time in a dword (SWAR), with
v_perm_b32 as the 8-entry byte lookup, v_alignbyte_b32 for the previous bytes, and the
previous dword's lookups carried.

Checked here, with v_perm_b32 / v_alignbyte_b32 emulated:
  1. the SWAR word function == the scalar rule (utf8_rule, phase B) at every byte position,
     exhaustively over every 4-byte context of 31 boundary byte values, and over random runs;
  2. the scalar rule at every position + the end-of-message check == CPython's strict UTF-8
     decoder, exhaustively over all strings of up to 4 bytes from those values and over
     random strings (a message is valid exactly when no position is flagged).
"""
import itertools

import numpy as np

M = 0xFFFFFFFF
H = 0x80808080

# error bits (simdutf / Keiser-Lemire)
TS, TL_, O3, TLG, SUR, O2, T1000, TC = 0x01, 0x02, 0x04, 0x08, 0x10, 0x20, 0x40, 0x80
O4 = T1000
CARRY = TS | TL_ | TC
B1H = [TL_] * 8 + [TC] * 4 + [TS | O2, TS, TS | O3 | SUR, TS | TLG | T1000 | O4]
B1L = [CARRY | O3 | O2 | O4, CARRY | O2, CARRY, CARRY, CARRY | TLG] + [CARRY | TLG | T1000] * 8 + [CARRY | TLG | T1000 | SUR] * 0
B1L = B1L[:13] + [CARRY | TLG | T1000 | SUR, CARRY | TLG | T1000, CARRY | TLG | T1000]
assert len(B1L) == 16
B2H = [TS] * 8 + [TL_ | O2 | TC | O3 | T1000 | O4, TL_ | O2 | TC | O3 | TLG, TL_ | O2 | TC | SUR | TLG,
                  TL_ | O2 | TC | SUR | TLG] + [TS] * 4
CLS = [0] * 14 + [0x80, 0xC0]   # high nibble E: lead of 3+ (bit 7), F: lead of 4+ (bits 7, 6)


def rule(b3, b2, b1, b0):
    """utf8_rule in ws_mask_gpu.hip: byte b0 with the 3 before it (0 before a message's start)."""
    special = B1H[b1 >> 4] & B1L[b1 & 15] & B2H[b0 >> 4]
    must = 0x80 if (b2 >= 0xE0 or b3 >= 0xF0) else 0
    return (special ^ must) != 0


def incomplete(b3, b2, b1):
    return b1 >= 0xC0 or b2 >= 0xE0 or b3 >= 0xF0


def valid_message(bs):
    h = [0, 0, 0]
    for b in bs:
        if rule(h[2], h[1], h[0], b):
            return False
        h = [b, h[0], h[1]]
    return not incomplete(h[2], h[1], h[0])


def alignbyte(hi, lo, s):
    return ((((hi & M) << 32) | (lo & M)) >> (8 * s)) & M


def perm(s0, s1, sel):   # v_perm_b32: bytes {s1 = 0..3, s0 = 4..7}; 8..11 sign of bytes 1,3,5,7; 12 -> 0, >= 13 -> 0xFF
    src = (s0 << 32) | s1
    out = 0
    for i in range(4):
        k = (sel >> (8 * i)) & 0xFF
        if k < 8:
            b = (src >> (8 * k)) & 0xFF
        elif k < 12:
            b = 0xFF if (src >> (16 * (k - 8) + 15)) & 1 else 0
        elif k == 12:
            b = 0
        else:
            b = 0xFF
        out |= b << (8 * i)
    return out


def tbl8(vals):   # 8 bytes -> (dword of entries 4..7, dword of entries 0..3): perm(hi, lo, idx)
    lo = sum(vals[i] << (8 * i) for i in range(4))
    hi = sum(vals[4 + i] << (8 * i) for i in range(4))
    return hi, lo


T_B1H = tbl8(B1H[8:])
T_B2H = tbl8(B2H[8:])
T_CLS = tbl8(CLS[8:])
T_B1L_LO = tbl8(B1L[:8])
T_B1L_HI = tbl8(B1L[8:])
SIGN = 0x090B080A


def sign_bytes(v):
    return perm((v << 8) & M, v, SIGN)


def carry(x):
    mx = sign_bytes(x)
    hx = (x >> 4) & 0x07070707
    b1hx = (mx & perm(*T_B1H, hx)) | (~mx & 0x02020202 & M)
    cls = mx & perm(*T_CLS, hx)
    return (x, b1hx, cls)


def word(x, c):
    xp, b1hp, clsp = c
    mx = sign_bytes(x)
    hx = (x >> 4) & 0x07070707
    b1hx = (mx & perm(*T_B1H, hx)) | (~mx & 0x02020202 & M)
    b2h = (mx & perm(*T_B2H, hx)) | (~mx & 0x01010101 & M)
    cls = mx & perm(*T_CLS, hx)
    p1 = alignbyte(x, xp, 3)
    b1h = alignbyte(b1hx, b1hp, 3)
    l1 = p1 & 0x07070707
    m3 = perm((p1 << 12) & M, (p1 << 4) & M, SIGN)
    b1l = (m3 & perm(*T_B1L_HI, l1)) | (~m3 & perm(*T_B1L_LO, l1) & M)
    special = b1h & b1l & b2h
    must = (alignbyte(cls, clsp, 2) | (alignbyte(cls, clsp, 1) << 1)) & H
    return (special ^ must) & M, (x, b1hx, cls)


def check_swar():
    reps = [0x00, 0x41, 0x7F, 0x80, 0x8F, 0x90, 0x9F, 0xA0, 0xBF, 0xC0, 0xC1, 0xC2, 0xDF, 0xE0, 0xE1, 0xEC, 0xED,
            0xEE, 0xEF, 0xF0, 0xF1, 0xF3, 0xF4, 0xF5, 0xF7, 0xFF, 0x30, 0x34, 0x3D, 0x10, 0x14]
    bad = n = 0
    for b3, b2, b1, b0 in itertools.product(reps, repeat=4):
        for pos in range(4):   # b0 at byte `pos` of x; the three before it in x / the previous dword
            seq = [0x61] * 8
            seq[4 + pos], seq[3 + pos], seq[2 + pos], seq[1 + pos] = b0, b1, b2, b3
            xp = sum(seq[i] << (8 * i) for i in range(4))
            x = sum(seq[4 + i] << (8 * i) for i in range(4))
            e, _ = word(x, carry(xp))
            got = ((e >> (8 * pos)) & 0xFF) != 0
            exp = rule(b3, b2, b1, b0)
            n += 1
            if got != exp:
                bad += 1
                if bad < 10:
                    print("swar mismatch", [hex(v) for v in (b3, b2, b1, b0)], pos, got, exp)
    rng = np.random.default_rng(1)
    for _ in range(30000):
        bs = [int(v) for v in rng.choice(reps, size=12)]
        d = [sum(bs[4 * k + i] << (8 * i) for i in range(4)) for k in range(3)]
        _, c = word(d[0], (0, 0x02020202, 0))
        _, c = word(d[1], c)
        e, _ = word(d[2], c)
        for i in range(4):
            p = 8 + i
            n += 1
            if (((e >> (8 * i)) & 0xFF) != 0) != rule(bs[p - 3], bs[p - 2], bs[p - 1], bs[p]):
                bad += 1
    print("SWAR vs scalar rule:", n, "positions,", bad, "mismatches")
    return bad


def check_decoder():
    vals = [0x00, 0x41, 0x7F, 0x80, 0x8F, 0x90, 0x9F, 0xA0, 0xBF, 0xC0, 0xC1, 0xC2, 0xDF, 0xE0, 0xE1, 0xEC, 0xED,
            0xEE, 0xEF, 0xF0, 0xF1, 0xF3, 0xF4, 0xF5, 0xF7, 0xF8, 0xFF]
    bad = n = 0
    for L in range(1, 5):
        for s in itertools.product(vals, repeat=L):
            b = bytes(s)
            try:
                b.decode("utf-8", "strict")
                ok = True
            except UnicodeDecodeError:
                ok = False
            n += 1
            if valid_message(b) != ok:
                bad += 1
                if bad < 10:
                    print("decoder mismatch", b.hex(), ok)
    rng = np.random.default_rng(2)
    pieces = ["a", "é", "€", "😀", "\x00", "ÿ", "￿", "\U0010ffff"]
    for _ in range(20000):
        s = "".join(rng.choice(pieces, size=int(rng.integers(1, 12)))).encode()
        b = bytearray(s)
        if rng.random() < 0.5 and b:
            b[int(rng.integers(0, len(b)))] = int(rng.choice(vals))
        try:
            bytes(b).decode("utf-8", "strict")
            ok = True
        except UnicodeDecodeError:
            ok = False
        n += 1
        if valid_message(bytes(b)) != ok:
            bad += 1
    print("rule + end check vs CPython strict decode:", n, "strings,", bad, "mismatches")
    return bad


if __name__ == "__main__":
    print("tables: B1H hi %08x %08x  B2H hi %08x %08x  CLS hi %08x %08x  B1L lo %08x %08x  B1L hi %08x %08x" %
          (*T_B1H, *T_B2H, *T_CLS, *T_B1L_LO, *T_B1L_HI))
    raise SystemExit(1 if check_swar() + check_decoder() else 0)
