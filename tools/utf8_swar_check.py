#!/usr/bin/env python3
"""Design-time check of the UTF-8 SWAR + nibble-lookup rule in ws_mask_gpu.hip (utf8_err_word):
a Python restatement of its operations (v_perm_b32 / v_alignbyte_b32 emulated) compared with the
scalar rule (utf8_rule, = the oracle decoder's local rules) over every 4-byte context of 31 boundary
byte values, plus random 12-byte runs through all four byte positions.  CPU only."""
import itertools, numpy as np
M = 0xFFFFFFFF
H = 0x80808080
def rule(b3,b2,b1,b0):
    need = b1 >= 0xC0 or b2 >= 0xE0 or b3 >= 0xF0
    cont = (b0 & 0xC0) == 0x80
    if need != cont: return True
    if b0 >= 0xF5 or b0 in (0xC0, 0xC1): return True
    if (b1 == 0xE0 and b0 < 0xA0) or (b1 == 0xED and b0 >= 0xA0) or (b1 == 0xF0 and b0 < 0x90) or (b1 == 0xF4 and b0 >= 0x90): return True
    return False
def alignbyte(hi, lo, s): return ((((hi & M) << 32) | (lo & M)) >> (8*s)) & M
def perm(s0, s1, sel):  # v_perm_b32: bytes {s1 = 0..3, s0 = 4..7}; 12 -> 0, >= 13 -> 0xFF
    src = (s0 << 32) | s1
    out = 0
    for i in range(4):
        k = (sel >> (8*i)) & 0xFF
        if k < 8: b = (src >> (8*k)) & 0xFF
        elif k < 12: b = 0xFF if (src >> (16*(k-8)+15)) & 1 else 0  # sign of bytes 1,3,5,7
        elif k == 12: b = 0
        else: b = 0xFF
        out |= b << (8*i)
    return out
def tbl(vals):  # 16 bytes -> 4 dwords
    return [sum(vals[4*d+i] << (8*i) for i in range(4)) for d in range(4)]
T1v = [0]*16; T1v[0x0] = 0x03; T1v[0x4] = 0x08; T1v[0xD] = 0x04
T1 = tbl(T1v)
T2v = [0x03, 0x09, 0x0C, 0x0C, 0, 0, 0, 0]
T2 = tbl(T2v + [0]*8)
def lookup16(T, idx):
    lo = perm(T[1], T[0], idx & 0x07070707)
    hi = perm(T[3], T[2], idx & 0x07070707)
    m = ((idx & 0x08080808) >> 3) * 0xFF
    return (m & hi) | (~m & lo & M)
def word(x, c):
    # c = (xprev, l2p, l3p, l4p)
    xp, l2p, l3p_, l4p = c
    s1 = (x << 1) & M
    l2 = x & s1 & H
    l3 = l2 & (x << 2) & M
    l4 = l3 & (x << 3) & M
    cont = x & ~s1 & H
    need = alignbyte(l2, l2p, 3) | alignbyte(l3, l3p_, 2) | alignbyte(l4, l4p, 1)
    err = need ^ cont
    z = (x & 0xFEFEFEFE) ^ 0xC0C0C0C0
    err |= ~(((z & 0x7F7F7F7F) + 0x7F7F7F7F) | z) & H
    err |= ((x & 0x7F7F7F7F) + 0x0B0B0B0B) & x & H
    p1 = alignbyte(x, xp, 3)
    lead3 = alignbyte(l3, l3p_, 3)
    t1 = lookup16(T1, p1 & 0x0F0F0F0F)
    sel = ((p1 & 0x10101010) >> 4) * 5 + 0x05050505
    t2 = perm(T2[1], T2[0], (x >> 4) & 0x07070707)
    sp = ((t1 & sel & t2) + 0x7F7F7F7F) & lead3
    err |= sp
    return err & H, (x, l2, l3, l4)

reps = [0x00, 0x41, 0x7F, 0x80, 0x8F, 0x90, 0x9F, 0xA0, 0xBF, 0xC0, 0xC1, 0xC2, 0xDF, 0xE0, 0xE1, 0xEC, 0xED, 0xEE, 0xEF, 0xF0, 0xF1, 0xF3, 0xF4, 0xF5, 0xF7, 0xFF, 0x30, 0x34, 0x3D, 0x10, 0x14]
bad = 0; n = 0
rng = np.random.default_rng(1)
# exhaustive over (b3,b2,b1,b0) from reps placed at byte 3 of dword x with prev context in xp
for b3, b2, b1, b0 in itertools.product(reps, repeat=4):
    # layout: xp bytes [.., b3, b2, b1] (bytes 1..3), x byte0 = b0, rest ASCII 'a'
    xp = (0x61) | (b3 << 8) | (b2 << 16) | (b1 << 24)
    # previous-previous context for xp's own lead flags: compute through word() on xp with ASCII before
    _, c = word(xp, (0x61616161, 0, 0, 0))
    x = b0 | (0x61 << 8) | (0x61 << 16) | (0x61 << 24)
    e, _ = word(x, c)
    got = bool(e & 0x80)
    exp = rule(b3, b2, b1, b0)
    n += 1
    if got != exp:
        bad += 1
        if bad < 10: print("mismatch", hex(b3), hex(b2), hex(b1), hex(b0), got, exp)
print("checked", n, "mismatches", bad)
# random full-dword check, all 4 positions
for _ in range(20000):
    xs = [int(v) for v in rng.choice(reps, size=12)]
    bs = xs
    d0 = sum(bs[i] << (8*i) for i in range(4)); d1 = sum(bs[4+i] << (8*i) for i in range(4)); d2 = sum(bs[8+i] << (8*i) for i in range(4))
    _, c = word(d0, (0, 0, 0, 0))
    _, c = word(d1, c)
    e, _ = word(d2, c)
    for i in range(4):
        p = 8 + i
        exp = rule(bs[p-3], bs[p-2], bs[p-1], bs[p])
        got = bool((e >> (8*i+7)) & 1)
        if got != exp:
            bad += 1
            if bad < 20: print("rand mismatch", [hex(v) for v in bs[p-3:p+1]], got, exp)
print("total mismatches", bad)
