/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C restatement of the reference's WebSocket masking path
 * (Altanis/netc @ 2024-08-07, src/ws/common.c), used as the checker for the
 * GPU kernels and the host framing library.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it; no product code links it.
 *
 * Pinned by: the reference's own round-trip payloads (tests/ws/test001.c:90,
 * 144, 248, 268), the RFC 6455 §5.7 known answer, and golden vectors produced
 * by the reference's compiled src/ws/common.c itself (oracle/_ref, recipe in
 * oracle/Makefile, generator tests/golden/make_golden.py) — see
 * tests/test_oracle.py.
 *
 * Every masking statement is the reference's exact expression, byte by byte,
 * with `%` (not `&`): the point is fidelity, not speed.
 */
#include <stddef.h>
#include <stdint.h>
#include <string.h>

/* src/ws/common.c:319-322 — unmask `n` received bytes at frame phase `received_length` */
void oracle_unmask(uint8_t *buffer_ptr, size_t n, const uint8_t masking_key[4], uint64_t received_length)
{
    for (size_t i = 0; i < n; ++i)
    {
        buffer_ptr[i] ^= masking_key[(received_length + i) % 4];
    }
}

/* src/ws/common.c:104-107 — mask one frame's payload copy (phase always 0) */
void oracle_mask(uint8_t *payload_data_encoded, uint64_t frame_payload_length, const uint8_t payload_masking_key[4])
{
    for (size_t i = 0; i < frame_payload_length; ++i)
    {
        payload_data_encoded[i] ^= payload_masking_key[i % 4];
    }
}

/*
 * A batch as the GPU C-ABI describes it (include/ws/mask.h): frame k covers
 * [off[k], off[k+1]) of buf, key32 packs the wire key bytes little-endian.
 * Each frame is unmasked from phase 0, as the reference's receive path does
 * for every frame (received_length reset at src/ws/common.c:337).
 */
void oracle_mask_batch(uint8_t *buf, const uint64_t *off, const uint32_t *keys, size_t nframes)
{
    for (size_t k = 0; k < nframes; ++k)
    {
        const uint8_t key[4] = {(uint8_t)keys[k], (uint8_t)(keys[k] >> 8), (uint8_t)(keys[k] >> 16),
                                (uint8_t)(keys[k] >> 24)};
        oracle_unmask(buf + off[k], (size_t)(off[k + 1] - off[k]), key, 0);
    }
}

/* src/ws/common.c:19-27 — the per-thread key sequence, with the seed made explicit */
void oracle_build_masking_key(uint8_t masking_key[4], int *seed)
{
    masking_key[0] = (uint8_t)((*seed)++ * 97);
    masking_key[1] = (uint8_t)((*seed)++ * 97);
    masking_key[2] = (uint8_t)((*seed)++ * 97);
    masking_key[3] = (uint8_t)((*seed)++ * 97);
}

/*
 * src/ws/common.c:53-125 for ONE frame of a message (the part of
 * ws_send_message with defined behaviour: a single frame, i.e. num_frames = 1).
 * Writes the wire bytes to out (capacity >= 14 + len) and returns their count.
 */
size_t oracle_encode_frame(uint8_t *out, int fin, uint8_t opcode, const uint8_t *payload, uint64_t len,
                           const uint8_t *masking_key)
{
    size_t h = 0;
    uint8_t header = 0;
    header |= (uint8_t)((fin ? 1 : 0) << 7);
    header |= opcode;                                                         /* :56-60 */
    const uint8_t payload_encoded = len <= 125 ? (uint8_t)len : (len <= 0xFFFF ? 126 : 127); /* :63 */
    uint8_t payload_length = 0;
    payload_length |= (uint8_t)((masking_key != NULL) << 7);
    payload_length |= payload_encoded;                                        /* :65-67 */
    out[h++] = header;
    out[h++] = payload_length;
    if (payload_encoded == 126)
    {
        out[h++] = (uint8_t)((len >> 8) & 0xFF);
        out[h++] = (uint8_t)(len & 0xFF);                                     /* :71-75 */
    }
    else if (payload_encoded == 127)
    {
        for (int i = 0; i < 8; ++i) out[h++] = (uint8_t)((len >> (8 * (7 - i))) & 0xFF); /* :76-82 */
    }
    if (masking_key != NULL && len != 0)
    {
        memcpy(out + h, masking_key, 4);                                      /* :119 */
        h += 4;
    }
    memcpy(out + h, payload, (size_t)len);
    if (masking_key != NULL) oracle_mask(out + h, len, masking_key);          /* :104-107 */
    return h + (size_t)len;
}

/*
 * A batch of frames as include/ws/frame.h describes it: frame k is payload
 * [off[k], off[k+1]) with first header byte header0[k] (FIN | RSV | opcode) and,
 * when masked, key32 keys[k]; each frame is oracle_encode_frame (the reference's
 * single-frame send, src/ws/common.c:53-125) and the frames are concatenated.
 * One deliberate deviation, defect B9: a masked frame with an
 * empty payload still carries its 4 key bytes (RFC 6455 §5.2); the reference
 * sets MASK but omits the key (:84-89,119).  wire_off receives n + 1 offsets.
 * Returns the wire length.
 */
size_t oracle_encode_batch(uint8_t *out, uint64_t *wire_off, const uint8_t *payload, const uint64_t *off,
                           const uint32_t *keys, const uint8_t *header0, size_t nframes, int masked)
{
    size_t w = 0;
    for (size_t k = 0; k < nframes; ++k)
    {
        const uint8_t b0 = header0 ? header0[k] : 0x82;
        const uint8_t key[4] = {(uint8_t)(masked ? keys[k] : 0), (uint8_t)(masked ? keys[k] >> 8 : 0),
                                (uint8_t)(masked ? keys[k] >> 16 : 0), (uint8_t)(masked ? keys[k] >> 24 : 0)};
        const uint64_t len = off[k + 1] - off[k];
        wire_off[k] = w;
        w += oracle_encode_frame(out + w, b0 >> 7, (uint8_t)(b0 & 0x7F), payload + off[k], len,
                                 masked ? key : NULL);
        if (masked && len == 0)
        {
            memcpy(out + w, key, 4); /* B9: the key follows MASK */
            w += 4;
        }
    }
    wire_off[nframes] = w;
    return w;
}

/*
 * The frame boundaries of a received byte stream (checker of the device frame
 * scan, include/ws/frame.h): the header decode of src/ws/common.c:146-296 walked
 * over wire[start, len) frame by frame —
 *   byte 0: FIN | RSV1-3 | opcode (:157-161); byte 1: MASK | 7-bit length (:180-181);
 *   126 → 16-bit, 127 → 64-bit big-endian extended length (:223-245);
 *   MASK → 4 key bytes (:273-289); then the payload.
 * For frame k it records the header offset, the packed key (0 if unmasked) and
 * byte 0.  The walk stops at the first frame not complete inside the stream
 * (*consumed = its header offset, or len when every byte was used) or, with
 * strict != 0, at the first header RFC 6455 forbids from a client (*error =
 * its offset, else UINT64_MAX): MASK clear, RSV set, a reserved opcode, or a
 * control frame (opcode >= 8) fragmented or longer than 125 (§5.1, §5.2, §5.5),
 * or a 64-bit length with its top bit set.  The reference checks none of these
 * (it accepts any header; strict = 0 reproduces that).  Returns the frames
 * found (at most cap are recorded).
 */
size_t oracle_scan_frames(const uint8_t *wire, uint64_t len, uint64_t start, int strict, uint64_t *hdr,
                          uint32_t *keys, uint8_t *b0, size_t cap, uint64_t *consumed, uint64_t *error)
{
    size_t n = 0;
    uint64_t p = start;
    *error = UINT64_MAX;
    for (;;)
    {
        if (p + 2 > len) break;
        const uint8_t first = wire[p], second = wire[p + 1];
        const uint8_t opcode = first & 0x0F, mask = second >> 7, code = second & 0x7F;
        const uint64_t ext = code == 126 ? 2 : (code == 127 ? 8 : 0);
        const uint64_t hl = 2 + ext + (mask ? 4 : 0);
        if (p + 2 + ext > len) break;
        uint64_t plen = code;
        if (ext)
        {
            plen = 0;
            for (uint64_t i = 0; i < ext; ++i) plen = plen << 8 | wire[p + 2 + i];
        }
        if (strict)
        {
            const int reserved = (opcode >= 3 && opcode <= 7) || opcode >= 11;
            const int control = opcode >= 8;
            if (!mask || (first & 0x70) || reserved || (control && (!(first & 0x80) || plen > 125)) ||
                (code == 127 && (plen >> 63)))
            {
                *error = p;
                break;
            }
        }
        if (p + hl > len || plen > len - (p + hl)) break;
        if (n < cap)
        {
            hdr[n] = p;
            keys[n] = mask ? ((uint32_t)wire[p + hl - 4] | (uint32_t)wire[p + hl - 3] << 8 |
                              (uint32_t)wire[p + hl - 2] << 16 | (uint32_t)wire[p + hl - 1] << 24)
                           : 0;
            b0[n] = first;
        }
        ++n;
        p += hl + plen;
    }
    *consumed = p;
    return n;
}

/*
 * UTF-8 validity (RFC 3629 §3-4: shortest form, no surrogates D800-DFFF, nothing
 * above U+10FFFF) — what RFC 6455 §8.1 requires of a TEXT message and the
 * reference never checks (src/ws/common.c:342 only appends a NUL).  A plain
 * byte-at-a-time decoder, the checker of the fused unmask + validate kernel.
 * Returns 1 if s[0, n) is valid UTF-8.
 */
int oracle_utf8_valid(const uint8_t *s, size_t n)
{
    size_t i = 0;
    while (i < n)
    {
        const uint8_t c = s[i];
        size_t need;
        uint32_t cp;
        if (c < 0x80)
        {
            ++i;
            continue;
        }
        else if (c >= 0xC2 && c <= 0xDF)
        {
            need = 1;
            cp = c & 0x1F;
        }
        else if (c >= 0xE0 && c <= 0xEF)
        {
            need = 2;
            cp = c & 0x0F;
        }
        else if (c >= 0xF0 && c <= 0xF4)
        {
            need = 3;
            cp = c & 0x07;
        }
        else
            return 0; /* continuation byte, C0 / C1, F5..FF */
        if (n - i - 1 < need) return 0; /* truncated sequence */
        for (size_t k = 1; k <= need; ++k)
        {
            if ((s[i + k] & 0xC0) != 0x80) return 0;
            cp = cp << 6 | (s[i + k] & 0x3F);
        }
        if ((need == 2 && cp < 0x800) || (need == 3 && cp < 0x10000)) return 0; /* overlong */
        if (cp >= 0xD800 && cp <= 0xDFFF) return 0;                            /* surrogate */
        if (cp > 0x10FFFF) return 0;
        i += need + 1;
    }
    return 1;
}

/*
 * The TEXT-message verdicts of a frame batch (include/ws/mask.h layout, payload
 * already unmasked, header0[k] = FIN | RSV | opcode): a TEXT message is a frame
 * with opcode 1 and the continuation frames (opcode 0) after it up to the first
 * with FIN set; control frames (opcode >= 8) in between are not part of it (RFC
 * 6455 §5.4).  valid[k] = 0 for the last frame of a TEXT message whose payload
 * bytes, concatenated, are not valid UTF-8; 1 everywhere else (other frames,
 * other messages, a message still open at the end of the batch, or abandoned by a
 * new data frame before its FIN).
 */
#include <stdlib.h>
void oracle_validate_batch(const uint8_t *payload, const uint64_t *off, const uint8_t *header0, size_t nframes,
                           uint8_t *valid)
{
    uint8_t *msg = NULL;
    size_t len = 0, cap = 0;
    int open = 0; /* a TEXT message is being collected */
    for (size_t k = 0; k < nframes; ++k)
    {
        valid[k] = 1;
        const uint8_t op = header0[k] & 0x0F, fin = header0[k] >> 7;
        if (op >= 8) continue; /* control frame */
        if (op != 0) open = 0; /* a new message starts (an open one is abandoned) */
        if (op == 1)
        {
            open = 1;
            len = 0;
        }
        if (!open) continue;
        const size_t n = (size_t)(off[k + 1] - off[k]);
        if (len + n > cap)
        {
            cap = (len + n) * 2 + 16;
            msg = (uint8_t *)realloc(msg, cap);
        }
        memcpy(msg + len, payload + off[k], n);
        len += n;
        if (fin)
        {
            valid[k] = (uint8_t)oracle_utf8_valid(msg, len);
            open = 0;
        }
    }
    free(msg);
}

/*
 * src/ws/common.c:146-347 as a pure function over a complete byte stream:
 * decodes frames until one with FIN completes a message.  On success returns
 * the wire bytes consumed and writes the message (payload bytes, unmasked, no
 * NUL appended) to out / *out_len and its opcode to *opcode.  Returns 0 when
 * the stream ends before a message completes.
 */
size_t oracle_decode_message(const uint8_t *wire, size_t wire_len, uint8_t *out, size_t out_cap, size_t *out_len,
                             uint8_t *opcode)
{
    size_t p = 0, n = 0;
    *opcode = 0;
    for (;;)
    {
        if (p + 2 > wire_len) return 0;
        const uint8_t b0 = wire[p++], b1 = wire[p++];
        const int fin = (b0 & 0x80) >> 7;                                     /* :157 */
        const uint8_t op = b0 & 0x0F;                                         /* :161 */
        if (op != 0) *opcode = op;                                            /* :163-164 */
        const int mask = (b1 & 0x80) >> 7;                                    /* :180 */
        uint64_t len = b1 & 0x7F;                                             /* :181 */
        if (len == 126 || len == 127)
        {
            const size_t nb = len == 126 ? 2 : 8;                             /* :226-227 */
            if (p + nb > wire_len) return 0;
            len = 0;
            for (size_t i = 0; i < nb; ++i) len = (len << 8) | wire[p++];     /* big endian, :245-257 */
        }
        uint8_t key[4] = {0, 0, 0, 0};
        if (mask)
        {
            if (p + 4 > wire_len) return 0;
            memcpy(key, wire + p, 4);                                         /* :278-296 */
            p += 4;
        }
        if (p + len > wire_len || n + len > out_cap) return 0;
        memcpy(out + n, wire + p, (size_t)len);
        if (mask) oracle_unmask(out + n, (size_t)len, key, 0);                /* :317-323 */
        n += (size_t)len;
        p += (size_t)len;
        if (fin)
        {
            *out_len = n;
            return p;
        }
    }
}
