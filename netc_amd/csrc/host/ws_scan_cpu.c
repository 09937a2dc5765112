/*
 * Host header walk: the frame boundaries of a received byte stream in host memory
 * (include/ws/frame.h, netc_ws_scan_frames_host) -- the CPU counterpart of
 * netc_gpu_scan_frames, with the same outputs and the same strict checks.
 *
 * It hops from header to header (src/ws/common.c:146-296: byte 0 :157-161, byte 1
 * MASK + 7-bit length :180-181, 16 / 64-bit big-endian extended length :223-245,
 * 4 key bytes :273-289), so its cost is O(frames), not O(bytes): for streams of
 * large frames it beats any scan that has to look at every byte, which is why the
 * ingest ring (ws_ingest.hip) uses it for slots whose frames are large.
 */
#include <stdint.h>
#include <string.h>

#include "../../../include/ws/frame.h"
#include "../../../include/ws/mask.h"

/* one decoded header (decode() returns 0 when byte 1 or the extended length is not in the stream yet) */
struct hdr_view
{
    uint64_t hlen;   /* header bytes: 2 + extended length + key */
    uint64_t plen;   /* payload bytes */
    uint32_t key;    /* packed key32 (0 if MASK is clear) */
    uint8_t first, second;
};

static int decode(const uint8_t *w, uint64_t avail, struct hdr_view *h)
{
    if (avail < 2) return 0;
    h->first = w[0];
    h->second = w[1];
    const unsigned code = h->second & 0x7Fu;
    const uint64_t ext = code == 126 ? 2 : code == 127 ? 8 : 0;
    const uint64_t key_bytes = (h->second & 0x80u) ? 4 : 0;
    if (avail < 2 + ext) return 0;
    uint64_t plen = code;
    if (ext) {
        plen = 0;
        for (uint64_t i = 0; i < ext; ++i) plen = (plen << 8) | w[2 + i];
    }
    h->hlen = 2 + ext + key_bytes;
    h->plen = plen;
    h->key = 0;
    if (key_bytes && avail >= h->hlen) {
        uint32_t k;
        memcpy(&k, w + 2 + ext, 4);   /* wire order k0 k1 k2 k3 -> little-endian key32 */
        h->key = k;
    }
    return 1;
}

/* RFC 6455 §5.1, §5.2, §5.5: what a server must not accept from a client */
static int forbidden(const struct hdr_view *h)
{
    const unsigned op = h->first & 0x0Fu;
    if (!(h->second & 0x80u)) return 1;               /* MASK clear */
    if (h->first & 0x70u) return 1;                   /* RSV1-3 */
    if ((op >= 3 && op <= 7) || op >= 11) return 1;   /* reserved opcodes */
    if (op >= 8 && (!(h->first & 0x80u) || h->plen > 125)) return 1;   /* control: FIN, <= 125 */
    if ((h->second & 0x7Fu) == 127 && (h->plen >> 63)) return 1;     /* 64-bit length, top bit */
    return 0;
}

int netc_ws_scan_frames_host(const void *wire, size_t len, uint64_t start, int flags, uint64_t *hdr,
                             uint32_t *keys, uint8_t *b0, size_t max_frames, uint64_t *result)
{
    if (!result || (len && !wire) || (max_frames && (!hdr || !keys || !b0)) || (flags & ~NETC_WS_SCAN_STRICT))
        return NETC_GPU_EINVAL;
    const uint8_t *w = (const uint8_t *)wire;
    const int strict = (flags & NETC_WS_SCAN_STRICT) != 0;
    uint64_t n = 0, p = start;
    uint64_t error = UINT64_MAX;
    struct hdr_view h;
    while (p < len && decode(w + p, len - p, &h)) {
        if (strict && forbidden(&h)) {
            error = p;
            break;
        }
        const uint64_t room = len - p;
        if (h.hlen > room || h.plen > room - h.hlen) break;   /* the frame is not complete yet */
        if (n < max_frames) {
            hdr[n] = p;
            keys[n] = h.key;
            b0[n] = h.first;
        }
        ++n;
        p += h.hlen + h.plen;
    }
    if (hdr && n <= max_frames) hdr[n] = p;
    result[NETC_WS_SCAN_FRAMES] = n;
    result[NETC_WS_SCAN_CONSUMED] = p;
    result[NETC_WS_SCAN_ERROR] = error;
    return 0;
}
