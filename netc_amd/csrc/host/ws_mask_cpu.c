/*
 * Host half of include/ws/mask.h: the CPU masking entry used by the framing
 * layer (ws_parse_frame / ws_send_message) and the byte-balanced shard planner
 * used to spread a frame batch over several GPUs.
 *
 * netc_ws_mask replaces the reference's per-byte loops
 *   src/ws/common.c:319-322  buffer_ptr[i] ^= masking_key[(received_length + i) % 4]
 *   src/ws/common.c:104-107  payload[i] ^= payload_masking_key[i % 4]
 * with a word-at-a-time XOR: the key is rotated once to the phase of the first
 * aligned word and replicated to 64 bits; every later 8-byte step keeps the
 * same rotation because 8 is a multiple of the key period 4.
 */
#include "../../../include/ws/mask.h"
#include "../../../include/ws/frame.h"

#include <stdint.h>
#include <string.h>

void netc_ws_mask(uint8_t *dst, const uint8_t *src, size_t len, const uint8_t key[4], size_t phase)
{
    size_t i = 0;
#if defined(__BYTE_ORDER__) && __BYTE_ORDER__ == __ORDER_LITTLE_ENDIAN__
    while (i < len && (((uintptr_t)(dst + i)) & 7u) != 0)
    {
        dst[i] = src[i] ^ key[(phase + i) & 3u];
        ++i;
    }
    if (len - i >= 8)
    {
        const size_t r = (phase + i) & 3u;
        const uint32_t k32 = (uint32_t)key[r] | ((uint32_t)key[(r + 1) & 3u] << 8) |
                             ((uint32_t)key[(r + 2) & 3u] << 16) | ((uint32_t)key[(r + 3) & 3u] << 24);
        const uint64_t k64 = (uint64_t)k32 | ((uint64_t)k32 << 32);
        for (; i + 8 <= len; i += 8)
        {
            uint64_t w;
            memcpy(&w, src + i, sizeof(w));
            w ^= k64;
            memcpy(dst + i, &w, sizeof(w));
        }
    }
#endif
    for (; i < len; ++i) dst[i] = src[i] ^ key[(phase + i) & 3u];
}

static size_t lower_bound_u64(const uint64_t *a, size_t lo, size_t hi, uint64_t x)
{
    while (lo < hi)
    {
        const size_t mid = lo + (hi - lo) / 2;
        if (a[mid] < x) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

int netc_shard_frames(const uint64_t *offsets, size_t nframes, size_t nshards, size_t *cuts)
{
    if (offsets == NULL || cuts == NULL || nshards == 0) return NETC_GPU_EINVAL;
    for (size_t k = 0; k < nframes; ++k)
        if (offsets[k + 1] < offsets[k]) return NETC_GPU_EINVAL;

    const uint64_t lo = offsets[0], span = offsets[nframes] - offsets[0];
    cuts[0] = 0;
    for (size_t i = 1; i < nshards; ++i)
    {
        /* ideal byte position of cut i, then the nearest frame boundary at or after the previous cut */
        const unsigned __int128 t = (unsigned __int128)span * i / nshards;
        const uint64_t target = lo + (uint64_t)t;
        size_t k = lower_bound_u64(offsets, cuts[i - 1], nframes + 1, target);
        if (k > nframes) k = nframes;
        if (k > cuts[i - 1] && offsets[k] - target > target - offsets[k - 1]) --k;
        cuts[i] = k;
    }
    cuts[nshards] = nframes;
    return 0;
}

/* include/ws/frame.h: header lengths as src/ws/common.c:63,69-82 (+ 4 key bytes when masked) */
uint64_t netc_ws_wire_size(const uint64_t *offsets, size_t nframes, int masked)
{
    uint64_t total = 0;
    for (size_t k = 0; k < nframes; ++k)
    {
        const uint64_t len = offsets[k + 1] - offsets[k];
        total += 2 + (len < 126 ? 0 : (len < 65536 ? 2 : 8)) + (masked ? 4 : 0) + len;
    }
    return total;
}
