// MI355X (gfx950 / CDNA4) frame-boundary scan — device kernels.
//
// Replaces the reference's header state machine (src/ws/common.c:146-296: byte 0
// FIN | RSV | opcode, byte 1 MASK | 7-bit length, 16 / 64-bit big-endian extended
// length, 4 key bytes) run over a received byte stream: it finds every frame of
// the stream (header offset, key, byte 0) in parallel.
//
// Frame starts form a chain: the next header follows the current frame's payload.
// The stream is cut into chunks of C = 4 KiB, chunks into tiles of 256 (1 MiB).
// Five launches (four up to 256 tiles = 256 MiB of stream, where K3b runs in the last K3a block to
// arrive: scan_tiles_resolve):
//   K1  scan_exits    one wavefront per chunk, straight from HBM (16-B loads, no
//                     LDS staging): the strict quick check on bytes 0-1 of every
//                     position, 4 positions per 5 VALU operations (SWAR).  A chain
//                     inside the chunk only steps between positions that pass it, so
//                     the places where chains LEAVE the chunk are direct exits of
//                     passing positions -- and only two kinds can exit: a 16/64-bit
//                     length (byte 1 & 0x7E == 0x7E) or a position in the chunk's last
//                     132 bytes.  Those few are parsed; their distinct exits become
//                     "candidate entries" (nodes) of the chunks they land in (the true
//                     chain enters each chunk at one of them).
//   K2  scan_links    per node: its chain walked inside its chunk (header bytes from
//                     global memory) to the node it exits to, counting frames; chains
//                     of more than 64 frames are finished by the workgroup in LDS
//                     (16-bit in-chunk links doubled to 8 / 16 hops), leaving an anchor
//                     every 8 frames for K4.
//   K3a scan_tiles    per tile, in LDS: list ranking over the tile's nodes (Wyllie
//                     pointer jumping): for every node the frames to the tile's exit
//                     (W) and the last node before it, and, for each of the tile's
//                     "external" nodes (entered from another tile: at most 32), a bit
//                     pushed along its path.
//   K3b scan_resolve  one workgroup: the same list ranking over the external nodes of
//                     all tiles (a few per tile), from the stream start: which external
//                     is each tile's true entry, the frames before it, and where the
//                     chain ends (the results).
//   K4  scan_emit     per chunk: its true entry (the node carrying its tile entry's
//                     bit), its first frame index (tile base + W(entry) - W(node)), and
//                     a walk writing the descriptors; past 64 frames one wavefront per
//                     chunk from K2's anchors, or the workgroup from LDS.
// Garbage chains (payload bytes parsed as headers) die within a hop or two under
// the strict checks, so chunks have few distinct exits; a stream whose exits
// overflow the fixed capacities (adversarial payloads, non-strict mode) is finished
// by a serial walk in K4 instead — same results, slower.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <map>
#include <memory>
#include <mutex>
#include <new>
#include <vector>
#include <type_traits>
#include <utility>

#include "gpu_util.h"
#include "ws_mask_gpu.h"

namespace netc_gpu {

static constexpr uint64_t kChunk = 4096;        // bytes per chunk
static constexpr int kScanT = 256;              // threads per K2 / K3a / K4 block
static constexpr int kPer = (int)(kChunk / kScanT);
static constexpr int kCand = 8;                 // candidate entries (node slots) per chunk
static constexpr int kSet = 64;                 // distinct exits per chunk
static constexpr uint64_t kTerm = 1ull << 63;   // link is terminal
static constexpr uint64_t kPosMask = (1ull << 61) - 1;
enum : uint64_t { kExit = 0, kEnd = 1, kDead = 2 };
static constexpr uint64_t kTileChunks = 256;                  // K3a: chunks per tile (1 MiB of stream)
static constexpr uint64_t kTileSlots = kTileChunks * kCand;   // node slots per tile
static constexpr int kExt = 32;                               // external nodes per tile (bits)
static constexpr int kResolveT = 1024;                        // K3b threads
static constexpr int kExtCap = 4096;                          // K3b: external nodes of the whole stream
static constexpr int kMaxTiles = 8192;                        // K3b: tiles (8 GiB of stream)
// K2 / K4 chunks per block.  Round 2 had 16 for both; at config 4 (65,537 chunks, most of them
// without a node) the blocks were the cost: 32 per K2 block (a thread per node slot, all 256
// busy) and 32 per K4 block took K2 13.5 -> 9.7 us and K4 9.4 -> 6.2 us at config 4 (r03h2),
// the scan 87.6 -> 81.3 us, config 2 unchanged (42.8); 64 per K4 block: config 4 80.1, config 2
// 43.2 (r03i2).
#ifndef NETC_SCAN_BLK
#define NETC_SCAN_BLK 32   // A/B builds
#endif
static constexpr int kBlkChunks = NETC_SCAN_BLK;              // K2: chunks per block
// K2 and K4 take twice the chunks per block above 128 MiB of stream, where most chunks hold no
// node and the blocks themselves are the cost (C4: 2,049 blocks of 32 take 1.6 rounds at 5 per
// CU; 1,025 of 64 fit one); K2 then runs two node slots per thread.  Up to 128 MiB 32 stay (C2:
// 64 per K4 block measured 43.2 against 42.5 us, r03i2).  Knob SCAN_BLOCK_CHUNKS picks either for
// any stream (tests, A/B).
static constexpr int kEmitChunks = 32;          // K4: chunks per block
static constexpr int kBlkChunksBig = 64;        // K2 and K4 above kBigBlocksAbove chunks
static constexpr uint64_t kBigBlocksAbove = 32768;   // chunks (128 MiB)
static_assert(kBlkChunks * kCand <= 256 && kTileChunks % kBlkChunks == 0, "K2: one thread per node slot");
static_assert(kEmitChunks <= 256 && kTileChunks % kEmitChunks == 0, "K4: one thread per chunk, blocks inside a tile");
static_assert(kBlkChunksBig <= 256 && kTileChunks % kBlkChunksBig == 0 && kBlkChunksBig * kCand < 0xFFFF,
              "K2 / K4: a thread per chunk (K4), node slots as 16-bit indexes (K2), blocks inside a tile");
static constexpr int32_t kDupLink = -2;                       // K2: slot repeats an earlier slot's position
static constexpr int kWalkHops = 64;                          // K2 / K4: frames walked one by one
static constexpr int kList = 8;                               // K2 -> K4: frames recorded per node
static constexpr int kListSlots = 4;                          // ... for node slots 0..3 of a chunk
static constexpr uint32_t kH = 0x80808080u;
// why a scan fell back to the serial walk (flags[9], read by netc_gpu_scan_diag): bits
// 0-7 flags[0] (K1 bucket full, K1 exit set full, K2 exit onto no candidate, K3a tile
// external list full, K1 candidate queue full), 8+ K3b's own reason
enum : uint32_t { kOvfBucket = 1, kOvfSet = 2, kOvfLink = 4, kOvfExt = 8, kOvfQueue = 16 };
enum : uint32_t { kWhyRoot = 1u << 8, kWhyTiles = 2u << 8, kWhyExtCap = 3u << 8, kWhySucc = 4u << 8 };
// bit 16: a speculative (non-strict) pass stopped at a header the filter rejects; the rest was walked serially
enum : uint32_t { kWhySpec = 1u << 16 };

#ifdef NETC_SCAN_STAMPS
// diagnostic build only (tools/scan_stamps.py): per kernel k (K1..K4 = 0..4) and block b
// < kStampBlocks, 8 wall-clock stamps (100 MHz): [0] start, [1..6] phases, [7] end
static constexpr int kStampBlocks = 8192;
__device__ uint64_t* g_scan_stamps;
extern "C" int netc_gpu_debug_scan_stamps(void* d_buf) {
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_scan_stamps), &d_buf, sizeof(d_buf));
}
__device__ __forceinline__ void scan_stamp(int k, int i) {
    if (threadIdx.x == 0 && g_scan_stamps && blockIdx.x < (unsigned)kStampBlocks)
        g_scan_stamps[((uint64_t)k * kStampBlocks + blockIdx.x) * 8 + i] = __builtin_amdgcn_s_memrealtime();
}
struct ScanStampScope {
    int k;
    __device__ explicit ScanStampScope(int kk) : k(kk) { scan_stamp(k, 0); }
    __device__ ~ScanStampScope() { scan_stamp(k, 7); }
};
__device__ __forceinline__ void scan_value(int k, int i, uint64_t v) {   // a count instead of a time (slots 5, 6)
    if (threadIdx.x == 0 && g_scan_stamps && blockIdx.x < (unsigned)kStampBlocks)
        g_scan_stamps[((uint64_t)k * kStampBlocks + blockIdx.x) * 8 + i] = v;
}
#define SCAN_SCOPE(k) ScanStampScope scan_scope_guard(k)
#define SCAN_STAMP(k, i) scan_stamp(k, i)
#define SCAN_VALUE(k, i, v) scan_value(k, i, v)
// K2's per-wavefront dense path: summed phase durations (100 MHz ticks) over every call, and calls
__device__ unsigned long long g_dense_phase[8];
extern "C" int netc_gpu_debug_dense_phases(unsigned long long* out8, int reset) {
    hipError_t e = hipMemcpyFromSymbol(out8, HIP_SYMBOL(g_dense_phase), sizeof(g_dense_phase));
    if (reset) {
        const unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        (void)hipMemcpyToSymbol(HIP_SYMBOL(g_dense_phase), z, sizeof(z));
    }
    return (int)e;
}
#define DENSE_T(i) uint64_t dense_t##i = (threadIdx.x & 63) == 0 ? __builtin_amdgcn_s_memrealtime() : 0
#define DENSE_ADD(i, a, b) (dacc[i] += dense_t##b - dense_t##a)
#define DENSE_COUNT() (dacc[7] += 1)
#define DENSE_ACC uint64_t dacc[8] = {0, 0, 0, 0, 0, 0, 0, 0}
#define DENSE_ARG , uint64_t (&dacc)[8]
#define DENSE_PASS , dacc
#define DENSE_FLUSH() \
    if ((threadIdx.x & 63) == 0 && dacc[7]) \
        for (int i_ = 0; i_ < 8; ++i_) atomicAdd(&g_dense_phase[i_], (unsigned long long)dacc[i_])
#else
#define SCAN_SCOPE(k) ((void)0)
#define SCAN_STAMP(k, i) ((void)0)
#define SCAN_VALUE(k, i, v) ((void)0)
#define DENSE_T(i) ((void)0)
#define DENSE_ADD(i, a, b) ((void)0)
#define DENSE_COUNT() ((void)0)
#define DENSE_ACC
#define DENSE_ARG
#define DENSE_PASS
#define DENSE_FLUSH() ((void)0)
#endif

#ifdef NETC_SCAN_TRACE
// diagnostic build only (tools/scan_probe.py): progress words in host-mapped memory, readable
// while a kernel still runs
__device__ uint32_t* g_op_trace;
extern "C" int netc_gpu_debug_scan_trace(void* host_mapped) {
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_op_trace), &host_mapped, sizeof(host_mapped));
}
#define OP_TRACE(i, v) \
    do { \
        if (g_op_trace) __hip_atomic_store(g_op_trace + (i), (uint32_t)(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); \
    } while (0)
// ... and a device buffer of 64-bit words (timestamps, counts) the probe copies after the call
__device__ uint64_t* g_op_stamp;
extern "C" int netc_gpu_debug_scan_stamps(void* device_buffer) {
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_op_stamp), &device_buffer, sizeof(device_buffer));
}
#define OP_STAMP(i, v) \
    do { \
        if (g_op_stamp) g_op_stamp[i] = (uint64_t)(v); \
    } while (0)
#define OP_STAMP_MAX(i, v) \
    do { \
        if (g_op_stamp) __hip_atomic_fetch_max(g_op_stamp + (i), (uint64_t)(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); \
    } while (0)
#define OP_STAMP_MIN(i, v) \
    do { \
        if (g_op_stamp) __hip_atomic_fetch_min(g_op_stamp + (i), (uint64_t)(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); \
    } while (0)
#define OP_STAMP_ADD(i, v) \
    do { \
        if (g_op_stamp) __hip_atomic_fetch_add(g_op_stamp + (i), (uint64_t)(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); \
    } while (0)
#else
#define OP_TRACE(i, v) ((void)0)
#define OP_STAMP(i, v) ((void)0)
#define OP_STAMP_MAX(i, v) ((void)0)
#define OP_STAMP_MIN(i, v) ((void)0)
#define OP_STAMP_ADD(i, v) ((void)0)
#endif
// OP_STAMP layout (trace build): [0] K1 first start (min), [1] K1 last wave's end (max), [5] [6]
// [7] [8] chunks whose T is None, Single, Multi, Fail

__device__ __forceinline__ uint64_t term(uint64_t type, uint64_t pos) { return kTerm | type << 61 | pos; }
__device__ __forceinline__ uint64_t term_type(uint64_t v) { return (v >> 61) & 3; }
__device__ __forceinline__ uint64_t term_pos(uint64_t v) { return v & kPosMask; }

// K3a -> K3b: an external node of a tile
struct TileExt {
    uint32_t slot;   // its global node slot
    uint32_t w;      // frames from it to the tile's exit
    int32_t xl;      // the node its path exits to (another tile), or -1: the chain ends in the tile
    uint32_t root;   // it is the stream start
    uint64_t term;   // K2's terminal of the path's last node in the tile
};
// K3a -> K3b records travel by relaxed agent-scope stores and loads (global_store / load
// ... sc1: through to the memory-side caches, past the XCD's own L2), so the K3b phase can
// run in the last block of the K3a launch (scan_tiles_resolve) with no L2 write-back or
// invalidate: every storing wave waits for its stores, the block then adds to an arrival
// counter, and the last block to arrive reads with sc1 loads only (MI355X_MICROARCH.md,
// cross-workgroup hand-offs, first row).
__device__ __forceinline__ void put_text(TileExt* p, const TileExt& e) {
    uint64_t w[3];
    __builtin_memcpy(w, &e, sizeof(w));
#pragma unroll
    for (int i = 0; i < 3; ++i) __hip_atomic_store((uint64_t*)p + i, w[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ TileExt get_text(const TileExt* p) {
    uint64_t w[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) w[i] = __hip_atomic_load((const uint64_t*)p + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    TileExt e;
    __builtin_memcpy(&e, w, sizeof(w));
    return e;
}
__device__ __forceinline__ uint32_t get_sc1(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
static_assert(sizeof(TileExt) == 24, "TileExt: three 8-byte words");

// K3b -> K4: a tile's true entry
struct TileInfo {
    int32_t j;       // its bit (index in the tile's external list), or -1: the chain does not enter the tile
    uint32_t we;     // its W
    uint64_t base;   // index of its first frame
};

struct ScanArgs {
    const uint8_t* wire;
    const uint8_t* pf_base;   // K1's clamped loads: wire, or a scratch word for a stream under 16 bytes
    uint64_t pf_lim;          // ... highest 16-byte load offset
    uint64_t len;          // stream bytes
    uint64_t start;        // offset of the first header
    uint64_t nc;           // chunks (the last one, index nc, is virtual: positions >= len)
    int strict;            // the header filter is on (always, see spec)
    int spec;              // the caller asked for no checks: the parallel pass runs with the strict
                           // filter minus the MASK and RSV1 checks, and K4 walks on serially, unchecked, from
                           // a header that filter rejects (speculative: RFC-clean streams never stop)
    uint32_t* flags;       // [8] K3b -> K4: serial fallback (big streams), [9] why the last call walked serially
    uint32_t* ovf;         // this call's overflow bits (flags[0] / flags[2] on alternate calls: the
    uint32_t* ovf_prev;    // ... reader is every K4 block, so K4 zeroes the previous call's word instead)
    uint32_t* ccount;      // nc + 1 candidate counters (zero when a call starts; K4 re-zeroes)
    uint8_t* ext;          // (nc + 1) * kCand: slot entered from another tile (or the root); K4 re-zeroes
    uint32_t* tarr;        // K2+ (fused): per-tile arrival counters (the last arrival re-zeroes)
    uint64_t* cand;        // (nc + 1) * kCand candidate positions
    int32_t* link;         // node -> next node, -1 = chain ends, kDupLink
    uint64_t* nterm;       // the terminal where the node's walk leaves its chunk
    uint32_t* ncnt;        // frames on that walk
    uint32_t* wsum;        // K3a: frames from the node to its tile's exit
    uint32_t* pbits;       // K3a: external nodes of the tile whose path holds the node
    TileExt* text;         // tiles * kExt
    uint32_t* tcount;      // tiles
    TileInfo* tinfo;       // tiles
    uint16_t* anc;         // K2' -> K4: 8-frame anchors of anchor slot q at anc[q * kAncSlot]
    uint32_t* anc_n;       // anchors in slot q
    uint32_t* anq;         // per node: its anchor slot, or ~0 when none was left
    uint64_t* flist;       // K2 -> K4: the frames of node slots 0..kListSlots-1 of each chunk, when
                           // the node's walk has at most kList of them: {offset in the chunk,
                           // header byte 0 << 16, key << 32} per frame
    uint64_t anc_cap;      // anchor slots
    uint64_t* hdr;         // outputs
    uint32_t* keys;
    uint8_t* b0;
    uint64_t max_frames;
    uint64_t* result;      // [0] frames, [1] consumed, [2] error offset or ~0
    int fast_rank;         // K3a / K3b may take their one-barrier-per-round ranking (0: the generic
                           // loop always; NETC_SCAN_FAST_RANK=0, tests)
    // the one-pass path (scan_exits<_, true>; see "One pass" below)
    int onepass;           // this call runs it (the host's choice: knob SCAN_ONEPASS, stream size)
    uint64_t op_walk;      // frames a chunk's walk may be projected to (kOpWalk; kOpRec when forced by the knob)
    uint32_t* opfail;      // this call's one-pass failure words: kFailCopies, kFailStride apart (two sets,
    uint32_t* opfail_prev; // ... alternate calls; K4 zeroes the previous call's, as for ovf)
    uint64_t* st_t;        // per chunk: its exit prediction T (epoch-tagged; K1)
    uint64_t* st_g;        // per block of kOpT chunks: its look-back status word
    uint64_t* opfl;        // per chunk: kOpRec frames {offset, byte 0 << 16, key << 32}
    uint64_t epoch;        // 1 .. 2^24 - 1, one per call on the scratch (words of other calls do not match)
};

// RSV bits the header filter rejects: all three in strict mode; in the speculative pass
// (non-strict: the caller accepts every header) RSV2 / RSV3 only -- RSV1 is what
// permessage-deflate sets on every data frame's first fragment (RFC 7692 §6), so such
// streams stay on the parallel path (a stop there walked the rest serially).
// Garbage positions then pass the filter twice as often, no more.
__device__ __forceinline__ uint32_t rsv_reject(const ScanArgs& a) { return a.spec ? 0x30u : 0x70u; }
// the same on 4 first-header bytes at once (quick_ok4's x): RSV1 cleared in the speculative pass
__device__ __forceinline__ uint32_t rsv_keep4(const ScanArgs& a) { return a.spec ? 0xBFBFBFBFu : 0xFFFFFFFFu; }

// One header at stream position p (bytes b[0..13] from p; bytes past len unused).
// Returns the link: the next header position, or a terminal.  (The serial fallback.)
template <typename Bytes>
__device__ __forceinline__ uint64_t parse_at(const ScanArgs& a, uint64_t p, const Bytes& b, uint32_t* key_out,
                                             uint8_t* b0_out) {
    if (p + 2 > a.len) return term(kEnd, p);
    const uint32_t first = b[0], second = b[1];
    const uint32_t code = second & 0x7F, mask = second >> 7, opcode = first & 0x0F;
    const uint64_t ext = code == 126 ? 2 : (code == 127 ? 8 : 0);
    if (p + 2 + ext > a.len) return term(kEnd, p);
    uint64_t plen = code;
    if (ext == 2) plen = (uint64_t)b[2] << 8 | b[3];
    if (ext == 8) {
        plen = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) plen = plen << 8 | b[2 + i];
    }
    if (a.strict) {
        const bool reserved = (opcode >= 3 && opcode <= 7) || opcode >= 11;
        const bool control = opcode >= 8;
        if ((!mask && !a.spec) || (first & rsv_reject(a)) || reserved || (control && (!(first & 0x80) || plen > 125)) ||
            (plen >> 63))
            return term(kDead, p);
    }
    const uint64_t hl = 2 + ext + (mask ? 4 : 0);
    if (p + hl > a.len || plen > a.len - (p + hl)) return term(kEnd, p);
    if (key_out) {   // key bytes at 2 + ext (constant offsets: no dynamic indexing)
        auto rd = [&](int o) {
            return (uint32_t)b[o] | (uint32_t)b[o + 1] << 8 | (uint32_t)b[o + 2] << 16 | (uint32_t)b[o + 3] << 24;
        };
        *key_out = mask ? (ext == 0 ? rd(2) : (ext == 2 ? rd(4) : rd(10))) : 0u;
        *b0_out = (uint8_t)first;
    }
    return p + hl + plen;
}

// Strict mode: can a header start at x at all?  (The two first bytes fail the
// checks.)  A chain reaching such an x dies there: DEAD(x).
__device__ __forceinline__ bool quick_reject(const ScanArgs& a, uint64_t x) {
    if (!a.strict || x + 2 > a.len) return false;
    const uint32_t first = gptr(a.wire)[x], second = gptr(a.wire)[x + 1];
    const uint32_t opcode = first & 0x0F;
    const bool reserved = (opcode >= 3 && opcode <= 7) || opcode >= 11;
    return (!(second & 0x80) && !a.spec) || (first & rsv_reject(a)) || reserved || (opcode >= 8 && !(first & 0x80));
}

// 16 stream bytes from LDS position i as 4 dwords (5 dword reads + v_alignbyte),
// indexed with constant byte offsets once the parse is unrolled.
struct Win {
    uint32_t d[4];
    __device__ __forceinline__ uint32_t operator[](int j) const { return (d[j >> 2] >> (8 * (j & 3))) & 0xFF; }
};

__device__ __forceinline__ Win window_at(const uint32_t* words, int i) {
    const int q = i >> 2;
    uint32_t w[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) w[k] = words[q + k];
    Win x;
#pragma unroll
    for (int k = 0; k < 4; ++k) x.d[k] = __builtin_amdgcn_alignbyte(w[k + 1], w[k], (uint32_t)(i & 3));
    return x;
}

// parse_at for a 16-byte window (every caller but the serial fallback): the same
// checks in the same order, computed without branches -- lanes of a wavefront parse
// different headers, and the branchy form cost about one scalar (exec-mask)
// instruction per vector instruction.  Window bytes past len are zero.
__device__ __forceinline__ uint64_t parse_at(const ScanArgs& a, uint64_t p, const Win& w, uint32_t* key_out,
                                             uint8_t* b0_out) {
    const uint32_t first = w.d[0] & 0xFF, second = (w.d[0] >> 8) & 0xFF;
    const uint32_t code = second & 0x7F, mask = second >> 7, opcode = first & 0x0F;
    const uint64_t ext = code == 126 ? 2 : (code == 127 ? 8 : 0);
    const uint32_t b25 = __builtin_amdgcn_alignbyte(w.d[1], w.d[0], 2);   // bytes 2..5
    const uint32_t b69 = __builtin_amdgcn_alignbyte(w.d[2], w.d[1], 2);   // bytes 6..9
    const uint64_t len16 = __builtin_bswap32(b25) >> 16;
    const uint64_t len64 = __builtin_bswap64((uint64_t)b69 << 32 | b25);
    const uint64_t plen = ext == 0 ? code : (ext == 2 ? len16 : len64);
    const uint64_t hl = 2 + ext + (mask ? 4 : 0);
    const bool hdr_short = p + 2 + ext > a.len;
    const bool reserved = (opcode >= 3) & ((opcode <= 7) | (opcode >= 11));
    const bool control = opcode >= 8;
    const bool dead = (a.strict != 0) & (((mask == 0) & (a.spec == 0)) | ((first & rsv_reject(a)) != 0) | reserved |
                                         (control & (((first & 0x80) == 0) | (plen > 125))) | ((plen >> 63) != 0));
    const bool pay_short = (p + hl > a.len) | (plen > a.len - (p + hl));
    if (key_out) {
        const uint32_t k = ext == 0 ? b25 : (ext == 2 ? w.d[1] : __builtin_amdgcn_alignbyte(w.d[3], w.d[2], 2));
        *key_out = mask ? k : 0u;
        *b0_out = (uint8_t)first;
    }
    return hdr_short ? term(kEnd, p) : (dead ? term(kDead, p) : (pay_short ? term(kEnd, p) : p + hl + plen));
}

// LDS copy of the chunk: stream bytes [B, B + kChunk + 32), zero past len.
static constexpr int kWords = (int)((kChunk + 32) / 4);

__device__ void load_chunk(const ScanArgs& a, uint64_t B, uint32_t* words) {
    typedef uint32_t u32x4u __attribute__((ext_vector_type(4), aligned(1)));
    const int tid = threadIdx.x, nt = blockDim.x;
    if (B + kChunk + 32 <= a.len) {
        for (int v = tid; v < kWords / 4; v += nt) {   // 16-B loads (any alignment of the stream)
            const u32x4 x = *(const NETC_GLOBAL u32x4u*)(a.wire + B + 16 * (uint64_t)v);
            words[4 * v] = x[0];
            words[4 * v + 1] = x[1];
            words[4 * v + 2] = x[2];
            words[4 * v + 3] = x[3];
        }
    } else {
        uint8_t* bytes = (uint8_t*)words;
        for (int i = tid; i < kWords * 4; i += nt) bytes[i] = B + i < a.len ? gptr(a.wire)[B + i] : 0;
    }
    __syncthreads();
}

// 16 stream bytes from p (zero past len) straight from global memory: the walks
// touch only the header bytes of the frames they visit, so they read them where
// they lie instead of staging the chunk in LDS.
__device__ __forceinline__ Win window_global(const ScanArgs& a, uint64_t p) {
    typedef uint32_t u32x4u __attribute__((ext_vector_type(4), aligned(1)));
    Win w;
    if (p + 16 <= a.len) {
        const u32x4 x = *(const NETC_GLOBAL u32x4u*)(a.wire + p);
#pragma unroll
        for (int k = 0; k < 4; ++k) w.d[k] = x[k];
    } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) w.d[k] = 0;
        for (int j = 0; j < 16; ++j)
            if (p + j < a.len) w.d[j >> 2] |= (uint32_t)gptr(a.wire)[p + j] << (8 * (j & 3));
    }
    return w;
}

// Walk the frames from e until the chain leaves the chunk [B, B + kChunk) (its
// terminal: EXIT, END or DEAD), calling emit(p, key, b0) for each complete frame;
// 0 if `hops` frames did not get there.  Windows from LDS (words, the chunk) or
// from global memory.
template <bool LDS, typename F>
__device__ uint64_t walk_frames(const ScanArgs& a, uint64_t B, const uint32_t* words, uint64_t e, int hops, F&& emit,
                                uint64_t* stop = nullptr) {
    const uint64_t Bend = B + kChunk;
    uint64_t p = e;
    for (int h = 0;; ++h) {
        if (p >= Bend) return term(kExit, p);
        if (h == hops) {
            if (stop) *stop = p;   // the next frame's header
            return 0;
        }
        uint32_t key;
        uint8_t b0;
        const uint64_t v = LDS ? parse_at(a, p, window_at(words, (int)(p - B)), &key, &b0)
                               : parse_at(a, p, window_global(a, p), &key, &b0);
        if (v & kTerm) return v;
        emit(p, key, b0);
        p = v;
    }
}

// The strict quick check for 4 positions at once: x = bytes 0 of positions 0..3,
// y = their bytes 1.  Bit 7 of a byte of the result is set when that position can
// start a client frame: MASK set, RSV clear, opcode 0/1/2/8/9/A, FIN on a control
// frame.  (first & 0x77) + 0x7D carries into bit 7 exactly when an RSV bit is set or
// (opcode & 7) >= 3 (the reserved opcodes 3-7, B-F); (x << 4) & ~x has bit 7 set for
// a control opcode (bit 3) without FIN (bit 7).  No carry crosses a byte; checked
// against quick_reject over all 65,536 byte pairs.  5 VALU operations.
__device__ __forceinline__ uint32_t quick_ok4(uint32_t x, uint32_t y) {
    return y & ~((x & 0x77777777u) + 0x7D7D7D7Du) & ~((x << 4) & ~x) & kH;
}

// x into the wavefront's LDS set of distinct exits (open addressing): true if it is
// new; *overflow when the set is full
__device__ __forceinline__ bool set_insert(unsigned long long* set, uint64_t x, bool* overflow) {
    uint32_t h = (uint32_t)((x * 0x9E3779B97F4A7C15ull) >> 58);
    for (int tries = 0; tries < kSet; ++tries, h = (h + 1) & (kSet - 1)) {
        const unsigned long long cur = set[h];
        if (cur == x) return false;
        if (cur == ~0ull) {
            const unsigned long long prev = atomicCAS(&set[h], ~0ull, (unsigned long long)x);
            if (prev == ~0ull) return true;
            if (prev == x) return false;
        }
    }
    *overflow = true;
    return false;
}

// x as a candidate entry (node slot) of the chunk it lies in; ext: appended from a
// chunk of another tile, or the stream start (K3a's external nodes)
__device__ __forceinline__ void append_cand(const ScanArgs& a, uint64_t x, bool ext) {
    const uint64_t t = x / kChunk;   // x <= len: t <= nc
    const uint32_t slot = atomicAdd(&a.ccount[t], 1u);
    if (slot < (uint32_t)kCand) {
        a.cand[t * kCand + slot] = x;
        if (ext) a.ext[t * kCand + slot] = 1;
    } else {
        atomicOr(a.ovf, kOvfBucket);
    }
}

__device__ __forceinline__ void put_frame(const ScanArgs& a, uint64_t k, uint64_t p, uint32_t key, uint8_t b0);
// a lane of the last vector of a chunk whose 16 positions can exit the chunk with a
// 7-bit length: p + 2 + 4 + 125 >= chunk end  <=>  offset >= 3965 (lane 55 holds 3952-3967)
static constexpr int kNearLane = 55;
// K1's LDS per 4-wave block: each wave's chunk (+ the 16 bytes after it, all a window at offset
// 4095 reads), exit set and candidate queue.  At 248 queue entries the block takes 20,480 B, so 8
// blocks (32 waves, the SIMDs' limit) fit a CU's 160 KiB where the 20,992 B of a 32-byte tail and
// 256 entries allowed 7.  NETC_K1_SLIM=0 restores that layout (A/B builds).
#ifndef NETC_K1_SLIM
#define NETC_K1_SLIM 1
#endif
static constexpr int kQCap = NETC_K1_SLIM ? 248 : 256;   // K1: exit-capable candidates queued per chunk (more: serial walk)
static constexpr int kStageWords = NETC_K1_SLIM ? (int)((kChunk + 16) / 4) : kWords;
static_assert(!NETC_K1_SLIM || 4 * (4 * kStageWords + 8 * kSet + 2 * kQCap) <= 20480,
              "K1: a 4-wave block must stay within 20,480 B of LDS (8 blocks per CU)");
static constexpr int kCheapMax = 64;   // K1: more from the cheap selection: the full quick check instead

__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t v);
// ------------------------------------------------------------------ one pass --
// The one-pass path for dense streams -- frames shorter than a chunk, so the chain
// visits every chunk from the start on (the C2 shape).  K1 publishes, per chunk c, T(c): where the
// chain leaves c if it visits it, from the distinct exits of c's exit-capable candidates that land
// on a position able to start a header (the nodes K1 appends): that exit when there is exactly one
// (Single), None (no such exit: a chain that visits c ends in it, or dies at an exit onto a
// position that cannot start a header), Multi, or Fail (K1's queue or set overflowed).  Garbage
// chains (payload bytes parsed as headers) land on header-capable positions with ~2 % odds, so
// nearly every chunk is Single.
//
// The next launch (scan_op_walk, a thread per chunk) SPECULATES each chunk's entry from its
// predecessor alone -- T(c-1) if Single, END if None, the predecessor's own walk exit W(c-1) if
// Multi, which it walks to itself from the nearest predecessor with a known T -- walks its frames
// from there (header bytes from global memory) to its exit W(c), and checks:
//   * an entry past the chunk's end (a frame covers it: not a dense stream) fails;
//   * a visited chunk's W(c) must equal T(c) when T(c) is Single (its successor used T(c));
//   * a chunk not visited (entry END) must not be Single (its successor would walk from T(c)).
// By induction from the start chunk (entry = the start), if no chunk fails every speculated entry
// is the true one.  Nothing waits but the blocks' decoupled look-back over their frame counts;
// then every chunk writes its descriptors and
// the chunk where the chain ends the results.  Any failure (a check, Fail, a speculative stop at a
// header the filter rejects, more than kOpRec frames in a chunk) sets the call's failure word, and
// K2-K4 then run the graph path from the nodes K1 appended all the same, overwriting everything;
// the results are the same either way.  T and the look-back words carry the call's epoch (never
// cleared per call).  (Round 6 first resolved the chunks inside K1 itself: with a frame counter
// per group and tile bumped by device-scope atomics, 126 us at config 2 -- hot-address atomics
// under K1's stream; without them still 34 us for K1 alone, the entry waits holding K1's waves.
// DESIGN.md §16.4.)
static constexpr uint64_t kOpBits = 40;
static constexpr uint64_t kOpMask = (1ull << kOpBits) - 1;
static constexpr uint64_t kTNone = kOpMask, kTMulti = kOpMask - 1, kTFail = kOpMask - 2;   // T values; else the exit
static constexpr uint64_t kXEnd = kOpMask;                              // W / entry: no chain here
static constexpr uint64_t kOnePassWait = 200000;                        // 2 ms at 100 MHz
static constexpr uint64_t kOnePassMax = 128ull << 20;                   // knob 2: streams up to 128 MiB
static constexpr uint64_t kOnePassCap = 256ull << 20;                   // knob 1: up to 256 MiB
static constexpr int kOpRec = 64;                                       // frames one chunk may hold
static constexpr int kOpT = 256;                                        // chunks per scan_op_walk block
static constexpr int kOpReg = 6;                                        // ... frames of a chunk held in registers
static constexpr uint64_t kOpWalk = 16;                                 // frames a chunk's walk is projected to at most
static constexpr uint64_t kOpDensest = 12;                              // frames per chunk a caller may expect (max_frames)
static constexpr int kFailCopies = kWave, kFailStride = 16;             // the failure word's copies, 64 B apart

__device__ __forceinline__ void op_put(uint64_t* p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t op_get(const uint64_t* p) {
    return __hip_atomic_load(const_cast<uint64_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// The failure word in kFailCopies copies on lines of their own: a failing chunk sets the copy its
// index picks (a store: set once, never cleared within the call), a reader ORs all of them (one
// load per lane; call it with the whole wavefront).  (One word -- an atomic OR by every failing
// chunk, a load by every poller -- held one memory channel busy, r06i.)
__device__ __forceinline__ bool op_failed(const ScanArgs& a) {
    const uint32_t v = __hip_atomic_load(a.opfail + (threadIdx.x & (kWave - 1)) * kFailStride, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
    return __ballot(v != 0) != 0;
}
__device__ __forceinline__ void op_fail(const ScanArgs& a, uint64_t c) {
    __hip_atomic_store(a.opfail + (c % kFailCopies) * kFailStride, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// K2-K4: the one-pass launch resolved this call (every chunk checked, none failed -- it has
// finished by then)
__device__ __forceinline__ bool onepass_done(const ScanArgs& a) { return a.onepass && !op_failed(a); }

// K1: T(c), for the next launch (a plain store)
__device__ __forceinline__ void op_publish_t(const ScanArgs& a, uint64_t c, uint64_t tval, int lane) {
    if (lane == 0 && c >= a.start / kChunk) a.st_t[c] = a.epoch << kOpBits | tval;
}
// T(c) as K1 published it (kTFail when this call's K1 did not: never on a finished K1)
__device__ __forceinline__ uint64_t op_t(const ScanArgs& a, uint64_t c) {
    const uint64_t w = a.st_t[c];
    return (w >> kOpBits) == a.epoch ? (w & kOpMask) : kTFail;
}

// a look-back status word: [63:62] 1 aggregate / 2 inclusive | [61:38] epoch | [37:0] frames
static constexpr int kGValBits = 38;
__device__ __forceinline__ uint64_t op_gword(uint64_t flag, uint64_t epoch, uint64_t v) {
    return flag << 62 | (epoch & 0xFFFFFF) << kGValBits | (v & ((1ull << kGValBits) - 1));
}

// the frames before block g (wave 0, every lane; its aggregate published first).  Every block
// publishes, failed or not, so no wait outlives its predecessors' work; false past kOnePassWait.
__device__ bool op_prefix(const ScanArgs& a, uint64_t g, uint64_t agg, int lane, uint64_t* out) {
    if (lane == 0) op_put(a.st_g + g, op_gword(1, a.epoch, agg));
    uint64_t acc = 0, t0 = 0;
    for (int64_t top = (int64_t)g - 1, n = 0; top >= 0; ++n) {
        const int64_t idx = top - lane;
        uint64_t v = 0;
        bool ok = true, incl = idx < 0;   // before block 0: an inclusive 0
        if (idx >= 0) {
            const uint64_t w = op_get(a.st_g + idx);
            ok = (w >> 62) != 0 && ((w >> kGValBits) & 0xFFFFFF) == (a.epoch & 0xFFFFFF);
            incl = ok && (w >> 62) == 2;
            v = w & ((1ull << kGValBits) - 1);
        }
        const uint64_t im = __ballot(incl);
        const int stop = im ? __builtin_ctzll(im) : kWave;   // the nearest inclusive prefix
        const uint64_t need = stop >= kWave - 1 ? ~0ull : ((2ull << stop) - 1);
        if ((__ballot(ok) & need) != need) {   // a predecessor has not published yet
            const uint64_t t = __builtin_amdgcn_s_memrealtime();
            if (n == 0) t0 = t;
            else if (t - t0 > kOnePassWait) return false;
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
        acc += wave_sum(lane <= stop && idx >= 0 ? v : 0);
        if (stop < kWave) break;
        top -= kWave;
    }
    if (lane == 0) op_put(a.st_g + g, op_gword(2, a.epoch, acc + agg));
    *out = acc;
    return true;
}

// The one-pass launch: chunks [b kOpT, (b + 1) kOpT), thread t the chunk b kOpT + t.  A chunk after
// Multi ones walks on from the nearest predecessor whose T is known (Single or None) through them
// to its own start, so no thread waits for another's walk (a wave waiting on its own lanes' walks
// took one walk round per Multi chunk in it: 19.6 us for this launch at config 2, r06_onepass).
static constexpr int kOpBack = 8;   // Multi predecessors walked through at most (more: the graph path)
__global__ __launch_bounds__(kOpT) void scan_op_walk(ScanArgs a) {
    __shared__ uint32_t wsum[kOpT / kWave];
    __shared__ uint64_t base;
    __shared__ int lb_ok;
    const int tid = threadIdx.x, lane = tid & (kWave - 1), wv = tid / kWave;
    const uint64_t g = blockIdx.x, c = g * kOpT + tid, c0 = a.start / kChunk;
    const bool mine = c >= c0 && c <= a.nc;
    const uint64_t B = c * kChunk, Bend = B + kChunk;
    const uint64_t tval = mine ? op_t(a, c) : kTNone;
    bool bad = mine && tval == kTFail;
    // the entry: the chain's position at or past B (kXEnd: it ended before)
    uint64_t e = kXEnd;
    if (mine && !bad) {
        if (c == c0) {
            e = a.start;
        } else {
            uint64_t k = 1, tp = op_t(a, c - 1);
            while (tp == kTMulti && c - k > c0 && k < (uint64_t)kOpBack) tp = op_t(a, c - ++k);
            if (tp == kTFail || (tp == kTMulti && c - k > c0)) {
                bad = true;   // (a failed prediction, or a run of more than kOpBack Multi chunks)
            } else {
                // p: where the chain enters chunk c - k + 1 (c - k == c0 with a Multi T: the start)
                uint64_t p = tp == kTMulti ? a.start : (tp == kTNone ? kXEnd : tp);
                for (uint64_t hops = 0; p < B && !bad; ++hops) {   // through the Multi chunks to B
                    if (hops == (uint64_t)kOpRec * k) {   // (each of them may hold kOpRec frames)
                        bad = true;
                        break;
                    }
                    const uint64_t v = parse_at(a, p, window_global(a, p), nullptr, nullptr);
                    p = (v & kTerm) ? kXEnd : v;   // (the chunk where it ends reports it)
                }
                e = p;
            }
        }
    }
    uint64_t cnt = 0, endpos = 0, Wx = kXEnd;
    uint32_t ended = 0;   // 1: the chain ends in this chunk (END), 2: it dies here (an error at endpos)
    uint64_t reg[kOpReg];
#pragma unroll
    for (int r = 0; r < kOpReg; ++r) reg[r] = 0;
    if (!mine || bad) {
    } else if (e == kXEnd) {
        if (tval != kTNone && tval != kTMulti) bad = true;   // not visited, yet Single
    } else if (e >= Bend) {
        bad = true;   // a frame covers this chunk: not dense
    } else {
        uint64_t p = e;
        for (;;) {
            if (p >= Bend) {   // the exit: a Single T must be it (checked below)
                if (tval == kTNone || tval == kTMulti) {
                    if (quick_reject(a, p)) {   // no header can start there: the chain dies at p
                        if (a.spec) bad = true;   // (the speculative pass walks on serially in K4)
                        ended = 2;
                        endpos = p;
                    } else if (tval == kTNone) {
                        bad = true;   // an exit K1's exit set did not hold
                    } else {
                        Wx = p;
                    }
                } else {
                    Wx = p;
                }
                break;
            }
            uint32_t key = 0;
            uint8_t b0 = 0;
            const uint64_t v = parse_at(a, p, window_global(a, p), &key, &b0);
            if (v & kTerm) {
                if (term_type(v) == kDead && a.spec) bad = true;
                ended = term_type(v) == kDead ? 2 : 1;
                endpos = term_pos(v);
                break;
            }
            // a chunk of more than kOpRec frames -- or one projected to hold more than kOpWalk, from
            // the mean length of its first ones (walked a hop at a time, such a chunk costs more
            // than the graph path) -- takes the graph path
            if (cnt == (uint64_t)kOpRec || (cnt >= 4 && (p - e) * (a.op_walk - cnt) < (Bend - p) * cnt)) {
                bad = true;
                break;
            }
            const uint64_t fr = (p - B) | (uint64_t)b0 << 16 | (uint64_t)key << 32;
            // the first kOpReg frames stay in registers (constant indices: selects, no scratch)
#pragma unroll
            for (int r = 0; r < kOpReg; ++r) reg[r] = cnt == (uint64_t)r ? fr : reg[r];
            if (cnt >= (uint64_t)kOpReg) a.opfl[c * kOpRec + cnt] = fr;
            ++cnt;
            p = v;
        }
        if (tval != kTMulti && tval != kTNone && Wx != tval) bad = true;
    }
    // one store per wavefront that failed (a store per failing chunk -- most chunks of a stream of
    // large frames -- queued on the 64 copies' lines)
    if (const uint64_t bm = __ballot(bad)) {
        if (lane == __builtin_ctzll(bm)) op_fail(a, c);
    }
    // the frames before each chunk: the block's scan, then the blocks' look-back (every block
    // publishes, failed or not, so no look-back waits on a block that gave up)
    const uint32_t incl = wave_incl_sum((uint32_t)cnt);
    if (lane == kWave - 1) wsum[wv] = incl;
    __syncthreads();
    uint64_t before = incl - (uint32_t)cnt;
    for (int k = 0; k < wv; ++k) before += wsum[k];
    if (wv == 0) {
        uint64_t agg = 0;
#pragma unroll
        for (int k = 0; k < kOpT / kWave; ++k) agg += wsum[k];
        uint64_t pre = 0;
        const bool ok = op_prefix(a, g, agg, lane, &pre);
        if (lane == 0) {
            base = pre;
            lb_ok = ok;
        }
    }
    __syncthreads();
    if (!lb_ok) {   // (block-uniform) a look-back that ran out: the graph path
        if (tid == 0) op_fail(a, c);
        return;
    }
    if (!mine) return;
    const uint64_t k0 = base + before;
#pragma unroll
    for (int r = 0; r < kOpReg; ++r)
        if ((uint64_t)r < cnt) put_frame(a, k0 + r, B + (reg[r] & 0xFFFFu), (uint32_t)(reg[r] >> 32), (uint8_t)(reg[r] >> 16));
    for (uint64_t i = kOpReg; i < cnt; ++i) {
        const uint64_t f = a.opfl[c * kOpRec + i];
        put_frame(a, k0 + i, B + (f & 0xFFFFu), (uint32_t)(f >> 32), (uint8_t)(f >> 16));
    }
    if (ended) {   // the chain ends in this chunk: the results
        const uint64_t total = k0 + cnt;
        a.result[0] = total;
        a.result[1] = endpos;
        a.result[2] = ended == 2 ? endpos : ~0ull;
        if (total <= a.max_frames) a.hdr[total] = endpos;
    }
}

// K4, both paths: the previous call's failure copies zeroed for the next call
__device__ __forceinline__ void op_clear_prev(const ScanArgs& a) {
    if (blockIdx.x == 0 && threadIdx.x < kFailCopies) a.opfail_prev[threadIdx.x * kFailStride] = 0;
}

typedef uint32_t u32x4u __attribute__((ext_vector_type(4), aligned(1)));

// Inclusive sum over the wavefront's lanes, in DPP moves (no LDS trip): row_shr 1/2/4/8
// within each row of 16, then row_bcast 15 / 31 carry the row totals up.
__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false);   // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false);   // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false);   // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false);   // row_shr:8
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);   // row_bcast:15 -> rows 1, 3
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);   // row_bcast:31 -> rows 2, 3
    return v;
}

// Bit 7 of each byte: the byte is x7E/x7F, or with hi = kH xFE/xFF -- a second header byte
// with a 16/64-bit length (and MASK set, for hi = the byte itself).  3 VALU operations.
__device__ __forceinline__ uint32_t long_len4(uint32_t r, uint32_t hi) {
    return ((r & 0x7E7E7E7Eu) + 0x02020202u) & hi & kH;
}

// The 4 stream bytes at p for the chunk at the end (clamped load; bytes at or past len
// undefined)
__device__ __forceinline__ uint32_t dword_clamped(const ScanArgs& a, uint64_t p) {
    typedef uint32_t u32u __attribute__((aligned(1)));
    const uint64_t lim = a.pf_lim + 12;   // len - 4 (a stream under 16 bytes: the scratch word)
    const uint64_t pc = p < lim ? p : lim;
    const uint32_t raw = *(const NETC_GLOBAL u32u*)(a.pf_base + pc);
    const uint64_t sh = p - pc;
    return sh >= 4 ? 0u : raw >> (8 * sh);
}

// K1: one wavefront per chunk (the mask kernel's lesson: one-shot waves over a covering
// grid stream HBM best).  Lane l holds bytes 1024 i + 16 l .. + 15 of the chunk (i = 0..3:
// four coalesced 16-B loads, addresses clamped into the buffer; the chunk at the end
// re-reads what the clamp moved), also written to the wave's LDS copy of the chunk.
// The quick check runs on the registers (the byte after a lane's 16 is the next lane's
// first; lane 63: the next vector's lane 0, or the next chunk).  The exit-capable
// candidates of the whole chunk are queued once and parsed round-robin by the lanes
// from the LDS copy -- one pass, a few lanes busy -- and their distinct exits become
// candidate entries of the chunks they land in.  (Parsing them vector by vector, a
// window cut from registers each time, cost 13 us of K1's 27 at config 2.)
// NT: non-temporal loads of the chunk.  Up to 128 MiB of stream K1 reads with plain loads, so
// the header bytes K2 and K4 read again soon after are still cached: config 2 41.2-41.4 against
// 42.3-42.6 us; above, the non-temporal stream is faster (config 4 80.8-82.9 against 82.7-84.3
// us with plain loads; r03t, profiles/r03t_scan_k1_loads.json).
template <bool NT>
__device__ __forceinline__ u32x4 k1_load(const uint8_t* p) {
    if constexpr (NT) return __builtin_nontemporal_load((const NETC_GLOBAL u32x4u*)p);
    return *(const NETC_GLOBAL u32x4u*)p;
}

// ONE: the one-pass path's prediction T(c) after the parse (op_publish_t).
template <bool NT, bool ONE>
__global__ __launch_bounds__(256) void scan_exits(ScanArgs a) {
    if (threadIdx.x == 0 && blockIdx.x == 0) OP_TRACE(0, 1);
    if (threadIdx.x == 0) OP_STAMP_MIN(0, __builtin_amdgcn_s_memrealtime());
    __shared__ uint32_t stage[4][kStageWords];   // per wave: its chunk's bytes (+ 16 after)
    __shared__ unsigned long long set[4][kSet];
    __shared__ uint16_t queue[4][kQCap];
#ifdef NETC_SCAN_K1_EXP
    __shared__ uint32_t qn[4];
    if ((threadIdx.x & 63) == 0) qn[threadIdx.x / 64] = 0;
#endif
    SCAN_SCOPE(0);
    // wv through readfirstlane: the chunk index, its bounds and the edge test below are
    // then scalar (SGPR arithmetic, scalar branches) instead of per-lane VALU
    const int tid = threadIdx.x, lane = tid & (kWave - 1), wv = __builtin_amdgcn_readfirstlane(tid / kWave);
    const uint64_t c = (uint64_t)blockIdx.x * 4 + wv;
    if (c > a.nc) return;
    const uint64_t B = c * kChunk, Bend = B + kChunk;
    if (lane == 0 && a.start / kChunk == c) append_cand(a, a.start, true);   // the root node
    if (B >= a.len) {   // the virtual chunk: no bytes
        if constexpr (ONE) op_publish_t(a, c, kTNone, lane);
        return;
    }
    uint32_t d[4][4], nx[4];
    if (Bend <= a.pf_lim) {   // wave-uniform: every load in place, no clamps (scalar base + lane offset)
        const uint8_t* base = a.pf_base + B;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const u32x4 v = k1_load<NT>(base + 1024 * i + 16 * lane);
#pragma unroll
            for (int k = 0; k < 4; ++k) d[i][k] = v[k];
        }
        const u32x4 v = *(const NETC_GLOBAL u32x4u*)(base + kChunk);
#pragma unroll
        for (int k = 0; k < 4; ++k) nx[k] = v[k];
    } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            uint64_t p = B + 1024 * i + 16 * (uint64_t)lane;
            p = p < a.pf_lim ? p : a.pf_lim;
            const u32x4 v = k1_load<NT>(a.pf_base + p);
#pragma unroll
            for (int k = 0; k < 4; ++k) d[i][k] = v[k];
        }
        const uint64_t q = Bend < a.pf_lim ? Bend : a.pf_lim;
        const u32x4 v = *(const NETC_GLOBAL u32x4u*)(a.pf_base + q);
#pragma unroll
        for (int k = 0; k < 4; ++k) nx[k] = v[k];
    }
    const bool fast = B >= a.start && Bend + 16 <= a.len;
    if (Bend + 16 > a.len) {
        // a vector the clamped 16-B load did not read in place is re-read by dwords,
        // clamped and shifted so a dword straddling len keeps its bytes below len.
        // Bytes at or past len may hold anything: no position there is a candidate, and
        // every parse checks its header and payload against len.
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint64_t p = B + 1024 * i + 16 * (uint64_t)lane;
            if (p > a.pf_lim)
#pragma unroll
                for (int k = 0; k < 4; ++k) d[i][k] = dword_clamped(a, p + 4 * k);
        }
        if (Bend > a.pf_lim)
#pragma unroll
            for (int k = 0; k < 4; ++k) nx[k] = dword_clamped(a, Bend + 4 * k);
    }
    uint32_t* st = stage[wv];
#pragma unroll
    for (int i = 0; i < 4; ++i)
        *(u32x4*)&st[(1024 * i + 16 * lane) / 4] = u32x4{d[i][0], d[i][1], d[i][2], d[i][3]};
    if (lane < 4) st[kChunk / 4 + lane] = nx[lane];
    SCAN_STAMP(0, 1);   // the chunk's bytes have arrived
    set[wv][lane] = ~0ull;   // the wave's exit set
    // the dword after each lane's 16 bytes (readfirstlane outside the lane-63 branch:
    // inside it lane 63 is the first active lane)
    const uint32_t f1 = (uint32_t)__builtin_amdgcn_readfirstlane((int)d[1][0]);
    const uint32_t f2 = (uint32_t)__builtin_amdgcn_readfirstlane((int)d[2][0]);
    const uint32_t f3 = (uint32_t)__builtin_amdgcn_readfirstlane((int)d[3][0]);
    uint32_t nb[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) nb[i] = (uint32_t)__shfl_down((int)d[i][0], 1, kWave);
    if (lane == kWave - 1) {
        nb[0] = f1;
        nb[1] = f2;
        nb[2] = f3;
        nb[3] = nx[0];
    }
    // exit-capable candidates: bit 32 h + 8 j + 4 (i & 1) + k <-> vector i = 2 h + (i & 1),
    // dword k, byte j.  The strict filter (always on: see ScanArgs::spec) is one branch
    // for the whole pass, not one per dword.
    uint32_t half[2] = {0, 0};
    const uint32_t specH = a.spec ? kH : 0u;
    const uint32_t specX = rsv_keep4(a);   // RSV1 cleared from the first bytes in the speculative pass
    // the quick check of every position (the first header byte's checks too), vectors 0-3
    auto full_pass = [&](auto strict_c) {
        constexpr bool kStrict = decltype(strict_c)::value;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            uint32_t ci = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t x = d[i][k];
                const uint32_t y = __builtin_amdgcn_alignbyte(k < 3 ? d[i][k + 1] : nb[i], x, 1);
                const uint32_t ok = kStrict ? quick_ok4(x & specX, y | specH) : kH;
                // a 7-bit length cannot leave the chunk unless the position is near its end
                // (a per-byte threshold test for those lanes cost more VALU than it saved)
                const uint32_t sel = ((i == 3 && lane >= kNearLane) ? kH : ((y & 0x7E7E7E7Eu) + 0x02020202u));
                ci |= (ok & sel & kH) >> (7 - k);
            }
            half[i >> 1] |= ci << (4 * (i & 1));
        }
    };
    // Vectors 0-2 lie wholly more than 131 bytes before the chunk's end, so only a 16/64-bit
    // length can exit from them: the second header byte is x7E/x7F (strict: xFE/xFF, MASK set).
    // The cheap pass selects them by that test alone (3 VALU per dword, on the raw dwords) and
    // leaves the first byte's checks to the parse (parse_at's `dead` holds every one of them):
    // a few more queued positions (about 2 in 256 payload bytes) for the quick check's 7 VALU
    // per dword.  The bit found at byte q is position q - 1's: byte j of dword k moves to byte
    // j - 1 (bit 8 j + k -> 8 (j - 1) + k), byte 0 to byte 3 of dword k - 1 (bit k -> 24 + k -
    // 1), and the lane's byte 0 to the previous lane's position 15 (bit 27).  Vector 3 (lanes
    // near the end exit with a 7-bit length) takes the full check.
    auto cheap_pass = [&](auto strict_c) {
        constexpr bool kStrict = decltype(strict_c)::value;
        const uint32_t hiR = kStrict ? specH : 0xFFFFFFFFu;   // OR'd into the byte itself: MASK test off
        uint32_t raw[3];
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            uint32_t ri = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t r = d[i][k];
                ri |= long_len4(r, r | hiR) >> (7 - k);
            }
            raw[i] = ri;
        }
        // bit 0 of each (byte 0 of the lane's 16) belongs to the previous lane; vector 3's byte 0
        // is vector 2's last position (lane 63)
        const uint32_t r3 = long_len4(d[3][0], d[3][0] | hiR) >> 7;
        const uint32_t b0s = (raw[0] & 1u) | (raw[1] & 1u) << 1 | (raw[2] & 1u) << 2 | (r3 & 1u) << 3;
        const uint32_t first = (uint32_t)__builtin_amdgcn_readfirstlane((int)b0s);
        uint32_t from_next = (uint32_t)__shfl_down((int)b0s, 1, kWave);
        from_next = lane == kWave - 1 ? first >> 1 : from_next;
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            const uint32_t ri = raw[i];
            const uint32_t ci = (ri >> 8) | ((ri & 0x0Eu) << 23) | (((from_next >> i) & 1u) << 27);
            half[i >> 1] |= ci << (4 * (i & 1));
        }
        uint32_t ci = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t x = d[3][k];
            const uint32_t y = __builtin_amdgcn_alignbyte(k < 3 ? d[3][k + 1] : nb[3], x, 1);
            const uint32_t ok = kStrict ? quick_ok4(x & specX, y | specH) : kH;
            const uint32_t sel = lane >= kNearLane ? kH : ((y & 0x7E7E7E7Eu) + 0x02020202u);
            ci |= (ok & sel & kH) >> (7 - k);
        }
        half[1] |= ci << 4;
    };
    // wave-uniform: an edge chunk; positions before the start or at / past the end are not candidates
    auto edge_mask = [&]() {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint64_t q0 = B + 1024 * i + 16 * (uint64_t)lane;
            const uint64_t lo = a.start <= q0 ? 0 : (a.start - q0 < 16 ? a.start - q0 : 16);
            const uint64_t hi = a.len <= q0 ? 0 : (a.len - q0 < 16 ? a.len - q0 : 16);
            const uint32_t valid = ((1u << hi) - 1u) & ~((1u << lo) - 1u);   // byte b <-> bit b
            uint32_t vm = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {   // byte j of dword k <-> bit 8 j + k
                const uint32_t m4 = (valid >> (4 * k)) & 0xFu;
                vm |= (((m4 * 0x00204081u) & 0x01010101u)) << k;
            }
            half[i >> 1] &= ~(0x0F0F0F0Fu << (4 * (i & 1))) | (vm << (4 * (i & 1)));
        }
    };
    // (non-strict: the two passes select the same positions)
    if (a.strict) cheap_pass(std::integral_constant<bool, true>{});
    else cheap_pass(std::integral_constant<bool, false>{});
    if (!fast) edge_mask();
    uint64_t rel = (uint64_t)half[1] << 32 | half[0];
    // queue them (chunk offsets), then parse round-robin
    uint32_t mine = (uint32_t)__popcll(rel);
    uint32_t incl = wave_incl_sum(mine);
    uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)incl, kWave - 1);
    if (a.strict && total > (uint32_t)kCheapMax) {
        // wave-uniform: payload bytes that repeat xFE/xFF (a run of one byte under a 4-byte key)
        // -- the full check keeps those chunks off the queue cap, as before the cheap pass
        half[0] = half[1] = 0;
        full_pass(std::integral_constant<bool, true>{});
        if (!fast) edge_mask();
        rel = (uint64_t)half[1] << 32 | half[0];
        mine = (uint32_t)__popcll(rel);
        incl = wave_incl_sum(mine);
        total = (uint32_t)__builtin_amdgcn_readlane((int)incl, kWave - 1);
    }
    if (total > (uint32_t)kQCap) {   // wave-uniform (adversarial payloads, non-strict mode)
        if (lane == 0) atomicOr(a.ovf, kOvfQueue);
        if constexpr (ONE) op_publish_t(a, c, kTFail, lane);
        return;
    }
    uint32_t at = incl - mine;
    for (; rel; rel &= rel - 1) {
        const int b = __builtin_ctzll(rel);
        const int q = b & 31, r = q & 7;
        const int i = 2 * (b >> 5) + (r >> 2), k = r & 3, j = q >> 3;
        queue[wv][at++] = (uint16_t)(1024 * i + 16 * lane + 4 * k + j);
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    SCAN_STAMP(0, 2);   // quick check done, candidates queued
    bool ovf = false;
    uint32_t nodes = 0;   // (one pass) exits this lane appended as nodes, and the last of them
    uint64_t ex = 0;
    for (uint32_t e = lane; e < total; e += kWave) {
        const uint32_t off = queue[wv][e];
        const uint64_t v = parse_at(a, B + off, window_at(st, (int)off), nullptr, nullptr);
        // strict mode prunes exits that cannot start a frame: payload bytes parsed as a
        // chain land on random positions, which pass with ~2 % odds, while the true chain
        // always lands on a real header
#ifdef NETC_SCAN_K1_EXP
        // diagnostic build only (tools/, timing of K1's tail): the exit written to a
        // per-source-chunk list with a plain store -- no target check, no atomic
        if (!(v & kTerm) && v >= Bend && set_insert(set[wv], v, &ovf)) {
            const uint32_t k = atomicAdd(&qn[wv], 1u);
            if (k < (uint32_t)kCand) a.cand[c * kCand + k] = v;
        }
#else
        if (!(v & kTerm) && v >= Bend && set_insert(set[wv], v, &ovf) && !quick_reject(a, v)) {
            append_cand(a, v, v / kChunk / kTileChunks != c / kTileChunks);
            ++nodes;
            ex = v;
        }
#endif
    }
    SCAN_STAMP(0, 3);   // parsed, exits checked and appended
    if (ovf) atomicOr(a.ovf, kOvfSet);
    if constexpr (ONE) {
        // T(c) from the distinct exits onto header-capable positions (a full set: unknown)
        const uint64_t bn = __ballot(nodes != 0);
        const uint32_t n = (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_sum(nodes), kWave - 1);
        const uint64_t t = __ballot(ovf) ? kTFail : (n == 0 ? kTNone : (n > 1 ? kTMulti : readlane64(ex, __builtin_ctzll(bn))));
        op_publish_t(a, c, t, lane);
        if (lane == 0) {
            OP_STAMP_ADD(t == kTNone ? 5 : t == kTMulti ? 7 : t == kTFail ? 8 : 6, 1);
            OP_STAMP_MAX(1, __builtin_amdgcn_s_memrealtime());
        }
    }
}

// K2 -> K3a words: plain, or (SC1: scan_links_fused, K3a in the same launch, maybe on another XCD)
// relaxed agent-scope stores and loads, which go through to the memory-side caches
template <bool SC1, typename T>
__device__ __forceinline__ void hand_st(T* p, T v) {
    if constexpr (SC1) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else *p = v;
}
template <bool SC1, typename T>
__device__ __forceinline__ T hand_ld(const T* p) {
    if constexpr (SC1) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else return *p;
}

// node -> the candidate its chain exits to (the first slot holding that position, or
// -1) and the terminal where it ends
template <bool SC1>
__device__ __forceinline__ void link_node(const ScanArgs& a, uint64_t node, uint64_t x, uint64_t v, uint32_t cnt) {
    int32_t next = -1;
    if (term_type(v) == kExit) {
        const uint64_t y = term_pos(v), t = y / kChunk;
        // the counter and the bucket's 8 positions (one line) in one trip
        const uint32_t n = min(a.ccount[t], (uint32_t)kCand);
        uint64_t ts[kCand];
#pragma unroll
        for (int j = 0; j < kCand; ++j) ts[j] = a.cand[t * kCand + j];
#pragma unroll
        for (int j = kCand - 1; j >= 0; --j)
            if ((uint32_t)j < n && ts[j] == y) next = (int32_t)(t * kCand + j);   // the first match
        // not a candidate: pruned by K1 (the chain dies at y), or its bucket overflowed
        if (next < 0 && !quick_reject(a, y)) atomicOr(a.ovf, kOvfLink);
    }
    hand_st<SC1>(&a.link[node], next);
    hand_st<SC1>(&a.nterm[node], v);
    hand_st<SC1>(&a.ncnt[node], cnt);
}

// Every position of the chunk that can start a header (strict: passes the quick
// check; else every position) parsed once into a 16-bit in-chunk link (kNoLink: the
// chain ends or leaves the chunk there), then four doubling passes: returns the
// 16-hop links (l1 keeps the 1-hop ones, lj the 8-hop ones).  The caller has loaded
// words.
static constexpr uint16_t kNoLink = 0xFFFF;
static constexpr int kStride = 16;   // hops per 16-hop link
static constexpr int kAncStride = 8;                              // frames per K2' anchor
static constexpr int kAncMax = (int)(kChunk / 2 / kAncStride) + 1;   // a frame is 2 bytes or more
static constexpr int kAncSlot = kAncMax + 1;                         // uint16 per slot (4-byte multiple)

__device__ __forceinline__ const uint16_t* chunk_links16(const ScanArgs& a, uint64_t B, const uint32_t* words, uint16_t* l1,
                                         uint16_t* lj, uint16_t* lk16) {
    const int tid = threadIdx.x;
    const uint64_t Bend = B + kChunk;
    const int i0 = kPer * tid;
    uint32_t w[kPer / 4 + 1];
#pragma unroll
    for (int k = 0; k < kPer / 4 + 1; ++k) w[k] = words[i0 / 4 + k];
    uint32_t cand = 0;   // this thread's positions that can start a header
#pragma unroll
    for (int k = 0; k < kPer / 4; ++k) {
        const uint32_t ok =
            a.strict ? quick_ok4(w[k] & rsv_keep4(a), __builtin_amdgcn_alignbyte(w[k + 1], w[k], 1) | (a.spec ? kH : 0u))
                     : kH;
#pragma unroll
        for (int j = 0; j < 4; ++j) cand |= ((ok >> (8 * j + 7)) & 1u) << (4 * k + j);
    }
    // no link anywhere first (bank-conflict-free order), then the candidates parsed:
    // the wave takes as many trips as its busiest lane has candidates (a few in
    // strict mode), not one full parse per position
#pragma unroll
    for (int k = 0; k < kPer; ++k) l1[k * kScanT + tid] = kNoLink;
    __syncthreads();
    while (cand) {
        const int j = __builtin_ctz(cand);
        cand &= cand - 1;
        const uint64_t v = parse_at(a, B + i0 + j, window_at(words, i0 + j), nullptr, nullptr);
        if (!(v & kTerm) && v < Bend) l1[i0 + j] = (uint16_t)(v - B);
    }
    __syncthreads();
    const uint16_t* src = l1;
    uint16_t* dst = lj;
#pragma unroll
    for (int pass = 0; pass < 4; ++pass) {   // 2, 4, 8, 16 hops
#pragma unroll
        for (int k = 0; k < kPer; ++k) {
            const int i = k * kScanT + tid;
            const uint16_t x = src[i];
            dst[i] = x == kNoLink ? kNoLink : src[x];
        }
        __syncthreads();
        src = dst;
        dst = dst == lj ? lk16 : lj;
    }
    return src;
}

// K2: nodes of BC chunks per block (kBlkChunks, or kBlkChunksBig: two slots per thread), one thread per slot: a repeated position
// defers to its first slot (passing on its external flag); a node's chain is walked
// from global memory to the candidate it exits to.  Chains of more than kWalkHops
// frames in the chunk are finished by the whole block afterwards: the chunk's 16-hop
// links built in LDS, one thread walks them from the entry -- count / 8 + at most 7
// hops, leaving an anchor every 8 frames -- and re-parses the last header for the exact
// terminal.
// K2's per-wavefront path for dense chunks (round 4): a node whose walk shows more than
// kWalkHops frames in its chunk -- small frames, e.g. 16-B payloads put ~190 frames in a
// chunk -- is finished by ONE wavefront from its own LDS instead of the whole block, so the
// block's four wavefronts take four such chunks at once (the block path ran a block's 32
// queued chunks one after another: 371 us of K2 at 64 MiB of 16-B frames, r04k).  Only
// positions that pass the strict quick check can be on a chain, so the wavefront keeps them
// compact: their sorted chunk offsets (at most kDenseCand; more, or a non-strict scan, leaves
// the node to the block path), each one's 1-hop successor as an index into that list (a
// bitmap of the list and a popcount), three doubling passes to 8-hop successors, then one lane walks the entry's chain
// -- count / 8 + at most 7 hops, an anchor every 8 frames as the block path leaves them.
static constexpr int kDenseCand = 392;   // 4 x 7.7 KB per block: K2 keeps 5 blocks per CU
static constexpr int kProbeHops = 8;     // K2: frames walked from global memory before judging density
struct DenseLds {
    uint32_t words[kWords];
    uint64_t bm[kWave];         // candidate bitmap: bit u of word L <-> chunk offset 64 L + u
    uint16_t pre[kWave];        // candidates before word L (the index of its first)
    uint16_t pos[kDenseCand];   // candidate positions (chunk offsets), ascending
    uint16_t s1[kDenseCand];    // 1-hop successor (index into pos), kNoLink: none in the list
    uint16_t sa[kDenseCand];    // doubling halves; sa ends with the 8-hop successors
    uint16_t sb[kDenseCand];
};

// BC chunks per block: kBlkChunks, or kBlkChunksBig for big streams (two node slots per thread)
template <int BC>
struct LinksLdsT {
    union {
        struct {
            uint32_t words[kWords];
            uint16_t l1[kChunk];
            uint16_t lj[kChunk];
            uint16_t lk16[kChunk];
        } b;
        DenseLds w[kScanT / kWave];
    };
    uint16_t queue[BC * kCand];   // queued nodes (slot in the block); kQTaken once the wavefront path took one
    int nq;
    uint32_t item;                // (one pass) the block of K2's work this block claimed
};
using LinksLds = LinksLdsT<kBlkChunks>;
static constexpr uint16_t kQTaken = 0xFFFF;

// the wavefront's LDS ops so far are visible to its other lanes
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// the chunk at B (+ 32 bytes, zero past len) into one wavefront's LDS words; the caller syncs
__device__ __forceinline__ void wave_load_chunk(const ScanArgs& a, uint64_t B, uint32_t* words, int lane) {
    typedef uint32_t u32x4u __attribute__((ext_vector_type(4), aligned(1)));
    if (B + kChunk + 32 <= a.len) {
        for (int v = lane; v < kWords / 4; v += kWave) {   // 16-B loads (any alignment of the stream)
            const u32x4 x = *(const NETC_GLOBAL u32x4u*)(a.wire + B + 16 * (uint64_t)v);
            words[4 * v] = x[0];
            words[4 * v + 1] = x[1];
            words[4 * v + 2] = x[2];
            words[4 * v + 3] = x[3];
        }
    } else {
        uint8_t* bytes = (uint8_t*)words;
        for (int i = lane; i < kWords * 4; i += kWave) bytes[i] = B + i < a.len ? gptr(a.wire)[B + i] : 0;
    }
}

// index of chunk offset t (< kChunk) in d.pos, or kNoLink: two LDS reads and a popcount
__device__ __forceinline__ uint16_t dense_find(const DenseLds& d, uint32_t t) {
    const uint64_t w = d.bm[t >> 6], below = w & ((1ull << (t & 63)) - 1);
    return (w >> (t & 63)) & 1 ? (uint16_t)(d.pre[t >> 6] + __popcll(below)) : kNoLink;
}

// One queued node by the calling wavefront (see DenseLds); false (wave-uniform, nothing
// written) leaves it to the block path.  qi: its queue index (anchor slot as the block path).
// a chunk's kWords words as the wavefront's registers: lane l holds 16-B vectors l + 64 i (the
// next chunk's loads stay in flight while the current one is processed); false on an edge chunk
// (the bytes past len must read as zero: wave_load_chunk's byte path then)
struct ChunkRegs {
    u32x4 v[(kWords / 4 + kWave - 1) / kWave];
};
__device__ __forceinline__ bool chunk_regs_load(const ScanArgs& a, uint64_t B, int lane, ChunkRegs& R) {
    typedef uint32_t u32x4u __attribute__((ext_vector_type(4), aligned(1)));
    if (B + kChunk + 32 > a.len) return false;   // wave-uniform
#pragma unroll
    for (int i = 0; i < (int)(sizeof(R.v) / sizeof(R.v[0])); ++i) {
        const int v = lane + kWave * i;
        const int vc = v < kWords / 4 ? v : kWords / 4 - 1;   // (the clamped loads are not stored)
        R.v[i] = *(const NETC_GLOBAL u32x4u*)(a.wire + B + 16 * (uint64_t)vc);
    }
    return true;
}
__device__ __forceinline__ void chunk_regs_store(uint32_t* words, const ChunkRegs& R, int lane) {
#pragma unroll
    for (int i = 0; i < (int)(sizeof(R.v) / sizeof(R.v[0])); ++i) {
        const int v = lane + kWave * i;
        if (v < kWords / 4) {
            words[4 * v] = R.v[i][0];
            words[4 * v + 1] = R.v[i][1];
            words[4 * v + 2] = R.v[i][2];
            words[4 * v + 3] = R.v[i][3];
        }
    }
}

// One queued node by the calling wavefront, its chunk's words already in d.words (see DenseLds);
// false (wave-uniform, nothing written) leaves it to the block path.  qi: its queue index
// (anchor slot as the block path).  x: the node's position (a.cand[node]).
template <bool SC1, int BC>
__device__ __forceinline__ bool dense_node(const ScanArgs& a, DenseLds& d, uint64_t node, uint64_t x, uint32_t qi, uint32_t bid DENSE_ARG) {
    const int lane = threadIdx.x & (kWave - 1);
    const uint64_t chunk = node / kCand, B = chunk * kChunk, Bend = B + kChunk;
    DENSE_T(1);
    // the lane's 64 positions [64 lane, 64 lane + 64) through the quick check
    uint64_t bits = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const uint32_t w0 = d.words[16 * lane + k], w1 = d.words[16 * lane + k + 1];
        const uint32_t ok = quick_ok4(w0 & rsv_keep4(a), __builtin_amdgcn_alignbyte(w1, w0, 1) | (a.spec ? kH : 0u));
#pragma unroll
        for (int j = 0; j < 4; ++j) bits |= (uint64_t)((ok >> (8 * j + 7)) & 1u) << (4 * k + j);
    }
    const uint32_t mine = (uint32_t)__popcll(bits);
    const uint32_t incl = wave_incl_sum(mine);
    const uint32_t m = (uint32_t)__builtin_amdgcn_readlane((int)incl, kWave - 1);
    if (m > (uint32_t)kDenseCand || m == 0) return false;   // wave-uniform
    uint32_t at = incl - mine;
    d.bm[lane] = bits;
    d.pre[lane] = (uint16_t)at;
    for (; bits; bits &= bits - 1) d.pos[at++] = (uint16_t)(64 * lane + __builtin_ctzll(bits));
    wave_lds_sync();
    DENSE_T(2);
    const uint16_t e = x - B < kChunk ? dense_find(d, (uint32_t)(x - B)) : kNoLink;   // the entry's index
    // 1-hop successors, as indexes into pos
    for (uint32_t i = lane; i < m; i += kWave) {
        const uint32_t p = d.pos[i];
        const uint64_t v = parse_at(a, B + p, window_at(d.words, (int)p), nullptr, nullptr);
        d.s1[i] = (!(v & kTerm) && v < Bend) ? dense_find(d, (uint32_t)(v - B)) : kNoLink;
    }
    wave_lds_sync();
    DENSE_T(3);
    // 2, 4, 8 hops (s8 in sa), then 16, 32, 64 (s64 in sb; s1 is reused for 32: the walk's last
    // hops re-parse from the words instead)
    uint16_t* const bufs[3] = {d.s1, d.sa, d.sb};
    constexpr int kFrom[6] = {0, 1, 2, 1, 2, 0}, kTo[6] = {1, 2, 1, 2, 0, 2};
#pragma unroll
    for (int pass = 0; pass < 6; ++pass) {
        const uint16_t* src = bufs[kFrom[pass]];
        uint16_t* dst = bufs[kTo[pass]];
        for (uint32_t i = lane; i < m; i += kWave) {
            const uint16_t y = src[i];
            dst[i] = y == kNoLink ? kNoLink : src[y];
        }
        wave_lds_sync();
    }
    const uint16_t* s8 = d.sa;
    const uint16_t* s64 = d.sb;
    DENSE_T(4);
    if (__builtin_amdgcn_readfirstlane((int)e) == (int)kNoLink) return false;   // wave-uniform (not listed)
    // anchor j (every 8 frames from the entry) by lane j mod 64: s64^(j/8), then s8^(j%8)
    const uint64_t q = (uint64_t)bid * BC + qi;
    const bool keep = qi < (uint32_t)BC && q < a.anc_cap;
    uint16_t* anc = a.anc + (keep ? q : 0) * kAncSlot;
    uint32_t na = 0;   // anchors (wave-uniform)
    for (int it = 0;; ++it) {
        const int j = lane + kWave * it;
        uint32_t p = e;
        for (int h = 0; h < j / 8 && p != kNoLink; ++h) p = s64[p];
        for (int h = 0; h < j % 8 && p != kNoLink; ++h) p = s8[p];
        const bool valid = p != kNoLink;
        if (valid && keep && j < kAncMax) anc[j] = d.pos[p];
        const uint64_t vm = __ballot(valid);
        na += (uint32_t)__popcll(vm);
        if (vm != ~0ull) break;   // (valid lanes are a prefix: anchor j exists when j + 1 does)
    }
    // the last anchor's position (lane (na - 1) % 64 of the last round holds it): recomputed by lane 0
    int ok = 0;
    if (lane == 0) {
        ok = 1;
        uint32_t p = e;
        for (uint32_t h = 0; h < (na - 1) / 8; ++h) p = s64[p];
        for (uint32_t h = 0; h < (na - 1) % 8; ++h) p = s8[p];
        uint32_t hops = (na - 1) * kAncStride;
        if (keep) a.anc_n[q] = na < (uint32_t)kAncMax ? na : (uint32_t)kAncMax;
        a.anq[node] = keep ? (uint32_t)q : ~0u;
        // at most 7 listed frames on from it (the 8th would be another anchor), by parsing
        uint64_t pp = B + d.pos[p], v;
        for (;;) {
            v = parse_at(a, pp, window_at(d.words, (int)(pp - B)), nullptr, nullptr);
            if (v & kTerm) break;
            ++hops;   // the frame at pp
            if (v >= Bend) {   // its successor is past the chunk
                v = term(kExit, v);
                break;
            }
            if (dense_find(d, (uint32_t)(v - B)) == kNoLink) {   // a position off the list: the chain dies there
                v = parse_at(a, v, window_at(d.words, (int)(v - B)), nullptr, nullptr);
                break;
            }
            pp = v;
        }
        DENSE_T(5);
        link_node<SC1>(a, node, x, v, hops);
        DENSE_T(6);
        DENSE_ADD(4, 4, 5);
        DENSE_ADD(5, 5, 6);
    }
    DENSE_ADD(1, 1, 2);
    DENSE_ADD(2, 2, 3);
    DENSE_ADD(3, 3, 4);
    DENSE_COUNT();
    return __builtin_amdgcn_readfirstlane(ok) != 0;
}

template <bool SC1, int BC>
__device__ __forceinline__ void links_body(const ScanArgs& a, LinksLdsT<BC>& sl, uint32_t bid) {
    uint32_t* words = sl.b.words;
    uint16_t* l1 = sl.b.l1;
    uint16_t* lj = sl.b.lj;
    uint16_t* lk16 = sl.b.lk16;
    uint16_t* queue = sl.queue;
    const uint64_t blk0 = (uint64_t)bid * (BC * kCand);   // the block's first node slot
    int& nq = sl.nq;
    const int tid = threadIdx.x;
    if (tid == 0) nq = 0;
    __syncthreads();
    for (int t = tid; t < BC * kCand; t += kScanT) {   // (two slots per thread when BC = 64)
        const uint64_t s = blk0 + (uint64_t)t, c = s / kCand;
        const uint32_t i = (uint32_t)(s % kCand);
        // the counter, the bucket (one line) and the external flags in one trip
        const uint32_t cc = c <= a.nc ? a.ccount[c] : 0;
        uint64_t cs[kCand];
#pragma unroll
        for (int j = 0; j < kCand; ++j) cs[j] = c <= a.nc ? a.cand[c * kCand + j] : 0;
        const uint64_t x = c <= a.nc ? a.cand[s] : 0;
        if (c <= a.nc && i < min(cc, (uint32_t)kCand)) {
            int dup = -1;
#pragma unroll
            for (int j = kCand - 1; j >= 0; --j)
                if ((uint32_t)j < i && cs[j] == x) dup = j;   // the first earlier slot with x
            if (dup >= 0) {
                hand_st<SC1>(&a.link[s], kDupLink);
                hand_st<SC1>(&a.ncnt[s], 0u);
                if (a.ext[s]) {   // (K1's flag, the previous launch) passed on to the first slot
                    const uint64_t b = c * kCand + (uint64_t)dup;
                    if constexpr (SC1)   // an atomic on the flag's 32-bit word
                        __hip_atomic_fetch_or((uint32_t*)(a.ext + (b & ~3ull)), 1u << (8 * (b & 3)), __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
                    else
                        a.ext[b] = 1;
                }
            } else {
                const uint64_t B = c * kChunk;
                uint32_t cnt = 0;
                // the walk's first kList frames, for K4 (read only if this node is the
                // chunk's true entry and its walk has at most kList frames)
                uint64_t* fl = a.flist + (c * kListSlots + (i < (uint32_t)kListSlots ? i : 0)) * kList;
                const bool rec = i < (uint32_t)kListSlots;
                auto emit = [&](uint64_t p, uint32_t key, uint8_t b0) {
                    if (rec && cnt < (uint32_t)kList) fl[cnt] = (p - B) | (uint64_t)b0 << 16 | (uint64_t)key << 32;
                    ++cnt;
                };
                uint64_t v = term(kEnd, x);   // x == len on a chunk edge
                if (x - B < kChunk) {
                    // kProbeHops frames first: a chain on course for more than kWalkHops frames in
                    // the chunk goes to the LDS paths now, not after kWalkHops dependent reads
                    uint64_t at = 0;
                    v = walk_frames<false>(a, B, nullptr, x, kProbeHops, emit, &at);
                    if (v == 0 && (at - x) * (kWalkHops / kProbeHops) >= B + kChunk - x)
                        v = walk_frames<false>(a, B, nullptr, at, kWalkHops - kProbeHops, emit);
                }
                if (v == 0) {
                    queue[atomicAdd(&nq, 1)] = (uint16_t)(s - blk0);
                } else {
                    a.anq[s] = ~0u;
                    link_node<SC1>(a, s, x, v, cnt);
                }
            }
        }
    }
    __syncthreads();
    SCAN_STAMP(1, 1);
    const int n = nq;
    if (n == 0) return;   // block-uniform
    // dense chunks: one wavefront each (DenseLds), the block's wavefronts side by side; each
    // wavefront's next chunk is loaded into registers while it works on the current one
    if (a.strict) {   // (non-strict: every position a candidate, the block path)
        const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / kWave));
        const int lane = threadIdx.x & (kWave - 1);
        DenseLds& d = sl.w[wv];
        DENSE_ACC;
        ChunkRegs R;
        bool rfast = wv < n && chunk_regs_load(a, (blk0 + queue[wv]) / kCand * kChunk, lane, R);
        for (int qi = wv; qi < n; qi += kScanT / kWave) {
            const uint64_t node = blk0 + queue[qi];

            const uint64_t x = a.cand[node];   // (before the prefetch: a wait for it must not wait for that)
            if (rfast) chunk_regs_store(d.words, R, lane);
            else wave_load_chunk(a, node / kCand * kChunk, d.words, lane);
            const int qn = qi + kScanT / kWave;
            rfast = qn < n && chunk_regs_load(a, (blk0 + queue[qn]) / kCand * kChunk, lane, R);
            wave_lds_sync();
            if (dense_node<SC1, BC>(a, d, node, x, (uint32_t)qi, bid DENSE_PASS) && lane == 0) queue[qi] = kQTaken;
            wave_lds_sync();   // (the next chunk overwrites d)
        }
        DENSE_FLUSH();
    }
    __syncthreads();
    SCAN_STAMP(1, 2);   // dense chunks done
    for (int qi = 0; qi < n; ++qi) {
        if (queue[qi] == kQTaken) continue;   // block-uniform: taken by a wavefront
        const uint64_t node = blk0 + queue[qi], chunk = node / kCand, B = chunk * kChunk;
        load_chunk(a, B, words);
        chunk_links16(a, B, words, l1, lj, lk16);
        const uint16_t* l8 = lj;   // the 8-hop links (the pass before the last)
        if (tid == 0) {
            const uint64_t x = a.cand[node];   // in [B, B + kChunk): the walk above started there
            uint32_t p = (uint32_t)(x - B), hops = 0;
            // the walk's positions every 8 frames are K4's anchors if this node turns out
            // to be its chunk's true entry: kept in the block's slots while they last
            const uint64_t q = (uint64_t)bid * BC + qi;
            const bool keep = qi < BC && q < a.anc_cap;
            uint16_t* anc = a.anc + (keep ? q : 0) * kAncSlot;
            int na = 0;
            if (keep) anc[na++] = (uint16_t)p;
            while (l8[p] != kNoLink) {
                p = l8[p];
                hops += kAncStride;
                if (keep && na < kAncMax) anc[na++] = (uint16_t)p;
            }
            if (keep) a.anc_n[q] = (uint32_t)na;
            a.anq[node] = keep ? (uint32_t)q : ~0u;
            while (l1[p] != kNoLink) {
                p = l1[p];
                ++hops;
            }
            uint64_t v = parse_at(a, B + p, window_at(words, (int)p), nullptr, nullptr);
            if (!(v & kTerm)) {   // the last frame of the chunk: its successor is past the chunk
                v = term(kExit, v);
                ++hops;
            }
            link_node<SC1>(a, node, x, v, hops);
        }
        __syncthreads();
    }
}

// K2: nothing when K1 resolved the call on the one-pass path (a flag read)
template <int BC>
__global__ __launch_bounds__(kScanT) void scan_links(ScanArgs a) {
    __shared__ LinksLdsT<BC> sl;
    SCAN_SCOPE(1);
    if (onepass_done(a)) return;
    links_body<false, BC>(a, sl, blockIdx.x);
}

// exclusive prefix sum over a block of NT threads; the block total in *total
template <int NT>
__device__ uint64_t block_scan(uint64_t v, uint64_t* total) {
    __shared__ uint64_t wsum[NT / kWave];
    const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
    uint64_t inc = v;
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
        const uint64_t o = (uint64_t)__shfl_up((unsigned long long)inc, d, kWave);
        if (lane >= d) inc += o;
    }
    if (lane == kWave - 1) wsum[w] = inc;
    __syncthreads();
    uint64_t before = 0, all = 0;
#pragma unroll
    for (int i = 0; i < NT / kWave; ++i) {
        before += i < w ? wsum[i] : 0;
        all += wsum[i];
    }
    __syncthreads();
    *total = all;
    return before + inc - v;
}

// K3a: one block per tile of kTileChunks chunks (thread t: chunk t).  The tile's
// nodes compacted into LDS; local links (to a node of the same tile) are followed by
// Wyllie pointer jumping: W = frames to the tile's exit, L = the last node before it,
// and each external node's bit pushed along its path (a node pushes its bits along
// its current jump; after round r every node holds the bits of the nodes up to 2^(r+1)
// - 1 links before it).  ~log2(path) rounds of a few LDS operations per node.
static constexpr uint16_t kNone = 0xFFFF;
static constexpr int kFastNodes = 2 * kScanT;   // K3a: up to this many nodes, each thread holds two

// Rounds of pointer jumping that finish every path among n nodes: a path has at most
// n - 1 links, and round r doubles the links a jump covers.
__device__ __forceinline__ int jump_rounds(int n) { return n <= 1 ? 0 : 32 - __clz(n - 1); }

// K3a's ranking for V <= kFastNodes, the usual tile: thread t holds nodes t and t +
// kScanT in registers; a round reads the jump targets from one half of a ping-pong
// pair in LDS and writes the thread's own nodes into the other, so a round is ONE
// barrier, and the round count is fixed (no block-wide OR to stop).  bits (monotone)
// is one array, as in the generic loop.  The results end in P / L / W.  (One
// wavefront doing all the rounds with no barriers was slower: a lone wavefront is
// instruction-issue-bound, 8 us at config-2 shape against 5.6 for the generic loop.)
__device__ void rank_tile_fast(uint16_t* P, uint16_t* L, uint32_t* W, uint32_t* bits, uint16_t* P2, uint16_t* L2,
                               uint32_t* W2, int n, int t) {
    uint16_t mp[2], ml[2];
    uint32_t mw[2];
#pragma unroll
    for (int r = 0; r < 2; ++r) {
        const int k = t + kScanT * r;
        mp[r] = k < n ? P[k] : kNone;
        ml[r] = k < n ? L[k] : 0;
        mw[r] = k < n ? W[k] : 0;
    }
    const int rounds = jump_rounds(n);
    for (int i = 0; i < rounds; ++i) {
        const uint16_t* sp = (i & 1) ? P2 : P;
        const uint16_t* sl = (i & 1) ? L2 : L;
        const uint32_t* sw = (i & 1) ? W2 : W;
        uint16_t* dp = (i & 1) ? P : P2;
        uint16_t* dl = (i & 1) ? L : L2;
        uint32_t* dw = (i & 1) ? W : W2;
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            const int k = t + kScanT * r;
            if (k < n) {
                const uint16_t p = mp[r];
                if (p != kNone) {
                    atomicOr(&bits[p], bits[k]);
                    mp[r] = sp[p];
                    ml[r] = sl[p];
                    mw[r] += sw[p];
                }
                dp[k] = mp[r];
                dl[k] = ml[r];
                dw[k] = mw[r];
            }
        }
        __syncthreads();
    }
    if (rounds & 1) {   // the last round wrote the second halves: the results go to P / L / W
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            const int k = t + kScanT * r;
            if (k < n) {
                P[k] = mp[r];
                L[k] = ml[r];
                W[k] = mw[r];
            }
        }
        __syncthreads();
    }
}

struct TilesLds {
    uint16_t cid[kTileSlots];   // tile slot -> compact node
    uint16_t gsl[kTileSlots];   // compact node -> tile slot
    uint16_t P[kTileSlots];     // current jump (compact), kNone: at the last node
    uint16_t L[kTileSlots];     // last node reached
    uint32_t W[kTileSlots];     // frames from the node to L's exit
    uint32_t bits[kTileSlots];
    uint16_t P2[kFastNodes], L2[kFastNodes];   // rank_tile_fast: the ping-pong halves
    uint32_t W2[kFastNodes];
    uint16_t elist[kExt];
    uint8_t eroot[kExt];
    int skip;
};

template <bool SC1>
__device__ __forceinline__ void tiles_body(const ScanArgs& a, uint64_t tile, TilesLds& st) {
    uint16_t* cid = st.cid;
    uint16_t* gsl = st.gsl;
    uint16_t* P = st.P;
    uint16_t* L = st.L;
    uint32_t* W = st.W;
    uint32_t* bits = st.bits;
    uint16_t* P2 = st.P2;
    uint16_t* L2 = st.L2;
    uint32_t* W2 = st.W2;
    uint16_t* elist = st.elist;
    uint8_t* eroot = st.eroot;
    int& skip = st.skip;
    const int t = threadIdx.x;
    // overflow: K4 walks serially.  Read once for the block (another tile may set it
    // meanwhile), in the same trip as the chunk data below; checked after the scans
    const uint32_t ovf0 = t == 0 ? __hip_atomic_load(a.ovf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
    const uint64_t c = tile * kTileChunks + t, s0 = tile * kTileSlots;
    // the chunk's counter, external flags, links and counts in one trip
    const bool live = c <= a.nc;
    const uint32_t cnt = live ? min(a.ccount[c], (uint32_t)kCand) : 0;
    // (SC1: K2's outputs handed over in the same launch, scan_links_fused)
    const uint64_t exf = live ? hand_ld<SC1>((const uint64_t*)(a.ext + c * kCand)) : 0;   // kCand == 8 flag bytes
    int32_t lks[kCand];
    uint32_t nws[kCand];
    uint32_t rootm = 0;   // the slot holding the stream start
#pragma unroll
    for (int j = 0; j < kCand; ++j) {
        lks[j] = live ? hand_ld<SC1>(&a.link[c * kCand + j]) : kDupLink;
        nws[j] = live ? hand_ld<SC1>(&a.ncnt[c * kCand + j]) : 0;
    }
    if (live && c == a.start / kChunk) {   // only the stream start's chunk holds the root
#pragma unroll
        for (int j = 0; j < kCand; ++j) rootm |= (a.cand[c * kCand + j] == a.start ? 1u : 0u) << j;
    }
    uint32_t extm = 0;
#pragma unroll
    for (int j = 0; j < kCand; ++j)
        if ((uint32_t)j < cnt && ((exf >> (8 * j)) & 0xFF) && lks[j] != kDupLink) extm |= 1u << j;
    uint64_t V64, E64;
    const uint32_t base = (uint32_t)block_scan<kScanT>(cnt, &V64);
    if (t == 0) skip = ovf0 != 0;
    uint32_t eidx = (uint32_t)block_scan<kScanT>((uint64_t)__popc(extm), &E64);   // its barriers publish skip
    SCAN_STAMP(2, 2);
    if (skip) return;   // block-uniform
    if (E64 > (uint64_t)kExt) {   // block-uniform
        if (t == 0) atomicOr(a.ovf, kOvfExt);
        return;
    }
    const int V = (int)V64, E = (int)E64;
    SCAN_VALUE(2, 5, V);
    for (uint32_t i = 0; i < cnt; ++i) {
        cid[t * kCand + i] = (uint16_t)(base + i);
        gsl[base + i] = (uint16_t)(t * kCand + i);
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kCand; ++i) {
        if ((uint32_t)i >= cnt) break;
        const uint32_t k = base + i;
        const int32_t lk = lks[i];
        P[k] = (lk >= 0 && (uint64_t)lk - s0 < kTileSlots) ? cid[(uint64_t)lk - s0] : kNone;
        W[k] = lk == kDupLink ? 0u : nws[i];
        L[k] = (uint16_t)k;
        if ((extm >> i) & 1) {
            bits[k] = 1u << eidx;
            elist[eidx] = (uint16_t)k;
            eroot[eidx] = (rootm >> i) & 1;
            ++eidx;
        } else {
            bits[k] = 0;
        }
    }
    __syncthreads();
    SCAN_STAMP(2, 3);
    constexpr int kR = (int)(kTileSlots / kScanT);
    if (a.fast_rank && V <= kFastNodes) {   // block-uniform: the usual tile (strict: about one node per chunk)
        rank_tile_fast(P, L, W, bits, P2, L2, W2, V, t);
        SCAN_VALUE(2, 6, jump_rounds(V));
    } else for (;;) {
        uint16_t np[kR], nl[kR];
        uint32_t nw[kR];
        int any = 0;
#pragma unroll
        for (int r = 0; r < kR; ++r) {
            const int k = t + kScanT * r;
            np[r] = kNone;
            if (k < V) {
                const uint16_t p = P[k];
                if (p != kNone) {
                    np[r] = P[p];
                    nw[r] = W[k] + W[p];
                    nl[r] = L[p];
                    atomicOr(&bits[p], bits[k]);
                    any |= np[r] != kNone;
                }
            }
        }
        __syncthreads();
#pragma unroll
        for (int r = 0; r < kR; ++r) {
            const int k = t + kScanT * r;
            if (k < V && P[k] != kNone) {
                P[k] = np[r];
                W[k] = nw[r];
                L[k] = nl[r];
            }
        }
        if (!__syncthreads_or(any)) break;
    }
    SCAN_STAMP(2, 4);
    for (uint32_t i = 0; i < cnt; ++i) {
        const uint64_t gs = c * kCand + i;
        const uint32_t k = base + i;
        a.wsum[gs] = W[k];
        a.pbits[gs] = bits[k];
    }
    if (t < E) {
        const uint32_t k = elist[t];
        const uint64_t last = s0 + gsl[L[k]];
        TileExt e;
        e.slot = (uint32_t)(s0 + gsl[k]);
        e.w = W[k];
        e.xl = hand_ld<SC1>(&a.link[last]);
        e.root = eroot[t];
        e.term = hand_ld<SC1>(&a.nterm[last]);
        put_text(&a.text[tile * kExt + t], e);
    }
    if (t == 0) __hip_atomic_store(&a.tcount[tile], (uint32_t)E, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(kScanT) void scan_tiles(ScanArgs a) {
    __shared__ TilesLds st;
    SCAN_SCOPE(2);
    if (onepass_done(a)) return;
    tiles_body<false>(a, blockIdx.x, st);
}

// Tile resolution (K3b): the external nodes of all tiles into LDS (tile by tile, in
// bit order); each one's successor is the external node its path exits to; Wyllie
// pointer jumping gives R = frames from the node to the end of its chain and marks
// the nodes reachable from the root.  A marked node is its tile's true entry: frames
// before it = R(root) - R(node).  The one whose path ends inside its tile holds the
// terminal: the results.  Beyond the capacities (MAXT tiles, CAP nodes) -> serial
// walk.  The tile counts and each tile's first two records are read in one trip (a
// tile rarely has more: the true entry, now and then a garbage one); the rest in a
// second.  (Tried: every K4 workgroup resolving the tiles itself in its prologue, no
// launch of its own: C2 51 -> 60 us -- the chain of trips, scans and rounds is paid
// per workgroup round, and K4 has several.)
static constexpr int kExtFirst = 2;

template <int MAXT, int CAP, int PP = kResolveT>
struct ResolveLds {
    uint32_t toff[MAXT + 1];
    uint32_t eslot[CAP];
    uint32_t ew[CAP];
    int32_t exl[CAP];
    uint64_t R[CAP];
    uint16_t succ[CAP];
    uint64_t R2[PP];      // resolve_fast: the ping-pong halves (its NT x PER nodes)
    uint16_t succ2[PP];
    uint8_t mark[CAP];
    uint8_t islast[CAP];   // its path ends in its tile (no successor)
    int bad, root_idx;
    uint32_t M, why;
};

__device__ __forceinline__ void put_ext(uint32_t* eslot, uint32_t* ew, int32_t* exl, uint64_t* R, uint8_t* mark,
                                        uint32_t idx, const TileExt& e) {
    eslot[idx] = e.slot;
    ew[idx] = e.w;
    exl[idx] = e.xl;
    R[idx] = e.w;
    mark[idx] = e.root != 0;
}

// K3b's ranking for m <= NT nodes (the usual stream: a few external nodes per tile):
// thread i holds node i in registers, one barrier per round over ping-pong halves, a
// fixed round count -- as rank_tile_fast.  The results end in succ / R; mark
// (monotone) is one array.
template <int NT, int PER>
__device__ void resolve_fast(uint16_t* succ, uint64_t* R, uint16_t* succ2, uint64_t* R2, uint8_t* mark, int m) {
    uint16_t ms[PER];
    uint64_t mr[PER];
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const int i = threadIdx.x + NT * q;
        ms[q] = i < m ? succ[i] : kNone;
        mr[q] = i < m ? R[i] : 0;
    }
    const int rounds = jump_rounds(m);
    for (int r = 0; r < rounds; ++r) {
        const uint16_t* ss = (r & 1) ? succ2 : succ;
        const uint64_t* sr = (r & 1) ? R2 : R;
        uint16_t* ds = (r & 1) ? succ : succ2;
        uint64_t* dr = (r & 1) ? R : R2;
#pragma unroll
        for (int q = 0; q < PER; ++q) {
            const int i = threadIdx.x + NT * q;
            if (i < m) {
                if (ms[q] != kNone) {
                    if (mark[i]) mark[ms[q]] = 1;
                    mr[q] += sr[ms[q]];
                    ms[q] = ss[ms[q]];
                }
                ds[i] = ms[q];
                dr[i] = mr[q];
            }
        }
        __syncthreads();
    }
    if (rounds & 1) {
#pragma unroll
        for (int q = 0; q < PER; ++q) {
            const int i = threadIdx.x + NT * q;
            if (i < m) {
                succ[i] = ms[q];
                R[i] = mr[q];
            }
        }
        __syncthreads();
    }
}

// every thread of the block; on return (after a barrier) sm.bad / sm.why say whether the
// parallel path holds, and R / mark / islast / toff answer per-tile queries
template <int NT, int PER, int MAXT, int CAP>
__device__ __forceinline__ void resolve_tiles(const ScanArgs& a, uint64_t tiles, ResolveLds<MAXT, CAP, NT * PER>& sm) {
    const int t = threadIdx.x;
    if (tiles > (uint64_t)MAXT) {   // kernel-uniform
        if (t == 0) {
            sm.bad = 1;
            sm.why = kWhyTiles;
        }
        __syncthreads();
        return;
    }
    constexpr int kTR = (MAXT + NT - 1) / NT;
    // trip 1: every tile's count, and the first records of the first NT tiles
    // (issued together, used after the scan)
    uint32_t tc[kTR];
    // the first two records of the tiles of the first kPre rounds (all of them when a thread
    // has at most two tiles: the merged launch up to 512 tiles) come in this trip too
    constexpr int kPre = kTR <= 2 ? kTR : 1;
    TileExt e0[kPre], e1[kPre];
#pragma unroll
    for (int r = 0; r < kTR; ++r) {
        const uint64_t tl = (uint64_t)t + (uint64_t)NT * r;
        tc[r] = tl < tiles ? get_sc1(&a.tcount[tl]) : 0;
    }
#pragma unroll
    for (int r = 0; r < kPre; ++r) {
        const uint64_t tl = (uint64_t)t + (uint64_t)NT * r;
        if (tl < tiles) {
            e0[r] = get_text(&a.text[tl * kExt]);
            e1[r] = get_text(&a.text[tl * kExt + 1]);
        }
    }
    if (t == 0) {   // the overflow word in the same trip
        const uint32_t ovf = __hip_atomic_load(a.ovf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        sm.bad = ovf != 0;
        sm.why = ovf;
        sm.root_idx = -1;
    }
    uint64_t run = 0;
#pragma unroll
    for (int r = 0; r < kTR; ++r) {
        if ((uint64_t)NT * r >= tiles) break;   // block-uniform
        const uint64_t tl = (uint64_t)t + (uint64_t)NT * r;
        uint64_t tot;
        const uint64_t ex = block_scan<NT>(tc[r], &tot);
        if (tl < tiles) sm.toff[tl] = (uint32_t)(run + ex);
        run += tot;
    }
    SCAN_STAMP(3, 1);
    if (t == 0) {
        sm.toff[tiles] = (uint32_t)run;
        sm.M = (uint32_t)run;
        if (run > (uint64_t)CAP) {
            sm.bad = 1;
            sm.why |= kWhyExtCap;
        }
    }
    __syncthreads();
    if (sm.bad) return;
    int more = 0;
#pragma unroll
    for (int r = 0; r < kTR; ++r) {
        const uint64_t tl = (uint64_t)t + (uint64_t)NT * r;
        if (tl >= tiles) break;
        const uint32_t o = sm.toff[tl];
        if (r < kPre) {
            const int rp = r < kPre ? r : 0;   // (a constant once unrolled)
            if (tc[r] > 0) put_ext(sm.eslot, sm.ew, sm.exl, sm.R, sm.mark, o, e0[rp]);
            if (tc[r] > 1) put_ext(sm.eslot, sm.ew, sm.exl, sm.R, sm.mark, o + 1, e1[rp]);
        } else {
            for (uint32_t j = 0; j < tc[r] && j < (uint32_t)kExtFirst; ++j)
                put_ext(sm.eslot, sm.ew, sm.exl, sm.R, sm.mark, o + j, get_text(&a.text[tl * kExt + j]));
        }
        more |= tc[r] > (uint32_t)kExtFirst;
    }
    if (__syncthreads_or(more)) {   // trip 2 (rare): tiles with more than two external nodes
#pragma unroll
        for (int r = 0; r < kTR; ++r) {
            const uint64_t tl = (uint64_t)t + (uint64_t)NT * r;
            if (tl >= tiles) break;
            for (uint32_t j = kExtFirst; j < tc[r]; ++j)
                put_ext(sm.eslot, sm.ew, sm.exl, sm.R, sm.mark, sm.toff[tl] + j, get_text(&a.text[tl * kExt + j]));
        }
        __syncthreads();
    }
    SCAN_STAMP(3, 2);
    const int m = (int)sm.M;
    SCAN_VALUE(3, 5, m);
    // successors: the external node (of a later tile) each path exits to, found in LDS
    for (int i = t; i < m; i += NT) {
        const int32_t xl = sm.exl[i];
        uint16_t sx = kNone;
        if (xl >= 0) {
            const uint64_t t2 = (uint64_t)xl / kTileSlots;
            for (uint32_t u = sm.toff[t2]; u < sm.toff[t2 + 1]; ++u)
                if (sm.eslot[u] == (uint32_t)xl) sx = (uint16_t)u;
            if (sx == kNone) {   // an exit onto a node no tile listed (defence in depth)
                sm.bad = 1;
                sm.why = kWhySucc;
            }
        }
        sm.succ[i] = sx;
        sm.islast[i] = xl < 0;
        if (sm.mark[i]) sm.root_idx = i;
    }
    __syncthreads();
    SCAN_STAMP(3, 3);
    if (sm.bad || sm.root_idx < 0) {   // block-uniform
        if (t == 0 && !sm.bad) {
            sm.bad = 1;
            sm.why = kWhyRoot;
        }
        __syncthreads();
        return;
    }
    if (a.fast_rank && m <= NT * PER) {   // block-uniform: the usual stream (a few external nodes per tile)
        resolve_fast<NT, PER>(sm.succ, sm.R, sm.succ2, sm.R2, sm.mark, m);
        SCAN_VALUE(3, 6, jump_rounds(m));
        SCAN_STAMP(3, 4);
        return;
    }
    constexpr int kR = (CAP + NT - 1) / NT;
    for (;;) {
        uint16_t ns[kR];
        uint64_t nr[kR];
        int any = 0;
#pragma unroll
        for (int r = 0; r < kR; ++r) {
            const int i = t + NT * r;
            ns[r] = kNone;
            if (i < m) {
                const uint16_t sx = sm.succ[i];
                if (sx != kNone) {
                    ns[r] = sm.succ[sx];
                    nr[r] = sm.R[i] + sm.R[sx];
                    if (sm.mark[i]) sm.mark[sx] = 1;
                    any |= ns[r] != kNone;
                }
            }
        }
        __syncthreads();
#pragma unroll
        for (int r = 0; r < kR; ++r) {
            const int i = t + NT * r;
            if (i < m && sm.succ[i] != kNone) {
                sm.succ[i] = ns[r];
                sm.R[i] = nr[r];
            }
        }
        if (!__syncthreads_or(any)) break;
    }
    SCAN_STAMP(3, 4);
}

// tile tl's true entry (at most one marked node: the chain enters a tile once); if the
// chain ends in it and `results`, the scan's results too
template <int MAXT, int CAP, int PP>
__device__ TileInfo tile_info(const ScanArgs& a, const ResolveLds<MAXT, CAP, PP>& sm, uint64_t tl, bool results) {
    TileInfo ti;
    ti.j = -1;
    ti.we = 0;
    ti.base = 0;
    const uint64_t total = sm.R[sm.root_idx];
    for (uint32_t i = sm.toff[tl]; i < sm.toff[tl + 1]; ++i)
        if (sm.mark[i]) {
            ti.j = (int32_t)(i - sm.toff[tl]);
            ti.we = sm.ew[i];
            ti.base = total - sm.R[i];
            if (results && sm.islast[i]) {   // the chain ends in this tile
                const uint64_t term_v = __hip_atomic_load(&a.text[tl * kExt + ti.j].term, __ATOMIC_RELAXED,
                                                          __HIP_MEMORY_SCOPE_AGENT);
                const uint64_t ty = term_type(term_v), pos = term_pos(term_v);
                // an exit onto a position K1 pruned: the chain dies there
                const bool dead = ty == kDead || ty == kExit;
                a.result[0] = total;
                a.result[1] = pos;
                a.result[2] = dead ? pos : ~0ull;
                if (total <= a.max_frames) a.hdr[total] = pos;
            }
        }
    return ti;
}

// K3b: one block resolves every tile, writes each tile's entry (tinfo) and whether K4
// walks serially (flags[8], the reason in flags[9])
template <int NT, int PER, int MAXT, int CAP>
__device__ __forceinline__ void resolve_body(const ScanArgs& a, uint64_t tiles, ResolveLds<MAXT, CAP, NT * PER>& sm) {
    resolve_tiles<NT, PER>(a, tiles, sm);
    if (!sm.bad)
        for (uint64_t tl = threadIdx.x; tl < tiles; tl += NT) a.tinfo[tl] = tile_info(a, sm, tl, true);
    if (threadIdx.x == 0) {
        a.flags[8] = sm.bad ? 1u : 0u;
        a.flags[9] = sm.bad ? sm.why : 0u;
    }
}

__global__ __launch_bounds__(kResolveT) void scan_resolve(ScanArgs a, uint64_t tiles) {
    __shared__ ResolveLds<kMaxTiles, kExtCap> sm;
    SCAN_SCOPE(3);
    if (onepass_done(a)) return;
    resolve_body<kResolveT, 1>(a, tiles, sm);
}

// K2 + K3a + K3b in one launch, for streams of up to kFuseTiles tiles: every block runs
// K2 on its 16 chunks; the last of a tile's blocks to finish (an arrival counter per
// tile) runs K3a for that tile, while other tiles' blocks are still in K2; the last tile
// to finish K3a (one more counter) runs K3b over all of them.  Two launch boundaries
// and their cold trips fewer, and K3a overlapped with K2.  Each arrival is one atomic
// after the block's own sc1 stores have completed (arrive_last below: no fences); the
// block that arrives last resets the counter for the next call and reads the other
// blocks' results with sc1 loads.  The phases' LDS share one union (36 KB: 4 blocks per CU).
static constexpr int kFuseTiles = 512;   // 512 MiB of stream
static constexpr int kFuseCap = 1024;    // external nodes
union FusedLds {
    LinksLds k2;
    TilesLds k3a;
    ResolveLds<kFuseTiles, kFuseCap> k3b;
};

// true in every thread of the block that arrives last at *counter (of `expect`)
// Round 4: the hand-offs need no fences.  Every byte a later phase of the launch reads is stored
// with a relaxed agent-scope (sc1) store and read with sc1 loads only (link_node, the dup flags,
// tiles_body's first trip and records, put_text / get_text); each wave waits for its stores, the
// block's barrier follows, then one lane adds to the arrival counter (MI355X_MICROARCH.md,
// cross-workgroup hand-offs).  The round-3 form -- a release fence by every block, an acquire by
// the last -- wrote back each XCD's L2 per block and measured 261 us at config 2.
__device__ __forceinline__ bool arrive_last(uint32_t* counter, uint32_t expect, int* flag) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's sc1 stores have completed
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t old = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *flag = old == expect - 1;
        if (*flag)   // every block has arrived: reset for the next call
            __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    return *flag != 0;
}

// On the one-pass path this launch (a flag read) and K4 follow K1: one launch boundary fewer
// than scan_links + scan_tiles_resolve.
__global__ __launch_bounds__(kScanT) void scan_links_fused(ScanArgs a, uint64_t tiles, uint32_t blocks) {
    __shared__ FusedLds sm;
    __shared__ int flag;
    SCAN_SCOPE(1);
    if (onepass_done(a)) return;
    links_body<true, kBlkChunks>(a, sm.k2, blockIdx.x);
    constexpr uint32_t kPerTile = (uint32_t)(kTileChunks / kBlkChunks);
    const uint32_t tile = blockIdx.x / kPerTile;
    const uint32_t in_tile = min(blocks - tile * kPerTile, kPerTile);
    if (!arrive_last(a.tarr + tile, in_tile, &flag)) return;   // block-uniform
    tiles_body<true>(a, tile, sm.k3a);
    if (!arrive_last(a.flags + 12, (uint32_t)tiles, &flag)) return;
    resolve_body<kScanT, kFuseCap / kScanT>(a, tiles, sm.k3b);
}

// K3a + K3b as one launch, for streams of up to kMergeTiles tiles (the default there): every
// block ranks its tile (K3a); the last block to arrive resolves all tiles (K3b) -- one launch
// boundary and K3b's cold first trip fewer.  Unlike scan_links_fused this needs no release
// fence: the only bytes K3b reads from this launch are the tiles' external-node records and
// counts, written and read with sc1 stores and loads (put_text / get_text), and the overflow
// word, set by atomics.  Each wave waits for its stores, the block's barrier follows, then
// one lane adds to the arrival counter (flags[13]); the block whose add returns tiles - 1
// resets it for the next call.  The phases' LDS share one union (62 KB: two blocks per CU):
// K3b with 256 threads, the one-barrier ranking up to 1,024 external nodes, the generic loop
// up to kMergeCap (more: the serial walk, as past kExtCap in the separate launch).  Up to 256
// tiles: at config 2 (65 tiles) the merge saves 0.9 us (42.8 against 43.7, r03g); at config 4
// (257 tiles) the merged launch measured 17.6 us against 7.2 + 7.6 for the separate ones, also
// with both rounds of tile records read in the first trip (r03j), so bigger streams keep them.
static constexpr int kMergeTiles = kScanT;   // 256 MiB of stream
static constexpr int kMergeCap = 2048;    // external nodes
union MergedLds {
    TilesLds k3a;
    ResolveLds<kMergeTiles, kMergeCap, 1024> k3b;
};

__global__ __launch_bounds__(kScanT) void scan_tiles_resolve(ScanArgs a, uint64_t tiles) {
    __shared__ MergedLds sm;
    __shared__ int last;
    SCAN_SCOPE(2);
    if (threadIdx.x == 0 && blockIdx.x == 0) OP_TRACE(7, 1);
    if (onepass_done(a)) return;
    tiles_body<false>(a, blockIdx.x, sm.k3a);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's sc1 stores have completed
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t old = __hip_atomic_fetch_add(a.flags + 13, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = old == (uint32_t)tiles - 1;
        if (last) __hip_atomic_store(a.flags + 13, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (!last) return;   // block-uniform
    resolve_body<kScanT, 1024 / kScanT>(a, tiles, sm.k3b);
}

// K4, serial fallback (capacities overflowed): one thread walks the whole stream.
__device__ void serial_walk(const ScanArgs& args) {
    ScanArgs a = args;
    if (a.spec) a.strict = 0;   // the caller's semantics: no checks
    uint64_t p = a.start, n = 0, err = ~0ull;
    for (;;) {
        uint32_t key;
        uint8_t b0;
        const uint64_t v = parse_at(a, p, window_global(a, p), &key, &b0);
        if (v & kTerm) {
            if (term_type(v) == kDead) err = p;
            break;
        }
        if (n < a.max_frames) {
            a.hdr[n] = p;
            a.keys[n] = key;
            a.b0[n] = b0;
        }
        ++n;
        p = v;
    }
    if (n <= a.max_frames) a.hdr[n] = p;
    a.result[0] = n;
    a.result[1] = p;
    a.result[2] = err;
}

// K4, speculative pass (spec): the parallel pass stopped at a header the strict filter
// (minus the MASK and RSV1 checks) rejects, which the caller accepts: one thread walks on from
// there, unchecked, appending frames after the ones found in parallel.
__device__ void spec_continue(const ScanArgs& args) {
    const uint64_t stop = args.result[2];
    if (stop == ~0ull) return;
    ScanArgs a = args;
    a.strict = 0;
    uint64_t p = stop, n = a.result[0];
    for (;;) {
        uint32_t key;
        uint8_t b0;
        const uint64_t v = parse_at(a, p, window_global(a, p), &key, &b0);
        if (v & kTerm) break;
        if (n < a.max_frames) {
            a.hdr[n] = p;
            a.keys[n] = key;
            a.b0[n] = b0;
        }
        ++n;
        p = v;
    }
    if (n <= a.max_frames) a.hdr[n] = p;
    a.result[0] = n;
    a.result[1] = p;
    a.result[2] = ~0ull;
    a.flags[9] |= kWhySpec;
}

// Write frame k's descriptors (if recorded)
__device__ __forceinline__ void put_frame(const ScanArgs& a, uint64_t k, uint64_t p, uint32_t key, uint8_t b0) {
    if (k < a.max_frames) {
        a.hdr[k] = p;
        a.keys[k] = key;
        a.b0[k] = b0;
    }
}

// K4: the chunks' descriptors, EC chunks per block (kEmitChunks or kBlkChunksBig).  Thread t < EC
// takes chunk t: its true entry is the node whose path bits hold the tile entry's bit;
// a chunk of at most kWalkHops frames is walked by that thread (header bytes from
// global memory).  Longer ones: with K2' anchors one wavefront per chunk, lane u
// parsing the 8 frames from anchor u; without, the whole block from LDS (16-hop links,
// an anchor every 16 frames, thread u the 16 frames from anchor u).  Every chunk's
// candidate counter and external flags are zeroed here, after their last reader:
// the next call needs no clearing launch.
// K4's anchored emit: anchors per round (their runs staged in LDS, then stored frame by frame)
static constexpr int kEmitGroup = 32;
static constexpr uint16_t kNoFrame = 0xFFFF;

template <int EC>
__global__ __launch_bounds__(kScanT) void scan_emit(ScanArgs a, uint64_t tiles) {
    __shared__ uint32_t words[kWords];
    __shared__ union {
        struct {
            uint16_t l1[kChunk];    // next header (local index) or kNoLink
            uint16_t lj[kChunk];    // 2^k hops (ping)
            uint16_t lk16[kChunk];  // 2^k hops (pong); 16 hops after the last pass
        } b;
        struct {
            uint32_t ww[kScanT / kWave][kWords];   // anchored chunks: each wavefront's chunk bytes
            uint32_t tkey[kScanT / kWave][kEmitGroup * kAncStride];   // ... and its frames, staged
            uint16_t tpos[kScanT / kWave][kEmitGroup * kAncStride];   //     for coalesced stores
            uint8_t tb0[kScanT / kWave][kEmitGroup * kAncStride];
        } w;
    } lu;
    uint16_t* const l1 = lu.b.l1;
    uint16_t* const lj = lu.b.lj;
    uint16_t* const lk16 = lu.b.lk16;
    __shared__ uint16_t anchor[kChunk / kStride + 1];
    __shared__ int nanchor, nqa, nqb;
    __shared__ uint32_t qa_node[EC], qb_node[EC], qa_slot[EC];
    __shared__ uint64_t qa_base[EC], qb_base[EC];
    __shared__ TileInfo bti;
    __shared__ int fbs;
    SCAN_SCOPE(4);
    (void)tiles;
    const int tid = threadIdx.x;
    const uint64_t tile = (uint64_t)blockIdx.x * EC / kTileChunks;   // EC divides kTileChunks
    if (tid == 0 && blockIdx.x == 0) OP_TRACE(8, 1);
    op_clear_prev(a);
    if (onepass_done(a)) {   // the one-pass launch wrote the frames and results: only the clearing
        if (tid < EC) {
            const uint64_t c = (uint64_t)blockIdx.x * EC + tid;
            if (c <= a.nc) {
                a.ccount[c] = 0;
                *(uint64_t*)(a.ext + c * kCand) = 0;
            }
        }
        if (blockIdx.x == 0 && tid == 0) {
            *a.ovf_prev = 0;
            a.flags[8] = 0;
            a.flags[9] = 0;    // no serial walk
            a.flags[10] = 1;   // the one-pass path (netc_gpu_scan_diag bit 32)
        }
        return;
    }
    if (blockIdx.x == 0 && tid == 0) {
        a.flags[10] = 0;
    }
    if (tid == 0) {
        fbs = __hip_atomic_load(&a.flags[8], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
        bti = a.tinfo[tile];
        if (blockIdx.x == 0) *a.ovf_prev = 0;   // the previous call's overflow word, for the next call
        nqa = 0;
        nqb = 0;
    }
    __syncthreads();
    const bool fb = fbs != 0;
    if (tid < EC) {
        const uint64_t c = (uint64_t)blockIdx.x * EC + tid;
        if (c <= a.nc) {
            // the chunk's counter, path bits, W, counts and positions, and its tile's entry, in one trip
            const uint32_t cnt = min(a.ccount[c], (uint32_t)kCand);
            const TileInfo ti = bti;
            uint32_t pb[kCand], ws[kCand], nct[kCand];
            uint64_t cd[kCand];
#pragma unroll
            for (int j = 0; j < kCand; ++j) {
                pb[j] = a.pbits[c * kCand + j];
                ws[j] = a.wsum[c * kCand + j];
                nct[j] = a.ncnt[c * kCand + j];
                cd[j] = a.cand[c * kCand + j];
            }
            // the true entry: the first slot whose path bits hold the tile entry's bit
            int ie = -1;
            uint32_t we = 0, count = 0;
            uint64_t x = 0;
#pragma unroll
            for (int j = kCand - 1; j >= 0; --j)
                if (!fb && ti.j >= 0 && (uint32_t)j < cnt && ((pb[j] >> ti.j) & 1u)) {
                    ie = j;
                    we = ws[j];
                    count = nct[j];
                    x = cd[j];
                }
            if (ie >= 0) {
                const uint64_t e = c * kCand + ie;
                const uint64_t base = ti.base + ti.we - we;
                if (count > (uint32_t)kWalkHops) {
                    const uint32_t slot = a.anq[e];
                    if (slot != ~0u) {
                        const int q = atomicAdd(&nqa, 1);
                        qa_node[q] = (uint32_t)e;
                        qa_slot[q] = slot;
                        qa_base[q] = base;
                    } else {
                        const int q = atomicAdd(&nqb, 1);
                        qb_node[q] = (uint32_t)e;
                        qb_base[q] = base;
                    }
                } else if (ie < kListSlots && count <= (uint32_t)kList) {
                    // K2 recorded the frames: one trip for the list instead of a walk of
                    // dependent header reads
                    const NETC_GLOBAL u32x4* fl = (const NETC_GLOBAL u32x4*)(a.flist + (c * kListSlots + ie) * kList);
                    u32x4 r[kList / 2];
#pragma unroll
                    for (int h = 0; h < kList / 2; ++h)
                        if ((uint32_t)(2 * h) < count) r[h] = fl[h];
#pragma unroll
                    for (int h = 0; h < kList; ++h)
                        if ((uint32_t)h < count) {
                            const uint32_t lo = r[h / 2][2 * (h & 1)], hi = r[h / 2][2 * (h & 1) + 1];
                            put_frame(a, base + h, c * kChunk + (lo & 0xFFFFu), hi, (uint8_t)(lo >> 16));
                        }
                } else {
                    uint64_t k = base;
                    walk_frames<false>(a, c * kChunk, nullptr, x, -1,
                                       [&](uint64_t p, uint32_t key, uint8_t b0) { put_frame(a, k++, p, key, b0); });
                }
            }
            a.ccount[c] = 0;
            *(uint64_t*)(a.ext + c * kCand) = 0;   // kCand == 8 flag bytes, 8-aligned
        }
    }
    if (fb) {   // block-uniform
        if (blockIdx.x == 0 && tid == 0) serial_walk(a);
        return;
    }
    __syncthreads();
    SCAN_STAMP(4, 1);
    // anchored chunks: one wavefront each, the chunk's bytes staged in the wavefront's LDS (one
    // coalesced 4-KiB read; the 8-frame runs from the anchors then parse from LDS instead of a
    // dependent global read per frame: K4 117 -> see DESIGN_ROUNDS.md §14 at 64 MiB of 16-B frames)
    const int lane = tid & (kWave - 1), wv = __builtin_amdgcn_readfirstlane(tid / kWave);
    for (int q = wv; q < nqa; q += kScanT / kWave) {
        const uint64_t node = qa_node[q], chunk = node / kCand, B = chunk * kChunk, Bend = B + kChunk;
        uint32_t* ww = lu.w.ww[wv];
        // one trip: the chunk, the anchor count and the first 64 anchors (a slot holds kAncSlot)
        const uint32_t slot = qa_slot[q];
        const uint16_t* anc = a.anc + (uint64_t)slot * kAncSlot;
        const uint32_t na_ld = a.anc_n[slot];
        const uint16_t anc0 = anc[lane];
        wave_load_chunk(a, B, ww, lane);
        const int na = (int)na_ld;
        wave_lds_sync();
        // kEmitGroup anchors per round: lane u < kEmitGroup parses the run of anchor ub + u into
        // entries 8 u .. 8 u + 7 of the staging arrays (kNoFrame past its end), then the wavefront
        // stores the round's frames with consecutive lanes on consecutive frames (the runs'
        // own order put each store instruction on 8-frame strides: 64 MiB of 16-B frames,
        // 4.2 M frames x 3 scattered stores)
        uint32_t* tkey = lu.w.tkey[wv];
        uint16_t* tpos = lu.w.tpos[wv];
        uint8_t* tb0 = lu.w.tb0[wv];
        for (int ub = 0; ub < na; ub += kEmitGroup) {
            const int u = ub + lane;
            if (lane < kEmitGroup) {
                uint64_t pos = u < na ? B + (ub == 0 ? anc0 : anc[u]) : Bend;   // (anc0 = anc[lane])
#pragma unroll 1
                for (int h = 0; h < kAncStride; ++h) {
                    const int i = lane * kAncStride + h;
                    uint64_t v = kTerm;
                    uint32_t key = 0;
                    uint8_t b0 = 0;
                    if (pos < Bend) v = parse_at(a, pos, window_at(ww, (int)(pos - B)), &key, &b0);
                    tpos[i] = (v & kTerm) ? kNoFrame : (uint16_t)(pos - B);
                    tkey[i] = key;
                    tb0[i] = b0;
                    if (!(v & kTerm)) pos = v;
                    else pos = Bend;
                }
            }
            wave_lds_sync();
            const uint64_t k0 = qa_base[q] + (uint64_t)ub * kAncStride;
            for (int i = lane; i < kEmitGroup * kAncStride; i += kWave)
                if (tpos[i] != kNoFrame) put_frame(a, k0 + i, B + tpos[i], tkey[i], tb0[i]);
            wave_lds_sync();   // (the next round overwrites the staging arrays)
        }
    }
    SCAN_STAMP(4, 2);   // (wave 0's) anchored chunks done
    // the rest: the block from LDS (its arrays overlay the wavefronts' chunk bytes)
    if (nqb) __syncthreads();   // block-uniform
    for (int q = 0; q < nqb; ++q) {
        const uint64_t node = qb_node[q], chunk = node / kCand, B = chunk * kChunk, Bend = B + kChunk;
        load_chunk(a, B, words);   // ends with a barrier
        const uint16_t* l16 = chunk_links16(a, B, words, l1, lj, lk16);
        if (tid == 0) {
            int na = 0;
            const uint64_t e = a.cand[node];
            if (e < Bend) {
                uint16_t p = (uint16_t)(e - B);
                anchor[na++] = p;
                while (na <= (int)(kChunk / kStride) && l16[p] != kNoLink) {
                    p = l16[p];
                    anchor[na++] = p;
                }
            }
            nanchor = na;
        }
        __syncthreads();
        const int na = nanchor;
        for (int u = tid; u < na; u += kScanT) {
            uint64_t k = qb_base[q] + (uint64_t)u * kStride;
            uint64_t pos = B + anchor[u];
            for (int h = 0; h < kStride && pos < Bend; ++h) {
                uint32_t key;
                uint8_t b0;
                const uint64_t v = parse_at(a, pos, window_at(words, (int)(pos - B)), &key, &b0);
                if (v & kTerm) break;
                put_frame(a, k++, pos, key, b0);
                pos = v;
            }
        }
        __syncthreads();
    }
    if (a.spec && blockIdx.x == 0 && tid == 0) spec_continue(a);   // after this block's own frames
}

// In-place unmask of scanned frames: the batch kernel reads each frame's header
// offset and key from the scan's outputs and its header length from the header bytes
// in the buffer (ArgsScan in ws_mask_gpu.hip); the frame count comes from the scan's
// result on the device, so scan -> unmask needs no host round trip and no view array.
hipError_t launch_unmask_scanned(uint8_t* wire, uint64_t len, const uint64_t* hdr, const uint32_t* keys,
                                 uint64_t max_frames, const uint64_t* result, hipStream_t stream,
                                 const LaunchCfg& cfg) {
    (void)cfg;
    return launch_mask_scanned(wire, len, hdr, keys, max_frames, result, stream);
}

// ------------------------------------------------------------------ launch --

struct ScanScratch {
    void* mem = nullptr;
    uint64_t bytes = 0;
    uint64_t cap = 0;      // chunks the layout is sized for
    bool dirty = false;    // a call did not launch all its kernels: clear before the next
    uint64_t calls = 0;    // the overflow word alternates per call
    uint64_t epoch = 0;    // the one-pass status words' epoch of the last call (1 .. 2^24 - 1)
    std::vector<void*> retired;   // outgrown allocations (queued work may still use them)
};

ScanScratch* scan_scratch_new() { return new (std::nothrow) ScanScratch(); }

void scan_scratch_free(ScanScratch* s) {
    if (!s) return;
    if (s->mem) (void)hipFree(s->mem);
    for (void* p : s->retired) (void)hipFree(p);
    delete s;
}

namespace {
// the per-(device, stream) scratch of the public netc_gpu_scan_frames entry
// shared_ptr: scan_diag keeps the scratch alive through its device read without holding the
// global lock (a concurrent release drops only the map's reference)
std::map<std::pair<int, hipStream_t>, std::shared_ptr<ScanScratch>>& stream_scratch() {
    static std::map<std::pair<int, hipStream_t>, std::shared_ptr<ScanScratch>> m;
    return m;
}
std::mutex& stream_scratch_mu() {
    static std::mutex mu;
    return mu;
}

// The scratch layout for `cap` chunks (cap a multiple of kTileChunks): offsets of the
// regions; flags, ccount and ext first -- the region every call leaves zeroed.
struct Layout {
    uint64_t flags, ccount, ext, tarr, cleared, cand, link, nterm, ncnt, wsum, pbits, anq, anc, anc_n, flist, text,
        tcount, tinfo, st_t, st_g, opfl, opf, total;
};
Layout layout_for(uint64_t cap) {
    auto align = [](uint64_t x) { return (x + 63) & ~63ull; };
    const uint64_t slots = cap * kCand, tiles = cap / kTileChunks;
    Layout l;
    uint64_t o = 0;
    l.flags = o;   o = 64;
    l.ccount = o;  o = align(o + cap * 4);
    l.ext = o;     o = align(o + slots);
    l.tarr = o;    o = align(o + tiles * 4);
    l.opf = o;     o = align(o + 2 * kFailCopies * kFailStride * 4);  // one-pass failure words, two sets
    l.cleared = o;
    l.cand = o;    o = align(o + slots * 8);
    l.link = o;    o = align(o + slots * 4);
    l.nterm = o;   o = align(o + slots * 8);
    l.ncnt = o;    o = align(o + slots * 4);
    l.wsum = o;    o = align(o + slots * 4);
    l.pbits = o;   o = align(o + slots * 4);
    l.anq = o;     o = align(o + slots * 4);
    l.anc = o;     o = align(o + cap * kAncSlot * 2);
    l.anc_n = o;   o = align(o + cap * 4);
    l.flist = o;   o = align(o + cap * kListSlots * kList * 8);   // (one pass: kOpRec frames per chunk)
    l.text = o;    o = align(o + tiles * kExt * sizeof(TileExt));
    l.tcount = o;  o = align(o + tiles * 4);
    l.tinfo = o;   o = align(o + tiles * sizeof(TileInfo));
    l.st_t = o;    o = align(o + cap * 8);   // one-pass status words (epochs: never cleared per call)
    l.st_g = o;    o = align(o + (cap / kOpT + 1) * 8);
    l.opfl = o;    o = align(o + cap * kOpRec * 8);
    l.total = o;
    return l;
}
}  // namespace

// grow to hold `chunks` (+1 virtual) chunks; outgrown allocations are kept until the
// scratch is freed (queued work may still use them)
static hipError_t scratch_grow(ScanScratch& s, uint64_t chunks, hipStream_t stream) {
    if (s.cap >= chunks) return hipSuccess;
    uint64_t cap = s.cap ? 2 * s.cap : kTileChunks;
    while (cap < chunks) cap *= 2;
    const uint64_t want = layout_for(cap).total;
    void* p = nullptr;
    hipError_t e;
    if ((e = hipMalloc(&p, want)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(p, 0, want, stream)) != hipSuccess) {   // zero flags, counters, ext flags
        (void)hipFree(p);
        return e;
    }
    if (s.mem) s.retired.push_back(s.mem);
    s.mem = p;
    s.bytes = want;
    s.cap = cap;
    s.dirty = false;
    return hipSuccess;
}

hipError_t scan_scratch_reserve(ScanScratch* s, uint64_t len, hipStream_t stream) {
    return scratch_grow(*s, (len + kChunk - 1) / kChunk + 1, stream);
}

// the word netc_gpu_scan_diag reads (flags[9]): written by every call's K3b, OR'd by K4's
// speculative continuation; valid until the scratch grows (ingest slots reserve up front)
const uint32_t* scan_scratch_diag_word(const ScanScratch* s) {
    return s && s->mem ? (const uint32_t*)((const uint8_t*)s->mem + 9 * sizeof(uint32_t)) : nullptr;
}

// Why the last scan on (device, stream) took the serial walk (0: it did not); the
// caller has synchronised the stream.  -1: no scratch for that stream.  The global lock is
// held only to find the scratch and read its address (a growing scan replaces s->mem under
// that lock and retires, never frees, the old allocation); the scratch itself stays alive
// through the shared_ptr while the word is copied on the caller's stream, so no other
// thread's scan, launch or release waits behind this device copy.
int64_t scan_diag(int device, hipStream_t stream) {
    std::shared_ptr<ScanScratch> keep;
    const uint8_t* word = nullptr;
    {
        std::lock_guard<std::mutex> g(stream_scratch_mu());
        auto it = stream_scratch().find({device, stream});
        if (it == stream_scratch().end()) return -1;
        keep = it->second;
        if (!keep->mem) return -1;
        word = (const uint8_t*)keep->mem + 9 * sizeof(uint32_t);
    }
    uint32_t w[2] = {0, 0};   // flags[9]: why the serial walk; flags[10]: 1 = the one-pass path
    if (hipMemcpyAsync(w, word, sizeof(w), hipMemcpyDeviceToHost, stream) != hipSuccess ||
        hipStreamSynchronize(stream) != hipSuccess)
        return -1;
    return (int64_t)w[0] | (int64_t)(w[1] & 1) << 32;
}

int release_stream_scratch(int device, hipStream_t stream) {
    std::shared_ptr<ScanScratch> s;
    {
        std::lock_guard<std::mutex> g(stream_scratch_mu());
        auto it = stream_scratch().find({device, stream});
        if (it == stream_scratch().end()) return 0;
        s = std::move(it->second);
        stream_scratch().erase(it);
    }
    return 1;   // freed (scan_scratch_free) when the last reference -- this one, or a scan_diag's -- drops
}

hipError_t launch_scan_frames(const uint8_t* wire, uint64_t len, uint64_t start, bool strict, uint64_t* hdr,
                              uint32_t* keys, uint8_t* b0, uint64_t max_frames, uint64_t* result,
                              hipStream_t stream, ScanScratch* own) {
    ScanArgs a;
    a.wire = wire;
    a.len = len;
    a.start = start;
    a.strict = 1;
    a.spec = strict ? 0 : 1;
    a.nc = (len + kChunk - 1) / kChunk;   // real chunks 0 .. nc-1; chunk nc is virtual (positions >= len)
    const uint64_t chunks = a.nc + 1, tiles = (chunks + kTileChunks - 1) / kTileChunks;
    a.hdr = hdr;
    a.keys = keys;
    a.b0 = b0;
    a.max_frames = max_frames;
    a.result = result;
    // scratch: sized for `cap` chunks (scratch_grow); the flags, the candidate counters
    // and the external flags must be zero when a call starts: a fresh allocation is
    // cleared once, and every call leaves them zeroed behind it (K3b the flags, K4 the
    // rest), so no clearing launch is needed per call.
    hipError_t e = hipSuccess;
    ScanScratch* sp = own;
    std::unique_lock<std::mutex> lk;
    if (!sp) {   // the public entry: scratch cached per (device, stream) until released
        int dev = 0;
        if ((e = hipGetDevice(&dev)) != hipSuccess) return e;
        lk = std::unique_lock<std::mutex>(stream_scratch_mu());
        std::shared_ptr<ScanScratch>& slot = stream_scratch()[{dev, stream}];
        if (!slot) {
            ScanScratch* fresh = scan_scratch_new();
            if (!fresh) return hipErrorOutOfMemory;
            slot = std::shared_ptr<ScanScratch>(fresh, scan_scratch_free);
        }
        sp = slot.get();
    }
    ScanScratch& s = *sp;
    if ((e = scratch_grow(s, chunks, stream)) != hipSuccess) return e;
    const Layout l = layout_for(s.cap);
    uint8_t* m = (uint8_t*)s.mem;
    if (s.dirty) {
        if ((e = hipMemsetAsync(m, 0, l.cleared, stream)) != hipSuccess) return e;
        s.dirty = false;
    }
    a.flags = (uint32_t*)(m + l.flags);
    a.ovf = a.flags + ((s.calls & 1) ? 2 : 0);
    a.ovf_prev = a.flags + ((s.calls & 1) ? 0 : 2);
    a.opfail = (uint32_t*)(m + l.opf) + ((s.calls & 1) ? kFailCopies * kFailStride : 0);
    a.opfail_prev = (uint32_t*)(m + l.opf) + ((s.calls & 1) ? 0 : kFailCopies * kFailStride);
    ++s.calls;
    // the one-pass path: knob SCAN_ONEPASS (0 never, 1 up to kOnePassCap, 2 up to kOnePassMax),
    // by default up to kOnePassMax of stream (config 2: 34.6-35.1 us against the graph path's
    // 41.5-41.8; a stream it cannot resolve pays its launch before the graph path).
    // Each call has its own epoch; when the 24-bit epoch wraps, the status words are cleared once,
    // so a word left from 2^24 calls ago cannot match.
    const int64_t op = knob(NETC_GPU_KNOB_SCAN_ONEPASS);
    const int64_t fuse = knob(NETC_GPU_KNOB_SCAN_FUSE);
    // A dense stream has a frame start in every chunk from the start on, so a caller whose frame
    // capacity is below that count (it expects larger frames) would only pay the launch (a 64 MiB
    // sample of config 4's mix: 46.0 against 35.9 us, r06t): no one-pass launch then.
    // ... and one expecting more than kOpDensest frames a chunk gets nothing from it either: each
    // chunk's thread walks its frames a hop at a time (uniform 128-B frames, ~30 a chunk: 111-118
    // against 86 us on the graph path; 16-B frames 390 against 270, r06x).
    const uint64_t span = (len - (start < len ? start : len)) / kChunk;
    const bool may_be_dense = max_frames >= span && max_frames <= kOpDensest * (span + 1);
    a.onepass = op != 0 && len <= (op == 1 ? kOnePassCap : kOnePassMax) && (may_be_dense || op > 0) ? 1 : 0;
    a.op_walk = op > 0 ? (uint64_t)kOpRec : kOpWalk;
    if (++s.epoch >= (1ull << 24) - 1) {   // (all-ones never: an exit-set entry's ~0 must not match)
        if ((e = hipMemsetAsync(m + l.st_t, 0, l.opfl - l.st_t, stream)) != hipSuccess) return e;
        s.epoch = 1;
    }
    a.epoch = s.epoch;
    a.st_t = (uint64_t*)(m + l.st_t);
    a.opfl = (uint64_t*)(m + l.opfl);
    a.st_g = (uint64_t*)(m + l.st_g);
    a.ccount = (uint32_t*)(m + l.ccount);
    a.ext = m + l.ext;
    a.tarr = (uint32_t*)(m + l.tarr);
    a.cand = (uint64_t*)(m + l.cand);
    a.link = (int32_t*)(m + l.link);
    a.nterm = (uint64_t*)(m + l.nterm);
    a.ncnt = (uint32_t*)(m + l.ncnt);
    a.wsum = (uint32_t*)(m + l.wsum);
    a.pbits = (uint32_t*)(m + l.pbits);
    a.anq = (uint32_t*)(m + l.anq);
    a.anc = (uint16_t*)(m + l.anc);
    a.anc_n = (uint32_t*)(m + l.anc_n);
    a.flist = (uint64_t*)(m + l.flist);
    a.text = (TileExt*)(m + l.text);
    a.tcount = (uint32_t*)(m + l.tcount);
    a.tinfo = (TileInfo*)(m + l.tinfo);
    a.anc_cap = s.cap;
    // tests: NETC_GPU_KNOB_SCAN_FAST_RANK = 0 sends every tile and stream through the generic
    // ranking loop; NETC_GPU_KNOB_SCAN_ANCHOR_SLOTS caps the anchor slots (0: none)
    a.fast_rank = knob(NETC_GPU_KNOB_SCAN_FAST_RANK) == 0 ? 0 : 1;
    if (const int64_t v = knob(NETC_GPU_KNOB_SCAN_ANCHOR_SLOTS); v >= 0)
        a.anc_cap = (uint64_t)v < a.anc_cap ? (uint64_t)v : a.anc_cap;
    a.pf_base = len >= 16 ? wire : m + l.flags;
    a.pf_lim = len >= 16 ? len - 16 : 0;
    const unsigned blk = (unsigned)((chunks + kBlkChunks - 1) / kBlkChunks);
    const dim3 g1((unsigned)((chunks + 3) / 4));
    if (len <= (128ull << 20)) {
        if (a.onepass) hipLaunchKernelGGL((scan_exits<false, true>), g1, dim3(256), 0, stream, a);
        else hipLaunchKernelGGL((scan_exits<false, false>), g1, dim3(256), 0, stream, a);
    } else {
        if (a.onepass) hipLaunchKernelGGL((scan_exits<true, true>), g1, dim3(256), 0, stream, a);
        else hipLaunchKernelGGL((scan_exits<true, false>), g1, dim3(256), 0, stream, a);
    }
#if defined(NETC_SCAN_K1_ONLY) || defined(NETC_SCAN_K1_EXP)
    return hipGetLastError();   // diagnostic builds only (tools/): K1 timed alone
#endif
    if (a.onepass) hipLaunchKernelGGL(scan_op_walk, dim3((unsigned)((chunks + kOpT - 1) / kOpT)), dim3(kOpT), 0, stream, a);
    // K2, K3a, K3b: by default K2 and then K3a + K3b as one launch up to kMergeTiles (256) tiles
    // (scan_tiles_resolve), three launches above.  NETC_GPU_KNOB_SCAN_FUSE (tests and A/B):
    // 0 three launches at every size; 1 K2 + K3a + K3b as one launch up to kFuseTiles tiles
    // (scan_links_fused.  Round 3 handed K2's outputs over with a release fence per block -- a
    // write-back of its XCD's L2 -- and measured 128 us against 43 us at config 2,
    // profiles/r03b_scan_fuse_ab.json.  Round 4 hands them over with sc1 stores and loads and no
    // fence (arrive_last), hand_st / hand_ld on this launch only: 56 against 41 us at config 2,
    // profiles/r04gg_scan_fuse_sc1.json; with the bodies inlined (no call, scratch 272 -> 36 B
    // per lane) 43.3 against 41.3 us at config 2, 96 against 82 us at config 4,
    // profiles/r04ii_scan_fuse.json -- the tiles' K3a still waits for each tile's slowest K2
    // block and K3b for the last tile, so the overlap saves little, while the launch runs at the
    // fused LDS footprint (4 blocks per CU against K2's 5).  Not the default.)
    const int64_t bk = knob(NETC_GPU_KNOB_SCAN_BLOCK_CHUNKS);
    const bool big = bk == kBlkChunksBig || (bk != kBlkChunks && chunks > kBigBlocksAbove);
    auto links = [&]() {
        if (big)
            hipLaunchKernelGGL(scan_links<kBlkChunksBig>, dim3((unsigned)((chunks + kBlkChunksBig - 1) / kBlkChunksBig)),
                               dim3(kScanT), 0, stream, a);
        else
            hipLaunchKernelGGL(scan_links<kBlkChunks>, dim3(blk), dim3(kScanT), 0, stream, a);
    };
    // the one-pass path: K2 + K3 fused by default (one gated launch; SCAN_FUSE 2: the split launches,
    // which measured 3.8 us slower at config 2 when the one-pass launch resolves the call, r06r)
    const bool fused = tiles <= (uint64_t)kFuseTiles && (fuse == 1 || (a.onepass && fuse < 0 && !big));
    if (fused) {   // (32 chunks per K2 block: the tiles' arrival counts)
        hipLaunchKernelGGL(scan_links_fused, dim3(blk), dim3(kScanT), 0, stream, a, tiles, blk);
    } else if (fuse != 0 && tiles <= (uint64_t)kMergeTiles) {
        links();
        hipLaunchKernelGGL(scan_tiles_resolve, dim3((unsigned)tiles), dim3(kScanT), 0, stream, a, tiles);
    } else {
        links();
        hipLaunchKernelGGL(scan_tiles, dim3((unsigned)tiles), dim3(kScanT), 0, stream, a);
        hipLaunchKernelGGL(scan_resolve, dim3(1), dim3(kResolveT), 0, stream, a, tiles);
    }
    if (big)
        hipLaunchKernelGGL(scan_emit<kBlkChunksBig>, dim3((unsigned)((chunks + kBlkChunksBig - 1) / kBlkChunksBig)),
                           dim3(kScanT), 0, stream, a, tiles);
    else
        hipLaunchKernelGGL(scan_emit<kEmitChunks>, dim3((unsigned)((chunks + kEmitChunks - 1) / kEmitChunks)), dim3(kScanT),
                           0, stream, a, tiles);
    e = hipGetLastError();
    if (e != hipSuccess) s.dirty = true;   // a launch failed: the flags may be left set (lock still held)
    return e;
}

}  // namespace netc_gpu
