// MI355X (gfx950 / CDNA4) frame-boundary scan — device kernels.
//
// Replaces the reference's header state machine (src/ws/common.c:146-296: byte 0
// FIN | RSV | opcode, byte 1 MASK | 7-bit length, 16 / 64-bit big-endian extended
// length, 4 key bytes) run over a received byte stream: it finds every frame of
// the stream (header offset, key, byte 0) in parallel.
//
// Frame starts form a chain: the next header follows the current frame's payload.
// The stream is cut into chunks of C bytes:
//   K1       per chunk, in LDS: every position that can start a header (strict
//            mode: passes the RFC checks on its first 2 bytes) is parsed once.  A
//            chain inside the chunk only steps between such positions, so the
//            distinct places where chains leave the chunk are the direct exits of
//            those positions; K1 publishes them as "candidate entries" of the
//            chunks they land in (the true chain enters each chunk at one of them).
//   K2       per candidate entry: its chain walked (header bytes from global
//            memory; past 64 frames K2' builds the chunk's 16-bit links in LDS,
//            doubles them to 8 / 16 hops and walks those, leaving an anchor every
//            8 frames for K4b') to the candidate it exits to: a graph of a few nodes
//            per chunk whose path from the stream start is the true chain, one node
//            per chunk it enters.
//   K3       pointer doubling over that graph, marking the nodes reachable from
//            the start node (log2(chunks) passes);
//   K4       per chunk: the true entry (its marked node) and its frame count from
//            K2, a chained scan of the counts (decoupled look-back), and a walk that
//            writes the descriptors (K4b'; past 64 frames one wavefront per chunk,
//            a lane per K2' anchor).
// Garbage chains (payload bytes parsed as headers) die within a hop or two under
// the strict checks, so chunks have few distinct exits; a stream whose exits
// overflow the fixed capacities (adversarial payloads) is finished by a serial
// walk in K4 instead — same results, slower.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <map>
#include <mutex>
#include <new>
#include <vector>
#include <utility>

#include "gpu_util.h"
#include "ws_mask_gpu.h"

namespace netc_gpu {

static constexpr uint64_t kChunk = 4096;        // bytes per chunk (LDS: bytes + 8 B link per byte)
static constexpr int kScanT = 256;              // threads per K1 / K2 block
static constexpr int kPer = (int)(kChunk / kScanT);
static constexpr int kCand = 8;                 // candidate entries per chunk
static constexpr int kSet = 64;                 // distinct exits per chunk
static constexpr uint64_t kTerm = 1ull << 63;   // link is terminal
static constexpr uint64_t kPosMask = (1ull << 61) - 1;
enum : uint64_t { kExit = 0, kEnd = 1, kDead = 2 };

__device__ __forceinline__ uint64_t term(uint64_t type, uint64_t pos) { return kTerm | type << 61 | pos; }
__device__ __forceinline__ uint64_t term_type(uint64_t v) { return (v >> 61) & 3; }
__device__ __forceinline__ uint64_t term_pos(uint64_t v) { return v & kPosMask; }

struct ScanArgs {
    const uint8_t* wire;
    uint64_t len;          // stream bytes
    uint64_t start;        // offset of the first header
    uint64_t nc;           // chunks (the last one, index nc, is virtual: positions >= len)
    int strict;
    uint32_t* ccount;      // nc + 1 candidate counters (zeroed per call)
    uint64_t* cand;        // (nc + 1) * kCand candidate positions
    int32_t* link;         // (nc + 1) * kCand: node -> next node, -1 = chain ends
    uint64_t* nterm;       // (nc + 1) * kCand: the terminal where the node's walk leaves its chunk
    uint32_t* ncnt;        // (nc + 1) * kCand: frames on that walk (~0: not counted, K2')
    uint8_t* mark;         // (nc + 1) * kCand: node is on the chain from the stream start
    uint32_t* flags;       // [0] overflow, [1] root node, [3] / [4] entries of slow2 / slow3
    uint32_t* slow2;       // K2 nodes left to the LDS kernel ((nc + 1) * kCand)
    uint32_t* slow3;       // K4 chunks of many frames left to the LDS emit kernel (nc + 1)
    uint64_t* cbase;       // K4: index of each chunk's first frame (nc + 1)
    uint16_t* anc;         // K2' -> K4b': 16-frame anchors of K2' slot q at anc[q * kAncSlot]
    uint32_t* anc_n;       // anchors in slot q
    uint32_t* anq;         // per node: its K2' slot (this call), or ~0 when none was left
    uint64_t anc_cap;      // anchor slots
    uint64_t* status;      // chained-scan status words (nc + 1)
    uint32_t epoch;
    uint64_t* hdr;         // outputs
    uint32_t* keys;
    uint8_t* b0;
    uint64_t max_frames;
    uint64_t* result;      // [0] frames, [1] consumed, [2] error offset or ~0
};

// One header at stream position p (bytes b[0..13] from p; bytes past len unused).
// Returns the link: the next header position, or a terminal.
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
        if (!mask || (first & 0x70) || reserved || (control && (!(first & 0x80) || plen > 125)) || (plen >> 63))
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
    return !(second & 0x80) || (first & 0x70) || reserved || (opcode >= 8 && !(first & 0x80));
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
    const bool dead = (a.strict != 0) & ((mask == 0) | ((first & 0x70) != 0) | reserved |
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
// of K2 and K4 touch only the header bytes of the frames they visit,
// so they read them where they lie instead of staging the chunk in LDS.
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
__device__ uint64_t walk_frames(const ScanArgs& a, uint64_t B, const uint32_t* words, uint64_t e, int hops, F&& emit) {
    const uint64_t Bend = B + kChunk;
    uint64_t p = e;
    for (int h = 0;; ++h) {
        if (p >= Bend) return term(kExit, p);
        if (h == hops) return 0;
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
// frame (the checks of quick_reject, SWAR).
__device__ __forceinline__ uint32_t quick_ok4(uint32_t x, uint32_t y) {
    const uint32_t H = 0x80808080u;
    const uint32_t rsv_ok = ~((x & 0x70707070u) + 0x70707070u) & H;   // bits 4-6 clear
    const uint32_t op_ok = ~((x << 5) | ((x << 7) & (x << 6))) & H;    // opcode & 7 in {0, 1, 2}
    const uint32_t ctl_bad = (x << 4) & ~x & H;                        // opcode >= 8 without FIN
    return y & rsv_ok & op_ok & ~ctl_bad & H;
}

// x into the chunk's LDS set of distinct exits (open addressing); *overflow when full
__device__ __forceinline__ void set_insert(unsigned long long* set, uint64_t x, int* overflow) {
    uint32_t h = (uint32_t)((x * 0x9E3779B97F4A7C15ull) >> 58);
    for (int tries = 0; tries < kSet; ++tries, h = (h + 1) & (kSet - 1)) {
        const unsigned long long cur = set[h];
        if (cur == x) return;
        if (cur == ~0ull) {
            const unsigned long long prev = atomicCAS(&set[h], ~0ull, (unsigned long long)x);
            if (prev == ~0ull || prev == x) return;
        }
    }
    *overflow = 1;
}

static constexpr int kWalkHops = 32;   // K1 / K2: hop budget of a direct chain walk

// publish a chunk's distinct exits as candidates of the chunks they land in, and the
// stream start as the candidate (root) of its chunk.  Strict mode prunes exits that
// cannot start a frame (2 header bytes fail the checks): payload bytes parsed as a
// chain land on random positions, and a random position passes with ~2 % odds,
// while the true chain always lands on a real header.  This keeps the candidate
// lists at about one entry per chunk.
__device__ __forceinline__ void publish_exits(const ScanArgs& a, uint64_t chunk, const unsigned long long* set,
                                              int overflow, int tid) {
    auto append = [&](uint64_t x) {
        const uint64_t t = x / kChunk;   // x <= len: t <= nc
        const uint32_t slot = atomicAdd(&a.ccount[t], 1u);
        if (slot < (uint32_t)kCand) a.cand[t * kCand + slot] = x;
        else atomicOr(&a.flags[0], 1u);
    };
    if (tid < kSet && set[tid] != ~0ull && !quick_reject(a, set[tid])) append(set[tid]);
    if (tid == 0) {
        if (overflow) atomicOr(&a.flags[0], 1u);
        if (a.start / kChunk == chunk) append(a.start);
    }
}

// K1: distinct exits of each chunk.  The chunk's candidates -- strict mode: the
// positions passing the quick check on their 2 first bytes (~2 % of payload
// positions, and every real header); otherwise every position -- are each parsed
// once, from the chunk's LDS copy.
__global__ __launch_bounds__(kScanT) void scan_exits(ScanArgs a) {
    __shared__ uint32_t words[kWords];
    __shared__ unsigned long long set[kSet];
    __shared__ int overflow;
    __shared__ uint16_t queue[kScanT / kWave][kChunk / (kScanT / kWave)];   // per wave: its candidates
    const uint64_t chunk = blockIdx.x;
    const uint64_t B = chunk * kChunk;
    const int tid = threadIdx.x;
    if (tid < kSet) set[tid] = ~0ull;
    if (tid == 0) overflow = 0;
    if (chunk == 0 && tid == 0) a.flags[4] = 0;   // K4b''s queue length, left set by the previous call
    load_chunk(a, B, words);   // 4 KiB in LDS: the walks' hops are LDS reads
    // this thread's kPer positions and the 4 bytes after them
    const uint64_t p0 = B + (uint64_t)kPer * tid;
    uint32_t w[kPer / 4 + 1];
#pragma unroll
    for (int k = 0; k < kPer / 4 + 1; ++k) w[k] = words[kPer / 4 * tid + k];
    // the quick check four positions at a time (bit 7 of each byte: position passes),
    // the four results interleaved into one word: bit 8 j + k <-> position 4 k + j;
    // without the strict checks every position is a candidate
    uint32_t cand = 0x0F0F0F0Fu;
    if (a.strict) {
        cand = 0;
#pragma unroll
        for (int k = 0; k < kPer / 4; ++k)
            cand |= quick_ok4(w[k], __builtin_amdgcn_alignbyte(w[k + 1], w[k], 1)) >> (7 - k);
    }
    // positions before the stream start or past its end are not candidates (only the
    // chunks holding either end: a wave-uniform test)
    if (B < a.start || B + kChunk > a.len) {
#pragma unroll
        for (int i = 0; i < kPer; ++i)
            if (p0 + i < a.start || p0 + i >= a.len) cand &= ~(1u << (8 * (i & 3) + (i >> 2)));
    }
    // the wavefront's candidates into its LDS queue (~2 % of positions pass, 0-3 per
    // lane), then parsed round-robin by its lanes
    const int lane = tid & (kWave - 1);
    uint16_t* q = queue[tid / kWave];
    const uint32_t mine = __popc(cand);
    uint32_t incl = mine;   // inclusive prefix of the counts over the wave
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
        const uint32_t o = __shfl_up(incl, d, kWave);
        if (lane >= d) incl += o;
    }
    const uint32_t total = __shfl(incl, kWave - 1, kWave);
    uint32_t at = incl - mine;
    for (uint32_t c = cand; c; c &= c - 1) {
        const int b = __builtin_ctz(c);
        q[at++] = (uint16_t)(kPer * tid + 4 * (b & 7) + (b >> 3));
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    // Each candidate is parsed once.  A chain inside the chunk moves from candidate
    // to candidate (a position that fails the quick check would parse DEAD), so a
    // chain leaves the chunk exactly where its last candidate's own frame does: the
    // chunk's exits are the direct exits of its candidates, and no chain is walked.
    // (An earlier form walked every candidate's chain to the chunk end, and handed
    // chunks of tiny frames, whose chains outran the hop budget, to an LDS
    // pointer-jumping kernel -- also the whole non-strict path.)
    const uint64_t Bend = B + kChunk;
    for (uint32_t i = lane; i < total; i += kWave) {
        const uint64_t p = B + q[i];
        const uint64_t v = parse_at(a, p, window_at(words, (int)(p - B)), nullptr, nullptr);
        if (!(v & kTerm) && v >= Bend) set_insert(set, v, &overflow);
    }
    __syncthreads();
    publish_exits(a, chunk, set, overflow, tid);
}

// node -> the candidate its chain exits to (or -1) and the terminal where it ends
__device__ __forceinline__ void link_node(const ScanArgs& a, uint64_t node, uint64_t x, uint64_t v, uint32_t cnt) {
    if (x == a.start) {
        a.flags[1] = (uint32_t)node;
        a.mark[node] = 1;
    }
    int32_t next = -1;
    if (term_type(v) == kExit) {
        const uint64_t y = term_pos(v), t = y / kChunk;
        const uint32_t cnt = min(a.ccount[t], (uint32_t)kCand);
        for (uint32_t i = 0; i < cnt; ++i)
            if (a.cand[t * kCand + i] == y) next = (int32_t)(t * kCand + i);
        // not a candidate: pruned by K1 (the chain dies at y), or its bucket overflowed
        if (next < 0 && !quick_reject(a, y)) atomicOr(&a.flags[0], 1u);
    }
    a.link[node] = next;
    a.nterm[node] = v;
    a.ncnt[node] = cnt;
}

// K2' / K4b': every position of the chunk that can start a header (strict: passes
// the quick check; else every position) parsed once into a 16-bit in-chunk link
// (kNoLink: the chain ends or leaves the chunk there), then four doubling passes:
// returns the 16-hop links (l1 keeps the 1-hop ones, lj the 8-hop ones).  The caller
// has loaded words.
static constexpr uint16_t kNoLink = 0xFFFF;
static constexpr int kStride = 16;   // hops per 16-hop link
static constexpr int kAncStride = 8;                              // frames per K2' anchor
static constexpr int kAncMax = (int)(kChunk / 2 / kAncStride) + 1;   // a frame is 2 bytes or more
static constexpr int kAncSlot = kAncMax + 1;                         // uint16 per slot (4-byte multiple)

__device__ const uint16_t* chunk_links16(const ScanArgs& a, uint64_t B, const uint32_t* words, uint16_t* l1,
                                         uint16_t* lj, uint16_t* lk16) {
    const int tid = threadIdx.x;
    const uint64_t Bend = B + kChunk;
    const int i0 = kPer * tid;
    uint32_t w[kPer / 4 + 1];
#pragma unroll
    for (int k = 0; k < kPer / 4 + 1; ++k) w[k] = words[i0 / 4 + k];
    auto byte_at = [&](int j) { return (w[j >> 2] >> (8 * (j & 3))) & 0xFFu; };
    uint32_t cand = 0;   // this thread's positions that can start a header
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
        const uint32_t first = byte_at(j), second = byte_at(j + 1), opcode = first & 0x0F;
        const bool reserved = (opcode >= 3 && opcode <= 7) || opcode >= 11;
        const bool reject =
            a.strict && (!(second & 0x80) || (first & 0x70) || reserved || (opcode >= 8 && !(first & 0x80)));
        if (!reject) cand |= 1u << j;
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

// K2: one thread per node (candidate slot): the candidate entry's chain walked from
// global memory to the candidate it exits to; a chain longer than kWalkHops goes
// to K2' (LDS).  Unused slots hold stale values from earlier calls: dead ends.
__global__ __launch_bounds__(256) void scan_links(ScanArgs a) {
    const uint64_t node = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t chunk = node / kCand;
    if (chunk > a.nc) return;
    const uint32_t i = (uint32_t)(node % kCand);
    if (i >= min(a.ccount[chunk], (uint32_t)kCand)) {
        a.link[node] = -1;
        return;
    }
    const uint64_t B = chunk * kChunk;
    const uint64_t x = a.cand[node];
    uint32_t cnt = 0;   // K4 takes the frame count of the true entry's walk from here
    const uint64_t v = x - B < kChunk ? walk_frames<false>(a, B, nullptr, x, 2 * kWalkHops,
                                                           [&](uint64_t, uint32_t, uint8_t) { ++cnt; })
                                      : term(kEnd, x);   // x == len on a chunk edge
    if (v == 0) {
        a.slow2[atomicAdd(&a.flags[3], 1u)] = (uint32_t)node;
        return;
    }
    link_node(a, node, x, v, cnt);
}

// K2': the nodes K2 left (chains of more than 2 kWalkHops frames in the chunk): the
// chunk's 16-hop links built in LDS, then one thread walks them from the entry --
// count / 16 + at most 15 hops -- and re-parses the last header for the exact
// terminal (EXIT to the next chunk, END or DEAD) and whether it adds a frame.
__global__ __launch_bounds__(kScanT) void scan_links_lds(ScanArgs a) {
    __shared__ uint32_t words[kWords];
    __shared__ uint16_t l1[kChunk];
    __shared__ uint16_t lj[kChunk];
    __shared__ uint16_t lk16[kChunk];
    const uint64_t count = __hip_atomic_load(&a.flags[3], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (uint64_t q = blockIdx.x; q < count; q += gridDim.x) {
        const uint64_t node = a.slow2[q], chunk = node / kCand, B = chunk * kChunk;
        load_chunk(a, B, words);
        chunk_links16(a, B, words, l1, lj, lk16);
        const uint16_t* l8 = lj;   // the 8-hop links (the pass before the last)
        if (threadIdx.x == 0) {
            const uint64_t x = a.cand[node];   // in [B, B + kChunk): K2's walk started there
            uint32_t p = (uint32_t)(x - B), hops = 0;
            // the walk's positions every 8 frames are K4b's anchors if this node turns out
            // to be its chunk's true entry: kept in slot q while slots last
            const bool keep = q < a.anc_cap;
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
            link_node(a, node, x, v, hops);
        }
        __syncthreads();
    }
}

// K3, pass k: src = J (the 8^k-th successor; J = link in pass 0).  Builds J^8 into
// dst (unless last) and marks the J .. J^7 successors of every marked node: after
// pass k every node within 8^(k+1) - 1 steps of the start is marked (a node d
// steps away is 0..7 J-steps past a node marked before the pass), so after
// ceil(log8(chunks)) passes exactly the chain's nodes are (one per chunk it
// enters).  The passes are launch-bound, hence 3 doubling levels each.  Marks set
// during a pass may be followed in the same pass: they are on the chain too.
__global__ void scan_lift(const int32_t* src, int32_t* dst, uint8_t* mark, uint64_t nodes) {
    const uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= nodes) return;
    auto step = [&](int32_t u) -> int32_t {   // (range check: defence in depth)
        return (u >= 0 && (uint64_t)u < nodes) ? src[u] : -1;
    };
    const bool marked = mark[v] != 0;
    int32_t u = step((int32_t)v);
#pragma unroll
    for (int h = 1; h < 8; ++h) {   // u = J^h(v)
        if (marked && u >= 0 && (uint64_t)u < nodes) mark[u] = 1;
        u = step(u);
    }
    if (dst) dst[v] = u;   // J^8(v)
}

__device__ __forceinline__ uint64_t cand_pos(const ScanArgs& a, int32_t node) { return a.cand[node]; }

static constexpr int kEmitHops = 64;   // K4: a chunk of more frames is emitted from LDS

// the marked (true) entry of a chunk: its node, or -1
__device__ __forceinline__ int64_t chunk_entry(const ScanArgs& a, uint64_t chunk) {
    int64_t enode = -1;
    const uint32_t cnt = min(a.ccount[chunk], (uint32_t)kCand);
    for (uint32_t i = 0; i < cnt; ++i)
        if (a.mark[chunk * kCand + i]) enode = (int64_t)(chunk * kCand + i);
    return enode;
}

// exclusive prefix sum over a 256-thread block; the block total in *total
__device__ uint64_t block_scan256(uint64_t v, uint64_t* total) {
    __shared__ uint64_t wsum[4];
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
    for (int i = 0; i < 4; ++i) {
        before += i < w ? wsum[i] : 0;
        all += wsum[i];
    }
    __syncthreads();
    *total = all;
    return before + inc - v;
}

// K4a: one thread per chunk.  The chain's frames in the chunk are the frames K2
// counted on its marked entry's walk; a chained scan over tiles of 256 chunks
// (decoupled look-back) gives each chunk's first frame index.  The chunk where
// the chain ends sets the results.  On candidate overflow, one thread walks the
// whole stream instead (serial fallback).
// The chunk's candidate counter and mark bytes are read here for the last time: the
// thread zeroes them, so the next call on this scratch needs no clearing launch.
__device__ __forceinline__ void clear_chunk(const ScanArgs& a, uint64_t chunk) {
    a.ccount[chunk] = 0;
    *(uint64_t*)(a.mark + chunk * kCand) = 0;   // kCand == 8 mark bytes, 8-aligned
}

__global__ __launch_bounds__(256) void scan_count(ScanArgs a) {
    __shared__ uint64_t tile_prefix;
    const uint64_t tile = blockIdx.x;
    const uint64_t chunk = tile * 256 + threadIdx.x;
    if (__hip_atomic_load(&a.flags[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) {
        if (chunk <= a.nc) clear_chunk(a, chunk);
        if (tile == 0 && threadIdx.x == 0) {
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
        return;
    }
    const int64_t enode = chunk <= a.nc ? chunk_entry(a, chunk) : -1;
    if (chunk <= a.nc) clear_chunk(a, chunk);
    const uint64_t count = enode >= 0 ? a.ncnt[enode] : 0;
    uint64_t agg;
    const uint64_t ex = block_scan256(count, &agg);
    if (threadIdx.x < kWave) {
        const int lane = threadIdx.x;
        if (lane == 0)
            __hip_atomic_store(&a.status[tile], status_word(tile == 0 ? 2 : 1, a.epoch, agg), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        const uint64_t prefix = tile == 0 ? 0 : look_back(a.status, (int64_t)tile, a.epoch, lane);
        if (lane == 0) {
            if (tile)
                __hip_atomic_store(&a.status[tile], status_word(2, a.epoch, prefix + agg), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            tile_prefix = prefix;
        }
    }
    __syncthreads();
    if (chunk > a.nc) return;
    const uint64_t base = tile_prefix + ex;
    a.cbase[chunk] = base;
    if (chunk == a.nc) a.result[0] = base + count;
    if (enode < 0) return;
    // the chain ends in this chunk, or leaves it onto a header K1 pruned
    uint64_t stop = a.nterm[enode];
    if (term_type(stop) == kExit && quick_reject(a, term_pos(stop))) stop = term(kDead, term_pos(stop));
    if (term_type(stop) != kExit) {
        const uint64_t end = term_pos(stop), k = base + count;
        a.result[1] = end;
        a.result[2] = term_type(stop) == kDead ? end : ~0ull;
        if (k <= a.max_frames) a.hdr[k] = end;
    }
    // K4b, in the same thread now that the base is known: the chunk's frames walked
    // from global memory (header bytes only), descriptors from the base on; a chunk
    // of more than kEmitHops frames goes to K4b' (LDS)
    if (count > (uint64_t)kEmitHops) {
        a.slow3[atomicAdd(&a.flags[4], 1u)] = (uint32_t)enode;   // the node: its mark is gone
        return;
    }
    uint64_t k = base;
    walk_frames<false>(a, chunk * kChunk, nullptr, a.cand[enode], -1, [&](uint64_t p, uint32_t key, uint8_t b0) {
        if (k < a.max_frames) {
            a.hdr[k] = p;
            a.keys[k] = key;
            a.b0[k] = b0;
        }
        ++k;
    });
}

// K4b' for the chunks whose entry K2' left anchors for (all of them unless the anchor
// slots ran out): one wavefront per chunk, lane t parses the kAncStride frames from
// anchor t, header bytes straight from global memory, and writes their descriptors
// from index cbase + kAncStride t.  No LDS: the chunk is never reloaded.  Runs at the
// start of scan_emit_lds (one launch fewer: at C2 shape nothing is queued at all).
__device__ void emit_anchored(const ScanArgs& a, uint64_t count) {
    const int lane = threadIdx.x & (kWave - 1);
    const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x / kWave);
    const uint64_t wave = (uint64_t)blockIdx.x * (blockDim.x / kWave) + threadIdx.x / kWave;
    for (uint64_t q = wave; q < count; q += nwaves) {
        const uint64_t node = a.slow3[q];
        const uint32_t slot = a.anq[node];
        if (slot == ~0u) continue;   // scan_emit_lds takes it
        const uint64_t chunk = node / kCand, B = chunk * kChunk, Bend = B + kChunk;
        const int na = (int)a.anc_n[slot];
        const uint64_t base = a.cbase[chunk];
        for (int t = lane; t < na; t += kWave) {
            uint64_t k = base + (uint64_t)t * kAncStride;
            uint64_t pos = B + a.anc[(uint64_t)slot * kAncSlot + t];
            for (int h = 0; h < kAncStride && pos < Bend; ++h) {
                uint32_t key;
                uint8_t b0;
                const uint64_t v = parse_at(a, pos, window_global(a, pos), &key, &b0);
                if (v & kTerm) break;
                if (k < a.max_frames) {
                    a.hdr[k] = pos;
                    a.keys[k] = key;
                    a.b0[k] = b0;
                }
                ++k;
                pos = v;
            }
        }
    }
}

// K4b': the chunks of many (tiny) frames, emitted from LDS in parallel.  Every
// position of the chunk that can start a header is parsed once into a 16-bit
// in-chunk link (kNoLink: the chain ends or leaves the chunk there); four doubling
// passes make the 16-hop links; one thread walks those from the entry, leaving an
// anchor every 16 frames; then thread t walks 16 frames from anchor t and writes
// their descriptors from index cbase + 16 t.  Serial depth count / 16 + 16 hops
// instead of count (a 4 KiB chunk of 16-B frames holds ~186).
// The last kernel of a scan: it also zeroes flags 0-3 for the next call (no longer
// read here; flag 4, this kernel's own queue length, is zeroed by the next call's K1,
// which runs before anything counts into it).  A last-block-done counter instead cost
// 1,024 same-address atomics per call (~10 us).
__global__ __launch_bounds__(kScanT) void scan_emit_lds(ScanArgs a) {
    __shared__ uint32_t words[kWords];
    __shared__ uint16_t l1[kChunk];    // next header (local index) or kNoLink
    __shared__ uint16_t lj[kChunk];    // 2^k hops (ping)
    __shared__ uint16_t lk16[kChunk];  // 2^k hops (pong); 16 hops after the last pass
    __shared__ uint16_t anchor[kChunk / kStride + 1];
    __shared__ int nanchor;
    const int tid = threadIdx.x;
    const uint64_t count = __hip_atomic_load(&a.flags[4], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (blockIdx.x == 0 && tid == 0)
        for (int i = 0; i < 4; ++i) a.flags[i] = 0;
    emit_anchored(a, count);
    for (uint64_t q = blockIdx.x; q < count; q += gridDim.x) {
        const uint64_t node = a.slow3[q], chunk = node / kCand, B = chunk * kChunk, Bend = B + kChunk;
        if (a.anq[node] != ~0u) continue;   // anchored: emit_anchored wrote it
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
        const uint64_t base = a.cbase[chunk];
        for (int t = tid; t < na; t += kScanT) {
            uint64_t k = base + (uint64_t)t * kStride;
            uint64_t pos = B + anchor[t];
            for (int h = 0; h < kStride && pos < Bend; ++h) {
                uint32_t key;
                uint8_t b0;
                const uint64_t v = parse_at(a, pos, window_at(words, (int)(pos - B)), &key, &b0);
                if (v & kTerm) break;
                if (k < a.max_frames) {
                    a.hdr[k] = pos;
                    a.keys[k] = key;
                    a.b0[k] = b0;
                }
                ++k;
                pos = v;
            }
        }
        __syncthreads();
    }
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
    uint32_t epoch = 0;
    bool dirty = false;    // a call did not launch all its kernels: clear before the next
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
std::map<std::pair<int, hipStream_t>, ScanScratch*>& stream_scratch() {
    static std::map<std::pair<int, hipStream_t>, ScanScratch*> m;
    return m;
}
std::mutex& stream_scratch_mu() {
    static std::mutex mu;
    return mu;
}
}  // namespace

// bytes of scratch for `c` chunks: flags, ccount, mark, cand, link, nterm, ncnt, status, jp, jq,
// slow2, slow3, cbase, anc (one anchor slot per chunk), anc_n, anq
static uint64_t scratch_need(uint64_t c) {
    const uint64_t n = c * kCand;
    return 64 + c * 4 + n + n * 8 + n * 4 + n * 8 + n * 4 + c * 8 + n * 4 + n * 4 + n * 4 + c * 4 + c * 8 +
           c * kAncSlot * 2 + c * 4 + n * 4 + 64 * 16;   // + alignment padding of the 16 regions
}

// grow to hold `chunks` (+1 virtual) chunks; outgrown allocations are kept until the
// scratch is freed (queued work may still use them)
static hipError_t scratch_grow(ScanScratch& s, uint64_t chunks, hipStream_t stream) {
    if (s.cap >= chunks) return hipSuccess;
    uint64_t cap = s.cap ? 2 * s.cap : 256;
    while (cap < chunks) cap *= 2;
    const uint64_t want = scratch_need(cap);
    void* p = nullptr;
    hipError_t e;
    if ((e = hipMalloc(&p, want)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(p, 0, want, stream)) != hipSuccess) {   // zero flags, epoch 0
        (void)hipFree(p);
        return e;
    }
    if (s.mem) s.retired.push_back(s.mem);
    s.mem = p;
    s.bytes = want;
    s.cap = cap;
    s.epoch = 0;
    s.dirty = false;
    return hipSuccess;
}

hipError_t scan_scratch_reserve(ScanScratch* s, uint64_t len, hipStream_t stream) {
    return scratch_grow(*s, (len + kChunk - 1) / kChunk + 1, stream);
}

int release_stream_scratch(int device, hipStream_t stream) {
    ScanScratch* s = nullptr;
    {
        std::lock_guard<std::mutex> g(stream_scratch_mu());
        auto it = stream_scratch().find({device, stream});
        if (it == stream_scratch().end()) return 0;
        s = it->second;
        stream_scratch().erase(it);
    }
    scan_scratch_free(s);
    return 1;
}


// workgroups of the LDS kernels K2' / K4b' (each loops over its queue); the queue
// lengths are only known on the device.  NETC_SCAN_SLOW_BLOCKS overrides (measurement).
static uint64_t slow_blocks() {
    const char* e = getenv("NETC_SCAN_SLOW_BLOCKS");
    const uint64_t v = e ? (uint64_t)strtoull(e, nullptr, 10) : 0;
    return v ? v : 1024;
}

hipError_t launch_scan_frames(const uint8_t* wire, uint64_t len, uint64_t start, bool strict, uint64_t* hdr,
                              uint32_t* keys, uint8_t* b0, uint64_t max_frames, uint64_t* result,
                              hipStream_t stream, ScanScratch* own) {
    ScanArgs a;
    a.wire = wire;
    a.len = len;
    a.start = start;
    a.strict = strict ? 1 : 0;
    a.nc = (len + kChunk - 1) / kChunk;   // real chunks 0 .. nc-1; chunk nc is virtual (positions >= len)
    const uint64_t chunks = a.nc + 1, nodes = chunks * kCand;
    int levels = 1;   // lifting passes: 8^levels - 1 >= chunks steps along the chain
    while ((1ull << (3 * levels)) < chunks + 1) ++levels;
    a.hdr = hdr;
    a.keys = keys;
    a.b0 = b0;
    a.max_frames = max_frames;
    a.result = result;
    // scratch: sized for `cap` chunks (scratch_grow); the flags, the candidate counters
    // and the mark bytes must be zero when a call starts: a fresh allocation is cleared
    // once, and every call leaves them zeroed behind it (K4a and K4b' clear them), so
    // no clearing launch is needed per call.
    hipError_t e = hipSuccess;
    ScanScratch* sp = own;
    std::unique_lock<std::mutex> lk;
    if (!sp) {   // the public entry: scratch cached per (device, stream) until released
        int dev = 0;
        if ((e = hipGetDevice(&dev)) != hipSuccess) return e;
        lk = std::unique_lock<std::mutex>(stream_scratch_mu());
        ScanScratch*& slot = stream_scratch()[{dev, stream}];
        if (!slot && !(slot = scan_scratch_new())) return hipErrorOutOfMemory;
        sp = slot;
    }
    uint8_t* m;
    int32_t *jp, *jq;   // ping-pong doubling tables
    uint64_t cleared = 0;
    bool* dirty_flag = nullptr;
    {
        ScanScratch& s = *sp;
        if ((e = scratch_grow(s, chunks, stream)) != hipSuccess) return e;
        s.epoch = (s.epoch + 1) & 0xFFFF;
        m = (uint8_t*)s.mem;
        auto align = [](uint64_t x) { return (x + 63) & ~63ull; };
        const uint64_t cap_nodes = s.cap * kCand;
        uint64_t o = 0;
        // flags, ccount and mark first, at capacity offsets: the region left zeroed
        a.flags = (uint32_t*)(m + o); o = 64;
        a.ccount = (uint32_t*)(m + o); o = align(o + s.cap * 4);
        a.mark = m + o; o = align(o + cap_nodes);
        cleared = o;
        if (s.dirty) {
            if ((e = hipMemsetAsync(m, 0, cleared, stream)) != hipSuccess) return e;
            s.dirty = false;
        }
        dirty_flag = &s.dirty;
        a.cand = (uint64_t*)(m + o); o = align(o + cap_nodes * 8);
        a.link = (int32_t*)(m + o); o = align(o + cap_nodes * 4);
        a.nterm = (uint64_t*)(m + o); o = align(o + cap_nodes * 8);
        a.ncnt = (uint32_t*)(m + o); o = align(o + cap_nodes * 4);
        a.status = (uint64_t*)(m + o); o = align(o + s.cap * 8);
        jp = (int32_t*)(m + o); o = align(o + cap_nodes * 4);
        jq = (int32_t*)(m + o); o = align(o + cap_nodes * 4);
        a.slow2 = (uint32_t*)(m + o); o = align(o + cap_nodes * 4);
        a.slow3 = (uint32_t*)(m + o); o = align(o + s.cap * 4);
        a.cbase = (uint64_t*)(m + o); o = align(o + s.cap * 8);
        a.anc = (uint16_t*)(m + o); o = align(o + s.cap * kAncSlot * 2);
        a.anc_n = (uint32_t*)(m + o); o = align(o + s.cap * 4);
        a.anq = (uint32_t*)(m + o);
        a.anc_cap = s.cap;
        if (const char* env = getenv("NETC_SCAN_ANCHOR_SLOTS")) {   // tests: fewer slots (0: none)
            const uint64_t v = (uint64_t)strtoull(env, nullptr, 10);
            a.anc_cap = v < a.anc_cap ? v : a.anc_cap;
        }
        if (o + cap_nodes * 4 > s.bytes) return hipErrorInvalidValue;   // layout and need_for disagree
        if (s.epoch == 0) {   // epochs wrapped: clear the status words
            if ((e = hipMemsetAsync(a.status, 0, s.cap * 8, stream)) != hipSuccess) return e;
            s.epoch = 1;
        }
        a.epoch = s.epoch;
    }
    (void)cleared;
    const uint64_t slow_cap = slow_blocks();
    const unsigned slow_grid = (unsigned)(chunks < slow_cap ? chunks : slow_cap);
    hipLaunchKernelGGL(scan_exits, dim3((unsigned)chunks), dim3(kScanT), 0, stream, a);
    hipLaunchKernelGGL(scan_links, dim3((unsigned)((nodes + 255) / 256)), dim3(256), 0, stream, a);
    hipLaunchKernelGGL(scan_links_lds, dim3(slow_grid), dim3(kScanT), 0, stream, a);
    const unsigned lb = (unsigned)((nodes + 255) / 256);
    const int32_t* src = a.link;
    for (int k = 0; k < levels; ++k) {
        int32_t* dst = k + 1 < levels ? ((k & 1) ? jq : jp) : nullptr;
        hipLaunchKernelGGL(scan_lift, dim3(lb), dim3(256), 0, stream, src, dst, a.mark, nodes);
        src = dst;
    }
    const unsigned cb = (unsigned)((chunks + 255) / 256);
    hipLaunchKernelGGL(scan_count, dim3(cb), dim3(256), 0, stream, a);
    hipLaunchKernelGGL(scan_emit_lds, dim3(slow_grid), dim3(kScanT), 0, stream, a);
    e = hipGetLastError();
    if (e != hipSuccess) *dirty_flag = true;   // a launch failed: the flags may be left set (lock still held)
    return e;
}

}  // namespace netc_gpu
