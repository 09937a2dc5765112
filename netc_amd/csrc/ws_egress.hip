// Host-resident messages framed and masked on the GPU into a pinned ring, then sent on a socket:
// include/ws/egress.h (SURVEY.md §8(f) row 2 from a caller's host buffers).
//
// The reference frames a message per frame with three copies and a byte loop
// (ws_send_message, src/ws/common.c:96-119) and one send() per frame (:121).  Here a
// message is appended to a page-locked payload slot (the one host copy) while its frame
// table -- payload offsets, key32, header byte 0 per frame, the reference's split
// (:42-49) -- is written beside it.  Per submitted slot, on the slot's own HIP stream:
//
//   H2D     the payload bytes, then the packed table (offsets | keys | header bytes: one copy)
//   encode  launch_encode_frames (ws_frame_gpu.hip): wire offsets, then every frame's header,
//           key and masked payload back to back -- one launch when every frame of the slot is
//           in one length class (the host saw each length: the offsets are affine, no scan)
//   D2H     the wire bytes into the slot's page-locked wire buffer (the host knows their
//           count: it summed the header lengths while queueing) and the device's own wire
//           length beside them, checked against it when the slot is taken; event "done"
//
// Slots are independent (each frame's wire position depends only on its own slot), so the
// next slot fills while this one is on the GPU and an older one goes out on the socket.
#include <hip/hip_runtime.h>

#include <errno.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/uio.h>

#include <new>

#include "ws_mask_gpu.h"

extern "C" {
#include "../../include/ws/mask.h"
#include "../../include/ws/frame.h"
#include "../../include/ws/egress.h"
#include "../../include/ws/common.h"
#include "../../include/ws/route.h"
extern __thread int netc_errno_reason;   // include/utils/error.h
}

using netc_gpu::api_fail;
using netc_gpu::api_fail_hip;

namespace {

constexpr int kBadSend = 9;   // netc's BADSEND reason (include/utils/error.h)

enum SlotState : int { kFree = 0, kFilling, kInflight, kTaken };

struct EgressSlot {
    uint8_t* h_pay = nullptr;     // pinned: queued payload bytes (slot_bytes)
    uint8_t* h_tab = nullptr;     // offsets [0, 8 (mf + 1)), keys and header bytes in their own
                                  // regions while filling
    uint8_t* h_pack = nullptr;    // pinned: the table packed at submit (offsets | keys | header
                                  // bytes), so a failed submission leaves h_tab intact for a retry
    uint8_t* h_wire = nullptr;    // pinned: the slot's wire bytes (D2H target)
    uint64_t* h_len = nullptr;    // pinned: the device's wire length (wo[n])
    uint8_t* d_pay = nullptr;
    uint8_t* d_tab = nullptr;
    uint8_t* d_wire = nullptr;
    uint64_t* d_wo = nullptr;     // wire offsets (n + 1)
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;
    int state = kFree;
    int masked = -1;              // the slot's frames are masked (1) or not (0); -1 while empty
    uint64_t fill = 0;            // payload bytes queued
    uint64_t frames = 0;
    uint64_t messages = 0;
    uint64_t wire = 0;            // wire bytes of the queued frames
    int ext = -2;                 // the frames' extended-length bytes: one class (0, 2, 8), mixed (-1),
                                  // none yet (-2); one class: the assembly launches without its scan
};

struct DeviceGuard {
    int prev = -1;
    bool switched = false;
    hipError_t err = hipSuccess;
    explicit DeviceGuard(int device) {
        err = hipGetDevice(&prev);
        if (err != hipSuccess || prev == device) return;
        err = hipSetDevice(device);
        switched = err == hipSuccess;
    }
    ~DeviceGuard() {
        if (switched) (void)hipSetDevice(prev);
    }
};

// header bytes of one frame (src/ws/common.c:55-82; include/ws/frame.h)
inline uint64_t header_len(uint64_t payload, bool masked) {
    return 2 + (payload <= 125 ? 0 : (payload <= 0xFFFF ? 2 : 8)) + (masked ? 4 : 0);
}

}  // namespace

struct netc_ws_egress {
    int device = 0;
    int flags = 0;
    int nslots = 0;
    uint64_t slot_bytes = 0, max_frames = 0, wire_cap = 0;
    uint64_t keys_at = 0, b0_at = 0;   // h_tab regions of the keys and header bytes while filling
    EgressSlot* slots = nullptr;
    int cur = -1;          // slot being filled, -1 = none
    int next_fill = 0;     // the slot to fill next (ring order)
    int fifo[16] = {0};    // submitted slots not yet handed out, in queue order
    int head = 0, count = 0;
    int owner_fd = -1;     // the socket served through ws_send_message (netc_ws_gpu_attach_send)
    uint64_t owner_dev = 0, owner_ino = 0;
};

namespace {

void free_slot(int device, EgressSlot& s) {
    if (s.stream) {
        (void)hipStreamSynchronize(s.stream);
        (void)netc_gpu::release_enc_scratch(device, s.stream);   // the encoder's per-stream scratch
    }
    if (s.h_pay) (void)hipHostFree(s.h_pay);
    if (s.h_tab) (void)hipHostFree(s.h_tab);
    if (s.h_pack) (void)hipHostFree(s.h_pack);
    if (s.h_wire) (void)hipHostFree(s.h_wire);
    if (s.h_len) (void)hipHostFree(s.h_len);
    if (s.d_pay) (void)hipFree(s.d_pay);
    if (s.d_tab) (void)hipFree(s.d_tab);
    if (s.d_wire) (void)hipFree(s.d_wire);
    if (s.d_wo) (void)hipFree(s.d_wo);
    if (s.done) (void)hipEventDestroy(s.done);
    if (s.stream) (void)hipStreamDestroy(s.stream);
    s = EgressSlot();
}

int alloc_slot(const netc_ws_egress* g, EgressSlot& s) {
    hipError_t e;
    const uint64_t mf = g->max_frames, tab = g->b0_at + mf;
    if ((e = hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking)) != hipSuccess ||
        (e = hipEventCreateWithFlags(&s.done, hipEventDisableTiming)) != hipSuccess)
        return api_fail_hip(NETC_GPU_ERUNTIME, "egress: stream / event create", e);
    if ((e = hipHostMalloc((void**)&s.h_pay, g->slot_bytes, hipHostMallocDefault)) != hipSuccess ||
        (e = hipHostMalloc((void**)&s.h_tab, tab, hipHostMallocDefault)) != hipSuccess ||
        (e = hipHostMalloc((void**)&s.h_pack, tab, hipHostMallocDefault)) != hipSuccess ||
        (e = hipHostMalloc((void**)&s.h_wire, g->wire_cap, hipHostMallocDefault)) != hipSuccess ||
        (e = hipHostMalloc((void**)&s.h_len, sizeof(uint64_t), hipHostMallocDefault)) != hipSuccess)
        return api_fail_hip(NETC_GPU_ENOMEM, "egress: pinned host allocation", e);
    if ((e = hipMalloc((void**)&s.d_pay, g->slot_bytes)) != hipSuccess ||
        (e = hipMalloc((void**)&s.d_tab, tab)) != hipSuccess ||
        (e = hipMalloc((void**)&s.d_wire, g->wire_cap)) != hipSuccess ||
        (e = hipMalloc((void**)&s.d_wo, (mf + 1) * sizeof(uint64_t))) != hipSuccess)
        return api_fail_hip(NETC_GPU_ENOMEM, "egress: device allocation", e);
    return 0;
}

// Queue the filling slot on the GPU (see the file comment).
int submit_cur(netc_ws_egress* g) {
    if (g->cur < 0) return 0;
    EgressSlot& s = g->slots[g->cur];
    if (s.frames == 0) return 0;
    if (netc_gpu::inject_fault())
        return api_fail(NETC_GPU_ELAUNCH, "egress: injected fault (NETC_GPU_KNOB_INJECT_FAULT)");
    const uint64_t n = s.frames;
    // pack the table: offsets (n + 1) | keys (n) | header bytes (n), one H2D copy
    uint64_t* off = (uint64_t*)s.h_pack;
    uint8_t* keys = s.h_pack + (n + 1) * sizeof(uint64_t);
    uint8_t* b0 = keys + n * sizeof(uint32_t);
    const bool masked = s.masked == 1;
    memcpy(off, s.h_tab, n * sizeof(uint64_t));
    if (masked) memcpy(keys, s.h_tab + g->keys_at, n * sizeof(uint32_t));
    memcpy(b0, s.h_tab + g->b0_at, n);
    off[n] = s.fill;
    const uint64_t tab = (uint64_t)(b0 + n - s.h_pack);
    const uint64_t bound = s.fill + n * NETC_WS_MAX_HEADER(masked);
    hipError_t e;
    if ((s.fill && (e = hipMemcpyAsync(s.d_pay, s.h_pay, s.fill, hipMemcpyHostToDevice, s.stream)) != hipSuccess) ||
        (e = hipMemcpyAsync(s.d_tab, s.h_pack, tab, hipMemcpyHostToDevice, s.stream)) != hipSuccess)
        return api_fail_hip(NETC_GPU_ERUNTIME, "egress: H2D copy", e);
    const uint8_t* d_keys = s.d_tab + (n + 1) * sizeof(uint64_t);
    if ((e = netc_gpu::launch_encode_frames(s.d_wire, bound, s.d_pay, s.fill, (const uint64_t*)s.d_tab,
                                            (const uint32_t*)d_keys, d_keys + n * sizeof(uint32_t), n, masked,
                                            s.d_wo, s.stream, netc_gpu::api_cfg(), s.ext >= 0 ? s.ext : -1)) !=
        hipSuccess)
        return api_fail_hip(e == hipErrorOutOfMemory ? NETC_GPU_ENOMEM : NETC_GPU_ELAUNCH, "egress: frame assembly",
                            e);
    *s.h_len = ~0ull;
    if ((e = hipMemcpyAsync(s.h_wire, s.d_wire, s.wire, hipMemcpyDeviceToHost, s.stream)) != hipSuccess ||
        (e = hipMemcpyAsync(s.h_len, s.d_wo + n, sizeof(uint64_t), hipMemcpyDeviceToHost, s.stream)) !=
            hipSuccess ||
        (e = hipEventRecord(s.done, s.stream)) != hipSuccess)
        return api_fail_hip(NETC_GPU_ERUNTIME, "egress: D2H copy", e);
    s.state = kInflight;
    g->fifo[(g->head + g->count) % 16] = g->cur;
    ++g->count;
    g->cur = -1;
    return 0;
}

// make a slot the filling one (ring order); NETC_WS_EGRESS_FULL if it is still in use
int acquire(netc_ws_egress* g) {
    if (g->cur >= 0) return 0;
    EgressSlot& s = g->slots[g->next_fill];
    if (s.state != kFree) return api_fail(NETC_WS_EGRESS_FULL, "egress: no free slot (send or release wire batches)");
    s.state = kFilling;
    s.masked = -1;
    s.fill = s.frames = s.messages = s.wire = 0;
    s.ext = -2;
    g->cur = g->next_fill;
    g->next_fill = (g->next_fill + 1) % g->nslots;
    return 0;
}

// [p, p + n) on fd without waiting for the peer: what the socket does not take joins the
// connection's send backlog (include/ws/route.h), ahead of its later bytes
int send_all(int fd, const uint8_t* p, uint64_t n) {
    struct iovec v = {(void*)p, (size_t)n};
    if (netc_ws_send_nb(fd, &v, 1, 1) == 1) return 0;
    const int saved = errno;
    api_fail(NETC_WS_EGRESS_ESEND, "egress: send: %s", strerror(saved));
    netc_errno_reason = kBadSend;
    errno = saved;
    return NETC_WS_EGRESS_ESEND;
}

}  // namespace

extern "C" {

int netc_ws_egress_create(struct netc_ws_egress** out, int device, size_t slot_bytes, int nslots, size_t max_frames,
                          int flags) {
    if (!out) return api_fail(NETC_GPU_EINVAL, "egress: null output pointer");
    *out = nullptr;
    if (int r = netc_gpu::api_check_device(device)) return r;
    if (flags & ~NETC_WS_EGRESS_DEFER) return api_fail(NETC_GPU_EINVAL, "egress: unknown flags 0x%x", flags);
    if (!slot_bytes) slot_bytes = 16u << 20;
    if (!nslots) nslots = 4;
    if (!max_frames) max_frames = slot_bytes / 64 + 64;
    if (slot_bytes < 4096 || slot_bytes > (1ull << 40) || nslots < 2 || nslots > 16 || max_frames > (1ull << 32))
        return api_fail(NETC_GPU_EINVAL, "egress: need 4096 <= slot_bytes <= 2^40, 2 <= nslots <= 16, "
                                         "max_frames <= 2^32");
    DeviceGuard dg(device);
    if (dg.err != hipSuccess) return api_fail_hip(NETC_GPU_ERUNTIME, "hipSetDevice", dg.err);
    netc_ws_egress* g = new (std::nothrow) netc_ws_egress();
    if (!g) return api_fail(NETC_GPU_ENOMEM, "egress: host allocation");
    g->device = device;
    g->flags = flags;
    g->nslots = nslots;
    g->slot_bytes = slot_bytes;
    g->max_frames = max_frames;
    g->wire_cap = slot_bytes + max_frames * NETC_WS_MAX_HEADER(1);
    g->keys_at = (max_frames + 1) * sizeof(uint64_t);
    g->b0_at = g->keys_at + max_frames * sizeof(uint32_t);
    g->slots = new (std::nothrow) EgressSlot[nslots];
    if (!g->slots) {
        delete g;
        return api_fail(NETC_GPU_ENOMEM, "egress: host allocation");
    }
    for (int i = 0; i < nslots; ++i) {
        if (int r = alloc_slot(g, g->slots[i])) {
            for (int j = 0; j <= i; ++j) free_slot(device, g->slots[j]);
            delete[] g->slots;
            delete g;
            return r;
        }
    }
    *out = g;
    return 0;
}

void netc_ws_egress_destroy(struct netc_ws_egress* g) {
    if (!g) return;
    DeviceGuard dg(g->device);
    for (int i = 0; i < g->nslots; ++i) free_slot(g->device, g->slots[i]);
    delete[] g->slots;
    delete g;
}

int netc_ws_egress_queue(struct netc_ws_egress* g, const void* payload, size_t len, uint8_t opcode,
                         const uint8_t* masking_key, size_t num_frames) {
    if (!g || (len && !payload)) return api_fail(NETC_GPU_EINVAL, "egress: null argument");
    const uint64_t nf = num_frames ? num_frames : 1;
    const int masked = masking_key ? 1 : 0;
    if (len > g->slot_bytes || nf > g->max_frames)
        return api_fail(NETC_WS_EGRESS_TOO_BIG, "egress: a message of %zu bytes in %llu frames exceeds a slot "
                        "(%llu bytes, %llu frames)", len, (unsigned long long)nf,
                        (unsigned long long)g->slot_bytes, (unsigned long long)g->max_frames);
    if (int r = acquire(g)) return r;
    {
        const EgressSlot& s = g->slots[g->cur];
        if (s.frames && (s.masked != masked || s.fill + len > g->slot_bytes || s.frames + nf > g->max_frames)) {
            DeviceGuard dg(g->device);   // (only here: a HIP call per queued message costs ~15 % at 1 KiB)
            if (dg.err != hipSuccess) return api_fail_hip(NETC_GPU_ERUNTIME, "hipSetDevice", dg.err);
            if (int e = submit_cur(g)) return e;
            if (int r = acquire(g)) return r;
        }
    }
    EgressSlot& s = g->slots[g->cur];
    s.masked = masked;
    if (len) memcpy(s.h_pay + s.fill, payload, len);
    // the reference's split (src/ws/common.c:42-49): equal parts, the remainder on the last
    const uint64_t split = len / nf, rem = len % nf;
    uint64_t* off = (uint64_t*)s.h_tab + s.frames;
    uint32_t* keys = (uint32_t*)(s.h_tab + g->keys_at) + s.frames;
    uint8_t* b0 = s.h_tab + g->b0_at + s.frames;
    const uint32_t key32 = masked ? (uint32_t)masking_key[0] | (uint32_t)masking_key[1] << 8 |
                                        (uint32_t)masking_key[2] << 16 | (uint32_t)masking_key[3] << 24
                                  : 0u;
    uint64_t wire = 0;
    for (uint64_t i = 0; i < nf; ++i) {
        const bool last = i + 1 == nf;
        const uint64_t flen = split + (last ? rem : 0);
        off[i] = s.fill + i * split;
        if (masked) keys[i] = key32;
        b0[i] = (uint8_t)((last ? 0x80 : 0x00) | (i == 0 ? (opcode & 0x0F) : WS_OPCODE_CONTINUE));   // :55-61
        wire += header_len(flen, masked) + flen;
        const int ext = flen <= 125 ? 0 : (flen <= 0xFFFF ? 2 : 8);
        s.ext = s.ext == -2 || s.ext == ext ? ext : -1;
    }
    s.fill += len;
    s.frames += nf;
    s.wire += wire;
    ++s.messages;
    return 0;
}

int netc_ws_egress_submit(struct netc_ws_egress* g) {
    if (!g) return api_fail(NETC_GPU_EINVAL, "egress: null egress");
    DeviceGuard dg(g->device);
    if (dg.err != hipSuccess) return api_fail_hip(NETC_GPU_ERUNTIME, "hipSetDevice", dg.err);
    return submit_cur(g);
}

int netc_ws_egress_next(struct netc_ws_egress* g, struct netc_ws_wire* out, int wait) {
    if (!g || !out) return api_fail(NETC_GPU_EINVAL, "egress: null argument");
    if (g->count == 0) return 0;
    DeviceGuard dg(g->device);
    if (dg.err != hipSuccess) return api_fail_hip(NETC_GPU_ERUNTIME, "hipSetDevice", dg.err);
    const int i = g->fifo[g->head];
    EgressSlot& s = g->slots[i];
    hipError_t e = wait ? hipEventSynchronize(s.done) : hipEventQuery(s.done);
    if (!wait && e == hipErrorNotReady) return 0;
    if (e != hipSuccess) return api_fail_hip(NETC_GPU_ERUNTIME, "egress: slot wait", e);
    g->head = (g->head + 1) % 16;
    --g->count;
    if (*s.h_len != s.wire) {   // the device's wire length against the host's header sum
        s.state = kFree;
        return api_fail(NETC_GPU_ERUNTIME, "egress: device wire length %llu, expected %llu",
                        (unsigned long long)*s.h_len, (unsigned long long)s.wire);
    }
    out->wire = s.h_wire;
    out->len = s.wire;
    out->nframes = s.frames;
    out->nmessages = s.messages;
    out->slot = i;
    s.state = kTaken;
    return 1;
}

int netc_ws_egress_release(struct netc_ws_egress* g, const struct netc_ws_wire* w) {
    if (!g || !w || w->slot < 0 || w->slot >= g->nslots || g->slots[w->slot].state != kTaken)
        return api_fail(NETC_GPU_EINVAL, "egress: not a wire batch handed out by this egress");
    g->slots[w->slot].state = kFree;
    return 0;
}

long netc_ws_egress_send(struct netc_ws_egress* g, int fd, int wait) {
    if (!g) return api_fail(NETC_GPU_EINVAL, "egress: null egress");
    long total = 0;
    for (;;) {
        struct netc_ws_wire w;
        const int r = netc_ws_egress_next(g, &w, wait);
        if (r < 0) return r;
        if (r == 0) return total;
        const int s = send_all(fd, w.wire, w.len);
        (void)netc_ws_egress_release(g, &w);
        if (s) return s;
        total += (long)w.len;
    }
}

long netc_ws_egress_flush(struct netc_ws_egress* g, int fd) {
    if (int r = netc_ws_egress_submit(g)) return r;
    return netc_ws_egress_send(g, fd, 1);
}

// ws_send_message on a socket attached to a ring (include/ws/route.h): the reference's send
// contract (src/ws/common.c:36-130: 1 once sent, else the failing send() result) served from
// the ring.  DEFER rings return once the message is queued and send what has finished.
static int gpu_send_route(void* ctx, int sockfd, struct ws_message* message, uint8_t masking_key[4],
                          size_t num_frames) {
    netc_ws_egress* g = (netc_ws_egress*)ctx;
    if (sockfd != g->owner_fd) {   // one ring, one connection: never another socket's bytes
        api_fail(NETC_GPU_EINVAL, "send route: the ring serves socket %d, not %d", g->owner_fd, sockfd);
        return -1;
    }
    int r = netc_ws_egress_queue(g, message->buffer, message->payload_length, message->opcode, masking_key,
                                 num_frames);
    if (r == NETC_WS_EGRESS_FULL) {   // every slot queued or unsent: put the oldest on the socket
        if (netc_ws_egress_send(g, sockfd, 1) < 0) return -1;
        r = netc_ws_egress_queue(g, message->buffer, message->payload_length, message->opcode, masking_key,
                                 num_frames);
    }
    if (r) return -1;
    // a DEFER ring sends what has finished; a close frame goes out at once, with everything
    // queued before it (netc closes the socket right after sending one, src/ws/server.c:123-124)
    const bool now = !(g->flags & NETC_WS_EGRESS_DEFER) || message->opcode == WS_OPCODE_CLOSE;
    const long s = now ? netc_ws_egress_flush(g, sockfd) : netc_ws_egress_send(g, sockfd, 0);
    return s < 0 ? -1 : 1;
}

// close() on the attached socket (close tracking, include/ws/route.h): what it queued goes out first
static void ring_close_hook(void* ctx, int sockfd) { (void)netc_ws_gpu_detach_send(sockfd); }

static bool sock_identity(int fd, uint64_t* dev, uint64_t* ino) {
    struct stat st;
    if (fstat(fd, &st) != 0 || !S_ISSOCK(st.st_mode)) return false;
    *dev = (uint64_t)st.st_dev;
    *ino = (uint64_t)st.st_ino;
    return true;
}

// a ring's messages queued but not yet on its socket (slots filling, on the GPU or finished)
static bool has_queued(const netc_ws_egress* g) {
    return g->count > 0 || (g->cur >= 0 && g->slots[g->cur].frames > 0);
}

int netc_ws_gpu_attach_send(int sockfd, struct netc_ws_egress* ring) {
    if (!ring) return api_fail(NETC_GPU_EINVAL, "attach_send: null ring");
    uint64_t dev = 0, ino = 0;
    if (!sock_identity(sockfd, &dev, &ino))
        return api_fail(NETC_GPU_EINVAL, "attach_send: %d is not an open socket", sockfd);
    if (ring->owner_fd >= 0) {
        if (ring->owner_fd == sockfd && ring->owner_dev == dev && ring->owner_ino == ino) return 0;
        uint64_t d2 = 0, i2 = 0;
        if (sock_identity(ring->owner_fd, &d2, &i2) && d2 == ring->owner_dev && i2 == ring->owner_ino)
            return api_fail(NETC_GPU_EINVAL, "attach_send: the ring already serves socket %d (one ring, one "
                            "connection)", ring->owner_fd);
        // its connection was closed without a detach
        void* ctx = nullptr;
        if (netc_ws_send_route_get_raw(ring->owner_fd, &ctx) && ctx == ring) (void)netc_ws_send_route_detach(ring->owner_fd);
        ring->owner_fd = -1;
    }
    if (has_queued(ring))   // they were queued for another connection
        return api_fail(NETC_GPU_EINVAL, "attach_send: the ring holds queued messages (flush or destroy it first)");
    if (netc_ws_send_route_attach(sockfd, gpu_send_route, ring) != 0)
        return api_fail(NETC_GPU_EINVAL, "attach_send: socket %d: %s", sockfd,
                        errno == EBUSY ? "another send route serves it" : "out of range");
    ring->owner_fd = sockfd;
    ring->owner_dev = dev;
    ring->owner_ino = ino;
    (void)netc_ws_send_route_on_close(sockfd, ring_close_hook);
    return 0;
}

int netc_ws_gpu_detach_send(int sockfd) {
    if (sockfd < 0) return api_fail(NETC_GPU_EINVAL, "detach_send: socket %d out of range", sockfd);
    void* ctx = nullptr;
    long flushed = 0;
    if (netc_ws_send_route_get_raw(sockfd, &ctx) == gpu_send_route && ctx) {
        netc_ws_egress* g = (netc_ws_egress*)ctx;
        if (g->owner_fd == sockfd) {
            // ws_send_message already returned 1 for a DEFER ring's queued messages: they go out now
            uint64_t d = 0, i = 0;
            if (has_queued(g)) {
                if (sock_identity(sockfd, &d, &i) && d == g->owner_dev && i == g->owner_ino)
                    flushed = netc_ws_egress_flush(g, sockfd);
                else
                    flushed = api_fail(NETC_WS_EGRESS_ESEND, "detach_send: socket %d was closed with queued "
                                       "messages", sockfd);
            }
            g->owner_fd = -1;
        }
    }
    if (netc_ws_send_route_detach(sockfd) != 0)
        return api_fail(NETC_GPU_EINVAL, "detach_send: socket %d out of range", sockfd);
    return flushed < 0 ? (int)flushed : 0;
}

}  // extern "C"
