// One GPU send ring shared by many connections: include/ws/egress_hub.h (the send side of
// include/ws/hub.h; SURVEY.md §8(f) row 2 in the shape of netc's server).
//
// Per ws_send_message on an attached socket (the event loop's thread): the message's payload is
// appended to the filling slot, its frames -- the reference's split (src/ws/common.c:42-49),
// one key, header byte per frame (:55-61) -- to the slot's frame table, and its wire span (where
// its frames will sit in the slot's wire, known on the host from the lengths) to the slot's
// message list.  Per slot, on its own stream:
//
//   submit   H2D of the payload and the packed table (offsets | keys | header bytes), the frame
//            assembly (launch_encode_frames: ONE launch when every frame of the slot is in one
//            length class -- the host saw each length -- else the wire-offsets scan first), D2H
//            of the wire into the slot's pinned wire buffer and of the device's wire length
//   send     once its event is done: per connection, one sendmsg(MSG_DONTWAIT) over iovecs of its
//            messages' runs in the wire (a connection's consecutive messages are one run); what
//            the socket does not take moves to the connection's send backlog (libnetc.so,
//            include/ws/route.h), which goes out ahead of its later bytes; then the slot is
//            free.  Slots go out in the order they were filled, so a connection's bytes keep its
//            queue order, and a peer that stops reading holds up nobody but itself.
#include <hip/hip_runtime.h>

#include <errno.h>
#include <limits.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/uio.h>

#include <deque>
#include <new>
#include <unordered_map>
#include <vector>

#include "ws_mask_gpu.h"

extern "C" {
#include "../../include/ws/mask.h"
#include "../../include/ws/frame.h"
#include "../../include/ws/egress.h"
#include "../../include/ws/egress_hub.h"
#include "../../include/ws/common.h"
#include "../../include/ws/route.h"
extern __thread int netc_errno_reason;   // include/utils/error.h
}

using netc_gpu::api_fail;
using netc_gpu::api_fail_hip;

namespace {

constexpr int kBadSend = 9;   // netc's BADSEND reason (include/utils/error.h)

enum SlotState : int { kFree = 0, kFilling, kInflight };

struct EhConn {
    int fd = -1;
    uint64_t dev = 0, ino = 0;
    int failed = 0;             // send() failed: its bytes are dropped, its calls return -1
    bool deferred = false;      // its send backlog holds bytes (on the hub's deferred list)
    uint64_t last_gen = 0;      // the slot filling this connection last queued into
    uint64_t queued = 0;        // its messages in slots not yet sent
    std::vector<struct iovec> iov;   // flush scratch: its runs in the slot being sent
};

struct Span {   // one message's wire bytes in its slot
    EhConn* conn;
    uint64_t w0, w1;
};

struct EhSlot {
    uint8_t* h_pay = nullptr;    // pinned: queued payload bytes (slot_bytes)
    uint8_t* h_tab = nullptr;    // offsets [0, 8 (mf + 1)), keys and header bytes in their regions
    uint8_t* h_pack = nullptr;   // pinned: the table packed at submit (a failed submission leaves h_tab)
    uint8_t* h_wire = nullptr;   // pinned: the slot's wire bytes (D2H target)
    uint64_t* h_len = nullptr;   // pinned: the device's wire length (wo[n])
    uint8_t* d_pay = nullptr;
    uint8_t* d_tab = nullptr;
    uint8_t* d_wire = nullptr;
    uint64_t* d_wo = nullptr;
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;
    int state = kFree;
    int masked = -1;             // the slot's frames are masked (1) or not (0); -1 while empty
    int ext = -2;                // one length class (0, 2, 8), mixed (-1), none yet (-2)
    uint64_t fill = 0, frames = 0, wire = 0, gen = 0;
    uint32_t nconn = 0;
    std::vector<Span> spans;
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

inline uint64_t header_len(uint64_t payload, bool masked) {   // src/ws/common.c:55-82
    return 2 + (payload <= 125 ? 0 : (payload <= 0xFFFF ? 2 : 8)) + (masked ? 4 : 0);
}

bool sock_identity(int fd, uint64_t* dev, uint64_t* ino) {
    struct stat st;
    if (fstat(fd, &st) != 0 || !S_ISSOCK(st.st_mode)) return false;
    *dev = (uint64_t)st.st_dev;
    *ino = (uint64_t)st.st_ino;
    return true;
}

}  // namespace

struct netc_ws_egress_hub {
    int device = 0;
    int nslots = 0;
    uint64_t slot_bytes = 0, max_frames = 0, wire_cap = 0, keys_at = 0, b0_at = 0;
    EhSlot* slots = nullptr;
    int cur = -1;                // the filling slot
    std::deque<int> fifo;        // submitted slots, oldest first
    uint64_t gens = 0;
    std::unordered_map<int, EhConn*> conns;
    std::vector<EhConn*> deferred;   // connections whose send backlog holds bytes
    struct netc_ws_egress_hub_stats st{};
};

namespace {

void free_slot(int device, EhSlot& s) {
    if (s.stream) {
        (void)hipStreamSynchronize(s.stream);
        (void)netc_gpu::release_enc_scratch(device, s.stream);
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
    s = EhSlot();
}

int alloc_slot(const netc_ws_egress_hub* h, EhSlot& s) {
    hipError_t e;
    const uint64_t tab = h->b0_at + h->max_frames;
    if ((e = hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking)) != hipSuccess ||
        (e = hipEventCreateWithFlags(&s.done, hipEventDisableTiming)) != hipSuccess)
        return api_fail_hip(NETC_GPU_ERUNTIME, "egress hub: stream / event create", e);
    if ((e = hipHostMalloc((void**)&s.h_pay, h->slot_bytes, hipHostMallocDefault)) != hipSuccess ||
        (e = hipHostMalloc((void**)&s.h_tab, tab, hipHostMallocDefault)) != hipSuccess ||
        (e = hipHostMalloc((void**)&s.h_pack, tab, hipHostMallocDefault)) != hipSuccess ||
        (e = hipHostMalloc((void**)&s.h_wire, h->wire_cap, hipHostMallocDefault)) != hipSuccess ||
        (e = hipHostMalloc((void**)&s.h_len, sizeof(uint64_t), hipHostMallocDefault)) != hipSuccess)
        return api_fail_hip(NETC_GPU_ENOMEM, "egress hub: pinned host allocation", e);
    if ((e = hipMalloc((void**)&s.d_pay, h->slot_bytes)) != hipSuccess ||
        (e = hipMalloc((void**)&s.d_tab, tab)) != hipSuccess ||
        (e = hipMalloc((void**)&s.d_wire, h->wire_cap)) != hipSuccess ||
        (e = hipMalloc((void**)&s.d_wo, (h->max_frames + 1) * sizeof(uint64_t))) != hipSuccess)
        return api_fail_hip(NETC_GPU_ENOMEM, "egress hub: device allocation", e);
    return 0;
}

// the filling slot goes to the GPU (see the file comment)
int submit(netc_ws_egress_hub* h) {
    if (h->cur < 0) return 0;
    EhSlot& s = h->slots[h->cur];
    if (s.frames == 0) return 0;
    if (netc_gpu::inject_fault())
        return api_fail(NETC_GPU_ELAUNCH, "egress hub: injected fault (NETC_GPU_KNOB_INJECT_FAULT)");
    DeviceGuard dg(h->device);
    if (dg.err != hipSuccess) return api_fail_hip(NETC_GPU_ERUNTIME, "hipSetDevice", dg.err);
    const uint64_t n = s.frames;
    uint64_t* off = (uint64_t*)s.h_pack;
    uint8_t* keys = s.h_pack + (n + 1) * sizeof(uint64_t);
    uint8_t* b0 = keys + n * sizeof(uint32_t);
    const bool masked = s.masked == 1;
    memcpy(off, s.h_tab, n * sizeof(uint64_t));
    if (masked) memcpy(keys, s.h_tab + h->keys_at, n * sizeof(uint32_t));
    memcpy(b0, s.h_tab + h->b0_at, n);
    off[n] = s.fill;
    const uint64_t tab = (uint64_t)(b0 + n - s.h_pack);
    const uint64_t bound = s.fill + n * NETC_WS_MAX_HEADER(masked);
    hipError_t e;
    if ((s.fill && (e = hipMemcpyAsync(s.d_pay, s.h_pay, s.fill, hipMemcpyHostToDevice, s.stream)) != hipSuccess) ||
        (e = hipMemcpyAsync(s.d_tab, s.h_pack, tab, hipMemcpyHostToDevice, s.stream)) != hipSuccess)
        return api_fail_hip(NETC_GPU_ERUNTIME, "egress hub: H2D copy", e);
    const uint8_t* d_keys = s.d_tab + (n + 1) * sizeof(uint64_t);
    if ((e = netc_gpu::launch_encode_frames(s.d_wire, bound, s.d_pay, s.fill, (const uint64_t*)s.d_tab,
                                            (const uint32_t*)d_keys, d_keys + n * sizeof(uint32_t), n, masked,
                                            s.d_wo, s.stream, netc_gpu::api_cfg(), s.ext >= 0 ? s.ext : -1)) !=
        hipSuccess)
        return api_fail_hip(e == hipErrorOutOfMemory ? NETC_GPU_ENOMEM : NETC_GPU_ELAUNCH, "egress hub: frame assembly",
                            e);
    *s.h_len = ~0ull;
    if ((e = hipMemcpyAsync(s.h_wire, s.d_wire, s.wire, hipMemcpyDeviceToHost, s.stream)) != hipSuccess ||
        (e = hipMemcpyAsync(s.h_len, s.d_wo + n, sizeof(uint64_t), hipMemcpyDeviceToHost, s.stream)) != hipSuccess ||
        (e = hipEventRecord(s.done, s.stream)) != hipSuccess)
        return api_fail_hip(NETC_GPU_ERUNTIME, "egress hub: D2H copy", e);
    s.state = kInflight;
    h->fifo.push_back(h->cur);
    h->cur = -1;
    h->st.launches++;
    h->st.messages += s.spans.size();
    h->st.frames += n;
    h->st.wire_bytes += s.wire;
    h->st.connection_slots += s.nconn;
    if (s.nconn > h->st.max_connections) h->st.max_connections = s.nconn;
    return 0;
}

// the connection's send backlog after a send: still holding bytes (kept on the deferred list), or
// failed past its bound
void note_backlog(netc_ws_egress_hub* h, EhConn* c) {
    const long p = netc_ws_send_pending(c->fd);
    if (p < 0) {
        c->failed = errno ? errno : ENOBUFS;
        h->st.send_errors++;
    } else if (p > 0 && !c->deferred) {
        c->deferred = true;
        h->deferred.push_back(c);
        h->st.deferred_sends++;
    }
}

// the deferred connections' backlogs, written as far as their sockets take them now
void drain_deferred(netc_ws_egress_hub* h) {
    size_t keep = 0;
    for (size_t i = 0; i < h->deferred.size(); ++i) {
        EhConn* c = h->deferred[i];
        const long r = c->failed ? -1 : netc_ws_send_flush(c->fd);
        if (r > 0) {
            h->deferred[keep++] = c;
            continue;
        }
        if (r < 0 && !c->failed) {
            c->failed = errno ? errno : EPIPE;
            h->st.send_errors++;
        }
        c->deferred = false;
    }
    h->deferred.resize(keep);
}

// wait for the oldest submitted slot and put its connections' bytes on their sockets; bytes sent.
// *dropped: the slot finished but its wire is not what was queued (the device's wire length differs
// from the host's); then each of its connections fails as on a failed send -- its bytes are gone,
// its next ws_send_message returns -1 and netc closes it -- and the slot is free for the others,
// so one bad slot does not hold up every later flush.  A failed wait (the device itself) stays
// sticky: the slot is left where it is.
long send_oldest(netc_ws_egress_hub* h, bool* dropped) {
    *dropped = false;
    const int i = h->fifo.front();
    EhSlot& s = h->slots[i];
    hipError_t e = hipEventSynchronize(s.done);
    if (e != hipSuccess) return api_fail_hip(NETC_GPU_ERUNTIME, "egress hub: slot wait", e);
    h->fifo.pop_front();
    if (*s.h_len != s.wire) {
        for (const Span& sp : s.spans)
            if (sp.conn && !sp.conn->failed) {
                sp.conn->failed = EIO;
                h->st.send_errors++;
            }
        s.spans.clear();
        s.state = kFree;
        *dropped = true;
        return api_fail(NETC_GPU_ERUNTIME, "egress hub: the device's wire length %llu is not the host's %llu; "
                        "the slot's connections fail", (unsigned long long)*s.h_len, (unsigned long long)s.wire);
    }
    // per connection, its runs in the wire, in queue order (consecutive messages: one run)
    std::vector<EhConn*> order;
    for (const Span& sp : s.spans) {
        EhConn* c = sp.conn;
        if (!c) continue;   // detached since
        if (c->queued) --c->queued;
        if (c->iov.empty()) order.push_back(c);
        struct iovec* last = c->iov.empty() ? nullptr : &c->iov.back();
        if (last && (uint8_t*)last->iov_base + last->iov_len == s.h_wire + sp.w0) last->iov_len += sp.w1 - sp.w0;
        else c->iov.push_back({s.h_wire + sp.w0, (size_t)(sp.w1 - sp.w0)});
    }
    long sent = 0;
    for (EhConn* c : order) {
        // a connection closed without a detach that close tracking did not see (a raw close, a
        // process where close() does not reach libnetc.so): its descriptor may name another
        // connection by now, which must not get these bytes.  One fstat per connection per slot.
        uint64_t d = 0, ino = 0;
        if (!c->failed && !(sock_identity(c->fd, &d, &ino) && d == c->dev && ino == c->ino)) {
            c->failed = EBADF;
            h->st.send_errors++;
        }
        if (!c->failed) {
            uint64_t n = 0;
            for (const struct iovec& v : c->iov) n += v.iov_len;
            if (netc_ws_send_nb(c->fd, c->iov.data(), (int)c->iov.size(), 1) == 1) {
                sent += (long)n;
                h->st.sendmsg_calls++;
                note_backlog(h, c);
            } else {
                c->failed = errno ? errno : EPIPE;
                h->st.send_errors++;
            }
        }
        c->iov.clear();
    }
    s.spans.clear();
    s.state = kFree;
    return sent;
}

// make a slot the filling one; with none free, the oldest submitted one is sent first
int acquire(netc_ws_egress_hub* h) {
    if (h->cur >= 0) return 0;
    for (;;) {
        for (int i = 0; i < h->nslots; ++i) {
            EhSlot& s = h->slots[i];
            if (s.state != kFree) continue;
            s.state = kFilling;
            s.masked = -1;
            s.ext = -2;
            s.fill = s.frames = s.wire = 0;
            s.nconn = 0;
            s.gen = ++h->gens;
            s.spans.clear();
            h->cur = i;
            return 0;
        }
        if (h->fifo.empty()) return api_fail(NETC_GPU_ERUNTIME, "egress hub: no slot to send");
        bool dropped = false;
        const long r = send_oldest(h, &dropped);
        if (r < 0 && !dropped) return (int)r;   // (dropped: its connections learn it on their next call)
    }
}

int queue(netc_ws_egress_hub* h, EhConn* c, const void* payload, size_t len, uint8_t opcode, const uint8_t* masking_key,
          size_t num_frames) {
    if (len && !payload) return api_fail(NETC_GPU_EINVAL, "egress hub: null payload");
    const uint64_t nf = num_frames ? num_frames : 1;
    const int masked = masking_key ? 1 : 0;
    if (len > h->slot_bytes || nf > h->max_frames)
        return api_fail(NETC_WS_EGRESS_TOO_BIG, "egress hub: a message of %zu bytes in %llu frames exceeds a slot "
                        "(%llu bytes, %llu frames)", len, (unsigned long long)nf,
                        (unsigned long long)h->slot_bytes, (unsigned long long)h->max_frames);
    if (int r = acquire(h)) return r;
    {
        const EhSlot& s = h->slots[h->cur];
        // a slot past its full mark is one whose submission failed: tried again (and reported)
        // before anything more is queued; a message that does not fit starts the next slot
        const bool full = s.fill + 4096 > h->slot_bytes || s.frames + 64 > h->max_frames;
        if (s.frames && (full || s.masked != masked || s.fill + len > h->slot_bytes || s.frames + nf > h->max_frames)) {
            if (int e = submit(h)) return e;
            if (int r = acquire(h)) return r;
        }
    }
    EhSlot& s = h->slots[h->cur];
    s.masked = masked;
    if (len) memcpy(s.h_pay + s.fill, payload, len);
    const uint64_t split = len / nf, rem = len % nf;   // the reference's split (src/ws/common.c:42-49)
    uint64_t* off = (uint64_t*)s.h_tab + s.frames;
    uint32_t* keys = (uint32_t*)(s.h_tab + h->keys_at) + s.frames;
    uint8_t* b0 = s.h_tab + h->b0_at + s.frames;
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
    s.spans.push_back(Span{c, s.wire, s.wire + wire});
    ++c->queued;
    if (c->last_gen != s.gen) {
        c->last_gen = s.gen;
        ++s.nconn;
    }
    s.fill += len;
    s.frames += nf;
    s.wire += wire;
    // full: on its way now.  The message is queued either way; a failed submission leaves the slot
    // filling, and the next queue or flush tries it again and reports it (before queueing anything).
    if (s.fill + 4096 > h->slot_bytes || s.frames + 64 > h->max_frames) (void)submit(h);
    return 0;
}

// every queued byte out; a dropped slot is reported (its code) once the later slots are sent
long flush(netc_ws_egress_hub* h) {
    if (int e = submit(h)) return e;
    long sent = 0, err = 0;
    while (!h->fifo.empty()) {
        bool dropped = false;
        const long r = send_oldest(h, &dropped);
        if (r < 0 && !dropped) return r;
        if (r < 0) err = r;
        else sent += r;
    }
    drain_deferred(h);
    return err ? err : sent;
}

// ws_send_message on a socket attached to an egress hub (include/ws/egress_hub.h)
int hub_send_route(void* ctx, int sockfd, struct ws_message* message, uint8_t masking_key[4], size_t num_frames) {
    netc_ws_egress_hub* h = (netc_ws_egress_hub*)ctx;
    auto it = h->conns.find(sockfd);
    if (it == h->conns.end()) {
        api_fail(NETC_GPU_EINVAL, "egress hub: socket %d is not attached", sockfd);
        return -1;
    }
    EhConn* c = it->second;
    if (c->failed) {   // an earlier flush's send() failed on it (src/ws/common.c:128-131: the send result)
        api_fail(NETC_WS_EGRESS_ESEND, "egress hub: send on socket %d failed: %s", sockfd, strerror(c->failed));
        netc_errno_reason = kBadSend;
        errno = c->failed;
        return -1;
    }
    if (c->deferred && netc_ws_send_pending(sockfd) < 0) {   // its backlog passed the bound
        c->failed = errno ? errno : ENOBUFS;
        h->st.send_errors++;
        api_fail(NETC_WS_EGRESS_ESEND, "egress hub: socket %d: %s", sockfd, strerror(c->failed));
        netc_errno_reason = kBadSend;
        errno = c->failed;
        return -1;
    }
    if (queue(h, c, message->buffer, message->payload_length, message->opcode, masking_key, num_frames)) return -1;
    // a close frame goes out now: netc closes the socket right after sending it
    // (src/ws/server.c:123-124), and everything queued before it must precede it on the wire
    if (message->opcode == WS_OPCODE_CLOSE) {
        DeviceGuard dg(h->device);
        if (flush(h) < 0) return -1;
    }
    return 1;
}

// close() on an attached socket (close tracking, include/ws/route.h): what was queued for it goes out
void hub_close_hook(void* ctx, int sockfd) { (void)netc_ws_gpu_detach_send_hub(sockfd); }

void forget(netc_ws_egress_hub* h, EhConn* c) {   // spans queued for it are skipped when sent
    for (int i = 0; i < h->nslots; ++i)
        for (Span& sp : h->slots[i].spans)
            if (sp.conn == c) sp.conn = nullptr;
    for (size_t i = 0; i < h->deferred.size(); ++i)
        if (h->deferred[i] == c) {
            h->deferred.erase(h->deferred.begin() + (long)i);
            break;
        }
    delete c;
}

}  // namespace

extern "C" {

int netc_ws_egress_hub_create(struct netc_ws_egress_hub** out, int device, size_t slot_bytes, int nslots,
                              size_t max_frames) {
    if (!out) return api_fail(NETC_GPU_EINVAL, "egress hub: null output pointer");
    *out = nullptr;
    if (int r = netc_gpu::api_check_device(device)) return r;
    if (!slot_bytes) slot_bytes = 16u << 20;
    if (!nslots) nslots = 4;
    if (!max_frames) max_frames = slot_bytes / 64 + 64;
    if (slot_bytes < 4096 || slot_bytes > (1ull << 40) || nslots < 2 || nslots > 16 || max_frames < 64 ||
        max_frames > (1ull << 32))
        return api_fail(NETC_GPU_EINVAL, "egress hub: need 4096 <= slot_bytes <= 2^40, 2 <= nslots <= 16, "
                                         "64 <= max_frames <= 2^32");
    DeviceGuard dg(device);
    if (dg.err != hipSuccess) return api_fail_hip(NETC_GPU_ERUNTIME, "hipSetDevice", dg.err);
    netc_ws_egress_hub* h = new (std::nothrow) netc_ws_egress_hub();
    if (!h) return api_fail(NETC_GPU_ENOMEM, "egress hub: host allocation");
    h->device = device;
    h->nslots = nslots;
    h->slot_bytes = slot_bytes;
    h->max_frames = max_frames;
    h->wire_cap = slot_bytes + max_frames * NETC_WS_MAX_HEADER(1);
    h->keys_at = (max_frames + 1) * sizeof(uint64_t);
    h->b0_at = h->keys_at + max_frames * sizeof(uint32_t);
    h->slots = new (std::nothrow) EhSlot[nslots];
    if (!h->slots) {
        delete h;
        return api_fail(NETC_GPU_ENOMEM, "egress hub: host allocation");
    }
    for (int i = 0; i < nslots; ++i) {
        if (int r = alloc_slot(h, h->slots[i])) {
            for (int j = 0; j <= i; ++j) free_slot(device, h->slots[j]);
            delete[] h->slots;
            delete h;
            return r;
        }
    }
    *out = h;
    return 0;
}

void netc_ws_egress_hub_destroy(struct netc_ws_egress_hub* h) {
    if (!h) return;
    DeviceGuard dg(h->device);
    (void)flush(h);
    for (auto& kv : h->conns) {
        void* ctx = nullptr;
        if (netc_ws_send_route_get_raw(kv.first, &ctx) == hub_send_route && ctx == h)
            (void)netc_ws_send_route_detach(kv.first);
        delete kv.second;
    }
    h->conns.clear();
    for (int i = 0; i < h->nslots; ++i) free_slot(h->device, h->slots[i]);
    delete[] h->slots;
    delete h;
}

int netc_ws_gpu_attach_send_hub(int sockfd, struct netc_ws_egress_hub* h) {
    if (!h) return api_fail(NETC_GPU_EINVAL, "attach_send_hub: null hub");
    uint64_t dev = 0, ino = 0;
    if (!sock_identity(sockfd, &dev, &ino))
        return api_fail(NETC_GPU_EINVAL, "attach_send_hub: %d is not an open socket", sockfd);
    auto it = h->conns.find(sockfd);
    if (it != h->conns.end()) {
        if (it->second->dev == dev && it->second->ino == ino) return 0;   // already this connection
        forget(h, it->second);                                             // closed without a detach
        h->conns.erase(it);
        void* ctx = nullptr;
        if (netc_ws_send_route_get_raw(sockfd, &ctx) == hub_send_route && ctx == h) (void)netc_ws_send_route_detach(sockfd);
    }
    EhConn* c = new (std::nothrow) EhConn();
    if (!c) return api_fail(NETC_GPU_ENOMEM, "attach_send_hub: host allocation");
    c->fd = sockfd;
    c->dev = dev;
    c->ino = ino;
    if (netc_ws_send_route_attach(sockfd, hub_send_route, h) != 0) {
        delete c;
        return api_fail(NETC_GPU_EINVAL, "attach_send_hub: socket %d: %s", sockfd,
                        errno == EBUSY ? "another send route serves it" : "out of range");
    }
    h->conns[sockfd] = c;
    h->st.connections = h->conns.size();
    (void)netc_ws_send_route_on_close(sockfd, hub_close_hook);
    return 0;
}

int netc_ws_gpu_detach_send_hub(int sockfd) {
    if (sockfd < 0) return api_fail(NETC_GPU_EINVAL, "detach_send_hub: socket %d out of range", sockfd);
    void* ctx = nullptr;
    long flushed = 0;
    if (netc_ws_send_route_get_raw(sockfd, &ctx) == hub_send_route && ctx) {
        netc_ws_egress_hub* h = (netc_ws_egress_hub*)ctx;
        auto it = h->conns.find(sockfd);
        if (it != h->conns.end()) {
            DeviceGuard dg(h->device);
            // ws_send_message already returned 1 for what it queued: it goes out first
            uint64_t d = 0, i = 0;
            if (!(sock_identity(sockfd, &d, &i) && d == it->second->dev && i == it->second->ino))
                it->second->failed = EBADF;   // closed without a detach: its bytes have nowhere to go
            if (it->second->queued || it->second->deferred) flushed = flush(h);
            forget(h, it->second);
            h->conns.erase(it);
            h->st.connections = h->conns.size();
        }
    }
    if (netc_ws_send_route_detach(sockfd) != 0)
        return api_fail(NETC_GPU_EINVAL, "detach_send_hub: socket %d out of range", sockfd);
    return flushed < 0 ? (int)flushed : 0;
}

long netc_ws_egress_hub_flush(struct netc_ws_egress_hub* h) {
    if (!h) return api_fail(NETC_GPU_EINVAL, "egress hub: null hub");
    DeviceGuard dg(h->device);
    if (dg.err != hipSuccess) return api_fail_hip(NETC_GPU_ERUNTIME, "hipSetDevice", dg.err);
    return flush(h);
}

long netc_ws_egress_hub_pending(const struct netc_ws_egress_hub* h) {
    if (!h) return api_fail(NETC_GPU_EINVAL, "egress hub: null hub");
    long n = 0;
    for (EhConn* c : h->deferred) {
        const long p = c->failed ? 0 : netc_ws_send_pending(c->fd);
        if (p > 0) n += p;
    }
    return n;
}

int netc_ws_egress_hub_stats(const struct netc_ws_egress_hub* h, struct netc_ws_egress_hub_stats* out) {
    if (!h || !out) return NETC_GPU_EINVAL;
    *out = h->st;
    out->pending_bytes = (uint64_t)netc_ws_egress_hub_pending(h);
    return 0;
}

}  // extern "C"
