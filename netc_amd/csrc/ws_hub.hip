// One GPU receive ring shared by many connections: include/ws/hub.h (SURVEY.md §8(f) row 4 in
// the shape of netc's server, which serves every client from one event loop --
// src/tcp/server.c:30-75, src/web/server.c:69-98).
//
// Per route call (ws_parse_frame on an attached socket, from the event loop's one thread):
//
//   take     the connection's carry (its incomplete frame) is copied into the filling slot,
//            then the socket's new bytes are peeked right behind it (MSG_PEEK), and the host
//            header walk finds the complete frames: they stay in the slot as one range of the
//            connection, the incomplete tail goes back to its carry.  The peeked bytes leave
//            the socket all but one (the hostage; see include/ws/hub.h).
//   submit   per slot, on the slot's own stream: H2D of the frames and their descriptors
//            (header offsets, key32), ONE unmask launch over the frames of every connection
//            in the slot (launch_unmask_scanned, the batch kernel of ws_mask_gpu.hip), D2H of
//            the unmasked frames back into the pinned slot, event "done".
//   deliver  the connection's ranges, oldest first: frames reassembled into messages with the
//            reference's rules (src/ws/common.c:163-164, 210-216, 303-309, 333-347).
//
// A slot is free again when every connection has consumed its ranges in it.
#include <hip/hip_runtime.h>

#include <errno.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <sys/ioctl.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/uio.h>

#include <deque>
#include <new>
#include <unordered_map>

#include "ws_mask_gpu.h"

extern "C" {
#include "../../include/ws/mask.h"
#include "../../include/ws/frame.h"
#include "../../include/ws/ingest.h"
#include "../../include/ws/hub.h"
#include "../../include/ws/common.h"
#include "../../include/ws/route.h"
extern __thread int netc_errno_reason;   // include/utils/error.h
}

using netc_gpu::api_fail;
using netc_gpu::api_fail_hip;

namespace {

constexpr int kBadRecv = 10;                 // netc's BADRECV reason (include/utils/error.h)
constexpr size_t kPeek = 256u << 10;         // bytes one take reads at most
constexpr size_t kScratch = 1u << 20;        // discard buffer of non-TCP sockets

enum SlotState : int { kFree = 0, kFilling, kInflight, kDone };

struct HubSlot {
    uint8_t* h_buf = nullptr;    // pinned: the frames of every connection, back to back
    uint8_t* d_buf = nullptr;
    uint64_t* h_tab = nullptr;   // pinned: result (3) | header offsets (max_frames + 1) | keys (max_frames, u32)
    uint64_t* d_tab = nullptr;
    uint8_t* b0 = nullptr;       // host: header byte 0 per frame
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;
    int state = kFree;
    uint64_t fill = 0, nframes = 0;
    uint32_t refs = 0;           // ranges of connections not yet consumed
    uint64_t gen = 0;            // which filling of the slot (ranges check it)
    uint32_t nconn = 0;          // connections with frames in it
    uint64_t* hdr() { return h_tab + 3; }
};

struct Range {
    int slot;
    uint64_t gen;
    uint64_t k0, n, next;        // frames [k0, k0 + n) of the slot; next: frames consumed
};

struct HubConn {
    int fd = -1;
    uint64_t dev = 0, ino = 0;
    int tcp = 0;
    uint64_t in_pos = 0, sock_pos = 0;   // stream bytes peeked / removed from the socket
    uint8_t* carry = nullptr;            // the incomplete frame's bytes
    size_t carry_len = 0, carry_cap = 0;
    uint8_t* mbuf = nullptr;             // the message so far
    size_t msize = 0, mcap = 0;
    uint8_t opcode = 0;
    std::deque<Range> ranges;
    uint64_t last_gen = 0;               // the slot filling this connection last added frames to
    int err = 0;                         // sticky (delivered)
    int pending = 0;                     // an error found behind frames not yet delivered
    bool carry_frames = false;           // the carry may hold complete frames (a full frame table
                                         // stopped the walk): walked before new bytes, hostage kept
    bool closed = false;
    uint8_t* scratch = nullptr;
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

}  // namespace

struct netc_ws_hub {
    int device = 0;
    int strict = 0;
    int nslots = 0;
    uint64_t slot_bytes = 0, max_frame = 0, max_frames = 0;
    HubSlot* slots = nullptr;
    int cur = -1;                // the filling slot
    uint64_t gens = 0;
    uint64_t swept_gen = ~0ull;  // the generation a full pool last looked for closed holders at
    std::unordered_map<int, HubConn*> conns;
    struct netc_ws_hub_stats st{};
};

namespace {

void free_slot(HubSlot& s) {
    if (s.stream) (void)hipStreamSynchronize(s.stream);
    if (s.h_buf) (void)hipHostFree(s.h_buf);
    if (s.h_tab) (void)hipHostFree(s.h_tab);
    if (s.d_buf) (void)hipFree(s.d_buf);
    if (s.d_tab) (void)hipFree(s.d_tab);
    free(s.b0);
    if (s.done) (void)hipEventDestroy(s.done);
    if (s.stream) (void)hipStreamDestroy(s.stream);
    s = HubSlot();
}

uint64_t tab_bytes(const netc_ws_hub* h) { return (3 + h->max_frames + 1) * 8 + h->max_frames * 4; }

int alloc_slot(const netc_ws_hub* h, HubSlot& s) {
    hipError_t e;
    if ((e = hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking)) != hipSuccess ||
        (e = hipEventCreateWithFlags(&s.done, hipEventDisableTiming)) != hipSuccess)
        return api_fail_hip(NETC_GPU_ERUNTIME, "hub: stream / event create", e);
    if ((e = hipHostMalloc((void**)&s.h_buf, h->slot_bytes, hipHostMallocDefault)) != hipSuccess ||
        (e = hipHostMalloc((void**)&s.h_tab, tab_bytes(h), hipHostMallocDefault)) != hipSuccess)
        return api_fail_hip(NETC_GPU_ENOMEM, "hub: pinned host allocation", e);
    if ((e = hipMalloc((void**)&s.d_buf, h->slot_bytes)) != hipSuccess ||
        (e = hipMalloc((void**)&s.d_tab, tab_bytes(h))) != hipSuccess)
        return api_fail_hip(NETC_GPU_ENOMEM, "hub: device allocation", e);
    if (!(s.b0 = (uint8_t*)malloc(h->max_frames))) return api_fail(NETC_GPU_ENOMEM, "hub: host allocation");
    return 0;
}

// a slot nobody needs any more goes back to the pool (its GPU work is done: every range that
// pointed into it was consumed after waiting for it)
void maybe_free(HubSlot& s) {
    if (s.refs == 0 && s.state == kDone) s.state = kFree;
}

void drop_conn(netc_ws_hub* h, HubConn* c);
bool sock_identity(int fd, uint64_t* dev, uint64_t* ino);
int hub_route(void* ctx, int sockfd, struct ws_frame_parsing_state* state, size_t max_payload_length);

// Connections closed without a detach that close tracking did not see (include/ws/route.h): their
// undelivered frames pin slots nobody will drain.  Dropped, with their routes; how many.
size_t sweep_closed(netc_ws_hub* h) {
    size_t n = 0;
    for (auto it = h->conns.begin(); it != h->conns.end();) {
        uint64_t d = 0, i = 0;
        HubConn* c = it->second;
        if (!c->ranges.empty() && !(sock_identity(c->fd, &d, &i) && d == c->dev && i == c->ino)) {
            void* ctx = nullptr;
            if (netc_ws_route_get_raw(c->fd, &ctx) == hub_route && ctx == h) (void)netc_ws_route_detach(c->fd);
            drop_conn(h, c);
            it = h->conns.erase(it);
            ++n;
        } else {
            ++it;
        }
    }
    h->st.connections = h->conns.size();
    return n;
}

// the filling slot, a new one if there is none; -1 (FULL) when every slot holds undelivered frames
int acquire(netc_ws_hub* h) {
    if (h->cur >= 0) return h->cur;
    for (int pass = 0; pass < 2; ++pass) {
        for (int i = 0; i < h->nslots; ++i) {
            HubSlot& s = h->slots[i];
            if (s.state == kInflight && s.refs == 0 && hipEventQuery(s.done) == hipSuccess) s.state = kDone;
            maybe_free(s);
            if (s.state != kFree) continue;
            s.state = kFilling;
            s.fill = s.nframes = 0;
            s.refs = s.nconn = 0;
            s.gen = ++h->gens;
            return h->cur = i;
        }
        // every slot is held: once per filling generation, look for holders that are gone
        if (pass || h->swept_gen == h->gens) break;
        h->swept_gen = h->gens;
        if (!sweep_closed(h)) break;
    }
    return -1;
}

// the filling slot goes to the GPU (see the file comment)
int submit(netc_ws_hub* h) {
    if (h->cur < 0) return 0;
    HubSlot& s = h->slots[h->cur];
    if (s.nframes == 0) return 0;
    if (netc_gpu::inject_fault()) return api_fail(NETC_GPU_ELAUNCH, "hub: injected fault (NETC_GPU_KNOB_INJECT_FAULT)");
    DeviceGuard dg(h->device);
    if (dg.err != hipSuccess) return api_fail_hip(NETC_GPU_ERUNTIME, "hipSetDevice", dg.err);
    const uint64_t n = s.nframes;
    uint64_t* res = s.h_tab;
    res[0] = n;
    res[1] = s.fill;
    res[2] = ~0ull;
    s.hdr()[n] = s.fill;
    // table: result | header offsets (one copy), keys where they were written (a second copy):
    // nothing is moved on the host, so a failed submission leaves the slot as it was
    const uint64_t keys_at = 3 + h->max_frames + 1;   // u64 index of the keys region
    hipError_t e;
    if ((e = hipMemcpyAsync(s.d_buf, s.h_buf, s.fill, hipMemcpyHostToDevice, s.stream)) != hipSuccess ||
        (e = hipMemcpyAsync(s.d_tab, s.h_tab, (3 + n + 1) * 8, hipMemcpyHostToDevice, s.stream)) != hipSuccess ||
        (e = hipMemcpyAsync(s.d_tab + keys_at, s.h_tab + keys_at, n * 4, hipMemcpyHostToDevice, s.stream)) !=
            hipSuccess)
        return api_fail_hip(NETC_GPU_ERUNTIME, "hub: H2D copy", e);
    const uint64_t* d_hdr = s.d_tab + 3;
    const uint32_t* d_keys = (const uint32_t*)(s.d_tab + keys_at);
    if ((e = netc_gpu::launch_unmask_scanned(s.d_buf, s.fill, d_hdr, d_keys, n, s.d_tab, s.stream,
                                             netc_gpu::api_cfg())) != hipSuccess)
        return api_fail_hip(NETC_GPU_ELAUNCH, "hub: unmask launch", e);
    if ((e = hipMemcpyAsync(s.h_buf, s.d_buf, s.fill, hipMemcpyDeviceToHost, s.stream)) != hipSuccess ||
        (e = hipEventRecord(s.done, s.stream)) != hipSuccess)
        return api_fail_hip(NETC_GPU_ERUNTIME, "hub: D2H copy", e);
    s.state = kInflight;
    h->cur = -1;
    h->st.launches++;
    h->st.frames += n;
    h->st.bytes += s.fill;
    h->st.connection_slots += s.nconn;
    if (s.nconn > h->st.max_connections) h->st.max_connections = s.nconn;
    return 0;
}

// header decode (src/ws/common.c:146-296): header length, payload length; false if the bytes
// there do not hold the whole header yet
bool decode(const uint8_t* p, size_t room, uint64_t* hl, uint64_t* pl) {
    if (room < 2) return false;
    const uint8_t second = p[1];
    const uint64_t code = second & 0x7F;
    const uint64_t ext = code == 126 ? 2 : code == 127 ? 8 : 0;
    const uint64_t h = 2 + ext + ((second & 0x80) ? 4 : 0);
    if (room < h) return false;
    uint64_t len = code;
    if (ext) {
        len = 0;
        for (uint64_t i = 0; i < ext; ++i) len = len << 8 | p[2 + i];
    }
    *hl = h;
    *pl = len;
    return true;
}

// the checks of NETC_WS_INGEST_STRICT (RFC 6455 §5.1-5.5; as ws_scan_cpu.c)
bool forbidden(const uint8_t* p, uint64_t pl) {
    const uint8_t first = p[0], second = p[1];
    const unsigned op = first & 0x0F;
    if (!(second & 0x80)) return true;
    if (first & 0x70) return true;
    if ((op >= 3 && op <= 7) || op >= 11) return true;
    if (op >= 8 && (!(first & 0x80) || pl > 125)) return true;
    if ((second & 0x7F) == 127 && (pl >> 63)) return true;
    return false;
}

// Complete frames of [buf, buf + len), recorded from table entry `at` on (at most cap of them):
// *cut = where the first frame not recorded starts; *err = the code that stops the stream
// there (PAYLOAD_TOO_BIG / INVALID_FRAME_LENGTH), 0 if it is only incomplete or the table full.
uint64_t walk(const netc_ws_hub* h, HubSlot& s, const uint8_t* buf, uint64_t base, uint64_t len, uint64_t cap,
              uint64_t* cut, int* err) {
    uint64_t p = 0, n = 0;
    *err = 0;
    uint32_t* keys = (uint32_t*)(s.hdr() + h->max_frames + 1);
    while (n < cap) {
        uint64_t hl = 0, pl = 0;
        if (!decode(buf + p, len - p, &hl, &pl)) break;
        if (h->strict && forbidden(buf + p, pl)) {
            *err = WS_FRAME_PARSE_ERROR_INVALID_FRAME_LENGTH;
            break;
        }
        if (pl > h->max_frame) {
            *err = WS_FRAME_PARSE_ERROR_PAYLOAD_TOO_BIG;
            break;
        }
        if (hl + pl > len - p) break;   // not complete yet
        const uint64_t k = s.nframes + n;
        s.hdr()[k] = base + p;
        uint32_t key = 0;
        if (buf[p + 1] & 0x80) memcpy(&key, buf + p + hl - 4, 4);
        keys[k] = key;
        s.b0[k] = buf[p];
        ++n;
        p += hl + pl;
    }
    *cut = p;
    return n;
}

// remove the socket's bytes up to stream position `to` (<= in_pos; the hub has them)
int sock_consume(HubConn& c, uint64_t to) {
    while (c.sock_pos < to) {
        const uint64_t want = to - c.sock_pos;
        ssize_t r;
        if (c.tcp) {
            r = recv(c.fd, nullptr, (size_t)want, MSG_TRUNC | MSG_DONTWAIT);
            if (r < 0 && errno == EFAULT) {
                c.tcp = 0;
                continue;
            }
        } else {
            if (!c.scratch && !(c.scratch = (uint8_t*)malloc(kScratch)))
                return api_fail(NETC_GPU_ENOMEM, "hub: discard buffer");
            r = recv(c.fd, c.scratch, (size_t)(want < kScratch ? want : kScratch), MSG_DONTWAIT);
        }
        if (r < 0 && errno == EINTR) continue;
        if (r <= 0) {
            const int saved = r < 0 ? errno : ECONNRESET;
            api_fail(NETC_WS_INGEST_ERECV, "hub: removing read bytes from socket %d: %s", c.fd, strerror(saved));
            netc_errno_reason = kBadRecv;
            errno = saved;
            return NETC_WS_INGEST_ERECV;
        }
        c.sock_pos += (uint64_t)r;
    }
    return 0;
}

bool grow(uint8_t*& buf, size_t& cap, size_t need) {
    if (need <= cap && buf) return true;
    size_t c = cap ? cap : 256;
    while (c < need) c *= 2;
    uint8_t* nb = (uint8_t*)realloc(buf, c);
    if (!nb) return false;
    buf = nb;
    cap = c;
    return true;
}

// One take (see the file comment): new bytes (> 0; *frames = complete frames added to the
// filling slot), 0 when the socket has nothing new, or a code (NETC_WS_INGEST_CLOSED / FULL / ...).
long take(netc_ws_hub* h, HubConn& c, uint64_t* frames) {
    *frames = 0;
    int cur = acquire(h);
    if (cur < 0) return NETC_WS_INGEST_FULL;
    // room for the carry and a useful read, else the next slot
    if (h->slots[cur].fill + c.carry_len + 4096 > h->slot_bytes ||
        h->slots[cur].nframes + 64 > h->max_frames) {
        if (int e = submit(h)) return e;
        if ((cur = acquire(h)) < 0) return NETC_WS_INGEST_FULL;
    }
    HubSlot& s = h->slots[cur];
    const uint64_t seg = s.fill;
    uint8_t* dst = s.h_buf + seg;
    if (c.carry_len) memcpy(dst, c.carry, c.carry_len);
    size_t room = (size_t)(h->slot_bytes - seg - c.carry_len);
    if (room > kPeek) room = kPeek;
    const int held = (int)(c.in_pos - c.sock_pos);
    if (held > 1) return api_fail(NETC_GPU_ERUNTIME, "hub: %d bytes held in socket %d", held, c.fd);
    // a carry with complete frames is walked even when the socket has nothing new, and the
    // hostage stays: the caller must come back for those frames' messages
    const bool stale = c.carry_frames;
    ssize_t r;
    bool eof = false;
    for (int pass = 0;; ++pass) {
        uint8_t skip[1];
        const int k = (int)(c.in_pos - c.sock_pos);
        struct iovec iov[2] = {{skip, (size_t)k}, {dst + c.carry_len, room}};
        struct msghdr mh;
        memset(&mh, 0, sizeof mh);
        mh.msg_iov = k ? iov : iov + 1;
        mh.msg_iovlen = k ? 2 : 1;
        do r = recvmsg(c.fd, &mh, MSG_PEEK | MSG_DONTWAIT);   // (never blocks the loop, blocking socket or not)
        while (r < 0 && errno == EINTR);
        if (r > 0 && r <= k) {   // only the hostage: release it and look once more
            if (pass == 0 && held && !stale) {
                if (int e = sock_consume(c, c.in_pos)) return e;
                continue;
            }
            r = 0;
            break;
        }
        if (r > 0) r -= k;
        else if (r == 0) eof = true;
        break;
    }
    if (r < 0) {
        if (errno != EAGAIN && errno != EWOULDBLOCK) {
            const int saved = errno;
            api_fail(NETC_WS_INGEST_ERECV, "hub: recv on socket %d: %s", c.fd, strerror(saved));
            netc_errno_reason = kBadRecv;
            errno = saved;
            return NETC_WS_INGEST_ERECV;
        }
        r = 0;
    }
    if (r == 0 && !stale) {
        if (eof) return api_fail(NETC_WS_INGEST_CLOSED, "hub: socket %d: the peer closed the connection", c.fd);
        return 0;
    }
    c.in_pos += (uint64_t)r;
    const uint64_t len = c.carry_len + (uint64_t)r;
    uint64_t cut = 0;
    int err = 0;
    const uint64_t cap = h->max_frames - s.nframes;
    const uint64_t n = walk(h, s, dst, seg, len, cap, &cut, &err);
    if (err) c.pending = err;
    c.carry_frames = !err && n == cap && cut < len;   // a full table: complete frames may follow
    if (n) {
        c.ranges.push_back(Range{cur, s.gen, s.nframes, n, 0});
        s.nframes += n;
        s.fill = seg + cut;
        ++s.refs;
        if (c.last_gen != s.gen) {
            c.last_gen = s.gen;
            ++s.nconn;
        }
    }
    // the incomplete tail (or, after an error, nothing more is needed) is the carry now
    const uint64_t tail = err ? 0 : len - cut;
    if (tail && !grow(c.carry, c.carry_cap, tail)) return api_fail(NETC_GPU_ENOMEM, "hub: carry buffer");
    if (tail) memmove(c.carry, dst + cut, tail);
    c.carry_len = tail;
    if (c.in_pos > c.sock_pos + 1)
        if (int e = sock_consume(c, c.in_pos - 1)) return e;
    *frames = n;
    if (s.fill + 4096 > h->slot_bytes || c.carry_frames) (void)submit(h);   // full: on its way now (errors resurface)
    return r > 0 ? r : (n > 0 || c.carry_frames ? 1 : 0);   // > 0: progress (new bytes or carried frames)
}

bool m_append(HubConn& c, const uint8_t* p, size_t n) {
    if (!grow(c.mbuf, c.mcap, c.msize + n)) return false;
    if (n) memcpy(c.mbuf + c.msize, p, n);
    c.msize += n;
    return true;
}

// The connection's next message from its ranges: 0 (filled), 1 (no frames pending), 2 (its next
// frames are in the filling slot, not launched yet), or a code.
int deliver(netc_ws_hub* h, HubConn& c, struct ws_message* out, size_t max_payload_length) {
    while (!c.ranges.empty()) {
        Range& r = c.ranges.front();
        HubSlot& s = h->slots[r.slot];
        if (s.gen != r.gen) return api_fail(NETC_GPU_ERUNTIME, "hub: a range outlived its slot");
        if (s.state == kFilling) return 2;
        if (s.state == kInflight) {
            hipError_t e = hipEventSynchronize(s.done);
            if (e != hipSuccess) return api_fail_hip(NETC_GPU_ERUNTIME, "hub: slot wait", e);
            s.state = kDone;
        }
        const uint64_t* hdr = s.hdr();
        while (r.next < r.n) {
            const uint64_t k = r.k0 + r.next++;
            const uint8_t* f = s.h_buf + hdr[k];
            uint64_t hl = 0, pl = 0;
            (void)decode(f, hdr[k + 1] - hdr[k], &hl, &pl);
            const uint8_t b0 = s.b0[k], op = b0 & 0x0F;
            if (op != WS_OPCODE_CONTINUE) c.opcode = op;                       // :163-164
            if (pl + c.msize > max_payload_length) return WS_FRAME_PARSE_ERROR_PAYLOAD_TOO_BIG;   // :210, :261
            if (!m_append(c, f + hl, (size_t)pl)) return api_fail(NETC_GPU_ENOMEM, "hub: message buffer");
            if (b0 & 0x80) {                                                   // FIN (:340-346)
                if (c.opcode == WS_OPCODE_TEXT && !m_append(c, (const uint8_t*)"", 1))
                    return api_fail(NETC_GPU_ENOMEM, "hub: message buffer");
                if (!c.mbuf && !(c.mbuf = (uint8_t*)malloc(1))) return api_fail(NETC_GPU_ENOMEM, "hub: message buffer");
                out->opcode = c.opcode;
                out->buffer = c.mbuf;
                out->payload_length = c.msize;
                c.mbuf = nullptr;
                c.msize = c.mcap = 0;
                if (r.next == r.n) {
                    --s.refs;
                    maybe_free(s);
                    c.ranges.pop_front();
                }
                return 0;
            }
        }
        --s.refs;
        maybe_free(s);
        c.ranges.pop_front();
    }
    return 1;
}

void drop_conn(netc_ws_hub* h, HubConn* c) {
    for (const Range& r : c->ranges) {
        HubSlot& s = h->slots[r.slot];
        if (s.gen == r.gen && s.refs) {
            if (s.state == kInflight) (void)hipEventSynchronize(s.done), s.state = kDone;
            --s.refs;
            maybe_free(s);
        }
    }
    free(c->carry);
    free(c->mbuf);
    free(c->scratch);
    delete c;
}

bool sock_identity(int fd, uint64_t* dev, uint64_t* ino) {
    struct stat st;
    if (fstat(fd, &st) != 0 || !S_ISSOCK(st.st_mode)) return false;
    *dev = (uint64_t)st.st_dev;
    *ino = (uint64_t)st.st_ino;
    return true;
}

// close() on an attached socket (close tracking, include/ws/route.h): its frames stop holding slots
void hub_close_hook(void* ctx, int sockfd) { (void)netc_ws_gpu_detach_hub(sockfd); }

// ws_parse_frame on a socket attached to a hub (include/ws/hub.h)
int hub_route(void* ctx, int sockfd, struct ws_frame_parsing_state* state, size_t max_payload_length) {
    netc_ws_hub* h = (netc_ws_hub*)ctx;
    auto it = h->conns.find(sockfd);
    if (it == h->conns.end()) return api_fail(NETC_GPU_EINVAL, "hub: socket %d is not attached", sockfd);
    HubConn& c = *it->second;
    if (c.err) return c.err;
    bool added = false;
    for (;;) {
        struct ws_message m;
        int r = deliver(h, c, &m, max_payload_length);
        if (r == 0) {
            // nothing of it left -- no frames, no error still to report, no carried frames (its
            // bytes are in the socket as far as the caller is concerned): no hostage
            if (c.ranges.empty() && !c.pending && !c.carry_frames) (void)sock_consume(c, c.in_pos);
            state->message = m;
            return 0;
        }
        if (r < 0) return c.err = r;
        if (r == 2) {
            // its frames wait in the filling slot: the first time, let the loop gather other
            // connections' frames into the same slot (the hostage keeps this socket readable)
            if (added) return 1;
            if (int e = submit(h)) return c.err = e;
            continue;
        }
        // nothing pending
        if (c.pending) return c.err = c.pending;
        if (c.closed) return c.err = WS_FRAME_PARSE_ERROR_RECV;   // the peer closed (:151-154)
        uint64_t frames = 0;
        const long n = take(h, c, &frames);
        if (n > 0) {
            added = added || frames > 0;
            continue;
        }
        if (n == 0) {
            if (c.ranges.empty() && !c.pending && !c.carry_frames) (void)sock_consume(c, c.in_pos);
            return 1;
        }
        if (n == NETC_WS_INGEST_CLOSED) {
            c.closed = true;
            continue;
        }
        if (n == NETC_WS_INGEST_FULL) return 1;   // every slot holds other connections' frames: they drain them
        if (n == NETC_WS_INGEST_ERECV) return c.err = WS_FRAME_PARSE_ERROR_RECV;
        return c.err = (int)n;
    }
}

}  // namespace

extern "C" {

int netc_ws_hub_create(struct netc_ws_hub** out, int device, size_t slot_bytes, int nslots, size_t max_frame_bytes,
                       int flags) {
    if (!out) return api_fail(NETC_GPU_EINVAL, "hub: null output pointer");
    *out = nullptr;
    if (int r = netc_gpu::api_check_device(device)) return r;
    if (flags & ~NETC_WS_INGEST_STRICT) return api_fail(NETC_GPU_EINVAL, "hub: unknown flags 0x%x", flags);
    if (!slot_bytes) slot_bytes = 16u << 20;
    if (!nslots) nslots = 8;
    if (!max_frame_bytes) max_frame_bytes = 65536;
    if (nslots < 2 || nslots > 64 || slot_bytes > (1ull << 40) || max_frame_bytes > (1ull << 40) ||
        slot_bytes < max_frame_bytes + 14 + 4096)
        return api_fail(NETC_GPU_EINVAL, "hub: need 2 <= nslots <= 64 and max_frame_bytes + 14 + 4096 <= slot_bytes "
                                         "<= 2^40");
    DeviceGuard dg(device);
    if (dg.err != hipSuccess) return api_fail_hip(NETC_GPU_ERUNTIME, "hipSetDevice", dg.err);
    netc_ws_hub* h = new (std::nothrow) netc_ws_hub();
    if (!h) return api_fail(NETC_GPU_ENOMEM, "hub: host allocation");
    h->device = device;
    h->strict = (flags & NETC_WS_INGEST_STRICT) ? 1 : 0;
    h->nslots = nslots;
    h->slot_bytes = slot_bytes;
    h->max_frame = max_frame_bytes;
    h->max_frames = slot_bytes / 64 + 64;   // a slot submits early when its table fills
    h->slots = new (std::nothrow) HubSlot[nslots];
    if (!h->slots) {
        delete h;
        return api_fail(NETC_GPU_ENOMEM, "hub: host allocation");
    }
    for (int i = 0; i < nslots; ++i) {
        if (int r = alloc_slot(h, h->slots[i])) {
            for (int j = 0; j <= i; ++j) free_slot(h->slots[j]);
            delete[] h->slots;
            delete h;
            return r;
        }
    }
    *out = h;
    return 0;
}

void netc_ws_hub_destroy(struct netc_ws_hub* h) {
    if (!h) return;
    DeviceGuard dg(h->device);
    for (auto& kv : h->conns) {
        void* ctx = nullptr;
        if (netc_ws_route_get_raw(kv.first, &ctx) == hub_route && ctx == h) (void)netc_ws_route_detach(kv.first);
        free(kv.second->carry);
        free(kv.second->mbuf);
        free(kv.second->scratch);
        delete kv.second;
    }
    h->conns.clear();
    for (int i = 0; i < h->nslots; ++i) free_slot(h->slots[i]);
    delete[] h->slots;
    delete h;
}

int netc_ws_gpu_attach_hub(int sockfd, struct netc_ws_hub* h) {
    if (!h) return api_fail(NETC_GPU_EINVAL, "attach_hub: null hub");
    uint64_t dev = 0, ino = 0;
    if (!sock_identity(sockfd, &dev, &ino)) return api_fail(NETC_GPU_EINVAL, "attach_hub: %d is not an open socket", sockfd);
    auto it = h->conns.find(sockfd);
    if (it != h->conns.end()) {
        if (it->second->dev == dev && it->second->ino == ino) return 0;   // already this connection
        drop_conn(h, it->second);                                          // closed without a detach
        h->conns.erase(it);
    }
    int type = 0, domain = 0;
    socklen_t tl = sizeof type, dl = sizeof domain;
    if (getsockopt(sockfd, SOL_SOCKET, SO_TYPE, &type, &tl) != 0 || type != SOCK_STREAM)
        return api_fail(NETC_GPU_EINVAL, "attach_hub: socket %d is not a stream socket", sockfd);
    (void)getsockopt(sockfd, SOL_SOCKET, SO_DOMAIN, &domain, &dl);
    HubConn* c = new (std::nothrow) HubConn();
    if (!c) return api_fail(NETC_GPU_ENOMEM, "attach_hub: host allocation");
    c->fd = sockfd;
    c->dev = dev;
    c->ino = ino;
    c->tcp = domain == AF_INET || domain == AF_INET6;
    if (netc_ws_route_attach(sockfd, hub_route, h) != 0) {
        delete c;
        return api_fail(NETC_GPU_EINVAL, "attach_hub: socket %d: %s", sockfd,
                        errno == EBUSY ? "another route serves it" : "out of range");
    }
    h->conns[sockfd] = c;
    h->st.connections = h->conns.size();
    (void)netc_ws_route_on_close(sockfd, hub_close_hook);
    return 0;
}

int netc_ws_gpu_detach_hub(int sockfd) {
    if (sockfd < 0) return api_fail(NETC_GPU_EINVAL, "detach_hub: socket %d out of range", sockfd);
    void* ctx = nullptr;
    if (netc_ws_route_get_raw(sockfd, &ctx) == hub_route && ctx) {
        netc_ws_hub* h = (netc_ws_hub*)ctx;
        auto it = h->conns.find(sockfd);
        if (it != h->conns.end()) {
            DeviceGuard dg(h->device);
            drop_conn(h, it->second);
            h->conns.erase(it);
            h->st.connections = h->conns.size();
        }
    }
    if (netc_ws_route_detach(sockfd) != 0) return api_fail(NETC_GPU_EINVAL, "detach_hub: socket %d out of range", sockfd);
    return 0;
}

int netc_ws_hub_stats(const struct netc_ws_hub* h, struct netc_ws_hub_stats* out) {
    if (!h || !out) return NETC_GPU_EINVAL;
    *out = h->st;
    return 0;
}

}  // extern "C"
