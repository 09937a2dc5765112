/*
 * Many connections, one event loop, one GPU egress hub (include/ws/egress_hub.h): the send side
 * of tests/drivers/ws_hub_server.c.
 *
 * Server (main thread): CONNS loopback TCP connections; per loop iteration it answers every
 * client with one message -- netc's ws_send_message (reference src/ws/common.c:36-131; netc's
 * server sends from its callbacks, src/web/server.c:112, :381) -- ROUNDS iterations.  Legs
 * (argv[1]):
 *   hub   every socket attached to one egress hub (netc_ws_gpu_attach_send_hub): the messages of
 *         an iteration share the hub's slots, netc_ws_egress_hub_flush after each iteration
 *   cpu   libnetc's ws_send_message on the CPU
 *   ref   the reference's own ws_send_message (oracle/_ref/libref_ws.so, its flags -O0); TEXT
 *         messages of printable bytes, unmasked (its masked BINARY path overflows the heap
 *         above 254 bytes: defect B1, src/ws/common.c:100)
 * Messages: size uniform in [0, MAX_BYTES], 1-3 frames, from an LCG seeded by (connection,
 * index), unmasked (server to client) unless MASKED = 1.  BURST (default 1): messages to each
 * client per loop iteration (a server fanning out updates), ROUNDS x BURST messages in all.
 *
 * Clients (4 threads, CONNS / 4 sockets each, epoll): read every byte and hash it per
 * connection (FNV-1a over the byte stream).  The server renders the frames it expects on each
 * connection -- the reference's split (src/ws/common.c:42-49), header forms (:55-82), one key
 * per message, each frame masked from its first byte -- and hashes them the same way; the run
 * fails unless every connection's hashes match.  The clock runs from the first send to the last
 * byte received.  One JSON line on stdout.
 *
 * usage: ws_egress_hub_server hub|cpu|ref CONNS ROUNDS MAX_BYTES [MASKED 0|1] [slot_bytes|0] [ref_lib|-] [BURST]
 */
#define _GNU_SOURCE
#include <arpa/inet.h>
#include <dlfcn.h>
#include <errno.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/epoll.h>
#include <sys/socket.h>
#include <time.h>
#include <unistd.h>

#include "tcp/server.h"
#include "ws/common.h"
#include "ws/egress_hub.h"
#include "ws/mask.h"

struct web_client_head {
    struct tcp_client *tcp_client;
};
struct peer {
    struct tcp_client tcp;
    struct web_client_head head;
};

static uint64_t now_ns(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (uint64_t)t.tv_sec * 1000000000ull + (uint64_t)t.tv_nsec;
}

static uint32_t lcg(uint64_t *s) {
    *s = *s * 6364136223846793005ull + 1442695040888963407ull;
    return (uint32_t)(*s >> 33);
}

static const uint64_t kFnv = 0xcbf29ce484222325ull;
static inline uint64_t fnv(uint64_t h, const uint8_t *p, size_t n) {
    for (size_t i = 0; i < n; ++i) h = (h ^ p[i]) * 0x100000001b3ull;
    return h;
}

static int g_conns, g_text;
static size_t g_max;
static int *g_cfd;
static uint64_t *g_got_hash, *g_got_bytes, *g_want_bytes;
static uint64_t g_last_ns;   /* when the last client had every byte (atomic max) */

/* the frames ws_send_message sends for one message, hashed into *h */
static uint64_t hash_frames(uint64_t h, uint8_t op, const uint8_t *msg, size_t len, size_t frames, const uint8_t *key,
                            uint64_t *bytes) {
    const size_t split = len / frames, rem = len % frames;
    uint8_t hdr[14], tmp[4096];
    for (size_t f = 0; f < frames; ++f) {
        const int last = f + 1 == frames;
        const size_t fl = split + (last ? rem : 0), at = f * split;
        size_t hl = 0;
        hdr[hl++] = (uint8_t)((last ? 0x80 : 0) | (f == 0 ? op : WS_OPCODE_CONTINUE));
        const uint8_t mbit = key ? 0x80 : 0;
        if (fl <= 125) {
            hdr[hl++] = (uint8_t)(mbit | fl);
        } else if (fl <= 0xFFFF) {
            hdr[hl++] = mbit | 126;
            hdr[hl++] = (uint8_t)(fl >> 8);
            hdr[hl++] = (uint8_t)fl;
        } else {
            hdr[hl++] = mbit | 127;
            for (int b = 7; b >= 0; --b) hdr[hl++] = (uint8_t)((uint64_t)fl >> (8 * b));
        }
        if (key) {
            memcpy(hdr + hl, key, 4);
            hl += 4;
        }
        h = fnv(h, hdr, hl);
        for (size_t i = 0; i < fl; i += sizeof tmp) {
            const size_t n = fl - i < sizeof tmp ? fl - i : sizeof tmp;
            for (size_t j = 0; j < n; ++j) tmp[j] = msg[at + i + j] ^ (key ? key[(i + j) & 3] : 0);
            h = fnv(h, tmp, n);
        }
        *bytes += hl + fl;
    }
    return h;
}

/* message i of connection c: opcode, bytes, frames */
static void message(int c, size_t i, uint8_t *buf, size_t *len, size_t *frames, uint8_t *op, uint8_t key[4]) {
    uint64_t s = 0x9E3779B97F4A7C15ull * (uint64_t)(c + 1) ^ (0xD1B54A32D192ED03ull * (uint64_t)(i + 1));
    lcg(&s);
    *op = g_text || (lcg(&s) & 1) ? WS_OPCODE_TEXT : WS_OPCODE_BINARY;
    *len = lcg(&s) % (g_max + 1);
    *frames = 1 + lcg(&s) % 3;
    if (*frames > *len && *len) *frames = *len;
    if (!*len) *frames = 1;
    const uint32_t kv = lcg(&s);
    memcpy(key, &kv, 4);
    for (size_t j = 0; j < *len; ++j) buf[j] = g_text ? (uint8_t)(32 + lcg(&s) % 95) : (uint8_t)lcg(&s);
    buf[*len] = 0;
}

struct client_arg {
    int first, count;
};

static void *client_main(void *p) {
    struct client_arg *a = p;
    const int ep = epoll_create1(0);
    for (int k = 0; k < a->count; ++k) {
        struct epoll_event ev = {.events = EPOLLIN, .data.u32 = (uint32_t)(a->first + k)};
        epoll_ctl(ep, EPOLL_CTL_ADD, g_cfd[a->first + k], &ev);
    }
    uint8_t *buf = malloc(1 << 20);
    int left = a->count;
    struct epoll_event evs[64];
    while (left) {
        const int n = epoll_wait(ep, evs, 64, 20000);
        if (n <= 0) {
            if (n < 0 && errno == EINTR) continue;
            fprintf(stderr, "client: epoll_wait timed out\n");
            exit(3);
        }
        for (int e = 0; e < n; ++e) {
            const int c = (int)evs[e].data.u32;
            const ssize_t r = recv(g_cfd[c], buf, 1 << 20, MSG_DONTWAIT);
            if (r <= 0) continue;
            g_got_hash[c] = fnv(g_got_hash[c], buf, (size_t)r);
            g_got_bytes[c] += (uint64_t)r;
            if (g_want_bytes[c] && g_got_bytes[c] == g_want_bytes[c]) {
                --left;
                epoll_ctl(ep, EPOLL_CTL_DEL, g_cfd[c], NULL);
            }
        }
    }
    const uint64_t t = now_ns();
    uint64_t seen = __atomic_load_n(&g_last_ns, __ATOMIC_RELAXED);
    while (t > seen && !__atomic_compare_exchange_n(&g_last_ns, &seen, t, 0, __ATOMIC_RELAXED, __ATOMIC_RELAXED)) {
    }
    free(buf);
    close(ep);
    return NULL;
}

typedef int (*send_fn)(struct web_client *, struct ws_message *, uint8_t *, size_t);

int main(int argc, char **argv) {
    if (argc < 5) {
        fprintf(stderr, "usage: %s hub|cpu|ref CONNS ROUNDS MAX_BYTES [MASKED] [slot_bytes] [ref_lib]\n", argv[0]);
        return 2;
    }
    const char *leg = argv[1];
    g_conns = atoi(argv[2]);
    const size_t rounds = (size_t)strtoull(argv[3], NULL, 10);
    g_max = (size_t)strtoull(argv[4], NULL, 10);
    const int masked = argc > 5 && atoi(argv[5]);
    const size_t slot_bytes = argc > 6 && strtoull(argv[6], NULL, 10) ? (size_t)strtoull(argv[6], NULL, 10) : (size_t)16 << 20;
    const char *ref_lib = argc > 7 && strcmp(argv[7], "-") ? argv[7] : "oracle/_ref/libref_ws.so";
    const size_t burst = argc > 8 && atoi(argv[8]) > 0 ? (size_t)atoi(argv[8]) : 1;
    const size_t nmsg = rounds * burst;   /* messages per connection */
    const int is_hub = !strcmp(leg, "hub") || !strcmp(leg, "hubcpu"), is_ref = !strcmp(leg, "ref");
    if (!is_hub && !is_ref && strcmp(leg, "cpu")) return 2;
    if (g_conns < 4 || g_conns % 4) {
        fprintf(stderr, "CONNS must be a multiple of 4\n");
        return 2;
    }
    g_text = is_ref;   /* the reference's sends: TEXT of printable bytes (B1 / B3) */
    if (is_ref && masked) {
        fprintf(stderr, "ref: unmasked only (B1)\n");
        return 2;
    }
    send_fn snd = ws_send_message;
    if (is_ref) {
        void *h = dlopen(ref_lib, RTLD_NOW | RTLD_LOCAL | RTLD_DEEPBIND);
        if (!h || !(snd = (send_fn)dlsym(h, "ws_send_message"))) {
            fprintf(stderr, "ref: %s\n", dlerror());
            return 2;
        }
    }
    struct netc_ws_egress_hub *hub = NULL;
    if (is_hub && (netc_gpu_init(0) || netc_ws_egress_hub_create(&hub, 0, slot_bytes, 4, 0))) {
        fprintf(stderr, "hub: %s\n", netc_gpu_strerror());
        return 2;
    }
    int ls = socket(AF_INET, SOCK_STREAM, 0);
    struct sockaddr_in a = {.sin_family = AF_INET, .sin_port = 0};
    a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    socklen_t al = sizeof a;
    if (ls < 0 || bind(ls, (struct sockaddr *)&a, sizeof a) || listen(ls, 1024) ||
        getsockname(ls, (struct sockaddr *)&a, &al)) {
        perror("listen");
        return 2;
    }
    g_cfd = malloc(sizeof(int) * (size_t)g_conns);
    int *sfd = malloc(sizeof(int) * (size_t)g_conns);
    struct peer *sp = calloc((size_t)g_conns, sizeof(struct peer));
    g_got_hash = malloc(sizeof(uint64_t) * (size_t)g_conns);
    g_got_bytes = calloc((size_t)g_conns, sizeof(uint64_t));
    g_want_bytes = calloc((size_t)g_conns, sizeof(uint64_t));
    uint64_t *want_hash = malloc(sizeof(uint64_t) * (size_t)g_conns);
    for (int c = 0; c < g_conns; ++c) {
        g_cfd[c] = socket(AF_INET, SOCK_STREAM, 0);
        if (connect(g_cfd[c], (struct sockaddr *)&a, sizeof a)) {
            perror("connect");
            return 2;
        }
        sfd[c] = accept(ls, NULL, NULL);
        int one = 1;
        setsockopt(sfd[c], IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
        sp[c].tcp.sockfd = sfd[c];
        sp[c].head.tcp_client = &sp[c].tcp;
        g_got_hash[c] = want_hash[c] = kFnv;
        if (hub && netc_ws_gpu_attach_send_hub(sfd[c], hub)) {
            fprintf(stderr, "attach: %s\n", netc_gpu_strerror());
            return 2;
        }
    }
    close(ls);
    /* every message rendered and hashed before the clock starts: the expected bytes per connection */
    uint8_t *buf = malloc(g_max + 16);
    uint64_t payload = 0, messages = 0;
    for (int c = 0; c < g_conns; ++c)
        for (size_t i = 0; i < nmsg; ++i) {
            size_t len, frames;
            uint8_t op, key[4];
            message(c, i, buf, &len, &frames, &op, key);
            uint64_t wb = 0;
            want_hash[c] = hash_frames(want_hash[c], op, buf, len, frames, masked ? key : NULL, &wb);
            g_want_bytes[c] += wb;
            payload += len;
            ++messages;
        }
    pthread_t th[4];
    struct client_arg ca[4];
    const uint64_t t0 = now_ns();
    for (int t = 0; t < 4; ++t) {
        ca[t].first = t * (g_conns / 4);
        ca[t].count = g_conns / 4;
        pthread_create(&th[t], NULL, client_main, &ca[t]);
    }
    /* the server's loop: one message to every client per iteration, then (hub) the flush */
    for (size_t i = 0; i < rounds; ++i) {
        for (int c = 0; c < g_conns; ++c) {
            for (size_t b = 0; b < burst; ++b) {
                size_t len, frames;
                uint8_t op, key[4];
                message(c, i * burst + b, buf, &len, &frames, &op, key);
                struct ws_message m;
                ws_build_message(&m, op, len, buf);
                if (snd((struct web_client *)&sp[c].head, &m, masked ? key : NULL, frames) != 1) {
                    fprintf(stderr, "server: connection %d: ws_send_message failed (%s)\n", c,
                            hub ? netc_gpu_strerror() : "");
                    return 3;
                }
            }
        }
        if (hub && netc_ws_egress_hub_flush(hub) < 0) {
            fprintf(stderr, "server: flush: %s\n", netc_gpu_strerror());
            return 3;
        }
    }
    /* what the sockets did not take yet (sends never wait): written as the clients read it */
    while (hub && netc_ws_egress_hub_pending(hub) > 0) {
        usleep(100);
        if (netc_ws_egress_hub_flush(hub) < 0) {
            fprintf(stderr, "server: flush: %s\n", netc_gpu_strerror());
            return 3;
        }
    }
    const uint64_t t_sent = now_ns();
    for (int t = 0; t < 4; ++t) pthread_join(th[t], NULL);
    struct netc_ws_egress_hub_stats hs;
    memset(&hs, 0, sizeof hs);
    if (hub) {
        netc_ws_egress_hub_stats(hub, &hs);
        for (int c = 0; c < g_conns; ++c) netc_ws_gpu_detach_send_hub(sfd[c]);
        netc_ws_egress_hub_destroy(hub);
    }
    size_t mismatched = 0;
    for (int c = 0; c < g_conns; ++c) mismatched += g_got_hash[c] != want_hash[c];
    const double secs = (double)(g_last_ns - t0) * 1e-9;
    printf("{\"leg\": \"%s\", \"conns\": %d, \"rounds\": %zu, \"burst\": %zu, \"max_bytes\": %zu, \"masked\": %d, \"messages\": %llu, "
           "\"payload_bytes\": %llu, \"seconds\": %.6f, \"server_seconds\": %.6f, \"msgs_per_s\": %.1f, "
           "\"gib_per_s\": %.4f, \"mismatched\": %zu, \"launches\": %llu, \"max_conns_per_launch\": %llu, "
           "\"mean_conns_per_launch\": %.2f, \"sendmsg_calls\": %llu, \"send_errors\": %llu}\n",
           leg, g_conns, rounds, burst, g_max, masked, (unsigned long long)messages, (unsigned long long)payload, secs,
           (double)(t_sent - t0) * 1e-9, (double)messages / secs, (double)payload / secs / (double)(1ull << 30),
           mismatched, (unsigned long long)hs.launches, (unsigned long long)hs.max_connections,
           hs.launches ? (double)hs.connection_slots / (double)hs.launches : 0.0,
           (unsigned long long)hs.sendmsg_calls, (unsigned long long)hs.send_errors);
    for (int c = 0; c < g_conns; ++c) {
        close(sfd[c]);
        close(g_cfd[c]);
    }
    free(buf);
    return mismatched != 0;
}
