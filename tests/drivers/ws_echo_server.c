/*
 * An echo server in netc's shape, GPU both ways: the receive hub (include/ws/hub.h) takes every
 * client's masked frames, the egress hub (include/ws/egress_hub.h) sends every reply.
 *
 * Server (main thread): CONNS loopback TCP connections, one level-triggered epoll over them
 * (reference src/tcp/server.c:30-75); per readable socket ONE ws_parse_frame (src/web/server.c:
 * 86-98); each message is answered with ws_send_message -- the same opcode and payload, unmasked
 * as a server sends, one frame -- and, on the hub leg, netc_ws_egress_hub_flush once per loop
 * iteration.  Legs (argv[1]):
 *   hub   every socket attached to one receive hub and one egress hub
 *   cpu   libnetc's ws_parse_frame / ws_send_message on the CPU
 * Clients: 4 writer threads send every connection's messages -- prerendered, masked, 1-3 frames,
 * sizes uniform in [0, MAX_BYTES], round robin, CHUNK bytes per send() (0: one message per
 * send) -- and 4 reader threads hash every byte that comes back per connection (FNV-1a) against
 * the frames of the expected replies.  The clock runs from the first send to the last reply byte.
 * One JSON line on stdout.
 *
 * usage: ws_echo_server hub|cpu CONNS MSGS MAX_BYTES [CHUNK]
 */
#define _GNU_SOURCE
#include <arpa/inet.h>
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
#include "ws/route.h"
#include "ws/hub.h"
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

static int g_conns;
static size_t g_msgs, g_max, g_chunk;
static int *g_cfd;
static uint8_t **g_wire;              /* per connection: every request, masked, back to back */
static size_t *g_wire_len;
static uint64_t *g_got_hash, *g_got_bytes, *g_want_hash, *g_want_bytes;
static uint64_t g_last_ns;

/* frames of one message (header, optional key, payload masked from the frame's first byte) appended */
static void frame(uint8_t **w, size_t *n, size_t *cap, uint8_t op, const uint8_t *msg, size_t len, size_t frames,
                  const uint8_t *key) {
    const size_t split = len / frames, rem = len % frames;
    for (size_t f = 0; f < frames; ++f) {
        const int last = f + 1 == frames;
        const size_t fl = split + (last ? rem : 0), at = f * split;
        while (*cap - *n < fl + 14) {
            *cap = *cap ? 2 * *cap : 1 << 16;
            if (!(*w = realloc(*w, *cap))) exit(4);
        }
        uint8_t *q = *w + *n;
        *q++ = (uint8_t)((last ? 0x80 : 0) | (f == 0 ? op : WS_OPCODE_CONTINUE));
        const uint8_t mbit = key ? 0x80 : 0;
        if (fl <= 125) {
            *q++ = (uint8_t)(mbit | fl);
        } else if (fl <= 0xFFFF) {
            *q++ = mbit | 126;
            *q++ = (uint8_t)(fl >> 8);
            *q++ = (uint8_t)fl;
        } else {
            *q++ = mbit | 127;
            for (int b = 7; b >= 0; --b) *q++ = (uint8_t)((uint64_t)fl >> (8 * b));
        }
        if (key) {
            memcpy(q, key, 4);
            q += 4;
        }
        for (size_t i = 0; i < fl; ++i) q[i] = msg[at + i] ^ (key ? key[i & 3] : 0);
        *n = (size_t)(q + fl - *w);
    }
}

static void message(int c, size_t i, uint8_t *buf, size_t *len, size_t *frames, uint8_t *op, uint8_t key[4]) {
    uint64_t s = 0x9E3779B97F4A7C15ull * (uint64_t)(c + 1) ^ (0xD1B54A32D192ED03ull * (uint64_t)(i + 1));
    lcg(&s);
    *op = (lcg(&s) & 1) ? WS_OPCODE_TEXT : WS_OPCODE_BINARY;
    *len = lcg(&s) % (g_max + 1);
    *frames = 1 + lcg(&s) % 3;
    if (*frames > *len && *len) *frames = *len;
    if (!*len) *frames = 1;
    const uint32_t kv = lcg(&s);
    memcpy(key, &kv, 4);
    for (size_t j = 0; j < *len; ++j) buf[j] = (uint8_t)lcg(&s);
}

struct client_arg {
    int first, count;
};

static void *writer_main(void *p) {
    struct client_arg *a = p;
    size_t *at = calloc((size_t)a->count, sizeof(size_t));
    for (size_t left = 1; left;) {
        left = 0;
        for (int k = 0; k < a->count; ++k) {
            const int c = a->first + k;
            if (at[k] == g_wire_len[c]) continue;
            size_t n = g_wire_len[c] - at[k];
            if (g_chunk && n > g_chunk) n = g_chunk;
            if (!g_chunk) {   /* one message: its frames up to the next FIN */
                const uint8_t *w = g_wire[c] + at[k];
                size_t q = 0;
                for (;;) {
                    const uint8_t code = w[q + 1] & 0x7F;
                    size_t hl = 2 + (code == 126 ? 2 : code == 127 ? 8 : 0) + 4, pl = code;
                    if (code == 126) pl = (size_t)w[q + 2] << 8 | w[q + 3];
                    if (code == 127) {
                        pl = 0;
                        for (int b = 0; b < 8; ++b) pl = pl << 8 | w[q + 2 + b];
                    }
                    const int fin = w[q] & 0x80;
                    q += hl + pl;
                    if (fin) break;
                }
                n = q;
            }
            for (size_t off = 0; off < n;) {
                const ssize_t r = send(g_cfd[c], g_wire[c] + at[k] + off, n - off, MSG_NOSIGNAL);
                if (r <= 0) {
                    if (r < 0 && errno == EINTR) continue;
                    perror("client send");
                    exit(4);
                }
                off += (size_t)r;
            }
            at[k] += n;
            left += g_wire_len[c] - at[k];
        }
    }
    free(at);
    return NULL;
}

static void *reader_main(void *p) {
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
            fprintf(stderr, "client: no reply for 20 s\n");
            exit(3);
        }
        for (int e = 0; e < n; ++e) {
            const int c = (int)evs[e].data.u32;
            const ssize_t r = recv(g_cfd[c], buf, 1 << 20, MSG_DONTWAIT);
            if (r <= 0) continue;
            g_got_hash[c] = fnv(g_got_hash[c], buf, (size_t)r);
            g_got_bytes[c] += (uint64_t)r;
            if (g_got_bytes[c] == g_want_bytes[c]) {
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

/* one pass over the send backlogs: the egress hub's flush, or (CPU leg) each socket's own; bytes
   still held, or -1 on a failure */
static long drain_once(struct netc_ws_egress_hub *tx, const int *sfd) {
    if (tx) {
        if (netc_ws_egress_hub_flush(tx) < 0) {
            fprintf(stderr, "server: flush: %s\n", netc_gpu_strerror());
            return -1;
        }
        return netc_ws_egress_hub_pending(tx);
    }
    long held = 0;
    for (int c = 0; c < g_conns; ++c) {
        const long p = netc_ws_send_pending(sfd[c]) > 0 ? netc_ws_send_flush(sfd[c]) : 0;
        if (p < 0) {
            fprintf(stderr, "server: connection %d: send failed\n", c);
            return -1;
        }
        held += p;
    }
    return held;
}

int main(int argc, char **argv) {
    if (argc < 5) {
        fprintf(stderr, "usage: %s hub|cpu CONNS MSGS MAX_BYTES [CHUNK]\n", argv[0]);
        return 2;
    }
    const int is_hub = !strcmp(argv[1], "hub") || !strcmp(argv[1], "hubcpu");
    if (!is_hub && strcmp(argv[1], "cpu")) return 2;
    g_conns = atoi(argv[2]);
    g_msgs = (size_t)strtoull(argv[3], NULL, 10);
    g_max = (size_t)strtoull(argv[4], NULL, 10);
    g_chunk = argc > 5 ? (size_t)strtoull(argv[5], NULL, 10) : 0;
    if (g_conns < 4 || g_conns % 4) {
        fprintf(stderr, "CONNS must be a multiple of 4\n");
        return 2;
    }
    struct netc_ws_hub *rx = NULL;
    struct netc_ws_egress_hub *tx = NULL;
    if (is_hub && (netc_gpu_init(0) || netc_ws_hub_create(&rx, 0, 16u << 20, 8, g_max > 65536 ? g_max : 65536, 0) ||
                   netc_ws_egress_hub_create(&tx, 0, 16u << 20, 4, 0))) {
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
    struct ws_frame_parsing_state *st = calloc((size_t)g_conns, sizeof(struct ws_frame_parsing_state));
    g_wire = calloc((size_t)g_conns, sizeof(uint8_t *));
    g_wire_len = calloc((size_t)g_conns, sizeof(size_t));
    g_got_hash = malloc(sizeof(uint64_t) * (size_t)g_conns);
    g_got_bytes = calloc((size_t)g_conns, sizeof(uint64_t));
    g_want_hash = malloc(sizeof(uint64_t) * (size_t)g_conns);
    g_want_bytes = calloc((size_t)g_conns, sizeof(uint64_t));
    const int ep = epoll_create1(0);
    uint8_t *buf = malloc(g_max + 16);
    uint64_t payload = 0;
    for (int c = 0; c < g_conns; ++c) {
        g_cfd[c] = socket(AF_INET, SOCK_STREAM, 0);
        if (connect(g_cfd[c], (struct sockaddr *)&a, sizeof a)) {
            perror("connect");
            return 2;
        }
        int one = 1;
        setsockopt(g_cfd[c], IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
        sfd[c] = accept(ls, NULL, NULL);
        setsockopt(sfd[c], IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
        fcntl(sfd[c], F_SETFL, fcntl(sfd[c], F_GETFL, 0) | O_NONBLOCK);
        sp[c].tcp.sockfd = sfd[c];
        sp[c].head.tcp_client = &sp[c].tcp;
        if (is_hub && (netc_ws_gpu_attach_hub(sfd[c], rx) || netc_ws_gpu_attach_send_hub(sfd[c], tx))) {
            fprintf(stderr, "attach: %s\n", netc_gpu_strerror());
            return 2;
        }
        struct epoll_event ev = {.events = EPOLLIN, .data.u32 = (uint32_t)c};
        epoll_ctl(ep, EPOLL_CTL_ADD, sfd[c], &ev);
        /* the requests (masked) and the replies' hash (unmasked, one frame) */
        size_t cap = 0, rn = 0, rcap = 0;
        uint8_t *reply = NULL;
        g_got_hash[c] = g_want_hash[c] = kFnv;
        for (size_t i = 0; i < g_msgs; ++i) {
            size_t len, frames;
            uint8_t op, key[4];
            message(c, i, buf, &len, &frames, &op, key);
            frame(&g_wire[c], &g_wire_len[c], &cap, op, buf, len, frames, key);
            rn = 0;
            frame(&reply, &rn, &rcap, op, buf, len, 1, NULL);
            g_want_hash[c] = fnv(g_want_hash[c], reply, rn);
            g_want_bytes[c] += rn;
            payload += len;
        }
        free(reply);
    }
    close(ls);
    pthread_t wt[4], rt[4];
    struct client_arg ca[4];
    const uint64_t t0 = now_ns();
    for (int t = 0; t < 4; ++t) {
        ca[t].first = t * (g_conns / 4);
        ca[t].count = g_conns / 4;
        pthread_create(&rt[t], NULL, reader_main, &ca[t]);
        pthread_create(&wt[t], NULL, writer_main, &ca[t]);
    }
    const size_t total = (size_t)g_conns * g_msgs;
    size_t done = 0;
    uint64_t iterations = 0;
    struct epoll_event *evs = malloc(sizeof(struct epoll_event) * (size_t)g_conns);
    uint64_t idle_since = 0;
    while (done < total) {
        const int n = epoll_wait(ep, evs, g_conns, 1);
        if (n < 0 && errno == EINTR) continue;
        if (n == 0) {
            /* nothing readable: sockets holding a send backlog (sends never wait) are written as
               far as their peers read; 20 s with neither is a stall */
            if (drain_once(tx, sfd) < 0) return 3;
            const uint64_t t = now_ns();
            if (!idle_since) idle_since = t;
            if (t - idle_since < 20000000000ull) continue;
        } else {
            idle_since = 0;
        }
        if (n <= 0) {
            fprintf(stderr, "server: epoll_wait timed out after %zu of %zu messages\n", done, total);
            return 3;
        }
        ++iterations;
        for (int e = 0; e < n; ++e) {   /* netc: on_data per readable client, once (src/tcp/server.c:72-75) */
            const int c = (int)evs[e].data.u32;
            const int r = ws_parse_frame((struct web_client *)&sp[c].head, &st[c], (size_t)1 << 40);
            if (r < 0) {
                fprintf(stderr, "server: connection %d: ws_parse_frame returned %d (%s)\n", c, r,
                        is_hub ? netc_gpu_strerror() : "");
                return 3;
            }
            if (r != 0) continue;
            struct ws_message *m = &st[c].message;
            struct ws_message reply;   /* the reference appends a NUL to TEXT: not echoed */
            ws_build_message(&reply, m->opcode, m->payload_length - (m->opcode == WS_OPCODE_TEXT), m->buffer);
            if (ws_send_message((struct web_client *)&sp[c].head, &reply, NULL, 1) != 1) {
                fprintf(stderr, "server: connection %d: ws_send_message failed (%s)\n", c,
                        is_hub ? netc_gpu_strerror() : "");
                return 3;
            }
            free(m->buffer);
            memset(&st[c], 0, sizeof st[c]);
            ++done;
        }
        if (tx && netc_ws_egress_hub_flush(tx) < 0) {   /* once per loop iteration */
            fprintf(stderr, "server: flush: %s\n", netc_gpu_strerror());
            return 3;
        }
    }
    /* what the sockets did not take yet (sends never wait): written as the clients read it */
    for (;;) {
        const long p = drain_once(tx, sfd);
        if (p < 0) return 3;
        if (p == 0) break;
        usleep(100);
    }
    for (int t = 0; t < 4; ++t) {
        pthread_join(wt[t], NULL);
        pthread_join(rt[t], NULL);
    }
    struct netc_ws_hub_stats rs;
    struct netc_ws_egress_hub_stats ts;
    memset(&rs, 0, sizeof rs);
    memset(&ts, 0, sizeof ts);
    if (is_hub) {
        netc_ws_hub_stats(rx, &rs);
        netc_ws_egress_hub_stats(tx, &ts);
        for (int c = 0; c < g_conns; ++c) {
            netc_ws_gpu_detach_hub(sfd[c]);
            netc_ws_gpu_detach_send_hub(sfd[c]);
        }
        netc_ws_hub_destroy(rx);
        netc_ws_egress_hub_destroy(tx);
    }
    size_t mismatched = 0;
    for (int c = 0; c < g_conns; ++c) mismatched += g_got_hash[c] != g_want_hash[c];
    const double secs = (double)(g_last_ns - t0) * 1e-9;
    printf("{\"leg\": \"%s\", \"conns\": %d, \"msgs_per_conn\": %zu, \"max_bytes\": %zu, \"chunk\": %zu, "
           "\"messages\": %zu, \"payload_bytes\": %llu, \"seconds\": %.6f, \"round_trips_per_s\": %.1f, "
           "\"gib_per_s_each_way\": %.4f, \"mismatched\": %zu, \"loop_iterations\": %llu, \"rx_launches\": %llu, "
           "\"rx_max_conns_per_launch\": %llu, \"tx_launches\": %llu, \"tx_max_conns_per_launch\": %llu, "
           "\"tx_sendmsg_calls\": %llu}\n",
           argv[1], g_conns, g_msgs, g_max, g_chunk, total, (unsigned long long)payload, secs, (double)total / secs,
           (double)payload / secs / (double)(1ull << 30), mismatched, (unsigned long long)iterations,
           (unsigned long long)rs.launches, (unsigned long long)rs.max_connections, (unsigned long long)ts.launches,
           (unsigned long long)ts.max_connections, (unsigned long long)ts.sendmsg_calls);
    for (int c = 0; c < g_conns; ++c) {
        close(sfd[c]);
        close(g_cfd[c]);
        free(g_wire[c]);
    }
    free(buf);
    return mismatched != 0;
}
