/*
 * Many connections, one event loop, one GPU hub (include/ws/hub.h; VERDICT r4 "next" #7).
 *
 * Server (main thread): netc's server loop (reference src/tcp/server.c:30-75): one
 * level-triggered epoll over every client socket; for each readable socket ONE ws_parse_frame
 * (src/web/server.c:86-98), then the message is checked, freed and the parser state cleared
 * (:139-140).  Legs (argv[1]):
 *   hub   every socket attached to one GPU hub (netc_ws_gpu_attach_hub): the frames of all
 *         connections share the hub's slots and unmask launches
 *   cpu   libnetc's ws_parse_frame on the CPU
 *   ref   the reference's own ws_parse_frame (oracle/_ref/libref_ws.so, its flags -O0); a
 *         frame is started only once its header and a payload byte are readable (its B6)
 * Clients (4 threads, CONNS / 4 sockets each): libnetc's ws_send_message, round robin over
 * their sockets, MSGS messages per connection: each message's size, fragment count, opcode
 * (TEXT / BINARY, a PING every 37th) and bytes come from an LCG seeded by (connection, index),
 * masked with a key of the same LCG -- so the server knows what each connection sent.
 *
 * Per connection the server keeps a running hash over (opcode, length, bytes) of every message
 * delivered, in order; each client keeps the same hash of what it sent (the message as
 * ws_parse_frame must return it, a TEXT message with its NUL).  Output, one JSON line: per-leg
 * rates, the hub's counters, "mismatched": connections whose hashes differ, and "conn_hash":
 * the per-connection hashes (the same for every leg that delivers exactly what was sent).
 *
 * With VERIFY = 1 the server also regenerates every message and compares it byte for byte.
 *
 * CHUNK (0: off) prerenders the clients' traffic: before the clock starts, each client renders
 * every message of its connections into memory -- the frames ws_send_message sends (the
 * reference's split, src/ws/common.c:42-49; one key, each frame masked from its own first byte);
 * the per-connection hashes check them -- and, timed, sends them round robin over its
 * connections, CHUNK bytes per send().  The clients
 * then cost a send per CHUNK, not a frame's ws_send_message, so the rate is the server's.  The
 * output also carries "clients_seconds": when the last client finished sending.
 *
 * usage: ws_hub_server hub|cpu|ref CONNS MSGS MAX_BYTES [slot_bytes|0] [VERIFY 0|1] [ref_lib|-] [CHUNK]
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
#include <sys/ioctl.h>
#include <sys/socket.h>
#include <time.h>
#include <unistd.h>

#include "tcp/server.h"
#include "ws/common.h"
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

/* message i of connection c: opcode, length, fragments, then the payload bytes from the same state */
struct spec {
    uint8_t op;
    size_t len, frames;
    uint64_t state;
};
static size_t g_max;
static struct spec spec_of(int c, size_t i) {
    struct spec s;
    s.state = 0x9E3779B97F4A7C15ull * (uint64_t)(c + 1) ^ (0xD1B54A32D192ED03ull * (uint64_t)(i + 1));
    lcg(&s.state);
    s.op = i % 37 == 36 ? WS_OPCODE_PING : (lcg(&s.state) & 1) ? WS_OPCODE_TEXT : WS_OPCODE_BINARY;
    s.len = s.op == WS_OPCODE_PING ? lcg(&s.state) % 126 : lcg(&s.state) % (g_max + 1);
    s.frames = s.op == WS_OPCODE_PING ? 1 : 1 + lcg(&s.state) % 3;
    if (s.frames > s.len && s.len) s.frames = s.len;
    if (!s.len) s.frames = 1;
    return s;
}
static void fill(struct spec *s, uint8_t *p) {   /* xorshift64*: 8 bytes a step */
    uint64_t x = s->state | 1;
    size_t j = 0;
    for (; j + 8 <= s->len; j += 8) {
        x ^= x >> 12, x ^= x << 25, x ^= x >> 27;
        const uint64_t v = x * 0x2545F4914F6CDD1Dull;
        memcpy(p + j, &v, 8);
    }
    x ^= x >> 12, x ^= x << 25, x ^= x >> 27;
    const uint64_t v = x * 0x2545F4914F6CDD1Dull;
    memcpy(p + j, &v, s->len - j);
}

/* a word-wise running hash of what a connection delivered (its messages in order) */
static uint64_t mix(uint64_t h, const void *p, size_t n) {
    const uint8_t *b = p;
    size_t i = 0;
    for (; i + 8 <= n; i += 8) {
        uint64_t w;
        memcpy(&w, b + i, 8);
        h = (h ^ w) * 0x9E3779B97F4A7C15ull;
        h ^= h >> 29;
    }
    uint64_t w = 0;
    memcpy(&w, b + i, n - i);
    h = (h ^ w ^ (uint64_t)n << 56) * 0xD1B54A32D192ED03ull;
    return h ^ (h >> 31);
}
static uint64_t msg_hash(uint64_t h, uint8_t op, const uint8_t *p, size_t n) {
    const uint64_t head = (uint64_t)op << 56 | n;
    h = mix(h, &head, 8);
    return mix(h, p, n);
}

static uint64_t *g_want;   /* per connection: the hash of what its client sent */
static int g_verify;

static int g_conns;
static size_t g_msgs;
static int *g_cfd;
static size_t g_chunk;                 /* CHUNK: prerendered traffic, bytes per send() (0: off) */
static pthread_barrier_t g_start;      /* CHUNK: the clients have rendered; the clock starts */
static uint64_t g_clients_end;         /* when the last client finished sending (ns) */
static pthread_mutex_t g_end_mu = PTHREAD_MUTEX_INITIALIZER;

struct client_arg {
    int first, count;
};

static void client_done(void) {
    const uint64_t t = now_ns();
    pthread_mutex_lock(&g_end_mu);
    if (t > g_clients_end) g_clients_end = t;
    pthread_mutex_unlock(&g_end_mu);
}

/* every byte of [p, p + n) on fd (blocking socket) */
static void send_all(int fd, const uint8_t *p, size_t n) {
    while (n) {
        const ssize_t r = send(fd, p, n, MSG_NOSIGNAL);
        if (r < 0 && errno == EINTR) continue;
        if (r <= 0) {
            perror("client send");
            exit(4);
        }
        p += r;
        n -= (size_t)r;
    }
}

struct wire {
    uint8_t *p;
    size_t n, cap, at;
};

/* append the frames of one message as ws_send_message sends them (masked) */
static void render(struct wire *w, uint8_t op, const uint8_t *msg, size_t len, size_t frames, const uint8_t key[4]) {
    const size_t split = len / frames, rem = len % frames;
    for (size_t f = 0; f < frames; ++f) {
        const int last = f + 1 == frames;
        const size_t fl = split + (last ? rem : 0), at = f * split;
        if (w->cap - w->n < fl + 14) {
            while (w->cap - w->n < fl + 14) w->cap = w->cap ? 2 * w->cap : 1 << 20;
            if (!(w->p = realloc(w->p, w->cap))) exit(4);
        }
        uint8_t *q = w->p + w->n;
        *q++ = (uint8_t)((last ? 0x80 : 0) | (f == 0 ? op : WS_OPCODE_CONTINUE));
        if (fl <= 125) {
            *q++ = (uint8_t)(0x80 | fl);
        } else if (fl <= 0xFFFF) {
            *q++ = 0x80 | 126;
            *q++ = (uint8_t)(fl >> 8);
            *q++ = (uint8_t)fl;
        } else {
            *q++ = 0x80 | 127;
            for (int b = 7; b >= 0; --b) *q++ = (uint8_t)((uint64_t)fl >> (8 * b));
        }
        memcpy(q, key, 4);
        q += 4;
        for (size_t i = 0; i < fl; ++i) q[i] = msg[at + i] ^ key[i & 3];
        w->n = (size_t)(q + fl - w->p);
    }
}

static void *client_main(void *p) {
    struct client_arg *a = p;
    struct peer *peers = calloc((size_t)a->count, sizeof(struct peer));
    struct wire *wires = g_chunk ? calloc((size_t)a->count, sizeof(struct wire)) : NULL;
    for (int k = 0; k < a->count; ++k) {
        peers[k].tcp.sockfd = g_cfd[a->first + k];
        peers[k].head.tcp_client = &peers[k].tcp;
    }
    uint8_t *buf = malloc(g_max + 16);
    for (size_t i = 0; i < g_msgs; ++i) {
        for (int k = 0; k < a->count; ++k) {
            const int c = a->first + k;
            struct spec s = spec_of(c, i);
            uint8_t key[4];
            const uint32_t kv = lcg(&s.state);
            memcpy(key, &kv, 4);
            fill(&s, buf);
            buf[s.len] = 0;   /* a TEXT message is delivered with a NUL appended (src/ws/common.c:342) */
            g_want[c] = msg_hash(g_want[c], s.op, buf, s.len + (s.op == WS_OPCODE_TEXT));
            if (g_chunk) {
                render(&wires[k], s.op, buf, s.len, s.frames, key);
                continue;
            }
            struct ws_message m;
            ws_build_message(&m, s.op, s.len, buf);
            if (ws_send_message((struct web_client *)&peers[k].head, &m, key, s.frames) != 1) {
                fprintf(stderr, "client %d: ws_send_message failed\n", c);
                exit(4);
            }
        }
    }
    free(buf);
    if (g_chunk) {
        pthread_barrier_wait(&g_start);   /* rendered: the clock starts */
        for (size_t left = 1; left;) {
            left = 0;
            for (int k = 0; k < a->count; ++k) {
                struct wire *w = &wires[k];
                if (w->at == w->n) continue;
                const size_t n = w->n - w->at < g_chunk ? w->n - w->at : g_chunk;
                send_all(g_cfd[a->first + k], w->p + w->at, n);
                w->at += n;
                left += w->n - w->at;
            }
        }
        for (int k = 0; k < a->count; ++k) free(wires[k].p);
        free(wires);
    }
    client_done();
    free(peers);
    return NULL;
}

typedef int (*parse_fn)(struct web_client *, struct ws_frame_parsing_state *, size_t);

int main(int argc, char **argv) {
    if (argc < 5) {
        fprintf(stderr, "usage: %s hub|cpu|ref CONNS MSGS MAX_BYTES [slot_bytes] [ref_lib]\n", argv[0]);
        return 2;
    }
    const char *leg = argv[1];
    g_conns = atoi(argv[2]);
    g_msgs = (size_t)strtoull(argv[3], NULL, 10);
    g_max = (size_t)strtoull(argv[4], NULL, 10);
    const size_t slot_bytes = argc > 5 && strtoull(argv[5], NULL, 10) ? (size_t)strtoull(argv[5], NULL, 10)
                                                                     : (size_t)16 << 20;
    g_verify = argc > 6 && atoi(argv[6]);
    const char *ref_lib = argc > 7 && strcmp(argv[7], "-") ? argv[7] : "oracle/_ref/libref_ws.so";
    g_chunk = argc > 8 ? (size_t)strtoull(argv[8], NULL, 10) : 0;
    const int is_hub = !strcmp(leg, "hub") || !strcmp(leg, "hubcpu"), is_ref = !strcmp(leg, "ref");
    if (!is_hub && !is_ref && strcmp(leg, "cpu")) return 2;
    if (g_conns < 4 || g_conns % 4) {
        fprintf(stderr, "CONNS must be a multiple of 4\n");
        return 2;
    }
    parse_fn parse = ws_parse_frame;
    if (is_ref) {
        void *h = dlopen(ref_lib, RTLD_NOW | RTLD_LOCAL | RTLD_DEEPBIND);
        if (!h || !(parse = (parse_fn)dlsym(h, "ws_parse_frame"))) {
            fprintf(stderr, "ref: %s\n", dlerror());
            return 2;
        }
    }
    struct netc_ws_hub *hub = NULL;
    if (is_hub) {
        if (netc_gpu_init(0) || netc_ws_hub_create(&hub, 0, slot_bytes, 8, g_max > 65536 ? g_max : 65536, 0)) {
            fprintf(stderr, "hub: %s\n", netc_gpu_strerror());
            return 2;
        }
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
    size_t *got = calloc((size_t)g_conns, sizeof(size_t));
    uint64_t *hash = malloc(sizeof(uint64_t) * (size_t)g_conns);
    g_want = malloc(sizeof(uint64_t) * (size_t)g_conns);
    const int ep = epoll_create1(0);
    int maxfd = 0;
    for (int c = 0; c < g_conns; ++c) {
        g_cfd[c] = socket(AF_INET, SOCK_STREAM, 0);
        if (connect(g_cfd[c], (struct sockaddr *)&a, sizeof a)) {
            perror("connect");
            return 2;
        }
        int one = 1;
        setsockopt(g_cfd[c], IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
        sfd[c] = accept(ls, NULL, NULL);
        fcntl(sfd[c], F_SETFL, fcntl(sfd[c], F_GETFL, 0) | O_NONBLOCK);
        if (sfd[c] > maxfd) maxfd = sfd[c];
        sp[c].tcp.sockfd = sfd[c];
        sp[c].head.tcp_client = &sp[c].tcp;
        hash[c] = g_want[c] = 0xcbf29ce484222325ull;
        if (hub && netc_ws_gpu_attach_hub(sfd[c], hub)) {
            fprintf(stderr, "attach: %s\n", netc_gpu_strerror());
            return 2;
        }
        struct epoll_event ev = {.events = EPOLLIN | EPOLLRDHUP, .data.u32 = (uint32_t)c};
        epoll_ctl(ep, EPOLL_CTL_ADD, sfd[c], &ev);
    }
    close(ls);
    uint8_t *want = malloc(g_max + 16);
    pthread_t th[4];
    struct client_arg ca[4];
    if (g_chunk) pthread_barrier_init(&g_start, NULL, 5);
    uint64_t t0 = now_ns();
    for (int t = 0; t < 4; ++t) {
        ca[t].first = t * (g_conns / 4);
        ca[t].count = g_conns / 4;
        pthread_create(&th[t], NULL, client_main, &ca[t]);
    }
    if (g_chunk) {   /* the clients render first; the clock starts when all have */
        pthread_barrier_wait(&g_start);
        t0 = now_ns();
    }
    const size_t total = (size_t)g_conns * g_msgs;
    size_t done = 0, bad = 0;
    uint64_t events = 0, bytes = 0, spins = 0;
    struct epoll_event *evs = malloc(sizeof(struct epoll_event) * (size_t)g_conns);
    while (done < total) {
        const int n = epoll_wait(ep, evs, g_conns, 20000);
        if (n < 0 && errno == EINTR) continue;
        if (n <= 0) {
            fprintf(stderr, "server: epoll_wait timed out after %zu of %zu messages\n", done, total);
            return 3;
        }
        for (int e = 0; e < n; ++e) {   /* netc: on_data per readable client, once (src/tcp/server.c:72-75) */
            const int c = (int)evs[e].data.u32;
            ++events;
            if (is_ref && st[c].parsing_state == WS_FRAME_NIL) {   /* (B6: header, key and a payload byte) */
                uint8_t h[14];
                const ssize_t k = recv(sfd[c], h, sizeof h, MSG_PEEK);
                size_t need = 2;
                if (k >= 2) {
                    const size_t code = h[1] & 0x7F, ext = code == 126 ? 2 : code == 127 ? 8 : 0;
                    need = 2 + ext + ((h[1] & 0x80) ? 4 : 0);
                    if ((size_t)k >= 2 + ext) {
                        size_t len = code;
                        if (ext) {
                            len = 0;
                            for (size_t b = 0; b < ext; ++b) len = len << 8 | h[2 + b];
                        }
                        need += len ? 1 : 0;
                    } else
                        need = 14;
                }
                int pend = 0;
                ioctl(sfd[c], FIONREAD, &pend);
                if ((size_t)pend < need) {
                    ++spins;
                    continue;
                }
            }
            const int r = parse((struct web_client *)&sp[c].head, &st[c], (size_t)1 << 40);
            if (r < 0) {
                fprintf(stderr, "server: connection %d: ws_parse_frame returned %d (%s)\n", c, r,
                        is_hub ? netc_gpu_strerror() : "");
                return 3;
            }
            if (r != 0) continue;
            const struct ws_message *m = &st[c].message;
            if (g_verify) {
                struct spec s = spec_of(c, got[c]);
                lcg(&s.state);   /* the key */
                fill(&s, want);
                size_t wl = s.len;
                if (s.op == WS_OPCODE_TEXT) want[wl++] = 0;   /* delivered with its NUL (src/ws/common.c:342) */
                if (m->opcode != s.op || m->payload_length != wl || memcmp(m->buffer, want, wl)) ++bad;
            }
            hash[c] = msg_hash(hash[c], m->opcode, m->buffer, m->payload_length);
            bytes += m->payload_length;
            free(m->buffer);
            memset(&st[c], 0, sizeof st[c]);
            ++got[c];
            ++done;
        }
    }
    const uint64_t t1 = now_ns();
    for (int t = 0; t < 4; ++t) pthread_join(th[t], NULL);
    struct netc_ws_hub_stats hs;
    memset(&hs, 0, sizeof hs);
    if (hub) {
        netc_ws_hub_stats(hub, &hs);
        for (int c = 0; c < g_conns; ++c) netc_ws_gpu_detach_hub(sfd[c]);
        netc_ws_hub_destroy(hub);
    }
    const double secs = (double)(t1 - t0) * 1e-9;
    const double csecs = g_clients_end > t0 ? (double)(g_clients_end - t0) * 1e-9 : 0.0;
    size_t mismatched = 0;
    for (int c = 0; c < g_conns; ++c) mismatched += hash[c] != g_want[c];
    printf("{\"leg\": \"%s\", \"conns\": %d, \"msgs_per_conn\": %zu, \"max_bytes\": %zu, \"messages\": %zu, "
           "\"payload_bytes\": %llu, \"seconds\": %.6f, \"msgs_per_s\": %.1f, \"gib_per_s\": %.4f, \"bad\": %zu, "
           "\"mismatched\": %zu, \"verified\": %d, \"chunk\": %zu, \"clients_seconds\": %.6f, "
           "\"events\": %llu, \"ref_spins\": %llu, \"launches\": %llu, \"frames\": %llu, \"max_conns_per_launch\": %llu, "
           "\"mean_conns_per_launch\": %.2f, \"mean_frames_per_launch\": %.1f, \"conn_hash\": [",
           leg, g_conns, g_msgs, g_max, total, (unsigned long long)bytes, secs, (double)total / secs,
           (double)bytes / secs / (double)(1ull << 30), bad, mismatched, g_verify, g_chunk, csecs, (unsigned long long)events, (unsigned long long)spins,
           (unsigned long long)hs.launches, (unsigned long long)hs.frames, (unsigned long long)hs.max_connections,
           hs.launches ? (double)hs.connection_slots / (double)hs.launches : 0.0,
           hs.launches ? (double)hs.frames / (double)hs.launches : 0.0);
    for (int c = 0; c < g_conns; ++c) printf("%s\"%016llx\"", c ? ", " : "", (unsigned long long)hash[c]);
    printf("]}\n");
    for (int c = 0; c < g_conns; ++c) {
        close(sfd[c]);
        close(g_cfd[c]);
    }
    return bad != 0 || mismatched != 0;
}
