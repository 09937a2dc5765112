/*
 * Receive rates and per-message latency of ws_parse_frame over loopback TCP, driven as netc's
 * server drives it (VERDICT r4 "next" #6): a level-triggered epoll loop that calls ws_parse_frame
 * ONCE per EPOLLIN and goes back to epoll_wait (reference src/tcp/server.c:72-75 ->
 * src/web/server.c:86-98), then frees the message and clears the parser state (:139-140).
 *
 * Legs (argv[1]):
 *   cpu   libnetc's ws_parse_frame on the CPU path (host/ws_common.c)
 *   gpu   the same call with the socket attached to a GPU ingest ring (netc_ws_gpu_attach):
 *         read-ahead with MSG_PEEK into pinned slots, GPU scan (or host walk) + GPU unmask
 *   ref   the REFERENCE's own ws_parse_frame (oracle/_ref/libref_ws.so, compiled from
 *         /root/reference/src/ws/common.c at its own flags, -O0), loaded with dlopen; a frame
 *         is started only once its header, key and one payload byte are readable, because its
 *         parser corrupts its buffer when the payload's first recv() would block (defect B6,
 *         src/ws/common.c:306-315; later recv()s run only on a readiness event, so have data)
 * Client (a second thread): libnetc's CPU ws_send_message, one masked frame per message, its
 * own key per message; the first 16 payload bytes carry the send time and the message index.
 *   open loop (default)   every message sent back to back: the receive rate, and the latency
 *                         of a message under that load (queueing included)
 *   closed loop (argv[4] = 1)   the next message is sent once the server has delivered the
 *                         previous one: the latency of one message alone
 * Every delivered message is checked (length, index, and its first and last 64 payload bytes).
 * One JSON line on stdout.
 *
 * usage: ws_route_bench cpu|gpu|ref MSG_BYTES COUNT [closed 0|1] [slot_bytes] [ref_lib]
 */
#define _GNU_SOURCE
#include <arpa/inet.h>
#include <dlfcn.h>
#include <errno.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <pthread.h>
#include <stdatomic.h>
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
#include "ws/ingest.h"
#include "ws/mask.h"

struct web_client_head {
    struct tcp_client *tcp_client;
};
struct peer {
    struct tcp_client tcp;
    struct web_client_head head;
};

static void peer_init(struct peer *p, int fd) {
    memset(p, 0, sizeof *p);
    p->tcp.sockfd = fd;
    p->head.tcp_client = &p->tcp;
}

static uint64_t now_ns(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (uint64_t)t.tv_sec * 1000000000ull + (uint64_t)t.tv_nsec;
}

static uint32_t lcg(uint64_t *s) {
    *s = *s * 6364136223846793005ull + 1442695040888963407ull;
    return (uint32_t)(*s >> 33);
}

typedef int (*parse_fn)(struct web_client *, struct ws_frame_parsing_state *, size_t);

static size_t g_bytes, g_count;
static int g_closed;
static int g_client_fd;
static const uint8_t *g_template;
static _Atomic uint64_t g_delivered;
static uint64_t g_t0;

static void *client_main(void *arg) {
    (void)arg;
    struct peer cp;
    peer_init(&cp, g_client_fd);
    uint8_t *msg = malloc(g_bytes > 16 ? g_bytes : 16);
    memcpy(msg, g_template, g_bytes);
    uint64_t seed = 0x6E657463;
    g_t0 = now_ns();
    for (size_t i = 0; i < g_count; ++i) {
        if (g_closed)
            while (atomic_load_explicit(&g_delivered, memory_order_acquire) < i) {
            }
        const uint64_t t = now_ns(), idx = i;
        if (g_bytes >= 16) {
            memcpy(msg, &t, 8);
            memcpy(msg + 8, &idx, 8);
        }
        uint8_t key[4];
        const uint32_t k = lcg(&seed);
        memcpy(key, &k, 4);
        struct ws_message m;
        ws_build_message(&m, WS_OPCODE_BINARY, g_bytes, msg);
        if (ws_send_message((struct web_client *)&cp.head, &m, key, 1) != 1) {
            fprintf(stderr, "client: ws_send_message failed\n");
            exit(4);
        }
    }
    free(msg);
    return NULL;
}

static int cmp_u64(const void *a, const void *b) {
    const uint64_t x = *(const uint64_t *)a, y = *(const uint64_t *)b;
    return x < y ? -1 : x > y;
}

int main(int argc, char **argv) {
    if (argc < 4) {
        fprintf(stderr, "usage: %s cpu|gpu|ref MSG_BYTES COUNT [closed 0|1] [slot_bytes] [ref_lib]\n", argv[0]);
        return 2;
    }
    const char *leg = argv[1];
    g_bytes = (size_t)strtoull(argv[2], NULL, 10);
    g_count = (size_t)strtoull(argv[3], NULL, 10);
    g_closed = argc > 4 && atoi(argv[4]) != 0;
    const size_t slot_bytes = argc > 5 ? (size_t)strtoull(argv[5], NULL, 10) : (size_t)16 << 20;
    const char *ref_lib = argc > 6 ? argv[6] : "oracle/_ref/libref_ws.so";
    const int is_gpu = !strcmp(leg, "gpu"), is_ref = !strcmp(leg, "ref");
    if (!is_gpu && !is_ref && strcmp(leg, "cpu")) return 2;

    parse_fn parse = ws_parse_frame;
    if (is_ref) {
        void *h = dlopen(ref_lib, RTLD_NOW | RTLD_LOCAL | RTLD_DEEPBIND);
        if (!h || !(parse = (parse_fn)dlsym(h, "ws_parse_frame"))) {
            fprintf(stderr, "ref: %s\n", dlerror());
            return 2;
        }
    }
    if (is_gpu && netc_gpu_init(0) != 0) {
        fprintf(stderr, "netc_gpu_init: %s\n", netc_gpu_strerror());
        return 2;
    }
    uint8_t *tmpl = malloc(g_bytes + 1);
    uint64_t seed = 0x5eed;
    for (size_t i = 0; i < g_bytes; ++i) tmpl[i] = (uint8_t)lcg(&seed);
    g_template = tmpl;

    int ls = socket(AF_INET, SOCK_STREAM, 0);
    struct sockaddr_in a = {.sin_family = AF_INET, .sin_port = 0};
    a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    socklen_t al = sizeof a;
    if (ls < 0 || bind(ls, (struct sockaddr *)&a, sizeof a) || listen(ls, 1) ||
        getsockname(ls, (struct sockaddr *)&a, &al)) {
        perror("listen");
        return 2;
    }
    g_client_fd = socket(AF_INET, SOCK_STREAM, 0);
    if (connect(g_client_fd, (struct sockaddr *)&a, sizeof a)) {
        perror("connect");
        return 2;
    }
    int one = 1;
    setsockopt(g_client_fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
    const int fd = accept(ls, NULL, NULL);
    close(ls);
    fcntl(fd, F_SETFL, fcntl(fd, F_GETFL, 0) | O_NONBLOCK);
    struct peer sp;
    peer_init(&sp, fd);
    struct netc_ws_ingest *ing = NULL;
    if (is_gpu) {
        const size_t maxf = g_bytes > 65536 ? g_bytes : 65536;
        if (netc_ws_ingest_create(&ing, 0, slot_bytes, 4, maxf, 0) || netc_ws_gpu_attach(fd, ing)) {
            fprintf(stderr, "gpu ring: %s\n", netc_gpu_strerror());
            return 2;
        }
    }
    const int ep = epoll_create1(0);
    struct epoll_event ev = {.events = EPOLLIN | EPOLLRDHUP, .data.fd = fd};
    epoll_ctl(ep, EPOLL_CTL_ADD, fd, &ev);

    uint64_t *lat = malloc(g_count * sizeof(uint64_t));
    const size_t frame_wire = 2 + (g_bytes < 126 ? 0 : g_bytes < 65536 ? 2 : 8) + 4 + g_bytes;
    struct ws_frame_parsing_state st;
    memset(&st, 0, sizeof st);
    uint64_t events = 0, bad = 0, spins = 0;
    pthread_t th;
    pthread_create(&th, NULL, client_main, NULL);
    size_t got = 0;
    while (got < g_count) {
        struct epoll_event e;
        const int n = epoll_wait(ep, &e, 1, 20000);
        if (n < 0 && errno == EINTR) continue;
        if (n <= 0) {
            fprintf(stderr, "server: epoll_wait timed out after %zu of %zu messages\n", got, g_count);
            return 3;
        }
        ++events;
        if (is_ref) {   // (B6: a frame is started only with its header and a payload byte readable)
            int pend = 0;
            ioctl(fd, FIONREAD, &pend);
            if (st.parsing_state == WS_FRAME_NIL && (size_t)pend < frame_wire - g_bytes + (g_bytes ? 1 : 0)) {
                ++spins;
                continue;
            }
        }
        const int r = parse((struct web_client *)&sp.head, &st, (size_t)1 << 40);   // once per event
        if (r < 0) {
            fprintf(stderr, "server: ws_parse_frame returned %d (%s)\n", r, is_gpu ? netc_gpu_strerror() : "");
            return 3;
        }
        if (r != 0) continue;
        const uint64_t t = now_ns();
        const struct ws_message *m = &st.message;
        uint64_t ts = 0, idx = got;
        if (g_bytes >= 16) {
            memcpy(&ts, m->buffer, 8);
            memcpy(&idx, m->buffer + 8, 8);
        }
        const size_t tail = g_bytes > 64 ? 64 : g_bytes;
        if (m->payload_length != g_bytes || idx != got ||
            (g_bytes > 16 && memcmp(m->buffer + 16, tmpl + 16, (g_bytes < 80 ? g_bytes : 80) - 16)) ||
            memcmp(m->buffer + g_bytes - tail, tmpl + g_bytes - tail, g_bytes >= 80 ? tail : 0))
            ++bad;
        lat[got] = g_bytes >= 16 ? t - ts : 0;
        free(m->buffer);                      // src/web/server.c:139
        memset(&st, 0, sizeof st);            // :140
        ++got;
        atomic_store_explicit(&g_delivered, got, memory_order_release);
    }
    const uint64_t t1 = now_ns();
    pthread_join(th, NULL);
    uint64_t gpu_slots = 0, host_slots = 0;
    if (ing) {
        netc_ws_ingest_scan_counts(ing, &gpu_slots, &host_slots);
        netc_ws_gpu_detach(fd);
        netc_ws_ingest_destroy(ing);
    }
    const double secs = (double)(t1 - g_t0) * 1e-9;
    qsort(lat, g_count, sizeof(uint64_t), cmp_u64);
    const double p50 = (double)lat[g_count / 2] * 1e-3, p99 = (double)lat[(g_count * 99) / 100] * 1e-3;
    printf("{\"leg\": \"%s\", \"msg_bytes\": %zu, \"count\": %zu, \"closed_loop\": %d, \"seconds\": %.6f, "
           "\"msgs_per_s\": %.1f, \"gib_per_s\": %.4f, \"lat_p50_us\": %.2f, \"lat_p99_us\": %.2f, \"events\": %llu, "
           "\"ref_spins\": %llu, \"bad\": %llu, \"gpu_slots\": %llu, \"host_slots\": %llu}\n",
           leg, g_bytes, g_count, g_closed, secs, (double)g_count / secs,
           (double)g_count * (double)g_bytes / secs / (double)(1ull << 30), p50, p99, (unsigned long long)events,
           (unsigned long long)spins, (unsigned long long)bad, (unsigned long long)gpu_slots,
           (unsigned long long)host_slots);
    close(fd);
    close(g_client_fd);
    return bad != 0;
}
