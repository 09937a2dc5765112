/*
 * The GPU receive route under netc's caller contract, over a real TCP connection
 * (VERDICT r2 "missing" #2; driven by tests/test_gpu_epoll.py).
 *
 * Server thread: an epoll loop on a loopback TCP connection, level-triggered like netc's
 * (reference src/tcp/server.c:32-75).  On EPOLLIN it does what netc's web layer does with
 * ws_parse_frame (reference src/web/server.c:69-140), with the GPU ingest ring in its place:
 *   netc_ws_ingest_recv(ing, fd), then netc_ws_ingest_next_message(ing, &m, limit, 1) until it
 *   stops returning 0; per message
 *     < 0             malformed: close 1002 "Malformed frame." (server.c:88-95)
 *     PING            PONG with the same payload, unmasked (server.c:105-113)
 *     PONG            heartbeat, recorded
 *     CLOSE           close frame back with the same code and reason, then the socket is closed
 *                     (server.c:115-136)
 *     TEXT / BINARY   the route's on_message (server.c:137): replies as the reference's own
 *                     test does (tests/ws/test001.c:83-170), plus the checks of this driver
 *   and free(m.buffer) (server.c:139).
 * Client (main thread): a blocking socket driven through libnetc.so's ws_send_message and
 * ws_parse_frame, replaying test001's message script (tests/ws/test001.c:192-273, keys from
 * ws_build_masking_key on a fresh thread), then a ping, one 16 MiB BINARY message in 256
 * frames, a burst of 2,000 fragmented messages sent without waiting, and close 1000 "test".
 *
 * Logs (for the test to compare with libnetc's own ws_parse_frame on the same bytes):
 *   server log: per delivered message  u8 kind ('M','P','Q','C'), u8 opcode, u64 length, payload
 *   client log: per sent message       u8 opcode, u8 masked, u8 key[4], u64 frames, u64 length, payload
 * Exit status 0 when every reply the client checks was right; stdout: one summary line.
 *
 * Route "parse1" (5th argument): the server is netc's own loop -- per EPOLLIN it calls ONLY
 * netc's ws_parse_frame (libnetc.so), exactly ONCE, and goes back to epoll_wait
 * (src/tcp/server.c:72-75 -> src/web/server.c:86-98), with the ring attached to the socket by
 * netc_ws_gpu_attach (include/ws/ingest.h): ws_parse_frame then reads ahead into the ring and
 * returns the GPU-unmasked messages, leaving each later message's bytes in the socket so the
 * level-triggered event fires again for it.  Route "parse": the same, calling
 * ws_parse_frame again after a 0 until it returns 1.  Either way the server memsets its parser
 * state after each message (server.c:139-140).  Route "ingest" (the default):
 * netc_ws_ingest_recv + netc_ws_ingest_next_message directly.
 *
 * usage: ws_gpu_epoll SERVER_LOG CLIENT_LOG [auto|gpu|host] [slot_bytes] [ingest|parse|parse1]
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
#include <unistd.h>

#include "tcp/server.h"
#include "ws/common.h"
#include "ws/ingest.h"
#include "ws/mask.h"

#define BIG_BYTES (16u << 20)
#define BIG_FRAMES 256
#define BURST 2000
#define SERVER_LIMIT (32u << 20)   /* the server's max_payload_len (reference include/web/server.h) */

struct peer {
    struct web_client *wc;   /* libnetc reads only the leading tcp_client pointer */
    struct tcp_client tcp;
};
struct web_client_head {
    struct tcp_client *tcp_client;
};

static void peer_init(struct peer *p, struct web_client_head *h, int fd) {
    memset(&p->tcp, 0, sizeof(p->tcp));
    p->tcp.sockfd = fd;
    h->tcp_client = &p->tcp;
    p->wc = (struct web_client *)h;
}

static uint64_t fnv1a(uint64_t h, const uint8_t *p, size_t n) {
    for (size_t i = 0; i < n; ++i) h = (h ^ p[i]) * 0x100000001b3ull;
    return h;
}
#define FNV0 0xcbf29ce484222325ull

static void log_put(FILE *f, const void *p, size_t n) {
    if (n && fwrite(p, 1, n, f) != n) {
        perror("log write");
        exit(3);
    }
}

/* ------------------------------------------------------------------ server -- */

struct server {
    int listen_fd;
    int port;
    const char *log_path;
    int scan_flags;
    int parse_route;           /* serve through ws_parse_frame on the attached socket: 1 until it
                                  returns 1, 2 once per readiness event (netc's own loop) */
    uint64_t events;           /* epoll wake-ups */
    size_t slot_bytes;
    int rc;                    /* 0 ok */
    uint64_t delivered, gpu_slots, host_slots;
};

static int send_text(struct web_client *wc, const char *s, int masked) {
    struct ws_message m;
    uint8_t key[4];
    ws_build_message(&m, WS_OPCODE_TEXT, strlen(s), (uint8_t *)s);
    if (masked) ws_build_masking_key(key);
    return ws_send_message(wc, &m, masked ? key : NULL, 1);
}

static void send_close(struct web_client *wc, uint16_t code, const uint8_t *reason, size_t rlen) {
    uint8_t buf[128];
    if (rlen > sizeof(buf) - 2) rlen = sizeof(buf) - 2;
    buf[0] = (uint8_t)(code >> 8);
    buf[1] = (uint8_t)code;
    if (rlen) memcpy(buf + 2, reason, rlen);
    struct ws_message m;
    ws_build_message(&m, WS_OPCODE_CLOSE, 2 + rlen, buf);
    ws_send_message(wc, &m, NULL, 1);
}

static void *server_main(void *arg) {
    struct server *S = arg;
    FILE *log = fopen(S->log_path, "wb");
    struct netc_ws_ingest *ing = NULL;
    int fd = -1, ep = -1;
    struct peer pr;
    struct web_client_head head;
    S->rc = 1;
    if (!log) return NULL;
    if (netc_ws_ingest_create(&ing, 0, S->slot_bytes, 4, 65536, S->scan_flags) != 0) {
        fprintf(stderr, "server: ingest create: %s\n", netc_gpu_strerror());
        goto out;
    }
    fd = accept(S->listen_fd, NULL, NULL);
    if (fd < 0) goto out;
    fcntl(fd, F_SETFL, fcntl(fd, F_GETFL, 0) | O_NONBLOCK);
    peer_init(&pr, &head, fd);
    ep = epoll_create1(0);
    struct epoll_event ev = {.events = EPOLLIN, .data.fd = fd};
    if (ep < 0 || epoll_ctl(ep, EPOLL_CTL_ADD, fd, &ev) != 0) goto out;

    if (S->parse_route && netc_ws_gpu_attach(fd, ing) != 0) {
        fprintf(stderr, "server: attach: %s\n", netc_gpu_strerror());
        goto out;
    }
    int burst_count = 0, open = 1;
    uint64_t burst_hash = FNV0;
    struct ws_frame_parsing_state st;   /* parse route: the connection's parser state (web_client's) */
    memset(&st, 0, sizeof st);
    while (open) {
        struct epoll_event got;
        int n = epoll_wait(ep, &got, 1, 20000);
        if (n < 0 && errno == EINTR) continue;
        if (n <= 0) {
            fprintf(stderr, "server: epoll_wait %s (%llu messages delivered)\n", n == 0 ? "timed out" : strerror(errno),
                    (unsigned long long)S->delivered);
            goto out;
        }
        ++S->events;
        if (!S->parse_route) {
            long r = netc_ws_ingest_recv(ing, fd);
            if (r == NETC_WS_INGEST_CLOSED) open = 0;   /* what it sent is still delivered below */
            else if (r < 0 && r != NETC_WS_INGEST_FULL) {
                fprintf(stderr, "server: recv: %ld %s\n", r, netc_gpu_strerror());
                goto out;
            }
        }
        struct ws_message m;
        int res;
        for (;;) {
            if (S->parse_route) {
                /* src/web/server.c:86, unchanged: the attached socket is served from the ring */
                res = ws_parse_frame(pr.wc, &st, SERVER_LIMIT);
                if (res == 0) m = st.message;
            } else {
                res = netc_ws_ingest_next_message(ing, &m, SERVER_LIMIT, 1);
            }
            if (res != 0) break;
            const uint8_t op = m.opcode;
            const uint8_t kind = op == WS_OPCODE_PING ? 'P' : op == WS_OPCODE_PONG ? 'Q' : op == WS_OPCODE_CLOSE ? 'C' : 'M';
            const uint64_t len = m.payload_length;
            log_put(log, &kind, 1);
            log_put(log, &op, 1);
            log_put(log, &len, 8);
            log_put(log, m.buffer, len);
            ++S->delivered;
            if (op == WS_OPCODE_PING) {
                struct ws_message pong;
                ws_build_message(&pong, WS_OPCODE_PONG, len, m.buffer);
                ws_send_message(pr.wc, &pong, NULL, 1);
            } else if (op == WS_OPCODE_CLOSE) {
                uint16_t code = len >= 2 ? (uint16_t)(m.buffer[0] << 8 | m.buffer[1]) : 1005;
                send_close(pr.wc, code, len > 2 ? m.buffer + 2 : NULL, len > 2 ? len - 2 : 0);
                open = 0;
            } else if (op != WS_OPCODE_PONG) {
                /* on_message: test001's replies (tests/ws/test001.c:83-170), then this driver's */
                static const uint8_t bin15[15] = {0, 233, 5, 11, 65, 115, 112, 101, 99, 116, 108, 44, 108, 44, 107};
                const char *t = (const char *)m.buffer;
                if (op == WS_OPCODE_BINARY && len == 15 && memcmp(m.buffer, bin15, 15) == 0)
                    send_text(pr.wc, "hello client masked", 1);
                else if (op == WS_OPCODE_TEXT && strcmp(t, "hello server basic") == 0)
                    send_text(pr.wc, "hello client basic", 0);
                else if (op == WS_OPCODE_TEXT && strcmp(t, "hello server multiple frames") == 0)
                    send_text(pr.wc, "hello client multiple frames", 0);
                else if (op == WS_OPCODE_TEXT && strcmp(t, "hello server multiple frames masked") == 0)
                    send_text(pr.wc, "hello client multiple frames masked", 1);
                else if (op == WS_OPCODE_BINARY && len == BIG_BYTES) {
                    char reply[96];
                    snprintf(reply, sizeof reply, "big fnv=%016llx len=%llu",
                             (unsigned long long)fnv1a(FNV0, m.buffer, len), (unsigned long long)len);
                    send_text(pr.wc, reply, 0);
                } else if (op == WS_OPCODE_TEXT && strcmp(t, "sync") == 0) {
                    char reply[96];
                    snprintf(reply, sizeof reply, "burst count=%d fnv=%016llx", burst_count,
                             (unsigned long long)burst_hash);
                    send_text(pr.wc, reply, 0);
                } else {
                    ++burst_count;
                    burst_hash = fnv1a(burst_hash, m.buffer, len);
                }
            }
            free(m.buffer);   /* the caller owns the message (src/web/server.c:139) */
            if (S->parse_route) memset(&st, 0, sizeof st);   /* src/web/server.c:140 */
            if (!open || S->parse_route == 2) break;         /* netc: back to epoll_wait */
        }
        if (res < 0) {   /* malformed: on_ws_malformed_frame + close 1002 (src/web/server.c:88-95) */
            if (S->parse_route && res == WS_FRAME_PARSE_ERROR_RECV) {
                open = 0;   /* the peer closed and every message before that was returned */
            } else if (open) {
                fprintf(stderr, "server: malformed frame (%d): %s\n", res, netc_gpu_strerror());
                send_close(pr.wc, 1002, (const uint8_t *)"Malformed frame.", 16);
                goto out;
            }
        }
    }
    netc_ws_ingest_scan_counts(ing, &S->gpu_slots, &S->host_slots);
    S->rc = 0;
out:
    if (S->parse_route && fd >= 0) netc_ws_gpu_detach(fd);
    if (ep >= 0) close(ep);
    if (fd >= 0) close(fd);
    if (ing) netc_ws_ingest_destroy(ing);
    fclose(log);
    return NULL;
}

/* ------------------------------------------------------------------ client -- */

static FILE *g_clog;
static int g_fail;

static void client_send(struct web_client *wc, uint8_t op, const uint8_t *payload, size_t len, int masked,
                        size_t frames) {
    uint8_t key[4] = {0, 0, 0, 0};
    struct ws_message m;
    if (masked) ws_build_masking_key(key);
    ws_build_message(&m, op, len, (uint8_t *)payload);
    const int r = ws_send_message(wc, &m, masked ? key : NULL, frames);
    if (r != 1) {
        fprintf(stderr, "client: ws_send_message returned %d\n", r);
        exit(4);
    }
    const uint8_t mk = (uint8_t)masked;
    const uint64_t fr = frames, ln = len;
    log_put(g_clog, &op, 1);
    log_put(g_clog, &mk, 1);
    log_put(g_clog, key, 4);
    log_put(g_clog, &fr, 8);
    log_put(g_clog, &ln, 8);
    log_put(g_clog, payload, len);
}

/* one server message through libnetc's ws_parse_frame (blocking socket) */
static struct ws_message client_recv(struct web_client *wc) {
    struct ws_frame_parsing_state st;
    memset(&st, 0, sizeof st);
    int r;
    while ((r = ws_parse_frame(wc, &st, (size_t)-1)) == 1) {
    }
    if (r < 0) {
        fprintf(stderr, "client: ws_parse_frame returned %d\n", r);
        exit(5);
    }
    return st.message;
}

static void expect_text(struct web_client *wc, const char *want) {
    struct ws_message m = client_recv(wc);
    if (m.opcode != WS_OPCODE_TEXT || strcmp((const char *)m.buffer, want) != 0) {
        fprintf(stderr, "client: expected \"%s\", got opcode %d \"%.*s\"\n", want, m.opcode, (int)m.payload_length,
                (const char *)m.buffer);
        g_fail = 1;
    }
    free(m.buffer);
}

static uint32_t lcg(uint64_t *s) {
    *s = *s * 6364136223846793005ull + 1442695040888963407ull;
    return (uint32_t)(*s >> 33);
}

int main(int argc, char **argv) {
    if (argc < 3) {
        fprintf(stderr, "usage: %s SERVER_LOG CLIENT_LOG [auto|gpu|host] [slot_bytes]\n", argv[0]);
        return 2;
    }
    struct server S;
    memset(&S, 0, sizeof S);
    S.log_path = argv[1];
    S.scan_flags = argc > 3 && !strcmp(argv[3], "gpu") ? NETC_WS_INGEST_SCAN_GPU
                   : argc > 3 && !strcmp(argv[3], "host") ? NETC_WS_INGEST_SCAN_HOST : 0;
    S.slot_bytes = argc > 4 ? (size_t)strtoull(argv[4], NULL, 10) : (size_t)1 << 20;
    S.parse_route = argc > 5 && !strcmp(argv[5], "parse") ? 1 : argc > 5 && !strcmp(argv[5], "parse1") ? 2 : 0;
    if (netc_gpu_init(0) != 0) {   /* keep runtime initialisation off the event loop */
        fprintf(stderr, "netc_gpu_init: %s\n", netc_gpu_strerror());
        return 2;
    }
    S.listen_fd = socket(AF_INET, SOCK_STREAM, 0);
    struct sockaddr_in a = {.sin_family = AF_INET, .sin_port = 0};
    a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    socklen_t al = sizeof a;
    if (S.listen_fd < 0 || bind(S.listen_fd, (struct sockaddr *)&a, sizeof a) != 0 || listen(S.listen_fd, 1) != 0 ||
        getsockname(S.listen_fd, (struct sockaddr *)&a, &al) != 0) {
        perror("listen");
        return 2;
    }
    pthread_t th;
    pthread_create(&th, NULL, server_main, &S);

    g_clog = fopen(argv[2], "wb");
    int cfd = socket(AF_INET, SOCK_STREAM, 0);
    if (!g_clog || cfd < 0 || connect(cfd, (struct sockaddr *)&a, sizeof a) != 0) {
        perror("connect");
        return 2;
    }
    int one = 1;
    setsockopt(cfd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
    struct peer cp;
    struct web_client_head ch;
    peer_init(&cp, &ch, cfd);
    struct web_client *wc = cp.wc;

    /* test001's script (tests/ws/test001.c:192-273), FRAME_SPLIT = 1 */
    const char *s1 = "hello server basic", *s2 = "hello server multiple frames",
               *s4 = "hello server multiple frames masked";
    static const uint8_t bin15[15] = {0, 233, 5, 11, 65, 115, 112, 101, 99, 116, 108, 44, 108, 44, 107};
    client_send(wc, WS_OPCODE_TEXT, (const uint8_t *)s1, strlen(s1), 0, 1);
    expect_text(wc, "hello client basic");
    client_send(wc, WS_OPCODE_TEXT, (const uint8_t *)s2, strlen(s2), 0, 1);
    expect_text(wc, "hello client multiple frames");
    client_send(wc, WS_OPCODE_BINARY, bin15, 15, 1, 1);   /* key 1 of the fresh thread: 00 61 c2 23 */
    expect_text(wc, "hello client masked");
    client_send(wc, WS_OPCODE_TEXT, (const uint8_t *)s4, strlen(s4), 1, 1);   /* key 2: 84 e5 46 a7 */
    expect_text(wc, "hello client multiple frames masked");

    /* heartbeat: PING -> PONG with the same payload (src/web/server.c:105-113) */
    const char *ping = "netc-ping-0123456789";
    client_send(wc, WS_OPCODE_PING, (const uint8_t *)ping, strlen(ping), 1, 1);
    struct ws_message pong = client_recv(wc);
    if (pong.opcode != WS_OPCODE_PONG || pong.payload_length != strlen(ping) ||
        memcmp(pong.buffer, ping, strlen(ping)) != 0) {
        fprintf(stderr, "client: bad pong (opcode %d, %zu bytes)\n", pong.opcode, pong.payload_length);
        g_fail = 1;
    }
    free(pong.buffer);

    /* one 16 MiB BINARY message in 256 masked frames of 64 KiB */
    uint8_t *big = malloc(BIG_BYTES);
    uint64_t seed = 0x6E657463;
    for (size_t i = 0; i < BIG_BYTES; i += 4) {
        const uint32_t v = lcg(&seed);
        memcpy(big + i, &v, 4);
    }
    client_send(wc, WS_OPCODE_BINARY, big, BIG_BYTES, 1, BIG_FRAMES);
    char want[96];
    snprintf(want, sizeof want, "big fnv=%016llx len=%llu", (unsigned long long)fnv1a(FNV0, big, BIG_BYTES),
             (unsigned long long)BIG_BYTES);
    expect_text(wc, want);

    /* a burst of fragmented messages, sent without waiting, then "sync" */
    uint64_t h = FNV0;
    for (int i = 0; i < BURST; ++i) {
        const size_t len = lcg(&seed) % 3001;
        const size_t frames = 1 + lcg(&seed) % 4;
        const uint8_t op = (lcg(&seed) & 1) ? WS_OPCODE_TEXT : WS_OPCODE_BINARY;
        uint8_t *p = big;   /* reuse the buffer: payloads of the burst */
        for (size_t j = 0; j < len; ++j) p[j] = op == WS_OPCODE_TEXT ? (uint8_t)('a' + lcg(&seed) % 26) : (uint8_t)lcg(&seed);
        client_send(wc, op, p, len, 1, len == 0 ? 1 : (frames > len ? len : frames));
        h = fnv1a(h, p, len);
        if (op == WS_OPCODE_TEXT) h = fnv1a(h, (const uint8_t *)"", 1);   /* delivered with its NUL (:342-343) */
    }
    client_send(wc, WS_OPCODE_TEXT, (const uint8_t *)"sync", 4, 1, 1);
    snprintf(want, sizeof want, "burst count=%d fnv=%016llx", BURST, (unsigned long long)h);
    expect_text(wc, want);
    free(big);

    /* close 1000 "test" (test001.c:273): the server answers with the same close */
    static const uint8_t close_payload[6] = {0x03, 0xE8, 't', 'e', 's', 't'};
    client_send(wc, WS_OPCODE_CLOSE, close_payload, 6, 1, 1);
    struct ws_message cl = client_recv(wc);
    if (cl.opcode != WS_OPCODE_CLOSE || cl.payload_length != 6 || memcmp(cl.buffer, close_payload, 6) != 0) {
        fprintf(stderr, "client: bad close reply (opcode %d, %zu bytes)\n", cl.opcode, cl.payload_length);
        g_fail = 1;
    }
    free(cl.buffer);
    close(cfd);
    fclose(g_clog);
    pthread_join(th, NULL);
    printf("{\"server_rc\": %d, \"client_ok\": %d, \"delivered\": %llu, \"gpu_slots\": %llu, \"host_slots\": %llu, "
           "\"events\": %llu, \"route\": \"%s\"}\n",
           S.rc, !g_fail, (unsigned long long)S.delivered, (unsigned long long)S.gpu_slots,
           (unsigned long long)S.host_slots, (unsigned long long)S.events,
           S.parse_route == 2 ? "parse1" : S.parse_route ? "parse" : "ingest");
    return S.rc || g_fail;
}
