/*
 * close() on routed sockets, in a process linked the way netc links libnetc.so (ahead of libc),
 * so close() binds to libnetc.so's definition (include/ws/route.h, "close tracking").
 *
 * netc closes clients without any hook of its own: ws_server_close_client sends a CLOSE frame and
 * closes at once (reference src/ws/server.c:108-125), an EPOLLRDHUP/HUP closes at once
 * (src/tcp/server.c:67-70), and accept() then reuses the descriptor number.  Checked, per MODE:
 *
 *   close  (close() reaches libnetc.so)
 *     1. netc_ws_route_close_tracked() == 1
 *     2. egress hub: messages queued on a socket (no flush), then close(): the peer gets every
 *        byte -- the close hook flushed the hub -- and the hub lets the connection go
 *     3. receive hub: connections whose delivered-but-unconsumed frames hold slots close without a
 *        detach; the hub releases them and a new connection is still served
 *     4. ingest ring and CPU send backlog: nothing of the closed connection is left behind
 *   raw    (close() bypasses libnetc.so: syscall(SYS_close) -- a close the hooks never see)
 *     2'. egress hub: the queued messages never reach a new, unattached socket that got the same
 *         descriptor number; the old connection fails alone
 *     3'. receive hub: the full pool finds the closed holders (identity sweep) and serves a new
 *         connection
 *
 * Linked against libnetc_ws_gpu.so (GPU) or tests/bin/libnetc_ingest_mock.so (the same host code
 * over the host-memory mock, CPU suite).  Prints "ok" and exits 0, else a reason and exits 1.
 *
 * usage: ws_close_track close|raw
 */
#define _GNU_SOURCE
#include <errno.h>
#include <fcntl.h>
#include <poll.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <sys/syscall.h>
#include <unistd.h>

#include "tcp/server.h"
#include "ws/common.h"
#include "ws/egress_hub.h"
#include "ws/hub.h"
#include "ws/ingest.h"
#include "ws/mask.h"
#include "ws/route.h"

struct web_client_head {
    struct tcp_client *tcp_client;
};
struct peer {
    struct tcp_client tcp;
    struct web_client_head head;
};

static int g_raw;

#define CHECK(cond, ...)                                                                            \
    do {                                                                                            \
        if (!(cond)) {                                                                              \
            fprintf(stderr, "%s:%d: ", __FILE__, __LINE__);                                         \
            fprintf(stderr, __VA_ARGS__);                                                           \
            fprintf(stderr, " [%s]\n", netc_gpu_strerror());                                        \
            exit(1);                                                                                \
        }                                                                                           \
    } while (0)

static int fcntl_nonblock(int fd) { return fcntl(fd, F_SETFL, fcntl(fd, F_GETFL, 0) | O_NONBLOCK) < 0 ? -1 : 0; }

static void do_close(int fd) {
    if (g_raw)
        (void)syscall(SYS_close, fd);
    else
        (void)close(fd);
}

static void bind_peer(struct peer *p, int fd) {
    memset(p, 0, sizeof *p);
    p->tcp.sockfd = fd;
    p->head.tcp_client = &p->tcp;
}

static void sockpair(int sv[2]) { CHECK(socketpair(AF_UNIX, SOCK_STREAM, 0, sv) == 0, "socketpair"); }

/* every byte readable on fd until it would block for 200 ms */
static size_t drain(int fd, uint8_t *out, size_t cap) {
    size_t n = 0;
    for (;;) {
        struct pollfd q = {fd, POLLIN, 0};
        if (poll(&q, 1, 200) <= 0) break;
        const ssize_t r = recv(fd, out + n, cap - n, 0);
        if (r <= 0) break;
        n += (size_t)r;
    }
    return n;
}

/* the frames of one unmasked single-frame message (src/ws/common.c:55-82) */
static size_t frame(uint8_t *out, uint8_t op, const uint8_t *p, size_t len) {
    size_t h = 0;
    out[h++] = (uint8_t)(0x80 | op);
    if (len <= 125) {
        out[h++] = (uint8_t)len;
    } else {
        out[h++] = 126;
        out[h++] = (uint8_t)(len >> 8);
        out[h++] = (uint8_t)len;
    }
    memcpy(out + h, p, len);
    return h + len;
}

static int send_msg(struct peer *p, uint8_t op, const uint8_t *buf, size_t len) {
    struct ws_message m;
    ws_build_message(&m, op, len, (uint8_t *)buf);
    return ws_send_message((struct web_client *)&p->head, &m, NULL, 1);
}

/* 2 / 2': queued sends, then the socket is closed */
static void egress_hub_close(void) {
    struct netc_ws_egress_hub *hub = NULL;
    CHECK(netc_ws_egress_hub_create(&hub, 0, 1 << 20, 2, 0) == 0, "egress hub create");
    int sv[2], keep[2];
    sockpair(sv);
    sockpair(keep);
    CHECK(netc_ws_gpu_attach_send_hub(sv[0], hub) == 0, "attach");
    CHECK(netc_ws_gpu_attach_send_hub(keep[0], hub) == 0, "attach");
    struct peer p, k;
    bind_peer(&p, sv[0]);
    bind_peer(&k, keep[0]);
    uint8_t msg[3][300], want[4096];
    size_t wlen = 0;
    for (int i = 0; i < 3; ++i) {
        memset(msg[i], 'a' + i, sizeof msg[i]);
        CHECK(send_msg(&p, WS_OPCODE_BINARY, msg[i], sizeof msg[i]) == 1, "queue");
        wlen += frame(want + wlen, WS_OPCODE_BINARY, msg[i], sizeof msg[i]);
    }
    CHECK(send_msg(&k, WS_OPCODE_TEXT, (const uint8_t *)"other", 5) == 1, "queue other");
    const int fd = sv[0];
    do_close(fd);   /* nothing flushed the hub yet */
    uint8_t got[8192];
    const size_t n = drain(sv[1], got, sizeof got);
    if (!g_raw) {
        CHECK(n == wlen && !memcmp(got, want, wlen), "close(): peer got %zu of %zu queued bytes", n, wlen);
        struct netc_ws_egress_hub_stats st;
        netc_ws_egress_hub_stats(hub, &st);
        CHECK(st.connections == 1, "the closed connection is still attached (%llu)", (unsigned long long)st.connections);
    } else {
        CHECK(n == 0, "raw close: %zu bytes reached the old peer before any flush", n);
        /* the number comes back for a socket nobody attached */
        int nv[2];
        sockpair(nv);
        if (nv[0] != fd) {
            CHECK(dup2(nv[0], fd) == fd, "dup2");
            (void)syscall(SYS_close, nv[0]);
            nv[0] = fd;
        }
        CHECK(netc_ws_egress_hub_flush(hub) >= 0, "flush");
        const size_t leak = drain(nv[1], got, sizeof got);
        CHECK(leak == 0, "a reused descriptor's new peer got %zu bytes of the old connection's frames", leak);
        struct netc_ws_egress_hub_stats st;
        netc_ws_egress_hub_stats(hub, &st);
        CHECK(st.send_errors == 1, "send_errors %llu", (unsigned long long)st.send_errors);
        (void)netc_ws_gpu_detach_send_hub(fd);
        (void)syscall(SYS_close, nv[0]);
        (void)syscall(SYS_close, nv[1]);
    }
    CHECK(netc_ws_egress_hub_flush(hub) >= 0, "flush");
    uint8_t ow[64];
    const size_t olen = frame(ow, WS_OPCODE_TEXT, (const uint8_t *)"other", 5);
    const size_t on = drain(keep[1], got, sizeof got);
    CHECK(on == olen && !memcmp(got, ow, olen), "the other connection got %zu of %zu bytes", on, olen);
    netc_ws_gpu_detach_send_hub(keep[0]);
    netc_ws_egress_hub_destroy(hub);
    do_close(sv[1]);
    do_close(keep[0]);
    do_close(keep[1]);
}

/* masked single-frame message from a client (RFC 6455 §5.3) */
static size_t client_frame(uint8_t *out, const uint8_t *p, size_t len, const uint8_t key[4]) {
    size_t h = 0;
    out[h++] = 0x82;
    out[h++] = (uint8_t)(0x80 | len);
    memcpy(out + h, key, 4);
    h += 4;
    for (size_t i = 0; i < len; ++i) out[h + i] = p[i] ^ key[i & 3];
    return h + len;
}

/* 3 / 3': connections holding slots close without a detach */
static void receive_hub_close(void) {
    struct netc_ws_hub *hub = NULL;
    CHECK(netc_ws_hub_create(&hub, 0, 70000 + 14 + 4096 + 16384, 2, 70000, 0) == 0, "hub create");
    const uint8_t key[4] = {0x37, 0xfa, 0x21, 0x3d};
    uint8_t wire[512], pay[100];
    memset(pay, 'x', sizeof pay);
    for (int round = 0; round < 6; ++round) {   /* more closed holders than slots */
        int sv[2];
        sockpair(sv);
        CHECK(netc_ws_gpu_attach_hub(sv[1], hub) == 0, "attach");
        struct peer p;
        bind_peer(&p, sv[1]);
        size_t n = client_frame(wire, pay, sizeof pay, key);
        n += client_frame(wire + n, pay, sizeof pay, key);   /* two messages: one stays in the hub */
        CHECK(send(sv[0], wire, n, 0) == (ssize_t)n, "send");
        struct ws_frame_parsing_state st;
        memset(&st, 0, sizeof st);
        int rc = 1;
        for (int t = 0; t < 100 && rc == 1; ++t) rc = ws_parse_frame((struct web_client *)&p.head, &st, 1 << 20);
        CHECK(rc == 0 && st.message.payload_length == sizeof pay, "round %d: first message (rc %d)", round, rc);
        free(st.message.buffer);
        do_close(sv[1]);   /* the second message still holds its slot */
        do_close(sv[0]);
    }
    /* a new connection must still get its message */
    int sv[2];
    sockpair(sv);
    CHECK(netc_ws_gpu_attach_hub(sv[1], hub) == 0, "attach");
    struct peer p;
    bind_peer(&p, sv[1]);
    const size_t n = client_frame(wire, pay, 50, key);
    CHECK(send(sv[0], wire, n, 0) == (ssize_t)n, "send");
    struct ws_frame_parsing_state st;
    memset(&st, 0, sizeof st);
    int rc = 1;
    for (int t = 0; t < 100 && rc == 1; ++t) rc = ws_parse_frame((struct web_client *)&p.head, &st, 1 << 20);
    CHECK(rc == 0 && st.message.payload_length == 50, "a new connection is not served (rc %d): slots stay pinned", rc);
    free(st.message.buffer);
    struct netc_ws_hub_stats hs;
    netc_ws_hub_stats(hub, &hs);
    CHECK(hs.connections == 1, "%llu connections still attached", (unsigned long long)hs.connections);
    netc_ws_gpu_detach_hub(sv[1]);
    netc_ws_hub_destroy(hub);
    do_close(sv[0]);
    do_close(sv[1]);
}

/* 4: the ingest ring and the CPU send backlog let go of a closed socket */
static void ring_and_backlog_close(void) {
    struct netc_ws_ingest *ring = NULL;
    CHECK(netc_ws_ingest_create(&ring, 0, 1 << 20, 2, 0, 0) == 0, "ingest create");
    int sv[2];
    sockpair(sv);
    CHECK(netc_ws_gpu_attach(sv[1], ring) == 0, "attach");
    void *ctx = NULL;
    CHECK(netc_ws_route_get_raw(sv[1], &ctx) != NULL, "no route after attach");
    const int fd = sv[1];
    do_close(fd);
    CHECK(netc_ws_route_get_raw(fd, &ctx) == NULL, "the route outlived close()");
    netc_ws_ingest_destroy(ring);
    do_close(sv[0]);

    /* a CPU-path backlog: a peer that does not read, a non-blocking socket */
    int bv[2];
    sockpair(bv);
    int sz = 1 << 14;
    setsockopt(bv[0], SOL_SOCKET, SO_SNDBUF, &sz, sizeof sz);
    setsockopt(bv[1], SOL_SOCKET, SO_RCVBUF, &sz, sizeof sz);
    CHECK(fcntl_nonblock(bv[0]) == 0, "nonblock");
    struct peer p;
    bind_peer(&p, bv[0]);
    static uint8_t big[65536];
    for (int i = 0; i < 8; ++i) CHECK(send_msg(&p, WS_OPCODE_BINARY, big, sizeof big) == 1, "backlogged send");
    CHECK(netc_ws_send_pending(bv[0]) > 0, "nothing held");
    const int bfd = bv[0];
    do_close(bfd);
    int nv[2];
    sockpair(nv);   /* the number again, most likely */
    CHECK(netc_ws_send_pending(nv[0]) == 0 && netc_ws_send_pending(bfd) == 0, "a backlog outlived its connection");
    do_close(bv[1]);
    do_close(nv[0]);
    do_close(nv[1]);
}

int main(int argc, char **argv) {
    if (argc < 2 || (strcmp(argv[1], "close") && strcmp(argv[1], "raw"))) {
        fprintf(stderr, "usage: %s close|raw\n", argv[0]);
        return 2;
    }
    g_raw = !strcmp(argv[1], "raw");
    const int tracked = netc_ws_route_close_tracked();
    const char *verify = getenv("NETC_WS_ROUTE_VERIFY");
    const int forced = verify && *verify && *verify != '0';   /* identity checks forced: not "tracked" */
    CHECK(tracked == !forced, "close() %s libnetc.so in a process linked against it", tracked ? "reaches" : "does not reach");
    egress_hub_close();
    receive_hub_close();
    if (!g_raw) ring_and_backlog_close();
    printf("ok %s tracked=%d\n", argv[1], tracked);
    return 0;
}
