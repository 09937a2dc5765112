/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * Drives the REFERENCE's own compiled framing code (Altanis/netc
 * src/ws/common.c: ws_parse_frame, ws_send_message, ws_build_masking_key),
 * built from /root/reference by oracle/Makefile into oracle/_ref/libref_ws.so
 * (never committed).  Used to generate and check golden vectors and as the
 * "reference" CPU baseline.  Not part of the product.
 *
 * Transport: an AF_UNIX socketpair stands in for the TCP connection; the
 * parser is only called while FIONREAD > 0 (level-triggered epoll, as
 * src/tcp/server.c:35-75 calls it), because calling it with nothing pending
 * corrupts its bookkeeping (reference defect B6).
 */
#include "web/client.h"   /* reference headers: -I$(REF)/include (oracle/Makefile) */
#include "ws/common.h"

#include <errno.h>
#include <fcntl.h>
#include <poll.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <sys/ioctl.h>
#include <sys/socket.h>
#include <time.h>
#include <unistd.h>

static int make_pair(int fds[2])
{
    if (socketpair(AF_UNIX, SOCK_STREAM, 0, fds) != 0) return -1;
    int sz = 4 << 20;
    setsockopt(fds[0], SOL_SOCKET, SO_SNDBUF, &sz, sizeof(sz));
    setsockopt(fds[1], SOL_SOCKET, SO_RCVBUF, &sz, sizeof(sz));
    return 0;
}

static size_t pending(int fd)
{
    int n = 0;
    if (ioctl(fd, FIONREAD, &n) != 0) return 0;
    return n > 0 ? (size_t)n : 0;
}

struct parse_ctx
{
    struct web_client client;
    struct tcp_client tcp;
    struct ws_frame_parsing_state st;
    uint8_t *out;          /* concatenated message payloads */
    size_t out_cap, out_len;
    size_t *msg_lens;      /* per message length (as reported by the reference: includes TEXT NUL) */
    uint8_t *msg_ops;
    size_t msg_cap, nmsg;
    size_t max_payload;
    int err;
};

/* call the reference parser while bytes are pending; collect finished messages */
static void drain(struct parse_ctx *c)
{
    while (c->err == 0 && pending(c->tcp.sockfd) > 0)
    {
        const int r = ws_parse_frame(&c->client, &c->st, c->max_payload);
        if (r < 0)
        {
            c->err = r;
            return;
        }
        if (r == 0)
        {
            const size_t n = c->st.message.payload_length;
            if (c->nmsg < c->msg_cap)
            {
                c->msg_lens[c->nmsg] = n;
                c->msg_ops[c->nmsg] = c->st.message.opcode;
            }
            if (c->out_len + n <= c->out_cap) memcpy(c->out + c->out_len, c->st.message.buffer, n);
            c->out_len += n;
            c->nmsg++;
            free(c->st.message.buffer);
            memset(&c->st, 0, sizeof(c->st)); /* as the caller does, src/web/server.c:139-140 */
        }
    }
}

/*
 * Feed `wire` to the reference's ws_parse_frame in chunks of the given sizes
 * (the remainder, if any, as a last chunk).  Returns the number of complete
 * messages (payloads concatenated into out, lengths / opcodes per message), or
 * a negative ws_frame_parsing_errors value, or -100 on a harness failure.
 */
long ref_parse(const uint8_t *wire, size_t wire_len, const size_t *chunks, size_t nchunks, size_t max_payload,
               uint8_t *out, size_t out_cap, size_t *msg_lens, uint8_t *msg_ops, size_t msg_cap)
{
    int fds[2];
    if (make_pair(fds) != 0) return -100;
    struct parse_ctx c;
    memset(&c, 0, sizeof(c));
    c.tcp.sockfd = fds[1];
    c.client.tcp_client = &c.tcp;
    c.out = out;
    c.out_cap = out_cap;
    c.msg_lens = msg_lens;
    c.msg_ops = msg_ops;
    c.msg_cap = msg_cap;
    c.max_payload = max_payload;
    fcntl(fds[1], F_SETFL, fcntl(fds[1], F_GETFL, 0) | O_NONBLOCK);
    fcntl(fds[0], F_SETFL, fcntl(fds[0], F_GETFL, 0) | O_NONBLOCK);

    size_t pos = 0, ci = 0;
    while (pos < wire_len && c.err == 0)
    {
        size_t len = ci < nchunks ? chunks[ci++] : wire_len - pos;
        if (len > wire_len - pos) len = wire_len - pos;
        size_t w = 0;
        while (w < len && c.err == 0)
        {
            const ssize_t r = send(fds[0], wire + pos + w, len - w, 0);
            if (r > 0) w += (size_t)r;
            else if (r < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) drain(&c); /* socket full: let the parser eat */
            else { c.err = -100; break; }
        }
        pos += len;
        drain(&c);
    }
    close(fds[0]);
    close(fds[1]);
    if (c.st.payload_data.elements) free(c.st.payload_data.elements);
    if (c.err) return c.err;
    return (long)c.nmsg;
}

struct reader_arg
{
    int fd;
    uint8_t *out;
    size_t cap, len;
};

static void *reader(void *p)
{
    struct reader_arg *a = p;
    uint8_t sink[65536];
    for (;;)
    {
        const ssize_t r = recv(a->fd, sink, sizeof(sink), 0);
        if (r <= 0) break;
        const size_t n = (size_t)r;
        if (a->len + n <= a->cap) memcpy(a->out + a->len, sink, n);
        a->len += n;
    }
    return NULL;
}

/*
 * Wire bytes the reference's ws_send_message puts on the socket for one
 * message.  key == NULL sends unmasked.  Returns the wire length or -1.  Only
 * call it where the reference has defined behaviour.
 */
long ref_send(uint8_t opcode, const uint8_t *payload, size_t len, const uint8_t *key, size_t num_frames, uint8_t *out,
              size_t out_cap)
{
    int fds[2];
    if (make_pair(fds) != 0) return -1;
    struct reader_arg ra = {fds[1], out, out_cap, 0};
    pthread_t th;
    if (pthread_create(&th, NULL, reader, &ra) != 0) return -1;
    struct tcp_client tcp;
    memset(&tcp, 0, sizeof(tcp));
    tcp.sockfd = fds[0];
    struct web_client client;
    memset(&client, 0, sizeof(client));
    client.tcp_client = &tcp;
    uint8_t *copy = malloc(len + 1);
    memcpy(copy, payload, len);
    copy[len] = 0; /* the reference strdup()s TEXT payloads (src/ws/common.c:96) */
    struct ws_message msg;
    ws_build_message(&msg, opcode, len, copy);
    uint8_t k[4];
    if (key) memcpy(k, key, 4);
    const int r = ws_send_message(&client, &msg, key ? k : NULL, num_frames);
    shutdown(fds[0], SHUT_WR);
    pthread_join(th, NULL);
    close(fds[0]);
    close(fds[1]);
    free(copy);
    if (r != 1) return -1;
    return (long)ra.len;
}

struct keyseq_arg
{
    size_t n;
    uint8_t *out;
};

static void *keyseq(void *p)
{
    struct keyseq_arg *a = p;
    for (size_t i = 0; i < a->n; ++i) ws_build_masking_key(a->out + 4 * i);
    return NULL;
}

/* The first n keys ws_build_masking_key returns on a fresh thread (4n bytes). */
int ref_key_sequence(size_t n, uint8_t *out)
{
    struct keyseq_arg a = {n, out};
    pthread_t th;
    if (pthread_create(&th, NULL, keyseq, &a) != 0) return -1;
    pthread_join(th, NULL);
    return 0;
}

struct writer_arg
{
    int fd;
    const uint8_t *wire;
    size_t len;
    volatile int done;
};

static void *writer(void *p)
{
    struct writer_arg *a = p;
    size_t w = 0;
    while (w < a->len)
    {
        const ssize_t r = send(a->fd, a->wire + w, a->len - w, 0);
        if (r <= 0) break;
        w += (size_t)r;
    }
    __atomic_store_n(&a->done, 1, __ATOMIC_RELEASE);
    return NULL;
}

/*
 * CPU baseline: receive `wire` (masked frames) through the reference's
 * ws_parse_frame exactly as its event loop would (writer thread on the peer,
 * poll + parse while bytes are pending).  Returns the payload bytes delivered
 * and the elapsed seconds in *seconds, or -1.
 */
long ref_receive_timed(const uint8_t *wire, size_t wire_len, size_t max_payload, double *seconds)
{
    int fds[2];
    if (make_pair(fds) != 0) return -1;
    fcntl(fds[1], F_SETFL, fcntl(fds[1], F_GETFL, 0) | O_NONBLOCK);
    struct parse_ctx c;
    memset(&c, 0, sizeof(c));
    c.tcp.sockfd = fds[1];
    c.client.tcp_client = &c.tcp;
    c.max_payload = max_payload;
    struct writer_arg wa = {fds[0], wire, wire_len, 0};
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    pthread_t th;
    if (pthread_create(&th, NULL, writer, &wa) != 0) return -1;
    size_t delivered = 0;
    while (c.err == 0)
    {
        struct pollfd p = {.fd = fds[1], .events = POLLIN};
        (void)poll(&p, 1, 10);
        while (c.err == 0 && pending(fds[1]) > 0)
        {
            const int r = ws_parse_frame(&c.client, &c.st, max_payload);
            if (r < 0) c.err = r;
            else if (r == 0)
            {
                delivered += c.st.message.payload_length;
                free(c.st.message.buffer);
                memset(&c.st, 0, sizeof(c.st));
            }
        }
        if (__atomic_load_n(&wa.done, __ATOMIC_ACQUIRE) && pending(fds[1]) == 0) break;
    }
    pthread_join(th, NULL);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    close(fds[0]);
    close(fds[1]);
    if (c.st.payload_data.elements) free(c.st.payload_data.elements);
    *seconds = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
    return c.err ? -1 : (long)delivered;
}
