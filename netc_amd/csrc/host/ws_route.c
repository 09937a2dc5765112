/*
 * Side table of per-connection state for ws_parse_frame and ws_send_message (include/ws/route.h):
 * the receive and send routes, their close hooks, and the connection's send backlog.
 *
 * Keyed by socket descriptor: pages of 1,024 entries allocated on first use (descriptors up to
 * 2^20).  A descriptor is a number the kernel reuses: a connection closed without a detach leaves
 * its entry behind, and the next accept() may get the same number (the reference closes clients
 * at src/web/server.c:94,135 and src/tcp/server.c:67-70, with no hook of its own before close()).
 * Two ways keep an entry from outliving its connection:
 *
 *   close tracking  libnetc.so defines close(): in a process where that definition is the one
 *                   the application's close() binds to (the library linked as netc's
 *                   replacement, ahead of libc), closing a socket with an entry first runs the
 *                   routes' close hooks (a hub flushes what it queued for it, a ring lets go of
 *                   it), makes one last non-blocking attempt at its send backlog, and clears the
 *                   entry; then the descriptor is closed.  A lookup is then two loads, no system
 *                   call.  Whether close() reaches this definition is probed once, at load, by
 *                   closing a spare descriptor through the symbol the process resolves.
 *   identity check  otherwise (loaded RTLD_LOCAL, e.g. by ctypes; NETC_WS_ROUTE_VERIFY=1), every
 *                   lookup that finds a route compares the socket's identity (device, inode; one
 *                   fstat) with the one recorded at attach: an entry whose socket is gone serves
 *                   nothing, and the new connection gets the CPU path.
 *
 * The send backlog (round 6): sends never wait for a peer.  What a non-blocking socket does not take
 * is kept here, per connection, and written ahead of any later byte of that connection, without
 * waiting, by the next ws_send_message, ws_parse_frame or netc_ws_send_flush on it (and by a hub's
 * flush).  It is bounded (netc_ws_send_backlog_limit, 64 MiB by default): past the bound the
 * connection fails alone (BADSEND, errno ENOBUFS) and its later sends return -1 until it is closed.
 * The reference sends with one send() and returns its result (src/tcp/server.c:219-225): on a full
 * socket buffer that is -1 with EAGAIN, and a short send is counted as sent (B5); neither waits.
 */
#define _GNU_SOURCE
#include "../../../include/ws/route.h"
#include "../../../include/utils/error.h"

#include <dlfcn.h>
#include <errno.h>
#include <limits.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <sys/uio.h>
#include <unistd.h>

#ifndef MSG_NOSIGNAL
#define MSG_NOSIGNAL 0
#endif

#define PAGE_BITS 10
#define PAGES 1024
#define PAGE_SIZE (1 << PAGE_BITS)

/* bytes a connection's send queue may hold before it fails (0: unbounded) */
#define BACKLOG_DEFAULT (64ull << 20)

struct backlog
{
    uint64_t dev, ino;   /* the socket's identity when the first byte was kept */
    uint8_t *buf;
    size_t head, len, cap;   /* pending bytes: buf[head, head + len) */
    int failed;              /* errno of the failure that ended the connection's sends, 0 if none */
};

struct route
{
    _Atomic(netc_ws_route_fn) fn;
    _Atomic(void *) ctx;
    _Atomic(uint64_t) dev, ino;   /* the socket's identity at attach */
    _Atomic(netc_ws_send_route_fn) send_fn;
    _Atomic(void *) send_ctx;
    _Atomic(uint64_t) send_dev, send_ino;
    _Atomic(netc_ws_route_close_fn) on_close, send_on_close;
    _Atomic(struct backlog *) backlog;
};

static _Atomic(struct route *) g_pages[PAGES];
static atomic_long g_attached, g_attached_send, g_backlogs;
static atomic_ullong g_backlog_limit = BACKLOG_DEFAULT;
static int (*g_real_close)(int);
static int g_tracked;            /* close() reaches the definition below: lookups skip the fstat */
static __thread int g_probe_seen;

/* (device, inode) of an open descriptor; 0 when it is not open */
static int identity(int fd, uint64_t *dev, uint64_t *ino)
{
    struct stat st;
    if (fstat(fd, &st) != 0) return 0;
    *dev = (uint64_t)st.st_dev;
    *ino = (uint64_t)st.st_ino;
    return 1;
}

/* the state recorded for (dev, ino) still belongs to the socket open as fd */
static int live(int fd, uint64_t dev, uint64_t ino)
{
    uint64_t d = 0, i = 0;
    return identity(fd, &d, &i) && d == dev && i == ino;
}

static struct route *entry(int fd, int create)
{
    if (fd < 0 || fd >= PAGES * PAGE_SIZE) return NULL;
    _Atomic(struct route *) *slot = &g_pages[fd >> PAGE_BITS];
    struct route *page = atomic_load_explicit(slot, memory_order_acquire);
    if (!page && create)
    {
        struct route *fresh = calloc(PAGE_SIZE, sizeof(struct route));
        if (!fresh) return NULL;
        struct route *expected = NULL;
        if (atomic_compare_exchange_strong_explicit(slot, &expected, fresh, memory_order_acq_rel, memory_order_acquire))
            page = fresh;
        else
        {
            free(fresh);   /* another thread installed this page first */
            page = expected;
        }
    }
    return page ? &page[fd & (PAGE_SIZE - 1)] : NULL;
}

/* ------------------------------------------------------------ close tracking -- */

static void close_hook(int fd);

static int real_close(int fd)
{
    return g_real_close ? g_real_close(fd) : (int)syscall(SYS_close, fd);
}

/*
 * close() as netc calls it (src/tcp/server.c:267, src/ws/server.c:124 through it): the
 * connection's routes and backlog are settled while the descriptor still names its socket.
 */
int close(int fd)
{
    if (fd == -2) /* the load-time probe's marker descriptor (never a valid one) */
    {
        g_probe_seen = 1;
        errno = EBADF;
        return -1;
    }
    if (fd >= 0 && (atomic_load_explicit(&g_attached, memory_order_relaxed) |
                    atomic_load_explicit(&g_attached_send, memory_order_relaxed) |
                    atomic_load_explicit(&g_backlogs, memory_order_relaxed)))
        close_hook(fd);
    return real_close(fd);
}

__attribute__((constructor)) static void route_init(void)
{
    g_real_close = (int (*)(int))dlsym(RTLD_NEXT, "close");
    const char *v = getenv("NETC_WS_ROUTE_VERIFY");
    if (v && *v && *v != '0') return; /* identity checks forced */
    int (*resolved)(int) = (int (*)(int))dlsym(RTLD_DEFAULT, "close");
    if (!resolved) return;
    /* the process's own close(), called with a descriptor no kernel hands out: it reaches the
       definition above only if that is the one (or is forwarded to by the one) the process uses */
    const int saved = errno;
    g_probe_seen = 0;
    (void)resolved(-2);
    g_tracked = g_probe_seen;
    errno = saved;
}

int netc_ws_route_close_tracked(void) { return g_tracked; }

static void backlog_free(struct route *e)
{
    struct backlog *b = atomic_exchange_explicit(&e->backlog, NULL, memory_order_acq_rel);
    if (!b) return;
    free(b->buf);
    free(b);
    atomic_fetch_sub_explicit(&g_backlogs, 1, memory_order_release);
}

static void close_hook(int fd)
{
    struct route *e = entry(fd, 0);
    if (!e) return;
    /* the hooks run first: a send hook flushes what its hub or ring queued for this socket */
    netc_ws_route_close_fn h;
    if (atomic_load_explicit(&e->send_fn, memory_order_acquire) &&
        (h = atomic_exchange_explicit(&e->send_on_close, NULL, memory_order_acq_rel)))
        h(atomic_load_explicit(&e->send_ctx, memory_order_relaxed), fd);
    if (atomic_load_explicit(&e->fn, memory_order_acquire) &&
        (h = atomic_exchange_explicit(&e->on_close, NULL, memory_order_acq_rel)))
        h(atomic_load_explicit(&e->ctx, memory_order_relaxed), fd);
    (void)netc_ws_send_route_detach(fd);
    (void)netc_ws_route_detach(fd);
    if (atomic_load_explicit(&e->backlog, memory_order_acquire))
    {
        (void)netc_ws_send_flush(fd); /* what the socket takes now still reaches the peer */
        backlog_free(e);
    }
}

/* ------------------------------------------------------------------ routes -- */

int netc_ws_route_attach(int sockfd, netc_ws_route_fn fn, void *ctx)
{
    uint64_t dev = 0, ino = 0;
    if (!fn || sockfd < 0 || sockfd >= PAGES * PAGE_SIZE || !identity(sockfd, &dev, &ino))
    {
        errno = EINVAL;
        return -1;
    }
    struct route *e = entry(sockfd, 1);
    if (!e)
    {
        errno = ENOMEM;
        return -1;
    }
    netc_ws_route_fn old = atomic_load_explicit(&e->fn, memory_order_acquire);
    if (old && (old != fn || atomic_load_explicit(&e->ctx, memory_order_relaxed) != ctx) &&
        live(sockfd, atomic_load_explicit(&e->dev, memory_order_relaxed), atomic_load_explicit(&e->ino, memory_order_relaxed)))
    {
        errno = EBUSY; /* another route serves this connection: detach it first */
        return -1;
    }
    if (old && old == fn && atomic_load_explicit(&e->ctx, memory_order_relaxed) == ctx &&
        atomic_load_explicit(&e->dev, memory_order_relaxed) == dev && atomic_load_explicit(&e->ino, memory_order_relaxed) == ino)
        return 0; /* already this route on this connection: its close hook stays */
    atomic_store_explicit(&e->fn, NULL, memory_order_relaxed);
    atomic_store_explicit(&e->on_close, NULL, memory_order_relaxed);
    atomic_store_explicit(&e->ctx, ctx, memory_order_relaxed);
    atomic_store_explicit(&e->dev, dev, memory_order_relaxed);
    atomic_store_explicit(&e->ino, ino, memory_order_relaxed);
    atomic_store_explicit(&e->fn, fn, memory_order_release); /* ctx and identity are visible with fn */
    if (!old) atomic_fetch_add_explicit(&g_attached, 1, memory_order_release);
    return 0;
}

int netc_ws_route_detach(int sockfd)
{
    if (sockfd < 0 || sockfd >= PAGES * PAGE_SIZE)
    {
        errno = EINVAL;
        return -1;
    }
    struct route *e = entry(sockfd, 0);
    if (!e) return 0;
    atomic_store_explicit(&e->on_close, NULL, memory_order_relaxed);
    if (atomic_exchange_explicit(&e->fn, NULL, memory_order_acq_rel) != NULL)
        atomic_fetch_sub_explicit(&g_attached, 1, memory_order_release);
    atomic_store_explicit(&e->ctx, NULL, memory_order_relaxed);
    return 0;
}

int netc_ws_route_on_close(int sockfd, netc_ws_route_close_fn hook)
{
    struct route *e = entry(sockfd, 0);
    if (!e || !atomic_load_explicit(&e->fn, memory_order_acquire))
    {
        errno = EINVAL;
        return -1;
    }
    atomic_store_explicit(&e->on_close, hook, memory_order_release);
    return 0;
}

netc_ws_route_fn netc_ws_route_get_raw(int sockfd, void **ctx)
{
    struct route *e = entry(sockfd, 0);
    if (!e) return NULL;
    netc_ws_route_fn fn = atomic_load_explicit(&e->fn, memory_order_acquire);
    if (fn && ctx) *ctx = atomic_load_explicit(&e->ctx, memory_order_relaxed);
    return fn;
}

netc_ws_route_fn netc_ws_route_get(int sockfd, void **ctx)
{
    if (atomic_load_explicit(&g_attached, memory_order_acquire) == 0) return NULL;
    struct route *e = entry(sockfd, 0);
    if (!e) return NULL;
    netc_ws_route_fn fn = atomic_load_explicit(&e->fn, memory_order_acquire);
    if (!fn) return NULL;
    if (!g_tracked &&
        !live(sockfd, atomic_load_explicit(&e->dev, memory_order_relaxed), atomic_load_explicit(&e->ino, memory_order_relaxed)))
        return NULL; /* left behind by a closed connection: this descriptor is another one now */
    if (ctx) *ctx = atomic_load_explicit(&e->ctx, memory_order_relaxed);
    return fn;
}

int netc_ws_send_route_attach(int sockfd, netc_ws_send_route_fn fn, void *ctx)
{
    uint64_t dev = 0, ino = 0;
    if (!fn || sockfd < 0 || sockfd >= PAGES * PAGE_SIZE || !identity(sockfd, &dev, &ino))
    {
        errno = EINVAL;
        return -1;
    }
    struct route *e = entry(sockfd, 1);
    if (!e)
    {
        errno = ENOMEM;
        return -1;
    }
    netc_ws_send_route_fn old = atomic_load_explicit(&e->send_fn, memory_order_acquire);
    if (old && (old != fn || atomic_load_explicit(&e->send_ctx, memory_order_relaxed) != ctx) &&
        live(sockfd, atomic_load_explicit(&e->send_dev, memory_order_relaxed),
             atomic_load_explicit(&e->send_ino, memory_order_relaxed)))
    {
        errno = EBUSY;
        return -1;
    }
    if (old && old == fn && atomic_load_explicit(&e->send_ctx, memory_order_relaxed) == ctx &&
        atomic_load_explicit(&e->send_dev, memory_order_relaxed) == dev &&
        atomic_load_explicit(&e->send_ino, memory_order_relaxed) == ino)
        return 0;
    atomic_store_explicit(&e->send_fn, NULL, memory_order_relaxed);
    atomic_store_explicit(&e->send_on_close, NULL, memory_order_relaxed);
    atomic_store_explicit(&e->send_ctx, ctx, memory_order_relaxed);
    atomic_store_explicit(&e->send_dev, dev, memory_order_relaxed);
    atomic_store_explicit(&e->send_ino, ino, memory_order_relaxed);
    atomic_store_explicit(&e->send_fn, fn, memory_order_release);
    if (!old) atomic_fetch_add_explicit(&g_attached_send, 1, memory_order_release);
    return 0;
}

int netc_ws_send_route_detach(int sockfd)
{
    if (sockfd < 0 || sockfd >= PAGES * PAGE_SIZE)
    {
        errno = EINVAL;
        return -1;
    }
    struct route *e = entry(sockfd, 0);
    if (!e) return 0;
    atomic_store_explicit(&e->send_on_close, NULL, memory_order_relaxed);
    if (atomic_exchange_explicit(&e->send_fn, NULL, memory_order_acq_rel) != NULL)
        atomic_fetch_sub_explicit(&g_attached_send, 1, memory_order_release);
    atomic_store_explicit(&e->send_ctx, NULL, memory_order_relaxed);
    return 0;
}

int netc_ws_send_route_on_close(int sockfd, netc_ws_route_close_fn hook)
{
    struct route *e = entry(sockfd, 0);
    if (!e || !atomic_load_explicit(&e->send_fn, memory_order_acquire))
    {
        errno = EINVAL;
        return -1;
    }
    atomic_store_explicit(&e->send_on_close, hook, memory_order_release);
    return 0;
}

netc_ws_send_route_fn netc_ws_send_route_get_raw(int sockfd, void **ctx)
{
    struct route *e = entry(sockfd, 0);
    if (!e) return NULL;
    netc_ws_send_route_fn fn = atomic_load_explicit(&e->send_fn, memory_order_acquire);
    if (fn && ctx) *ctx = atomic_load_explicit(&e->send_ctx, memory_order_relaxed);
    return fn;
}

netc_ws_send_route_fn netc_ws_send_route_get(int sockfd, void **ctx)
{
    if (atomic_load_explicit(&g_attached_send, memory_order_acquire) == 0) return NULL;
    struct route *e = entry(sockfd, 0);
    if (!e) return NULL;
    netc_ws_send_route_fn fn = atomic_load_explicit(&e->send_fn, memory_order_acquire);
    if (!fn) return NULL;
    if (!g_tracked && !live(sockfd, atomic_load_explicit(&e->send_dev, memory_order_relaxed),
                            atomic_load_explicit(&e->send_ino, memory_order_relaxed)))
        return NULL;
    if (ctx) *ctx = atomic_load_explicit(&e->send_ctx, memory_order_relaxed);
    return fn;
}

/* ----------------------------------------------------------- send backlog -- */

/* the connection's backlog, or NULL; one left by a closed connection (untracked processes) is freed */
static struct backlog *backlog_of(int fd, struct route **out)
{
    if (atomic_load_explicit(&g_backlogs, memory_order_acquire) == 0) return NULL;
    struct route *e = entry(fd, 0);
    if (!e) return NULL;
    struct backlog *b = atomic_load_explicit(&e->backlog, memory_order_acquire);
    if (!b) return NULL;
    if (!g_tracked && !live(fd, b->dev, b->ino))
    {
        backlog_free(e);
        return NULL;
    }
    if (out) *out = e;
    return b;
}

/* fails the connection's sends: its kept bytes are dropped, later sends return -1 */
static int backlog_fail(struct backlog *b, int err)
{
    free(b->buf);
    b->buf = NULL;
    b->head = b->len = b->cap = 0;
    b->failed = err ? err : EPIPE;
    errno = b->failed;
    (void)netc_error(BADSEND);
    return -1;
}

/* appends the iovecs' bytes past `skip` to the backlog; -1 (connection failed) past the bound */
static int backlog_append(struct backlog *b, const struct iovec *iov, int cnt, size_t skip)
{
    size_t n = 0;
    for (int i = 0; i < cnt; ++i) n += iov[i].iov_len;
    n -= skip;
    const unsigned long long limit = atomic_load_explicit(&g_backlog_limit, memory_order_relaxed);
    if (limit && b->len + n > limit) return backlog_fail(b, ENOBUFS);
    if (b->head + b->len + n > b->cap)
    {
        if (b->head) /* compact first */
        {
            memmove(b->buf, b->buf + b->head, b->len);
            b->head = 0;
        }
        if (b->len + n > b->cap)
        {
            size_t cap = b->cap ? b->cap : 4096;
            while (cap < b->len + n) cap *= 2;
            uint8_t *nb = realloc(b->buf, cap);
            if (!nb) return backlog_fail(b, ENOMEM);
            b->buf = nb;
            b->cap = cap;
        }
    }
    uint8_t *dst = b->buf + b->head + b->len;
    for (int i = 0; i < cnt; ++i)
    {
        size_t l = iov[i].iov_len;
        const uint8_t *p = iov[i].iov_base;
        if (skip >= l)
        {
            skip -= l;
            continue;
        }
        p += skip;
        l -= skip;
        skip = 0;
        memcpy(dst, p, l);
        dst += l;
    }
    b->len += n;
    return 0;
}

static struct backlog *backlog_create(int fd)
{
    struct route *e = entry(fd, 1);
    if (!e) return NULL;
    struct backlog *b = atomic_load_explicit(&e->backlog, memory_order_acquire);
    if (b) return b;
    uint64_t dev = 0, ino = 0;
    if (!identity(fd, &dev, &ino)) return NULL;
    if (!(b = calloc(1, sizeof *b))) return NULL;
    b->dev = dev;
    b->ino = ino;
    atomic_store_explicit(&e->backlog, b, memory_order_release);
    atomic_fetch_add_explicit(&g_backlogs, 1, memory_order_release);
    return b;
}

/* one sendmsg of up to IOV_MAX entries; bytes written, 0 when it would block, -1 on an error */
static ssize_t send_once(int fd, const struct iovec *iov, int cnt, int flags)
{
    struct msghdr mh;
    memset(&mh, 0, sizeof mh);
    mh.msg_iov = (struct iovec *)iov;
    mh.msg_iovlen = (size_t)(cnt < IOV_MAX ? cnt : IOV_MAX);
    for (;;)
    {
        const ssize_t r = sendmsg(fd, &mh, flags | MSG_NOSIGNAL);
        if (r >= 0) return r;
        if (errno == EINTR) continue;
        if (errno == EAGAIN || errno == EWOULDBLOCK) return 0;
        return -1;
    }
}

long netc_ws_send_flush(int sockfd)
{
    struct route *e = NULL;
    struct backlog *b = backlog_of(sockfd, &e);
    if (!b) return 0;
    if (b->failed)
    {
        errno = b->failed;
        (void)netc_error(BADSEND);
        return -1;
    }
    while (b->len)
    {
        struct iovec v = {b->buf + b->head, b->len};
        const ssize_t r = send_once(sockfd, &v, 1, MSG_DONTWAIT);
        if (r < 0) return backlog_fail(b, errno);
        if (r == 0) break;
        b->head += (size_t)r;
        b->len -= (size_t)r;
    }
    const long held = (long)b->len;
    if (!held) backlog_free(e); /* emptied: the connection's sends take the direct path again */
    return held;
}

long netc_ws_send_pending(int sockfd)
{
    struct backlog *b = backlog_of(sockfd, NULL);
    if (!b) return 0;
    if (b->failed)
    {
        errno = b->failed;
        return -1;
    }
    return (long)b->len;
}

int netc_ws_send_nb(int sockfd, const struct iovec *iov, int iovcnt, int dontwait)
{
    struct backlog *b = backlog_of(sockfd, NULL);
    if (b && b->failed)
    {
        errno = b->failed;
        (void)netc_error(BADSEND);
        return -1;
    }
    if (b && b->len)
    {
        const long held = netc_ws_send_flush(sockfd);
        if (held < 0) return -1;                                           /* failed just now */
        if (held > 0) return backlog_append(b, iov, iovcnt, 0) == 0 ? 1 : -1; /* behind earlier bytes */
        b = NULL; /* emptied (and freed) */
    }

    /* written in place while the socket takes them; the rest into the queue */
    struct iovec local[64];
    struct iovec *v = iovcnt <= 64 ? local : malloc(sizeof(struct iovec) * (size_t)iovcnt);
    if (!v)
    {
        errno = ENOMEM;
        (void)netc_error(BADSEND);
        return -1;
    }
    memcpy(v, iov, sizeof(struct iovec) * (size_t)iovcnt);
    struct iovec *cur = v;
    int left = iovcnt;
    int rc = 1;
    while (left > 0 && cur->iov_len == 0) ++cur, --left;
    while (left > 0)
    {
        const ssize_t r = send_once(sockfd, cur, left, dontwait ? MSG_DONTWAIT : 0);
        if (r < 0)
        {
            const int saved = errno;
            if (b) (void)backlog_fail(b, saved);
            errno = saved;
            (void)netc_error(BADSEND);
            rc = -1;
            break;
        }
        if (r == 0) /* the socket is full: the rest waits in the connection's queue */
        {
            if (!b && !(b = backlog_create(sockfd)))
            {
                errno = ENOMEM;
                (void)netc_error(BADSEND);
                rc = -1;
                break;
            }
            rc = backlog_append(b, cur, left, 0) == 0 ? 1 : -1;
            break;
        }
        size_t done = (size_t)r;
        while (left > 0 && done >= cur->iov_len)
        {
            done -= cur->iov_len;
            ++cur;
            --left;
        }
        if (left > 0)
        {
            cur->iov_base = (uint8_t *)cur->iov_base + done;
            cur->iov_len -= done;
        }
    }
    if (v != local) free(v);
    return rc;
}

size_t netc_ws_send_backlog_limit(size_t bytes)
{
    return (size_t)atomic_exchange_explicit(&g_backlog_limit, (unsigned long long)bytes, memory_order_relaxed);
}
