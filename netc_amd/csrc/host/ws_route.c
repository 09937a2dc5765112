/*
 * Side table of per-connection routes for ws_parse_frame and ws_send_message (include/ws/route.h).
 *
 * Keyed by socket descriptor: pages of 1,024 entries allocated on first use (descriptors up to
 * 2^20), each entry two atomic {fn, ctx} pairs (receive, send) with the identity (device, inode)
 * the socket had when its route was attached.  A descriptor is a number the kernel reuses: a
 * connection closed without a detach leaves its route behind, and the next accept() may get the
 * same number (the reference closes clients at src/web/server.c:94,135).  So a lookup checks the
 * socket's identity (one fstat) and a route whose socket is gone serves nothing: the new
 * connection gets the CPU path.  A call on a socket without a route costs one load of that
 * direction's attached count while no socket anywhere has one, and one page and entry load
 * otherwise.
 */
#include "../../../include/ws/route.h"

#include <errno.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdlib.h>
#include <sys/stat.h>

#define PAGE_BITS 10
#define PAGES 1024
#define PAGE_SIZE (1 << PAGE_BITS)

struct route
{
    _Atomic(netc_ws_route_fn) fn;
    _Atomic(void *) ctx;
    _Atomic(uint64_t) dev, ino;   /* the socket's identity at attach */
    _Atomic(netc_ws_send_route_fn) send_fn;
    _Atomic(void *) send_ctx;
    _Atomic(uint64_t) send_dev, send_ino;
};

/* (device, inode) of an open descriptor; 0 when it is not open */
static int identity(int fd, uint64_t *dev, uint64_t *ino)
{
    struct stat st;
    if (fstat(fd, &st) != 0) return 0;
    *dev = (uint64_t)st.st_dev;
    *ino = (uint64_t)st.st_ino;
    return 1;
}

/* the route recorded for (dev, ino) still belongs to the socket open as fd */
static int live(int fd, uint64_t dev, uint64_t ino)
{
    uint64_t d = 0, i = 0;
    return identity(fd, &d, &i) && d == dev && i == ino;
}

static _Atomic(struct route *) g_pages[PAGES];
static atomic_long g_attached, g_attached_send;

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
    atomic_store_explicit(&e->fn, NULL, memory_order_relaxed);
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
    if (atomic_exchange_explicit(&e->fn, NULL, memory_order_acq_rel) != NULL)
        atomic_fetch_sub_explicit(&g_attached, 1, memory_order_release);
    atomic_store_explicit(&e->ctx, NULL, memory_order_relaxed);
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
    if (!live(sockfd, atomic_load_explicit(&e->dev, memory_order_relaxed), atomic_load_explicit(&e->ino, memory_order_relaxed)))
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
    atomic_store_explicit(&e->send_fn, NULL, memory_order_relaxed);
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
    if (atomic_exchange_explicit(&e->send_fn, NULL, memory_order_acq_rel) != NULL)
        atomic_fetch_sub_explicit(&g_attached_send, 1, memory_order_release);
    atomic_store_explicit(&e->send_ctx, NULL, memory_order_relaxed);
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
    if (!live(sockfd, atomic_load_explicit(&e->send_dev, memory_order_relaxed),
              atomic_load_explicit(&e->send_ino, memory_order_relaxed)))
        return NULL;
    if (ctx) *ctx = atomic_load_explicit(&e->send_ctx, memory_order_relaxed);
    return fn;
}
