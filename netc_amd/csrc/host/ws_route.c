/*
 * Side table of per-connection routes for ws_parse_frame and ws_send_message (include/ws/route.h).
 *
 * Keyed by socket descriptor: pages of 1,024 entries allocated on first use (descriptors up to
 * 2^20), each entry two atomic {fn, ctx} pairs (receive, send).  A call on a socket without a
 * route costs one load of that direction's attached count while no socket anywhere has one, and
 * one page and entry load otherwise.
 */
#include "../../../include/ws/route.h"

#include <errno.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdlib.h>

#define PAGE_BITS 10
#define PAGES 1024
#define PAGE_SIZE (1 << PAGE_BITS)

struct route
{
    _Atomic(netc_ws_route_fn) fn;
    _Atomic(void *) ctx;
    _Atomic(netc_ws_send_route_fn) send_fn;
    _Atomic(void *) send_ctx;
};

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
    if (!fn || sockfd < 0 || sockfd >= PAGES * PAGE_SIZE)
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
    const int had = atomic_load_explicit(&e->fn, memory_order_relaxed) != NULL;
    atomic_store_explicit(&e->ctx, ctx, memory_order_relaxed);
    atomic_store_explicit(&e->fn, fn, memory_order_release);   /* ctx is visible with fn */
    if (!had) atomic_fetch_add_explicit(&g_attached, 1, memory_order_release);
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

netc_ws_route_fn netc_ws_route_get(int sockfd, void **ctx)
{
    if (atomic_load_explicit(&g_attached, memory_order_acquire) == 0) return NULL;
    struct route *e = entry(sockfd, 0);
    if (!e) return NULL;
    netc_ws_route_fn fn = atomic_load_explicit(&e->fn, memory_order_acquire);
    if (fn && ctx) *ctx = atomic_load_explicit(&e->ctx, memory_order_relaxed);
    return fn;
}

int netc_ws_send_route_attach(int sockfd, netc_ws_send_route_fn fn, void *ctx)
{
    if (!fn || sockfd < 0 || sockfd >= PAGES * PAGE_SIZE)
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
    const int had = atomic_load_explicit(&e->send_fn, memory_order_relaxed) != NULL;
    atomic_store_explicit(&e->send_ctx, ctx, memory_order_relaxed);
    atomic_store_explicit(&e->send_fn, fn, memory_order_release);   /* ctx is visible with fn */
    if (!had) atomic_fetch_add_explicit(&g_attached_send, 1, memory_order_release);
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

netc_ws_send_route_fn netc_ws_send_route_get(int sockfd, void **ctx)
{
    if (atomic_load_explicit(&g_attached_send, memory_order_acquire) == 0) return NULL;
    struct route *e = entry(sockfd, 0);
    if (!e) return NULL;
    netc_ws_send_route_fn fn = atomic_load_explicit(&e->send_fn, memory_order_acquire);
    if (fn && ctx) *ctx = atomic_load_explicit(&e->send_ctx, memory_order_relaxed);
    return fn;
}
