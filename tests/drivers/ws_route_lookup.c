/*
 * What an attached socket's route lookup costs per call (VERDICT r5 "next" #6): the lookups
 * ws_parse_frame and ws_send_message do on every call -- netc_ws_send_pending (the send backlog),
 * netc_ws_route_get, netc_ws_send_route_get -- timed over N calls on one attached socket.  In a
 * process whose close() reaches libnetc.so's (netc's link), identity is settled at close time and a
 * lookup is a table read; NETC_WS_ROUTE_VERIFY=1 forces the fstat per lookup that untracked
 * processes pay.  Host only.  Prints one JSON line.
 *
 *   tests/bin/ws_route_lookup [calls]
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <sys/socket.h>
#include <sys/uio.h>
#include <time.h>
#include <unistd.h>

#include "ws/route.h"

static int route_fn(void *ctx, int fd, struct ws_frame_parsing_state *st, size_t max_payload_length)
{
    (void)ctx; (void)fd; (void)st; (void)max_payload_length;
    return 0;
}

static int send_fn(void *ctx, int fd, struct ws_message *message, uint8_t masking_key[4], size_t num_frames)
{
    (void)ctx; (void)fd; (void)message; (void)masking_key; (void)num_frames;
    return 0;
}

static double now(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

int main(int argc, char **argv)
{
    const long n = argc > 1 ? atol(argv[1]) : 2000000;
    int sv[2];
    if (socketpair(AF_UNIX, SOCK_STREAM, 0, sv) != 0) return 2;
    if (netc_ws_route_attach(sv[0], route_fn, NULL) != 0) return 3;
    if (netc_ws_send_route_attach(sv[0], send_fn, NULL) != 0) return 4;
    long hits = 0;
    double t0 = now();
    for (long i = 0; i < n; ++i)
    {
        void *ctx = NULL;
        hits += netc_ws_send_pending(sv[0]) == 0;
        hits += netc_ws_route_get(sv[0], &ctx) != NULL;
        hits += netc_ws_send_route_get(sv[0], &ctx) != NULL;
    }
    const double dt = now() - t0;
    printf("{\"tracked\": %d, \"calls\": %ld, \"ns_per_call\": %.1f, \"ok\": %s}\n", netc_ws_route_close_tracked(), n,
           dt * 1e9 / (double)n, hits == 3 * n ? "true" : "false");
    netc_ws_route_detach(sv[0]);
    netc_ws_send_route_detach(sv[0]);
    close(sv[0]);
    close(sv[1]);
    return hits == 3 * n ? 0 : 1;
}
