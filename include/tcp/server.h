#ifndef TCP_SERVER_H
#define TCP_SERVER_H

/*
 * The part of the reference's include/tcp/server.h that the WebSocket path
 * touches: struct tcp_client (include/tcp/server.h:16-41, same layout; the WS
 * path reads only .sockfd) and the send/receive wrappers
 * (include/tcp/server.h:90-93; src/tcp/server.c:219-233).  The TCP event loop,
 * accept/bind/listen and struct tcp_server are netc's networking layer and are
 * out of scope for this library ("Scope").
 */

#include <stdbool.h>
#include <sys/socket.h>

#include "../socket.h"

struct tcp_client
{
    socket_t sockfd;
    struct sockaddr *sockaddr;
    int listening;
    int pfd;
    void *data;
    void (*on_connect)(struct tcp_client *client);
    void (*on_data)(struct tcp_client *client);
    void (*on_disconnect)(struct tcp_client *client, bool is_error);
};

/** send() wrapper. Returns the send() result; on -1 sets netc_errno_reason = BADSEND. */
int tcp_server_send(socket_t sockfd, const char *message, size_t msglen, int flags);
/** recv() wrapper. Returns the recv() result; on -1 sets netc_errno_reason = BADRECV. */
int tcp_server_receive(socket_t sockfd, const char *message, size_t msglen, int flags);

#endif // TCP_SERVER_H
