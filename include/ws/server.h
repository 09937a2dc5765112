#ifndef WS_SERVER_H
#define WS_SERVER_H

/*
 * WebSocket server handshake — same declarations as the reference's
 * include/ws/server.h:9-12.  NOT implemented by this repo's libraries: the
 * handshake (Sec-WebSocket-Accept = base64(SHA1(key + GUID)), the 101 response,
 * src/ws/server.c:13-106) runs once per connection on the control plane and stays
 * netc's own src/ws/server.c.  A netc program links that
 * file next to libnetc.so; tests/test_dropin.py builds exactly
 * that.  Kept here so the boundary's headers are complete; struct http_request is
 * only passed by pointer, so a forward declaration keeps the signature identical
 * without the reference's include/http/common.h.
 */

#include <stdint.h>

struct web_server;
struct web_client;
struct http_request;

/** Upgrades the connection to WebSocket. Returns `-1` if the upgrade was not able to occur. */
int ws_server_upgrade_connection(struct web_server *server, struct web_client *client, struct http_request *request);
/** Closes a WebSocket client. */
int ws_server_close_client(struct web_server *server, struct web_client *client, uint16_t code, const char *reason);

#endif // WS_SERVER_H
