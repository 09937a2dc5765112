#ifndef WS_CLIENT_H
#define WS_CLIENT_H

/*
 * WebSocket client handshake — same declaration as the reference's
 * include/ws/client.h:9-13.  NOT implemented by this repo's libraries: the upgrade
 * request (src/ws/client.c:11-40) is once-per-connection control plane and stays
 * netc's own src/ws/client.c, linked next to libnetc.so (INTEGRATION.md §1,
 * tests/test_dropin.py).  See include/ws/server.h.
 */

struct web_server;
struct web_client;

/**
 * Upgrades an existing HTTP connection. Ensure `url` includes the host. Returns `1` if the request was successful.
 * NOTE: This does not guarantee that the server will accept the upgrade request. The callback will be called with the response.
 */
int ws_client_connect(struct web_client *client, const char *hostname, const char *path);

#endif // WS_CLIENT_H
