#ifndef SOCKET_H
#define SOCKET_H

/*
 * Socket helpers — same declarations as the reference's include/socket.h:1-28
 * (POSIX build; the reference's WinSock branch is out of scope here).  The header is
 * part of the kept C API (BASELINE.json north_star); the implementations are NOT in
 * this repo's libraries: they stay netc's own src/socket.c ("header API
 * kept verbatim; implementation out of scope"), linked next to libnetc.so
 * (tests/test_dropin.py).
 */

#include "./utils/vector.h"
#include "./utils/string.h"

#include <sys/types.h>
#include <fcntl.h>

typedef int socket_t;

/** Receives byte by byte into `string` until `bytes` is seen (or max_bytes_received). -2 if the pattern never came. */
int socket_recv_until_dynamic(socket_t sockfd, string_t *string, const char *bytes, int remove_delimiter, size_t max_bytes_received);
/** Receives byte by byte into `buffer` until `bytes` is seen or the buffer is full. -2 if the pattern never came. */
int socket_recv_until_fixed(socket_t sockfd, char *buffer, size_t buffer_size, const char *bytes, int remove_delimiter);

/** Sets O_NONBLOCK. Returns 0 or errno (netc_errno_reason = FD_CTL). */
int socket_set_non_blocking(socket_t sockfd);

#endif // SOCKET_H
