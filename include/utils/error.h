#ifndef ERROR_H
#define ERROR_H

/*
 * netc's error side channel, as in the reference include/utils/error.h:19-45:
 * a failing call stores *which* operation failed in the thread-local
 * netc_errno_reason and returns / leaves the OS reason in errno.
 */

#include <errno.h>
#include <stdio.h>
#include <stdarg.h>

/** Sets the netc reason and evaluates to errno. */
#define netc_error(reason) (netc_errno_reason = reason, errno)

/** The operation `errno` originates from (one of the codes below). */
extern __thread int netc_errno_reason;

#define EVCREATE        1     /** kqueue / epoll_create1 */
#define SOCKET_C        2     /** socket() */
#define POLL_FD         3     /** kevent / epoll_wait */
#define EVENT_SELECT    4     /** WSAEventSelect */
#define NETWORK_EVENT   5     /** WSAEnumNetworkEvents */
#define WSA_WAIT        6     /** WSAWaitForMultipleEvents */
#define BIND            6     /** bind() (shares 6 with WSA_WAIT, as in the reference) */
#define LISTEN          7     /** listen() */
#define ACCEPT          8     /** accept() */
#define BADSEND         9     /** send() */
#define BADRECV        10     /** recv() */
#define CLOSE          11     /** close() */
#define FD_CTL         12     /** ioctl / fcntl */
#define CONNECT        13     /** connect() */
#define HANGUP         14     /** unexpected hangup */
#define INETPTON       15     /** inet_pton() */
#define WSA_STARTUP    16     /** WSAStartup() */
#define SIGNAL         17     /** signal() */
/* 18 = NETC_REASON_GPU, include/ws/mask.h */

/** Writes strerror(errno) into buffer (at least 1024 bytes). */
void netc_strerror(char *buffer);
/** Prints "<formatted message>: <strerror(errno)>" to stderr. */
void netc_perror(const char *message, ...);

#endif // ERROR_H
