/* send/recv wrappers of include/tcp/server.h; as the reference's src/tcp/server.c:219-233. */
#include "../../../include/tcp/server.h"
#include "../../../include/utils/error.h"

#include <sys/socket.h>

int tcp_server_send(socket_t sockfd, const char *message, size_t msglen, int flags)
{
    const int r = (int)send(sockfd, message, msglen, flags);
    if (r == -1) (void)netc_error(BADSEND);
    return r;
}

int tcp_server_receive(socket_t sockfd, const char *message, size_t msglen, int flags)
{
    const int r = (int)recv(sockfd, (void *)message, msglen, flags);
    if (r == -1) (void)netc_error(BADRECV);
    return r;
}
