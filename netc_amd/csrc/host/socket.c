/* Socket helpers (include/socket.h); behaviour as the reference's src/socket.c:16-111 (POSIX branch). */
#include "../../../include/socket.h"
#include "../../../include/utils/error.h"

#include <errno.h>
#include <string.h>
#include <sys/socket.h>

int socket_recv_until_dynamic(socket_t sockfd, string_t *string, const char *bytes, int remove_delimiter, size_t max_bytes_received)
{
    const size_t blen = bytes ? strlen(bytes) : 0;
    size_t got = 0;
    int found = 0;
    while (got < max_bytes_received)
    {
        char c;
        const ssize_t r = recv(sockfd, &c, 1, 0);
        if (r <= 0)
        {
            if (r == -1 && errno != EWOULDBLOCK && errno != EAGAIN) (void)netc_error(BADRECV);
            return (int)r;
        }
        ++got;
        sso_string_concat_char(string, c);
        if (bytes && got >= blen && memcmp(sso_string_get(string) + string->length - blen, bytes, blen) == 0)
        {
            found = 1;
            if (remove_delimiter)
            {
                sso_string_backspace(string, blen);
                got -= blen;
            }
            break;
        }
    }
    if (bytes && !found) return -2;
    return (int)got;
}

int socket_recv_until_fixed(socket_t sockfd, char *buffer, size_t buffer_size, const char *bytes, int remove_delimiter)
{
    const size_t blen = bytes ? strlen(bytes) : 0;
    size_t got = 0;
    int found = 0;
    while (got + blen < buffer_size)
    {
        const ssize_t r = recv(sockfd, buffer + got, 1, 0);
        if (r <= 0)
        {
            if (r == -1)
            {
                if (errno == EAGAIN || errno == EWOULDBLOCK) break;
                (void)netc_error(BADRECV);
            }
            return (int)r;
        }
        got += (size_t)r;
        if (bytes && got >= blen && strncmp(buffer + got - blen, bytes, blen) == 0)
        {
            found = 1;
            if (remove_delimiter)
            {
                buffer[got - blen] = '\0';
                --got;
            }
            break;
        }
    }
    if (bytes && !found) return -2;
    return (int)got;
}

int socket_set_non_blocking(socket_t sockfd)
{
    const int flags = fcntl(sockfd, F_GETFL, 0);
    if (flags == -1) return netc_error(FD_CTL);
    if (flags & O_NONBLOCK) return 0;
    if (fcntl(sockfd, F_SETFL, flags | O_NONBLOCK) == -1) return netc_error(FD_CTL);
    return 0;
}
