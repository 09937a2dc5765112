/* Error side channel (include/utils/error.h); as the reference's src/utils/error.c:5-50 (POSIX branch). */
#include "../../../include/utils/error.h"

#include <string.h>

__thread int netc_errno_reason = 0;

void netc_strerror(char *buffer)
{
    char msg[1024] = {0};
    const int e = errno;
#if (_POSIX_C_SOURCE >= 200112L) && !defined(_GNU_SOURCE)
    if (strerror_r(e, msg, sizeof(msg) - 1) != 0) snprintf(msg, sizeof(msg), "errno %d", e);
    strcpy(buffer, msg);
#else
    strcpy(buffer, strerror_r(e, msg, sizeof(msg) - 1));
#endif
}

void netc_perror(const char *message, ...)
{
    char err[1024] = {0};
    netc_strerror(err);
    va_list args;
    va_start(args, message);
    vfprintf(stderr, message, args);
    va_end(args);
    fprintf(stderr, ": %s\n", err);
}
