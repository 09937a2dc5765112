#ifndef STRING_H
#define STRING_H

/*
 * Small-string-optimised string used by the socket helpers; same layout and
 * functions as the reference's include/utils/string.h:6-49.  Declarations only:
 * the implementation stays netc's own src/utils/string.c (out of scope).
 */

#include <stddef.h>

#define SSO_STRING_MAX_LENGTH 15

typedef struct sso_string {
    /** Characters in use (excluding the NUL). */
    size_t length;
    /** Heap capacity in characters when long (0 while short). */
    size_t capacity;
    union
    {
        char short_string[SSO_STRING_MAX_LENGTH + 1];
        char *long_string;
    };
} string_t;

void sso_string_init(string_t *string, const char *data);
void sso_string_set(string_t *string, const char *data);
const char *sso_string_get(string_t *string);

void sso_string_concat(string_t *dest, string_t *src);
void sso_string_concat_buffer(string_t *dest, const char *src);
void sso_string_concat_char(string_t *dest, const char src);
/** Drops the last n characters. */
void sso_string_backspace(string_t *string, size_t n);

void sso_string_copy(string_t *dest, string_t *src);
void sso_string_copy_buffer(char *dest, string_t *src);

int sso_string_compare(string_t *string1, string_t *string2);

void sso_string_ensure_null_terminated(string_t *string);

void sso_string_free(string_t *string);

#endif // STRING_H
