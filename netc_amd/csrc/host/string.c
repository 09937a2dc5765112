/* SSO string (include/utils/string.h); behaviour as the reference's src/utils/string.c. */
#include "../../../include/utils/string.h"

#include <stdlib.h>
#include <string.h>

static int is_long(const string_t *s)
{
    return s->capacity > SSO_STRING_MAX_LENGTH;
}

static char *data_of(string_t *s)
{
    return is_long(s) ? s->long_string : s->short_string;
}

/* make room for `need` characters + NUL */
static void reserve(string_t *s, size_t need)
{
    if (need <= SSO_STRING_MAX_LENGTH && !is_long(s)) return;
    if (is_long(s) && need <= s->capacity) return;
    size_t cap = is_long(s) ? s->capacity : 2 * SSO_STRING_MAX_LENGTH;
    while (cap < need) cap *= 2;
    char *p = malloc(cap + 1);
    if (p == NULL) return;
    memcpy(p, data_of(s), s->length);
    p[s->length] = '\0';
    if (is_long(s)) free(s->long_string);
    s->long_string = p;
    s->capacity = cap;
}

void sso_string_init(string_t *string, const char *data)
{
    memset(string, 0, sizeof(*string));
    if (data != NULL) sso_string_set(string, data);
}

void sso_string_set(string_t *string, const char *data)
{
    const size_t n = data ? strlen(data) : 0;
    string->length = 0;
    reserve(string, n);
    char *d = data_of(string);
    if (n) memcpy(d, data, n);
    d[n] = '\0';
    string->length = n;
}

const char *sso_string_get(string_t *string)
{
    return data_of(string);
}

void sso_string_concat_buffer(string_t *dest, const char *src)
{
    const size_t n = strlen(src);
    reserve(dest, dest->length + n);
    char *d = data_of(dest);
    memcpy(d + dest->length, src, n);
    dest->length += n;
    d[dest->length] = '\0';
}

void sso_string_concat(string_t *dest, string_t *src)
{
    sso_string_concat_buffer(dest, sso_string_get(src));
}

void sso_string_concat_char(string_t *dest, const char src)
{
    reserve(dest, dest->length + 1);
    char *d = data_of(dest);
    d[dest->length++] = src;
    d[dest->length] = '\0';
}

void sso_string_backspace(string_t *string, size_t n)
{
    if (n > string->length) n = string->length;
    string->length -= n;
    data_of(string)[string->length] = '\0';
}

void sso_string_copy(string_t *dest, string_t *src)
{
    sso_string_set(dest, sso_string_get(src));
}

void sso_string_copy_buffer(char *dest, string_t *src)
{
    memcpy(dest, sso_string_get(src), src->length + 1);
}

int sso_string_compare(string_t *string1, string_t *string2)
{
    return strcmp(sso_string_get(string1), sso_string_get(string2));
}

void sso_string_ensure_null_terminated(string_t *string)
{
    data_of(string)[string->length] = '\0';
}

void sso_string_free(string_t *string)
{
    if (is_long(string)) free(string->long_string);
    memset(string, 0, sizeof(*string));
}
