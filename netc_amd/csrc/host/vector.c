/*
 * struct vector (include/utils/vector.h) with the reference's semantics,
 * src/utils/vector.c:8-90 — libnetc.so exports these under netc's own names, and a
 * netc program that links its own src/utils/vector.c interposes them (the drop-in
 * check, tests/test_dropin.py, shows libnetc.so binding the program's copies), so
 * the two must behave alike: vector_set_index grows size when it writes at or past
 * it (:38-44), vector_get does no range check (:46-49), vector_get_buffer is the
 * end of the data — where the next element goes (:51-54), vector_free leaves the
 * capacity field as it was (:84-89).  Departures only where the reference has
 * undefined behaviour: a push into capacity 0 grows to 1 (the reference asks for
 * 0 * 2 and writes past the allocation, :31-33), and deleting at or past size is a
 * no-op (the reference's memmove length underflows, :60).
 */
#include "../../../include/utils/vector.h"

#include <stdlib.h>
#include <string.h>

void vector_init(struct vector *vec, size_t capacity, size_t element_size)
{
    vec->size = 0;
    vec->capacity = capacity;
    vec->element_size = element_size;
    /* calloc(0, n) may return NULL; keep a valid pointer so later pushes work */
    vec->elements = calloc(capacity ? capacity : 1, element_size ? element_size : 1);
}

int vector_resize(struct vector *vec, size_t new_capacity)
{
    if (vec->capacity >= new_capacity) return -1;
    void *p = realloc(vec->elements, vec->element_size * new_capacity);
    if (p == NULL) return -1;
    vec->elements = p;
    vec->capacity = new_capacity;
    return 0;
}

void vector_push(struct vector *vec, void *element)
{
    if (vec->size + 1 > vec->capacity) vector_resize(vec, vec->capacity ? vec->capacity * 2 : 1);
    memcpy((char *)vec->elements + vec->element_size * vec->size, element, vec->element_size);
    ++vec->size;
}

void vector_set_index(struct vector *vec, void *element, size_t index)
{
    memcpy((char *)vec->elements + vec->element_size * index, element, vec->element_size);
    if (index >= vec->size) ++vec->size;
}

void *vector_get(struct vector *vec, size_t index)
{
    return (char *)vec->elements + vec->element_size * index;
}

void *vector_get_buffer(struct vector *vec)
{
    return (char *)vec->elements + vec->element_size * vec->size;
}

void vector_delete(struct vector *vec, size_t index)
{
    if (index >= vec->size) return;
    char *base = vec->elements;
    memmove(base + vec->element_size * index, base + vec->element_size * (index + 1),
            vec->element_size * (vec->size - index - 1));
    --vec->size;
}

void vector_clear(struct vector *vec)
{
    vec->size = 0;
}

void vector_reset(struct vector *vec)
{
    memset(vec->elements, 0, vec->element_size * vec->size);
}

void vector_free(struct vector *vec)
{
    vec->size = 0;
    free(vec->elements);
    vec->elements = NULL;
}
