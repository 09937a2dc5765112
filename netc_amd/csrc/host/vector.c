/* struct vector (include/utils/vector.h); behaviour as the reference's src/utils/vector.c:8-90. */
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
}

void *vector_get(struct vector *vec, size_t index)
{
    if (index >= vec->size) return NULL;
    return (char *)vec->elements + vec->element_size * index;
}

void *vector_get_buffer(struct vector *vec)
{
    return vec->elements;
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
    free(vec->elements);
    vec->elements = NULL;
    vec->size = 0;
    vec->capacity = 0;
}
