#ifndef VECTOR_H
#define VECTOR_H

/*
 * Growable array used as the WS reassembly buffer.  Same struct layout and
 * functions as the reference's include/utils/vector.h:7-41 (the buffer is
 * embedded in struct ws_frame_parsing_state, so its layout is ABI).
 */

#include <stddef.h>

struct vector
{
    /** Elements in use. */
    size_t size;
    /** Elements allocated. */
    size_t capacity;
    /** Bytes per element. */
    size_t element_size;
    /** Storage (malloc-family; freed with free()). */
    void *elements;
};

/** Allocates zeroed storage for `capacity` elements; size = 0. */
void vector_init(struct vector *vec, size_t capacity, size_t element_size);
/** Grows storage to `new_capacity` elements. Returns 0 if it grew, -1 if no growth was needed or realloc failed. */
int vector_resize(struct vector *vec, size_t new_capacity);

/** Appends one element, doubling capacity when full. */
void vector_push(struct vector *vec, void *element);
/** Overwrites the element at `index`; size grows by one when index >= size (as the reference). */
void vector_set_index(struct vector *vec, void *element, size_t index);
/** Pointer to the element at `index` (no range check, as the reference). */
void *vector_get(struct vector *vec, size_t index);
/** Pointer to the end of the data (elements + size * element_size): where the next element goes. */
void *vector_get_buffer(struct vector *vec);
/** Removes the element at `index`, shifting the tail down. */
void vector_delete(struct vector *vec, size_t index);

/** Removes every element (size = 0), keeping storage. */
void vector_clear(struct vector *vec);
/** Zeroes every element in use, keeping size. */
void vector_reset(struct vector *vec);

/** Releases storage; size = 0, elements = NULL (capacity is left as it was, as the reference). */
void vector_free(struct vector *vec);

#endif // VECTOR_H
