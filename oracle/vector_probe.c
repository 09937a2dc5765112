/*
 * TEST INFRASTRUCTURE ONLY — tests/test_dropin.py compiles this twice, once with the
 * reference's src/utils/vector.c (from /root/reference, where it lies) and once with
 * netc_amd/csrc/host/vector.c, and requires the same output: libnetc.so exports
 * netc's vector_* names, and a netc program that links its own copy interposes them,
 * so the two must behave alike on every defined path (include/utils/vector.h).
 */
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include VECTOR_HEADER

#define SHOW(tag) printf("%s size=%zu cap=%zu\n", tag, v.size, v.capacity)
#define OFF(p) ((long)((char *)(p) - (char *)v.elements))

int main(void)
{
    struct vector v;
    vector_init(&v, 2, sizeof(uint32_t));
    SHOW("init");
    for (uint32_t i = 0; i < 5; ++i) vector_push(&v, &i);
    SHOW("push5");
    printf("get_buffer off=%ld\n", OFF(vector_get_buffer(&v)));
    printf("get(3) off=%ld val=%u\n", OFF(vector_get(&v, 3)), *(uint32_t *)vector_get(&v, 3));
    uint32_t x = 77;
    vector_set_index(&v, &x, 1); /* inside: size unchanged */
    SHOW("set1");
    vector_set_index(&v, &x, 5); /* at size: size grows */
    SHOW("set5");
    printf("get_buffer off=%ld\n", OFF(vector_get_buffer(&v)));
    printf("resize-smaller=%d resize-bigger=%d\n", vector_resize(&v, 4), vector_resize(&v, 64));
    SHOW("resize");
    vector_delete(&v, 0);
    SHOW("delete0");
    for (size_t i = 0; i < v.size; ++i) printf("%u ", *(uint32_t *)vector_get(&v, i));
    printf("\n");
    vector_reset(&v);
    printf("after reset first=%u size=%zu\n", *(uint32_t *)vector_get(&v, 0), v.size);
    vector_clear(&v);
    SHOW("clear");
    printf("get_buffer off=%ld\n", OFF(vector_get_buffer(&v)));
    vector_push(&v, &x);
    SHOW("push-after-clear");
    vector_free(&v);
    printf("free elements=%s size=%zu cap=%zu\n", v.elements ? "set" : "NULL", v.size, v.capacity);
    /* the WS path's own use: byte vector grown by resize, NUL pushed (src/ws/common.c:213-216,303,342) */
    struct vector b;
    vector_init(&b, 5, 1);
    memcpy(b.elements, "hello", 5);
    b.size = 5;
    vector_push(&b, &(char){'\0'});
    printf("bytes size=%zu cap=%zu str=%s\n", b.size, b.capacity, (char *)b.elements);
    vector_free(&b);
    return 0;
}
