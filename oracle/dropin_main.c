/*
 * TEST INFRASTRUCTURE ONLY — the drop-in check.
 *
 * Runs the reference's own WebSocket integration test, tests/ws/test001.c, as the
 * reference's main.c does (main.c:11,40), but alone (in the full
 * suite it fails on the shared port 8923).  The test file is #included from where it
 * lies under /root/reference (-DREF_WS_TEST=...); nothing is copied.  oracle/Makefile
 * links it twice against the reference's own callers (src/web, src/http, src/tcp,
 * src/ws/{server,client}.c, src/utils, src/socket.c):
 *   _ref/ws_test001_reference : + the reference's src/ws/common.c (the baseline)
 *   _ref/ws_test001_libnetc   : + libnetc.so of this repo INSTEAD of src/ws/common.c
 * Prints one line per symbol of interest with the object that defines the copy the
 * process binds (dladdr), then the test's result; exits with the test's result.
 */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <stdio.h>

/* brings in the reference's include/web, include/ws, include/utils headers */
#include REF_WS_TEST

static void where(const char *name, void *addr)
{
    Dl_info info;
    if (addr && dladdr(addr, &info) && info.dli_fname)
        printf("bind %s %s\n", name, info.dli_fname);
    else
        printf("bind %s ?\n", name);
}

int main(void)
{
    setvbuf(stdout, NULL, _IOLBF, 0);
    /* function addresses as the executable resolves them (PLT / its own copies) */
    where("ws_parse_frame", (void *)&ws_parse_frame);
    where("ws_send_message", (void *)&ws_send_message);
    where("ws_build_masking_key", (void *)&ws_build_masking_key);
    where("vector_init", (void *)&vector_init);
    where("vector_get_buffer", (void *)&vector_get_buffer);
    where("tcp_server_send", (void *)&tcp_server_send);
    /* what libnetc.so itself binds for the utilities it calls (default symbol search) */
    where("dlsym:vector_resize", dlsym(RTLD_DEFAULT, "vector_resize"));
    where("dlsym:netc_ws_mask", dlsym(RTLD_DEFAULT, "netc_ws_mask"));
    const int r = ws_test001();
    printf("ws_test001 result %d\n", r);
    return r;
}
