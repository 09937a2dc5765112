// TEST INFRASTRUCTURE ONLY: host stand-ins for the netc_gpu:: kernel launches and C-ABI helpers
// that ws_ingest.hip calls (see hip/hip_runtime.h here).  The frame scan is libnetc's host header
// walk (netc_ws_scan_frames_host, pinned against the oracle in tests/test_scan_host.py); the XOR of
// the unmask and of the frame assembly is libnetc's netc_ws_mask (pinned against the oracle in
// tests/test_mask_cpu.py), so the same build serves as the "hubcpu" measurement control
// (tests/bin/libnetc_hub_cpu.so): the hubs' host code with their device work done on the host.
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include "../../netc_amd/csrc/ws_mask_gpu.h"
extern "C" {
#include "../../include/ws/frame.h"
#include "../../include/ws/mask.h"
extern __thread int netc_errno_reason;
}

namespace netc_gpu {
namespace {
char g_err[512];
int g_fault = -1;
int g_bad_wire = -1;   // netc_mock_bad_wire: the assembly launch this many launches on reports no wire
}
struct ScanScratch {
    uint32_t diag;
};
ScanScratch* scan_scratch_new() { return new ScanScratch{0}; }
void scan_scratch_free(ScanScratch* s) { delete s; }
hipError_t scan_scratch_reserve(ScanScratch*, uint64_t, hipStream_t) { return hipSuccess; }
const uint32_t* scan_scratch_diag_word(const ScanScratch* s) { return &s->diag; }
hipError_t launch_scan_frames(const uint8_t* wire, uint64_t len, uint64_t start, bool strict, uint64_t* hdr,
                              uint32_t* keys, uint8_t* b0, uint64_t max_frames, uint64_t* result, hipStream_t,
                              ScanScratch*) {
    return netc_ws_scan_frames_host(wire, len, start, strict ? NETC_WS_SCAN_STRICT : 0, hdr, keys, b0, max_frames,
                                    result) == 0 ? hipSuccess : hipErrorInvalidValue;
}
hipError_t launch_unmask_scanned(uint8_t* wire, uint64_t, const uint64_t* hdr, const uint32_t* keys,
                                 uint64_t max_frames, const uint64_t* result, hipStream_t, const LaunchCfg&) {
    const uint64_t n = result[0] < max_frames ? result[0] : max_frames;
    for (uint64_t k = 0; k < n; ++k) {
        const uint64_t h = hdr[k];
        const uint8_t second = wire[h + 1];
        const uint64_t code = second & 0x7F;
        if (!(second & 0x80)) continue;
        const uint64_t p = h + 2 + (code == 126 ? 2 : code == 127 ? 8 : 0) + 4;
        uint8_t key[4];
        memcpy(key, wire + p - 4, 4);
        netc_ws_mask(wire + p, wire + p, (size_t)(hdr[k + 1] - p), key, 0);
    }
    return hipSuccess;
}
// the frame assembly (include/ws/frame.h, netc_gpu_encode_frames): each frame's header, key and
// masked payload back to back, frame by frame (src/ws/common.c:55-125 without B1/B2); with a
// length class, a frame outside it sets wo[n] to UINT64_MAX as the kernel's check does
hipError_t launch_encode_frames(uint8_t* wire, uint64_t, const uint8_t* src, uint64_t, const uint64_t* off,
                                const uint32_t* keys, const uint8_t* b0, uint64_t n, bool masked, uint64_t* wo,
                                hipStream_t, const LaunchCfg&, int ext_class) {
    uint64_t w = 0;
    bool broken = false;
    for (uint64_t k = 0; k < n; ++k) {
        const uint64_t len = off[k + 1] - off[k];
        const int ext = len <= 125 ? 0 : (len <= 0xFFFF ? 2 : 8);
        broken |= ext_class >= 0 && ext != ext_class;
        wo[k] = w;
        uint8_t* p = wire + w;
        *p++ = b0 ? b0[k] : 0x82;
        if (ext == 0) {
            *p++ = (uint8_t)((masked ? 0x80 : 0) | len);
        } else if (ext == 2) {
            *p++ = (uint8_t)((masked ? 0x80 : 0) | 126);
            *p++ = (uint8_t)(len >> 8);
            *p++ = (uint8_t)len;
        } else {
            *p++ = (uint8_t)((masked ? 0x80 : 0) | 127);
            for (int b = 7; b >= 0; --b) *p++ = (uint8_t)(len >> (8 * b));
        }
        uint8_t key[4] = {0, 0, 0, 0};
        if (masked) {
            memcpy(key, &keys[k], 4);
            memcpy(p, key, 4);
            p += 4;
        }
        netc_ws_mask(p, src + off[k], (size_t)len, key, 0);
        w = (uint64_t)(p + len - wire);
    }
    if (g_bad_wire >= 0 && g_bad_wire-- == 0) broken = true;
    wo[n] = broken ? ~0ull : w;
    return hipSuccess;
}
int release_enc_scratch(int, hipStream_t) { return 0; }
int api_fail(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof g_err, fmt, ap);
    va_end(ap);
    netc_errno_reason = NETC_REASON_GPU;
    return code;
}
int api_fail_hip(int code, const char* what, hipError_t) { return api_fail(code, "%s: mock failure", what); }
int api_check_device(int) { return 0; }
LaunchCfg api_cfg() { return LaunchCfg(); }
int64_t knob(int) { return -1; }
bool inject_fault() {
    if (g_fault < 0) return false;
    return g_fault-- == 0;
}
}  // namespace netc_gpu

extern "C" const char* netc_gpu_strerror(void) { return netc_gpu::g_err; }
extern "C" int netc_gpu_init(int) { return 0; }
extern "C" int netc_mock_inject_fault(int countdown) {
    netc_gpu::g_fault = countdown;
    return 0;
}
// the frame assembly launch `countdown` launches from now writes wo[n] = UINT64_MAX (a wire the
// device does not vouch for, as a broken length-class promise reports it); -1 disarms
extern "C" int netc_mock_bad_wire(int countdown) {
    netc_gpu::g_bad_wire = countdown;
    return 0;
}
