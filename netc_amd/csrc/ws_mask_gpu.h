// Internal interface between the gfx950 kernels (ws_mask_gpu.hip) and the
// C-ABI layer (ws_mask_api.hip).  Not installed; the public surface is
// include/ws/mask.h.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ws/mask.h"   // NETC_GPU_KNOB_*

namespace netc_gpu {

// Kernel arguments (passed by value in the kernarg segment).
struct Args {
    uint8_t* dst_base;         // dst rounded down to 16 B
    const uint8_t* src_base;   // src - (dst & 15): same P coordinates as dst_base
    uint64_t total;            // payload bytes in the batch
    const uint64_t* off;       // n + 1 frame offsets (payload coordinates)
    const uint32_t* keys;      // n packed keys
    uint64_t n;                // frames
    uint64_t mis;              // dst & 15
    uint64_t nwin;             // windows (chunks) of U KiB covering [0, mis + total)
    double density;            // n / total: frames per payload byte (table-base guesses)
    const uint64_t* n_dev;     // if set: the frame count is read from device memory at kernel start
    uint8_t* verr;             // TEXT validation (VAL kernels): per-frame "local UTF-8 rule broken" flags
    uint8_t vtag;              // ... written as this call's tag (verr[f] == vtag: flagged by this call)
    uint8_t xcd_remap;         // one-window-per-wave walk: give each XCD a contiguous share of the windows
    int32_t probe_e;           // one-window-per-wave walk: entries of a window's first table probe (<= 64)
    int32_t probe_bias;        // ... and the frames its base sits before the density's guess
    uint8_t seam_src;          // VAL, out of place: a window checks the first bytes after its start itself
                               // (the 4 bytes before it unmasked from src); utf8_messages skips the seams
    uint64_t full_win;         // one-window-per-wave walk, K > 1 steps: windows from this one on are ONE step
                               // (the batch's tapered end, NETC_GPU_KNOB_MASK_TAPER); ~0: none
};

// LaunchCfg::flags (NETC_GPU_TUNE_*): bits 0-1 non-temporal payload stream, 2 the
// persistent grid-stride walk (round-1 kernel), 3 two steps per wavefront window,
// 4 XCD-contiguous window order, 5 XCD-grouped window order (8 consecutive blocks per XCD)
enum : int { kNtLoads = 1, kNtStores = 2, kPersistent = 4, kTwoSteps = 8, kXcdRemap = 16, kXcdGroups = 32 };

struct LaunchCfg {
    int unroll = 1;            // KiB loaded per wavefront at once (1, 2, 4, 8)
    int max_blocks = 0;        // persistent walk only: cap on 256-thread workgroups; 0 = one resident round
    int flags = -1;            // -1 (auto: non-temporal, one window of two steps per wavefront) or a kNt* | k* mix
};

hipError_t launch_mask_frames(uint8_t* dst, const uint8_t* src, uint64_t total, const uint64_t* off,
                              const uint32_t* keys, uint64_t n, hipStream_t stream, const LaunchCfg& cfg,
                              const uint64_t* n_dev = nullptr);

// Unmask + UTF-8 verdicts of the batch's TEXT messages (include/ws/mask.h,
// netc_gpu_unmask_validate): verr is n bytes of scratch holding no byte equal to
// tag (flags of earlier calls carry other tags), valid the n-byte output.
hipError_t launch_mask_validate(uint8_t* dst, const uint8_t* src, uint64_t total, const uint64_t* off,
                                const uint32_t* keys, const uint8_t* header0, uint64_t n, uint8_t* verr, uint8_t tag,
                                uint8_t* valid, hipStream_t stream, const LaunchCfg& cfg);

// ws_frame_gpu.hip: wire offsets (n + 1 entries into wo), then the wire bytes of
// every frame (header, key, masked payload) into wire.  wire_bound >= wo[n].
hipError_t launch_wire_offsets(const uint64_t* off, uint64_t n, bool masked, uint64_t* wo, hipStream_t stream);
// ws_scan_gpu.hip: frame boundaries of a received stream (include/ws/frame.h).  Scratch:
// caller-owned (`own`, e.g. one per ingest slot, freed with it) or, with own == nullptr,
// cached per (device, stream) until release_stream_scratch (netc_gpu_scan_release).
struct ScanScratch;
ScanScratch* scan_scratch_new();
void scan_scratch_free(ScanScratch* s);   // no work using it may be queued
hipError_t scan_scratch_reserve(ScanScratch* s, uint64_t len, hipStream_t stream);   // sized for a len-byte stream
const uint32_t* scan_scratch_diag_word(const ScanScratch* s);   // device: why the last scan walked serially (0: it did not)
int release_stream_scratch(int device, hipStream_t stream);   // 1 if there was a cached entry
int64_t scan_diag(int device, hipStream_t stream);            // why the last scan walked serially (0: it did not)
hipError_t launch_scan_frames(const uint8_t* wire, uint64_t len, uint64_t start, bool strict, uint64_t* hdr,
                              uint32_t* keys, uint8_t* b0, uint64_t max_frames, uint64_t* result,
                              hipStream_t stream, ScanScratch* own = nullptr);
hipError_t launch_unmask_scanned(uint8_t* wire, uint64_t len, const uint64_t* hdr, const uint32_t* keys,
                                 uint64_t max_frames, const uint64_t* result, hipStream_t stream,
                                 const LaunchCfg& cfg);
// ws_mask_gpu.hip: the batch kernel over the frames a scan found (no view array)
hipError_t launch_mask_scanned(uint8_t* wire, uint64_t len, const uint64_t* hdr, const uint32_t* keys,
                               uint64_t max_frames, const uint64_t* result, hipStream_t stream);

// ws_mask_api.hip: the C-ABI's error side channel and process-wide launch shape
int api_fail(int code, const char* fmt, ...);                 // sets the message + netc_errno_reason, returns code
int api_fail_hip(int code, const char* what, hipError_t e);
int api_check_device(int device);                            // 0 or NETC_GPU_ENODEV (message set)
LaunchCfg api_cfg();                                         // snapshot of netc_gpu_tune's shape (one atomic word)
// measurement / test knobs (netc_gpu_knob, include/ws/mask.h NETC_GPU_KNOB_*): one atomic
// word each, seeded once from the environment; < 0 = the built-in default
int64_t knob(int k);
// fault injection for tests (NETC_GPU_KNOB_INJECT_FAULT): true when this ring submission must fail
bool inject_fault();
// per-(device, stream) scratch of the public entries, released by netc_gpu_stream_release
int release_enc_scratch(int device, hipStream_t stream);     // ws_frame_gpu.hip

hipError_t launch_encode_frames(uint8_t* wire, uint64_t wire_bound, const uint8_t* src, uint64_t src_total,
                                const uint64_t* off, const uint32_t* keys, const uint8_t* b0, uint64_t n, bool masked,
                                uint64_t* wo, hipStream_t stream, const LaunchCfg& cfg, int ext_class = -1);
// ext_class: -1, or every frame's extended-length bytes (0, 2, 8) as the caller promises
// (netc_gpu_encode_frames_class; wo[n] = UINT64_MAX after the call if a frame breaks it)

}  // namespace netc_gpu
