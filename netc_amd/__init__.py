"""netc-mi355x: MI355X (gfx950) WebSocket payload masking for netc.

The product is two C-ABI shared libraries built in-tree (``make``):

* ``netc_amd/lib/libnetc.so``        host C: the netc WebSocket framing API
  (``include/ws/common.h``) and the CPU masking entry ``netc_ws_mask``;
* ``netc_amd/lib/libnetc_ws_gpu.so`` HIP / gfx950: the device batch masking
  entries of ``include/ws/mask.h``.

This Python package is a thin ctypes mirror of that C-ABI (``netc_amd.mask``),
used by the tests and ``bench.py``; PyTorch only supplies device memory and
streams.
"""

from .mask import (  # noqa: F401
    NetcGpuError,
    device_count,
    gpu_init,
    mask_batch,
    mask_batch_multi,
    mask_host,
    mask_stream_host,
    pack_keys,
    shard_frames,
    tune,
)
