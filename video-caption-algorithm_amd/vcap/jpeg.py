"""JPEG frames -> uint8 RGB on the GPU (vcap_jpeg_decode_batch).

Replaces the host `Image.open(path).convert("RGB")` of core/preprocessing/frame_loader.py:42-44 for
baseline JPEGs: the library parses and entropy-decodes on host threads and runs libjpeg-turbo's
islow IDCT, fancy chroma upsampling and YCbCr -> RGB on the device, bit-identical to Pillow
(tests/test_gpu_jpeg.py).  Images the decoder does not take (progressive, arithmetic-coded, CMYK,
4:4:0 ...) raise VcapError; there is no host fallback.
"""
from __future__ import annotations

import ctypes as C
from typing import Sequence

import torch

from . import _native as N


def probe(data: bytes):
    """(width, height, components) of one JPEG; raises VcapError for what the decoder refuses."""
    w, h, c = C.c_int(), C.c_int(), C.c_int()
    N.check(N.lib().vcap_jpeg_probe(data, len(data), C.byref(w), C.byref(h), C.byref(c)), "vcap_jpeg_probe")
    return w.value, h.value, c.value


def decode_jpegs(blobs: Sequence[bytes], device) -> torch.Tensor:
    """JPEG byte strings (one size, sampling and quantisation tables) -> uint8 [n, H, W, 3] on device."""
    if not blobs:
        raise ValueError("no images")
    device = torch.device(device)
    w, h, _ = probe(blobs[0])
    lib = N.lib()
    n = len(blobs)
    ws_bytes = int(lib.vcap_jpeg_workspace_bytes(blobs[0], len(blobs[0]), n))
    if ws_bytes == 0:
        raise N.VcapError("vcap_jpeg_workspace_bytes: unsupported JPEG")
    out = torch.empty(n, h, w, 3, dtype=torch.uint8, device=device)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=device)
    keep = [C.create_string_buffer(b, len(b)) for b in blobs]     # stable host pointers for the call
    ptrs = (C.c_void_p * n)(*[C.cast(k, C.c_void_p) for k in keep])
    lens = (C.c_size_t * n)(*[len(b) for b in blobs])
    with torch.cuda.device(device):
        stream = torch.cuda.current_stream(device).cuda_stream
        N.check(lib.vcap_jpeg_decode_batch(ptrs, lens, n, out.data_ptr(), ws.data_ptr(), ws_bytes, stream),
                "vcap_jpeg_decode_batch")
    return out
