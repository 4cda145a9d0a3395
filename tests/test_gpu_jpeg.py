"""GPU JPEG frame decode (vcap_jpeg_decode_batch: host entropy decode, device islow IDCT + fancy
upsampling + YCbCr -> RGB) bit-identical to Pillow's Image.open(...).convert("RGB"), the call the
reference makes (core/preprocessing/frame_loader.py:42-44), and to the CPU oracle; the frame loader's
GPU path (decode + resize + normalise on the device) equals the host PIL path fed to the same GPU
preprocessing."""
import io

import numpy as np
import pytest
import torch
from PIL import Image

from helpers import jpeg_cases
from vcap import _native as N
from vcap.jpeg import decode_jpegs

pytestmark = pytest.mark.gpu
CASES = jpeg_cases()


@pytest.mark.parametrize("name,data", CASES, ids=[c[0] for c in CASES])
def test_decode_bit_exact_vs_pillow(device, name, data):
    ref = np.asarray(Image.open(io.BytesIO(data)).convert("RGB"))
    got = decode_jpegs([data], device)
    torch.cuda.synchronize()
    assert np.array_equal(got[0].cpu().numpy(), ref)


def test_decode_batch_of_frames(device):
    """16 frames of one clip (same encoder settings, different content) in one call."""
    g = np.random.default_rng(3)
    blobs, refs = [], []
    for i in range(16):
        a = np.clip(np.add.outer(np.arange(180), np.arange(320))[:, :, None] * (i + 1) % 256 +
                    g.normal(0, 20, (180, 320, 3)), 0, 255).astype(np.uint8)
        b = io.BytesIO()
        Image.fromarray(a).save(b, format="JPEG", quality=90)
        blobs.append(b.getvalue())
        refs.append(np.asarray(Image.open(io.BytesIO(blobs[-1])).convert("RGB")))
    got = decode_jpegs(blobs, device).cpu().numpy()
    assert np.array_equal(got, np.stack(refs))


def test_decode_batch_mixed_quantisation_tables(device):
    """Frames of one clip written with different quantisation tables in one call (ffmpeg's MJPEG
    rate control writes a per-frame qscale into each frame's DQT): every frame bit-identical to
    Pillow's decode of it."""
    g = np.random.default_rng(11)
    blobs, refs = [], []
    for i, q in enumerate([55, 70, 95, 80, 62, 99, 75, 88]):
        a = np.clip(np.add.outer(np.arange(96), 2 * np.arange(128))[:, :, None] * (i + 3) % 256 +
                    g.normal(0, 18, (96, 128, 3)), 0, 255).astype(np.uint8)
        b = io.BytesIO()
        Image.fromarray(a).save(b, format="JPEG", quality=q, subsampling=2)
        blobs.append(b.getvalue())
        refs.append(np.asarray(Image.open(io.BytesIO(blobs[-1])).convert("RGB")))
    got = decode_jpegs(blobs, device).cpu().numpy()
    assert np.array_equal(got, np.stack(refs))


def _segments(data):
    """(marker, start, end) of the header segments of a JPEG up to SOS."""
    out, i = [], 2
    while i + 4 <= len(data):
        m = data[i + 1]
        n = (data[i + 2] << 8) | data[i + 3]
        out.append((m, i, i + 2 + n))
        if m == 0xDA:
            break
        i += 2 + n
    return out


def _jpeg(h=40, w=56, mode="RGB", **kw):
    g = np.random.default_rng(h * w)
    a = np.clip(np.add.outer(np.arange(h), np.arange(w))[:, :, None] * np.array([1, 3, 5]) % 256 +
                g.normal(0, 15, (h, w, 3)), 0, 255).astype(np.uint8)
    b = io.BytesIO()
    Image.fromarray(a).convert(mode).save(b, format="JPEG", quality=90, **kw)
    return b.getvalue()


def test_rgb_coded_jpeg_refused_ycbcr_adobe_decoded(device):
    """libjpeg's colour-space rule (jdapimin.c default_decompress_parms): a 3-component JPEG with no
    JFIF marker and an APP14 Adobe transform of 0 is RGB-coded (Pillow returns the samples as RGB)
    and the decoder refuses it; with the JFIF marker kept the same APP14 is ignored (YCbCr) and the
    decode stays bit-identical to Pillow, APP14 placed before the SOF as encoders write it."""
    data = _jpeg(subsampling=0)
    seg = _segments(data)
    app0 = next(s for s in seg if s[0] == 0xE0)
    app14 = b"\xff\xee\x00\x0eAdobe\x00\x64\x00\x00\x00\x00\x00"   # transform = 0
    no_jfif = data[:app0[1]] + app14 + data[app0[2]:]
    with pytest.raises(N.VcapError):
        decode_jpegs([no_jfif], device)
    with_jfif = data[:app0[2]] + app14 + data[app0[2]:]
    ref = np.asarray(Image.open(io.BytesIO(with_jfif)).convert("RGB"))
    assert np.array_equal(decode_jpegs([with_jfif], device)[0].cpu().numpy(), ref)


def test_greyscale_with_declared_sampling_factors(device):
    """A one-component JPEG is a non-interleaved scan whatever sampling factors its SOF declares
    (T.81 A.2.2): the block walk is raster order over ceil(W/8) x ceil(H/8), as libjpeg decodes it."""
    data = bytearray(_jpeg(37, 53, "L"))
    sof = next(s for s in _segments(bytes(data)) if s[0] == 0xC0)
    data[sof[1] + 2 + 2 + 6 + 1] = 0x22          # component 0's H/V sampling byte: 1x1 -> 2x2
    data = bytes(data)
    ref = np.asarray(Image.open(io.BytesIO(data)).convert("RGB"))
    assert np.array_equal(decode_jpegs([data], device)[0].cpu().numpy(), ref)


def test_loader_auto_falls_back_to_host_decode_for_refused_frames(device, tmp_path):
    """load_video_tensor(backend='auto') on progressive JPEGs (refused by the GPU decoder): PIL
    decodes them on the host and the device resizes / normalises, = the PIL path bit for bit;
    backend='hip' raises."""
    from core.preprocessing.frame_loader import load_video_tensor
    from vcap.preprocess import frames_to_video
    for i in range(8):
        (tmp_path / f"frame_{i:04d}.jpg").write_bytes(_jpeg(60 + 0 * i, 80, progressive=True))
    got = load_video_tensor(tmp_path, 8, 224, device=str(device), backend="auto")
    pil = [np.asarray(Image.open(p).convert("RGB")) for p in sorted(tmp_path.glob("frame_*.jpg"))]
    assert torch.equal(got, frames_to_video(pil, 224, device))
    with pytest.raises(N.VcapError):
        load_video_tensor(tmp_path, 8, 224, device=str(device), backend="hip")


def test_decode_refuses_mixed_shapes(device):
    with pytest.raises(N.VcapError):
        decode_jpegs([CASES[0][1], CASES[3][1]], device)


def test_loader_gpu_decode_equals_pil_decode(device, tmp_path):
    """load_video_tensor(backend='hip') (GPU decode + GPU resize / normalise) == PIL decode + the
    same GPU resize / normalise, bit for bit."""
    from core.preprocessing.frame_loader import load_video_tensor
    from vcap.preprocess import frames_to_video
    g = np.random.default_rng(7)
    for i in range(20):
        yy, xx = np.mgrid[0:240, 0:320]
        a = np.clip(np.stack([128 + 90 * np.sin(xx / (9.0 + i) + c) for c in range(3)], -1) +
                    g.normal(0, 25, (240, 320, 3)), 0, 255).astype(np.uint8)
        Image.fromarray(a).save(tmp_path / f"frame_{i:04d}.jpg", quality=88)
    got = load_video_tensor(tmp_path, 16, 224, device=str(device), backend="hip")
    files = sorted(tmp_path.glob("frame_*.jpg"))[::1][:16]
    pil = [np.asarray(Image.open(p).convert("RGB")) for p in files]
    ref = frames_to_video(pil, 224, device)
    torch.cuda.synchronize()
    assert torch.equal(got, ref)
