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
