"""GPU frame preprocessing (vcap_frames_preprocess) against PIL itself and the reference's
transform chain (core/preprocessing/frame_loader.py:34-45): resized pixels bit-identical to
PIL Image.resize(BILINEAR) (integer parity), normalised f32 bit-identical to ToTensor + Normalize
on those pixels (oracle.frames_to_tensor restates the chain; PIL is the resize oracle)."""
import numpy as np
import pytest
import torch
from PIL import Image

from oracle import vcap_oracle as O
from vcap.preprocess import preprocess_frames

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("hw", [(240, 320), (360, 480), (224, 224), (100, 150), (1080, 1920), (224, 300),
                                (300, 224), (37, 500)])
def test_preprocess_bit_exact_vs_pil(device, hw):
    h, w = hw
    g = np.random.default_rng(h + 3 * w)
    frames = np.stack([g.integers(0, 256, (h, w, 3), dtype=np.uint8),
                       (np.add.outer(np.arange(h), 3 * np.arange(w))[:, :, None] * np.array([1, 2, 5]) % 256)
                       .astype(np.uint8)])
    out, u8 = preprocess_frames(torch.from_numpy(frames).to(device), 224, out_u8=True)
    torch.cuda.synchronize()
    ref_u8 = np.stack([np.asarray(Image.fromarray(f).resize((224, 224), Image.BILINEAR)) for f in frames])
    assert np.array_equal(u8.cpu().numpy(), ref_u8)
    assert np.array_equal(out.cpu().numpy(), O.frames_to_tensor(frames, 224))


def test_loader_hip_matches_pil_backend(device, tmp_path):
    """core.preprocessing.load_video_tensor: GPU path == host PIL path on real JPEG files."""
    from core.preprocessing.frame_loader import load_video_tensor
    g = np.random.default_rng(5)
    for i in range(20):
        img = (g.random((180, 320, 3)) * 255).astype(np.uint8)
        Image.fromarray(img).save(tmp_path / f"frame_{i:04d}.jpg", quality=90)
    a = load_video_tensor(tmp_path, 8, 224, device=str(device), backend="hip")
    b = load_video_tensor(tmp_path, 8, 224, device="cpu", backend="pil")
    assert a.shape == (1, 8, 3, 224, 224)
    assert torch.equal(a.cpu(), b)
