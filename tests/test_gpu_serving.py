"""Batched engine path on the GPU: InferenceEngine.infer_batch (one encode + batched decodes for
several frames directories) gives every video the captions its own infer() gives, for the greedy
and beam presets (per-sequence decoding; sampling is excluded: one RNG stream per batch), and the
request batcher (core/serving.py) returns the same results through futures."""
import numpy as np
import pytest
from PIL import Image

pytestmark = pytest.mark.gpu


def _frames(tmp_path, n_videos=3, n_frames=6):
    dirs = []
    g = np.random.default_rng(11)
    for v in range(n_videos):
        d = tmp_path / f"clip{v}"
        d.mkdir()
        for i in range(n_frames):
            img = (g.random((120, 160, 3)) * 255).astype(np.uint8)
            Image.fromarray(img).save(d / f"frame_{i:04d}.jpg", quality=92)
        dirs.append(str(d))
    return dirs


def _cfg():
    from core.config import InferenceConfig
    return InferenceConfig(vit_name="vit_tiny_test", gpt2_name="gpt2_tiny_test", num_frames=4, precision="fp32",
                           device="cuda:0", weights_seed=1, preset1="precise", preset2="detailed",
                           preset3="precise", prompt2="ids:5 900", prompt3="ids:17")


def test_infer_batch_equals_single_video_infer(device, tmp_path):
    from core.engine import InferenceEngine
    dirs = _frames(tmp_path)
    eng = InferenceEngine(_cfg())
    single = [eng.infer(d).to_api_dict() for d in dirs]
    batched = [r.to_api_dict() for r in eng.infer_batch(dirs)]
    assert batched == single


def test_batching_service_end_to_end(device, tmp_path):
    from core.engine import InferenceEngine
    from core.serving import BatchingInferenceService
    dirs = _frames(tmp_path, n_videos=5)
    cfg = _cfg()
    ref = [r.to_api_dict() for r in InferenceEngine(cfg).infer_batch(dirs)]
    svc = BatchingInferenceService(max_batch=8, max_wait_ms=50)
    futs = [svc.submit(d, cfg) for d in dirs]
    got = [f.result(timeout=120).to_api_dict() for f in futs]
    svc.close()
    assert got == ref and sum(svc.batches) == 5
