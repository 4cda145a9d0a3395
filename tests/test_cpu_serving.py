"""Serving batcher (core/serving.py) on a fake engine: requests coalesce into engine calls of at
most max_batch per engine key, results route back to their request, errors reach every request
of the failed call are retried alone (only the offending request fails), videos of different
shapes never share a call, validation mirrors server/services/inference_service.py:50-55."""
import threading
from dataclasses import replace

import pytest

from core.config import InferenceConfig
from core.serving import BatchingInferenceService, GpuTaskManager, ModelRegistry, engine_key


class FakeEngine:
    def __init__(self, config):
        self.config = config
        self.calls = []

    def infer_batch(self, dirs):
        self.calls.append(list(dirs))
        if any(d.endswith("boom") for d in dirs):
            raise RuntimeError("engine failure")
        return [f"{self.config.preset1}:{d}" for d in dirs]


def _dirs(tmp_path, n, tag="v"):
    out = []
    for i in range(n):
        p = tmp_path / f"{tag}{i}"
        p.mkdir()
        out.append(str(p))
    return out


def test_requests_coalesce_and_route(tmp_path):
    engines = {}

    def factory(cfg):
        engines[engine_key(cfg)] = FakeEngine(cfg)
        return engines[engine_key(cfg)]

    svc = BatchingInferenceService(ModelRegistry(factory), max_batch=8, max_wait_ms=200)
    cfg = InferenceConfig(weights_seed=1)
    dirs = _dirs(tmp_path, 20)
    futs = [None] * len(dirs)

    def client(i):
        futs[i] = svc.submit(dirs[i], cfg)

    ts = [threading.Thread(target=client, args=(i,)) for i in range(len(dirs))]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert [f.result(timeout=30) for f in futs] == [f"precise:{d}" for d in dirs]
    svc.close()
    assert sum(svc.batches) == 20 and max(svc.batches) <= 8 and len(svc.batches) < 20
    assert len(engines) == 1


def test_engines_per_config_and_errors(tmp_path):
    reg = ModelRegistry(FakeEngine)
    svc = BatchingInferenceService(reg, GpuTaskManager(1), max_batch=4, max_wait_ms=100)
    a, b = InferenceConfig(weights_seed=1), replace(InferenceConfig(weights_seed=1), preset1="detailed")
    da, db = _dirs(tmp_path, 3, "a"), _dirs(tmp_path, 3, "b")
    bad = tmp_path / "boom"
    bad.mkdir()
    fa = [svc.submit(d, a) for d in da]
    fb = [svc.submit(d, b) for d in db]
    fbad = svc.submit(str(bad), b)
    assert [f.result(timeout=30) for f in fa] == [f"precise:{d}" for d in da]
    got_b = []
    for f in fb + [fbad]:
        try:
            got_b.append(f.result(timeout=30))
        except RuntimeError as e:
            got_b.append(str(e))
    svc.close()
    # the failing request poisons only the engine call it was part of
    assert "engine failure" in got_b[-1]
    assert reg.get_engine(a) is not reg.get_engine(b)
    assert all(len(c) <= 4 for c in reg.get_engine(b).calls)


def test_validation_matches_reference_service(tmp_path):
    svc = BatchingInferenceService(ModelRegistry(FakeEngine))
    with pytest.raises(FileNotFoundError):
        svc.submit(str(tmp_path / "missing"), InferenceConfig())
    d = _dirs(tmp_path, 1)[0]
    with pytest.raises(FileNotFoundError):
        svc.submit(d, InferenceConfig(ckpt=str(tmp_path / "nope.pt")))
    svc.close()
    with pytest.raises(RuntimeError):
        svc.submit(d, InferenceConfig())


class FakeVideoEngine:
    """load_video / infer_videos protocol: frames_dir names encode the clip shape ("t4" = 4 frames)."""

    def __init__(self, config):
        self.config = config
        self.calls = []

    def load_video(self, d):
        import torch
        if d.endswith("unreadable"):
            raise FileNotFoundError("no frames")
        t = int(d.rsplit("t", 1)[1].split("_")[0])
        v = torch.zeros(1, t, 3, 4, 4)
        v[0, 0, 0, 0, 0] = float(d.rsplit("_", 1)[1])
        return v

    def max_batch_videos(self):
        return 3

    def infer_videos(self, videos):
        self.calls.append(tuple(videos.shape))
        ids = [int(x) for x in videos[:, 0, 0, 0, 0].tolist()]
        if 13 in ids:
            raise RuntimeError("bad video 13")
        return [f"T{videos.shape[1]}:{i}" for i in ids]


def test_video_batches_group_by_shape_cap_and_isolate_errors(tmp_path):
    eng = {}

    def factory(cfg):
        eng["e"] = FakeVideoEngine(cfg)
        return eng["e"]

    svc = BatchingInferenceService(ModelRegistry(factory), max_batch=8, max_wait_ms=300)
    cfg = InferenceConfig(weights_seed=1)
    names = [f"t4_{i}" for i in range(5)] + [f"t8_{i}" for i in range(10, 15)] + ["t4_unreadable"]
    dirs = []
    for n in names:
        (tmp_path / n).mkdir()
        dirs.append(str(tmp_path / n))
    futs = [svc.submit(d, cfg) for d in dirs]
    out = []
    for f in futs:
        try:
            out.append(f.result(timeout=30))
        except Exception as e:  # noqa: BLE001
            out.append(type(e).__name__)
    svc.close()
    assert out[:5] == [f"T4:{i}" for i in range(5)]
    assert out[5:10] == ["T8:10", "T8:11", "T8:12", "RuntimeError", "T8:14"]
    assert out[10] == "FileNotFoundError"
    shapes = eng["e"].calls
    assert all(s[0] <= 3 for s in shapes)               # engine.max_batch_videos cap
    assert {s[1] for s in shapes} == {4, 8}             # never mixed in one call
