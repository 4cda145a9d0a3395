"""BASELINE configs[0]: the north-star CLI (`src/cli/inference.py --video_path <frames dir>
--num_frames 16`, README.md:79) end to end on a 16-frame JPEG directory with ViT-B/16 + GPT-2.

The reference's frames layout (core/preprocessing/frame_loader.py:13-49: frames_dir/frame_*.jpg,
strided pick, PIL bilinear resize, ImageNet normalise) is written here from seeded pixels; the CLI
output must equal the engine API on the same directory (InferenceEngine.infer for the default
3-candidate mode, _generate_once on load_video_tensor for --greedy and for S1 / S2)."""
import json

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

SEED = 3


def _frames_dir(tmp_path, n=40, h=240, w=320):
    from PIL import Image
    d = tmp_path / "clip"
    d.mkdir()
    g = np.random.default_rng(7)
    base = g.integers(0, 256, (h // 8, w // 8, 3), dtype=np.uint8)
    for i in range(n):   # a smooth moving pattern (JPEG-friendly) plus per-frame noise
        img = np.kron(np.roll(base, i, axis=1), np.ones((8, 8, 1), dtype=np.uint8))
        img = np.clip(img.astype(np.int16) + g.integers(-8, 9, img.shape), 0, 255).astype(np.uint8)
        Image.fromarray(img).save(d / f"frame_{i:04d}.jpg", quality=90)
    return d


def _run_cli(argv, capsys):
    from src.cli import inference as cli
    capsys.readouterr()
    cli.main(argv)
    out = capsys.readouterr().out.strip().splitlines()[-1]
    return json.loads(out)


def test_cli_main_matches_engine(device, tmp_path, capsys):
    from core.config import InferenceConfig
    from core.engine import InferenceEngine
    from core.inference import preset_to_kwargs
    from core.preprocessing.frame_loader import load_video_tensor
    d = _frames_dir(tmp_path)
    # explicit-id prompts: the reference's default prompt texts need the GPT-2 vocab, absent offline
    prompts = dict(prompt1="", prompt2="ids:16594 257 1790 11", prompt3="ids:16594 257")
    common = ["--video_path", str(d), "--num_frames", "16", "--weights_seed", str(SEED), "--device", str(device)]
    common += [x for k, v in prompts.items() for x in (f"--{k}", v)]
    greedy = _run_cli(common + ["--greedy"], capsys)
    full = _run_cli(common, capsys)
    eng = InferenceEngine(InferenceConfig(num_frames=16, device=str(device), weights_seed=SEED, **prompts))
    video = load_video_tensor(str(d), 16, 224, str(device))
    assert tuple(video.shape) == (1, 16, 3, 224, 224)
    exp_greedy = eng._generate_once(video, "", **dict(preset_to_kwargs("precise"), num_beams=1, temperature=1.0))
    assert greedy == {"caption": exp_greedy}
    res = eng.infer(str(d)).to_api_dict()
    assert full == res
    c = eng.config
    assert full["S1"] == eng._generate_once(video, c.prompt1, **preset_to_kwargs(c.preset1))
    assert full["S2"] == eng._generate_once(video, c.prompt2, **preset_to_kwargs(c.preset2))
    torch.cuda.synchronize()
