"""Command-line caption inference: `python -m src.cli.inference --video_path <dir|file> --num_frames 16`.

The north-star CLI of the reference README (README.md:79), which the reference itself does not
ship (its src/cli/infer_once.py imports a missing module).  Flags follow README.md:79 and
experiments/inference.py:388-436 (--frames_dir --ckpt --num_frames --preset* --prompt*).

--video_path may be a directory of frame_*.jpg (the reference's pre-extracted layout) or a video
file; decoding a video file needs a frame extractor (ffmpeg / OpenCV / PyAV), none of which is in
this image, so files are rejected with a message instead of silently falling back.
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))

from core.config import InferenceConfig  # noqa: E402


def _frames_dir(args) -> str:
    path = args.frames_dir or args.video_path
    if not path:
        raise SystemExit("give --video_path (frame directory or video file) or --frames_dir")
    p = Path(path)
    if p.is_dir():
        return str(p)
    if p.is_file():
        for mod in ("cv2", "av", "decord"):
            try:
                __import__(mod)
            except ImportError:
                continue
            raise SystemExit(f"video decode through {mod} is not wired yet; extract frames to <dir>/frame_*.jpg")
        raise SystemExit("no video decoder (ffmpeg/cv2/av/decord) in this environment; pass a directory of "
                         "frame_*.jpg (e.g. from `ffmpeg -i clip.mp4 -vf fps=2 dir/frame_%04d.jpg`)")
    raise SystemExit(f"{path} does not exist")


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--video_path", default="")
    ap.add_argument("--frames_dir", default="")
    ap.add_argument("--checkpoint", "--ckpt", dest="ckpt", default="")
    ap.add_argument("--num_frames", type=int, default=16)
    ap.add_argument("--vit_name", default="vit_base_patch16_224")
    ap.add_argument("--gpt2_name", default="gpt2")
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp32", "fp8"],
                    help="ViT arithmetic: bf16 = the reference's half-precision autocast; fp32 = the parity mode; "
                         "fp8 = MXFP8 ViT GEMMs")
    ap.add_argument("--decoder_precision", default="auto", choices=["auto", "fp32", "bf16"],
                    help="GPT-2 decoder arithmetic: auto = fp32, the reference's (token-exact captions); "
                         "bf16 = the throughput mode")
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--preset", default="", help="decode a single candidate with this preset (precise/detailed/"
                                                 "natural/safe_sample); default runs the 3-candidate infer()")
    ap.add_argument("--greedy", action="store_true", help="single greedy candidate (num_beams=1, temperature=1)")
    ap.add_argument("--prompt", default="", help="prompt text, or 'ids:<id> <id> ...' without a local vocab")
    ap.add_argument("--preset1", default="precise")
    ap.add_argument("--preset2", default="precise")
    ap.add_argument("--preset3", default="natural")
    ap.add_argument("--prompt1", default="")
    ap.add_argument("--prompt2", default="")
    ap.add_argument("--prompt3", default="")
    ap.add_argument("--tokenizer_dir", default="", help="directory with GPT-2 vocab.json + merges.txt")
    ap.add_argument("--weights_seed", type=int, default=None, help="seeded random-init weights when no --checkpoint")
    return ap.parse_args(argv)


def main(argv=None):
    args = parse(argv)
    frames = _frames_dir(args)
    cfg = InferenceConfig(ckpt=args.ckpt, vit_name=args.vit_name, gpt2_name=args.gpt2_name,
                          num_frames=args.num_frames, precision=args.precision,
                          decoder_precision=args.decoder_precision, device=args.device,
                          preset1=args.preset1, preset2=args.preset2, preset3=args.preset3, prompt1=args.prompt1,
                          prompt2=args.prompt2, prompt3=args.prompt3, tokenizer_dir=args.tokenizer_dir,
                          weights_seed=args.weights_seed)
    from core.engine import InferenceEngine
    from core.inference import preset_to_kwargs
    from core.preprocessing.frame_loader import load_video_tensor
    engine = InferenceEngine(cfg)
    if args.greedy or args.preset:
        kw = preset_to_kwargs(args.preset) if args.preset else {}
        if args.greedy:
            kw.update(num_beams=1, temperature=1.0)
        video = load_video_tensor(frames, cfg.num_frames, cfg.image_size, cfg.device)
        print(json.dumps({"caption": engine._generate_once(video, args.prompt, **kw)}))
    else:
        print(json.dumps(engine.infer(frames).to_api_dict()))


if __name__ == "__main__":
    main()
