"""Encode throughput of 8 ViT-B/16 clips (16 frames) split over S concurrent HIP streams (B/S clips
per stream, each stream its own workspace): does overlapping two half-batch encodes fill the
GEMM epilogue / memory-bound gaps of a single encode?  bf16, alone on the GPU."""
import sys, time
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "video-caption-algorithm_amd"))
import torch
from vcap import configs, prng, weights
from vcap.model import HipPrefix, HipViTEncoder, _Workspace

va, ga = configs.vit_arch("vit_base_patch16_224"), configs.gpt2_arch("gpt2")
dev = torch.device("cuda:0")
sd = weights.synthetic_state_dict(1, va, ga)
enc = HipViTEncoder(sd, va, "bf16", dev)
pre = HipPrefix(sd, ga.n_embd, device=dev)
B = 8
video = torch.from_numpy(prng.imagenet_frames(1000, (B, 16, 3, 224, 224))).to(dev)
for S in (1, 2, 4):
    streams = [torch.cuda.Stream(dev) for _ in range(S)]
    wss = [_Workspace(dev) for _ in range(S)]
    per = B // S

    def run():
        for i, st in enumerate(streams):
            with torch.cuda.stream(st):
                enc.ws = wss[i]
                enc.encode(video[i * per:(i + 1) * per], pre)
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    t = time.perf_counter()
    n = 20
    for _ in range(n):
        run()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t) / n * 1e3
    print(f"streams {S} x {per} clips: {ms:.2f} ms per 8 clips ({B / ms * 1e3:.0f} clips/s)", flush=True)
