"""Minimal decode driver for counter collection (eager launches, B=8, 24 tokens, 3 runs)."""
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "video-caption-algorithm_amd"))
import torch
from vcap import configs, weights
from vcap.model import GenConfig, HipGPT2Decoder

ga = configs.gpt2_arch("gpt2")
dec = HipGPT2Decoder(weights.synthetic_gpt2(1, ga), ga, "bf16", torch.device("cuda:0"))
pre = torch.randn(8, 4, 768, device="cuda:0") * 0.1
for _ in range(3):
    dec.generate_ids(pre, [50256], GenConfig(24, 8, 3, 1.1, 50256, 50256, False))
torch.cuda.synchronize()
print("done")
