"""Decode timing probe: per-token step cost vs batch, graph vs eager (run on the GPU box)."""
import sys, time
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "video-caption-algorithm_amd"))
import torch
from vcap import configs, weights
from vcap.model import GenConfig, HipGPT2Decoder

ga = configs.gpt2_arch("gpt2")
sd = weights.synthetic_gpt2(1, ga)
dev = torch.device("cuda:0")
dec = HipGPT2Decoder(sd, ga, "bf16", dev)
s = torch.cuda.Stream()
with torch.cuda.stream(s):
    for B in (1, 8, 32):
        pre = torch.randn(B, 4, 768, device=dev) * 0.1
        for graph in (True, False):
            res = {}
            for mx in (1, 24):
                cfg = GenConfig(mx, 8, 3, 1.1, 50256, 50256, graph)
                for _ in range(3):
                    dec.generate_ids(pre, [50256], cfg)
                torch.cuda.synchronize()
                t = time.perf_counter()
                n = 10
                for _ in range(n):
                    dec.generate_ids(pre, [50256], cfg)
                torch.cuda.synchronize()
                res[mx] = (time.perf_counter() - t) / n * 1e3
            print(f"B={B:3d} graph={graph}: prefill-only {res[1]:.3f} ms, 24 tokens {res[24]:.3f} ms, "
                  f"per decode step {(res[24]-res[1])/23*1e3:.1f} us", flush=True)
