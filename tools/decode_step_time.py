"""Per-token decode step cost (B=8, hipGraph) for the library named by VCAP_LIB (ablation builds)."""
import os, sys, time
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "video-caption-algorithm_amd"))
import torch
from vcap import configs, weights
from vcap.model import GenConfig, HipGPT2Decoder

ga = configs.gpt2_arch("gpt2")
dev = torch.device("cuda:0")
dec = HipGPT2Decoder(weights.synthetic_gpt2(1, ga), ga, "bf16", dev)
from vcap import _native as N
N.check(N.lib().vcap_set_gemm_policy(int(os.environ.get("VCAP_GEMM_POLICY", "0"))), "policy")
s = torch.cuda.Stream()
B = int(os.environ.get("B", "8"))
with torch.cuda.stream(s):
    pre = torch.randn(B, 4, 768, device=dev) * 0.1
    res = {}
    for mx in (1, 24):
        cfg = GenConfig(mx, 8, 3, 1.1, 50256, 50256, True)
        for _ in range(3):
            dec.generate_ids(pre, [50256], cfg)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(10):
            dec.generate_ids(pre, [50256], cfg)
        torch.cuda.synchronize()
        res[mx] = (time.perf_counter() - t) / 10 * 1e3
print(f"{Path(os.environ.get('VCAP_LIB', 'base')).name} policy {os.environ.get('VCAP_GEMM_POLICY', '0')}: B={B} step {(res[24]-res[1])/23*1e3:.1f} us prefill {res[1]*1e3:.0f} us")
