"""configs[3] beam decode step cost: the device beam search (one hipGraph) vs the host-bookkeeping
search, GPT-2-medium, B=4 sequences x 4 beams (preset "detailed", max_new 40), bf16 / fp32."""
import os, sys, time
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "video-caption-algorithm_amd"))
import torch
from vcap import configs, weights, search
from vcap.model import HipGPT2Decoder

ga = configs.gpt2_arch("gpt2-medium")
dev = torch.device("cuda:0")
prec = os.environ.get("PREC", "bf16")
dec = HipGPT2Decoder(weights.synthetic_gpt2(3, ga), ga, prec, dev)
B = int(os.environ.get("B", "4"))
pre = torch.randn(B, 4, ga.n_embd, device=dev) * 0.1
kw = dict(num_beams=4, min_new_tokens=8, no_repeat_ngram_size=3, repetition_penalty=1.1, eos=ga.eos_token_id)
res = {}
for impl in ("device", "host"):
    fn = search.beam_search_device if impl == "device" else search.beam_search
    for mx in (2, 40):
        for _ in range(2):
            fn(dec, pre, [ga.bos_token_id], max_new_tokens=mx, **kw)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(5):
            fn(dec, pre, [ga.bos_token_id], max_new_tokens=mx, **kw)
        torch.cuda.synchronize()
        res[(impl, mx)] = (time.perf_counter() - t) / 5
    print(f"{impl} {prec} B={B}x4: search 40 steps {res[(impl, 40)] * 1e3:.1f} ms, "
          f"per step {(res[(impl, 40)] - res[(impl, 2)]) / 38 * 1e3:.3f} ms", flush=True)
