"""Per-token decode step cost (hipGraph, alone on the GPU) for the library named by VCAP_LIB
(ablation builds).  Environment: B (sequences, default 8), GPT2 (arch, default gpt2), BEAMS
(default 1 = HF-greedy graph; > 1 = the device beam search graph, preset "detailed" shape), CAP
(decode grid cap), PREC (decoder arithmetic, bf16 or fp32)."""
import os, sys, time
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "video-caption-algorithm_amd"))
import torch
from vcap import configs, weights, search
from vcap.model import GenConfig, HipGPT2Decoder

name = os.environ.get("GPT2", "gpt2")
ga = configs.gpt2_arch(name)
dev = torch.device("cuda:0")
dec = HipGPT2Decoder(weights.synthetic_gpt2(1, ga), ga, os.environ.get("PREC", "bf16"), dev)
from vcap import _native as N
N.check(N.lib().vcap_set_gemm_policy(int(os.environ.get("VCAP_GEMM_POLICY", "0"))), "policy")
s = torch.cuda.Stream()
B = int(os.environ.get("B", "8"))
beams = int(os.environ.get("BEAMS", "1"))
lo, hi = (1, 24) if beams == 1 else (2, 40)
with torch.cuda.stream(s):
    pre = torch.randn(B, 4, ga.n_embd, device=dev) * 0.1
    res = {}
    for mx in (lo, hi):
        if beams == 1:
            cfg = GenConfig(mx, 8, 3, 1.1, ga.eos_token_id, ga.eos_token_id, True,
                            max_blocks=int(os.environ.get("CAP", "0")))
            run = lambda: dec.generate_ids(pre, [ga.bos_token_id], cfg)
        else:
            run = lambda: search.beam_search_device(dec, pre, [ga.bos_token_id], num_beams=beams, max_new_tokens=mx,
                                                    min_new_tokens=8, no_repeat_ngram_size=3,
                                                    repetition_penalty=1.1, eos=ga.eos_token_id)
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(10):
            run()
        torch.cuda.synchronize()
        res[mx] = (time.perf_counter() - t) / 10 * 1e3
print(f"{Path(os.environ.get('VCAP_LIB', 'base')).name} {name} {os.environ.get('PREC', 'bf16')} B={B} beams={beams} "
      f"cap={os.environ.get('CAP', '0')}: "
      f"step {(res[hi]-res[lo])/(hi-lo)*1e3:.1f} us first {res[lo]*1e3:.0f} us")
