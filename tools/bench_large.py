"""BASELINE configs[3] measurement (informational; bench.py's headline is configs[1]):
32-frame synthetic clips, ViT-L/14 encoder + GPT-2-medium decoder, beam_size=4 with the
reference's `detailed` preset (max_new 40, no_repeat_ngram 3, repetition_penalty 1.1,
min_new_tokens 8) on one MI355X, bf16.  Serial per batch: encode (vcap_vit_encode) then the
host-driven beam search over the step ABI (vcap/search.py).  Prints one JSON line.
usage: python tools/bench_large.py [--batch B] [--steps K] [--warmup W]"""
import argparse
import json
import statistics
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "video-caption-algorithm_amd"))
import torch  # noqa: E402

from vcap import configs, prng, search, weights  # noqa: E402
from vcap.model import HipGPT2Decoder, HipPrefix, HipViTEncoder  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=4)
ap.add_argument("--frames", type=int, default=32)
ap.add_argument("--steps", type=int, default=5)
ap.add_argument("--warmup", type=int, default=1)
ap.add_argument("--beams", type=int, default=4)
ap.add_argument("--max-new", type=int, default=40)
args = ap.parse_args()

dev = torch.device("cuda:0")
va, ga = configs.vit_arch("vit_large_patch14_224"), configs.gpt2_arch("gpt2-medium")
sd = weights.synthetic_state_dict(1, va, ga)
video = torch.from_numpy(prng.imagenet_frames(2000, (args.batch, args.frames, 3, va.image, va.image))).to(dev)
enc, pre, dec = HipViTEncoder(sd, va, "bf16", dev), HipPrefix(sd, ga.n_embd, device=dev), HipGPT2Decoder(sd, ga, "bf16", dev)


def step():
    t0 = time.perf_counter()
    _, prefix = enc.encode(video, pre)
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    rows = search.beam_search(dec, prefix, [ga.bos_token_id], num_beams=args.beams, max_new_tokens=args.max_new,
                              min_new_tokens=8, no_repeat_ngram_size=3, repetition_penalty=1.1,
                              eos=ga.eos_token_id)
    torch.cuda.synchronize(dev)
    return t1 - t0, time.perf_counter() - t1, rows


for _ in range(args.warmup):
    step()
enc_t, dec_t, tot = [], [], []
for _ in range(args.steps):
    a, b, rows = step()
    enc_t.append(a), dec_t.append(b), tot.append(a + b)
p50 = statistics.median(tot)
print(json.dumps({"metric": "captions/s, BASELINE configs[3] shape (informational)", "value": args.batch / p50,
                  "unit": "captions/s", "p50_latency_ms": p50 * 1e3,
                  "stage_ms_p50": {"vit_l14_encode": statistics.median(enc_t) * 1e3,
                                   "beam4_decode": statistics.median(dec_t) * 1e3},
                  "config": {"vit": "vit_large_patch14_224", "gpt2": "gpt2-medium", "batch": args.batch,
                             "frames": args.frames, "num_beams": args.beams, "max_new_tokens": args.max_new,
                             "dtype": "bf16", "schedule": "serial (encode, then host-driven beam search)"},
                  "vit_tflop_per_batch": args.batch * args.frames * va.flops_per_frame(cls_tail=True) / 1e12,
                  "new_tokens": [len(r) for r in rows]}), flush=True)
