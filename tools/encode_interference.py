"""What slows the 16-video encode beside the decodes?  Times the encode (CU-reserved stream, as in the
pipeline) alone and beside interferers queued on another stream:
  empty62   a hipGraph of 62 dependent one-workgroup kernels (the decode step's launch count, no work)
  wide62    the same with 16 x 768 f32 adds (12 workgroups each, a decode activation's size)
  decode    the real greedy decode graph (16 rows, grid cap 96), back to back
  decode_conf  the same on a stream masked to the encode's reserved CUs
Prints the median encode time per mode and the interferer's own rate."""
import ctypes as C
import os
import statistics
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "video-caption-algorithm_amd"))
import torch

from vcap import _native as N, configs, prng, weights
from vcap.model import GenConfig, HipGPT2Decoder, HipPrefix, HipViTEncoder

dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
va, ga = configs.vit_arch("vit_base_patch16_224"), configs.gpt2_arch("gpt2")
sd = weights.synthetic_state_dict(1, va, ga)
enc = HipViTEncoder(sd, va, "bf16", dev)
pre = HipPrefix(sd, ga.n_embd, device=dev)
dec = HipGPT2Decoder(sd, ga, "bf16", dev)
video = torch.from_numpy(prng.imagenet_frames(1000, (16, 16, 3, va.image, va.image))).to(dev)

h = C.c_void_p()
N.check(N.lib().vcap_stream_create_cu_reserved(int(os.environ.get("RESERVE", "32")), C.byref(h)), "stream")
s_enc = torch.cuda.ExternalStream(h.value, device=dev)
s_int = torch.cuda.Stream(dev)
# the reserved CUs only (pipeline confine_decode): decode workgroups never take an encode CU
words = (torch.cuda.get_device_properties(dev).multi_processor_count + 31) // 32
mask = (C.c_uint32 * words)()
for c in range(int(os.environ.get("RESERVE", "32"))):
    mask[c // 32] |= 1 << (c % 32)
hc = C.c_void_p()
N.check(N.lib().vcap_stream_create_cu_mask(mask, words, C.byref(hc)), "confined stream")
s_conf = torch.cuda.ExternalStream(hc.value, device=dev)
ENC = int(os.environ.get("ENC", "8"))

# interferers
one = torch.zeros(1, device=dev)
act = torch.zeros(16, 768, device=dev)
graphs = {}
for name, t in (("empty62", one), ("wide62", act)):
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s_int):
        for _ in range(3):
            t.add_(1.0)
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s_int):
            for _ in range(62):
                t.add_(1.0)
    graphs[name] = g
dpre = torch.randn(16, 4, ga.n_embd, device=dev) * 0.1
cfg = GenConfig(24, 8, 3, 1.1, ga.eos_token_id, ga.eos_token_id, True, max_blocks=96)


def interfere(mode, n):
    with torch.cuda.stream(s_conf if mode == "decode_conf" else s_int):
        for _ in range(n):
            if mode.startswith("decode"):
                dec.generate_ids(dpre, [ga.bos_token_id], cfg)
            else:
                graphs[mode].replay()


def rate(mode, n):
    torch.cuda.synchronize()
    t = time.perf_counter()
    interfere(mode, n)
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e3


def encodes():
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(ENC + 1)]
    with torch.cuda.stream(s_enc):
        ev[0].record(s_enc)
        for i in range(ENC):
            enc.encode(video, pre)
            ev[i + 1].record(s_enc)
    return ev


for _ in range(2):
    encodes()
interfere("decode", 2)
torch.cuda.synchronize()
print(f"interferer alone: empty62 {rate('empty62', 200) * 1e3:.0f} us/graph, wide62 {rate('wide62', 200) * 1e3:.0f} "
      f"us/graph, decode {rate('decode', 6):.2f} ms/call", flush=True)
print(f"confined decode alone {rate('decode_conf', 6):.2f} ms/call", flush=True)
per_ms = {"empty62": 0.11, "wide62": 0.12, "decode": 7.5, "decode_conf": 7.5}
for rnd in range(2):
    for mode in ("alone", "decode", "decode_conf"):
        torch.cuda.synchronize()
        if mode != "alone":
            interfere(mode, int(ENC * 12.5 / per_ms[mode] * 1.3) + 4)
        ev = encodes()
        torch.cuda.synchronize()
        ts = [ev[i].elapsed_time(ev[i + 1]) for i in range(1, ENC)]
        print(f"round {rnd} {mode:8s} encode median {statistics.median(ts):.3f} ms  min {min(ts):.3f}", flush=True)
