"""Encode throughput, ViT-B/16 bf16 16-frame clips, alone on the GPU: one encode of 2B clips on the whole
chip against two encodes of B clips on two streams CU-masked to disjoint halves of the chip (XCDs 0-3 /
4-7), started half an encode apart so their memory-bound phases (GEMM residual epilogues, LayerNorms)
fall beside the other half's MFMA-bound ones.  Also two unmasked streams, for reference."""
import ctypes as C
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "video-caption-algorithm_amd"))
import torch  # noqa: E402

from vcap import _native as N, configs, prng, weights  # noqa: E402
from vcap.model import HipPrefix, HipViTEncoder, _Workspace  # noqa: E402

B = int(os.environ.get("B", "8"))
ITERS = int(os.environ.get("ITERS", "12"))
va, ga = configs.vit_arch("vit_base_patch16_224"), configs.gpt2_arch("gpt2")
dev = torch.device("cuda:0")
sd = weights.synthetic_state_dict(1, va, ga)
enc = HipViTEncoder(sd, va, "bf16", dev)
pre = HipPrefix(sd, ga.n_embd, device=dev)
lib = N.lib()
video = torch.from_numpy(prng.imagenet_frames(1000, (2 * B, 16, 3, 224, 224))).to(dev)
ncu = torch.cuda.get_device_properties(dev).multi_processor_count


def masked(lo, hi):
    words = (ncu + 31) // 32
    m = (C.c_uint32 * words)()
    for c in range(lo, hi):
        m[c // 32] |= 1 << (c % 32)
    h = C.c_void_p()
    N.check(lib.vcap_stream_create_cu_mask(m, words, C.byref(h)), "stream")
    return torch.cuda.ExternalStream(h.value, device=dev)


def timed(fn, n):
    fn(2)
    torch.cuda.synchronize()
    t = time.perf_counter()
    fn(n)
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e3


ws_full = _Workspace(dev)


def one_stream(n):
    enc.ws = ws_full
    for _ in range(n):
        enc.encode(video, pre)


ms = timed(one_stream, ITERS)
print(f"one stream, {2 * B} clips per encode: {ms:.2f} ms per {2 * B} clips ({2 * B / ms * 1e3:.0f} clips/s)", flush=True)
# the same on CU-masked streams: every CU enabled (mask overhead alone), and the bench's 32 reserved
for label, st in (("all-CU mask", masked(0, ncu)), ("reserve-32 mask", masked(32, ncu))):
    def one_masked(n, st=st):
        with torch.cuda.stream(st):
            one_stream(n)
    ms = timed(one_masked, ITERS)
    print(f"one {label} stream, {2 * B} clips per encode: {ms:.2f} ms ({2 * B / ms * 1e3:.0f} clips/s)", flush=True)

for label, streams in (("two half-chip masked streams", [masked(0, ncu // 2), masked(ncu // 2, ncu)]),
                       ("two unmasked streams", [torch.cuda.Stream(dev), torch.cuda.Stream(dev)])):
    wss = [_Workspace(dev), _Workspace(dev)]

    def two(n, streams=streams, wss=wss):
        # stream 1 first runs a half-size encode, so the two loops stay about half an encode apart
        with torch.cuda.stream(streams[1]):
            enc.ws = wss[1]
            enc.encode(video[:B // 2], pre)
        for _ in range(n):
            for i in (0, 1):
                with torch.cuda.stream(streams[i]):
                    enc.ws = wss[i]
                    enc.encode(video[i * B:(i + 1) * B], pre)
    ms = timed(two, ITERS)
    print(f"{label}, {B} clips each: {ms:.2f} ms per {2 * B} clips ({2 * B / ms * 1e3:.0f} clips/s)", flush=True)
