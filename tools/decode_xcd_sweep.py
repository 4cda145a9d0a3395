"""Decode step time beside a running encode for different CU-mask layouts of the two streams:
'spread' = the decode's CUs are mask bits [0, R) (spread over XCDs by the driver), 'xcd<k>' =
mask bits i with i % 8 < k (k whole XCDs if the driver maps bit i to XCD i % 8)."""
import ctypes as C
import sys
import threading
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "video-caption-algorithm_amd"))
import torch  # noqa: E402

from vcap import _native as N, configs, prng, weights  # noqa: E402
from vcap.model import GenConfig, HipGPT2Decoder, HipPrefix, HipViTEncoder  # noqa: E402

dev = torch.device("cuda:0")
va, ga = configs.vit_arch("vit_base_patch16_224"), configs.gpt2_arch("gpt2")
sd = weights.synthetic_state_dict(1, va, ga)
enc = HipViTEncoder(sd, va, "bf16", dev)
pre = HipPrefix(sd, ga.n_embd, device=dev)
dec = HipGPT2Decoder(sd, ga, "bf16", dev)
video = torch.from_numpy(prng.imagenet_frames(1000, (8, 16, 3, 224, 224))).to(dev)
prefix = torch.randn(8, 4, 768, device=dev) * 0.1
lib = N.lib()
NCU = 256


def stream_of(bits):
    words = [0] * (NCU // 32)
    for b in bits:
        words[b // 32] |= 1 << (b % 32)
    arr = (C.c_uint32 * len(words))(*words)
    h = C.c_void_p()
    N.check(lib.vcap_stream_create_cu_mask(arr, len(words), C.byref(h)), "mask stream")
    return torch.cuda.ExternalStream(h.value, device=dev)


def step_us(s, cap):
    res = {}
    with torch.cuda.stream(s):
        for mx in (1, 24):
            cfg = GenConfig(mx, 8, 3, 1.1, 50256, 50256, True, cap)
            for _ in range(2):
                dec.generate_ids(prefix, [50256], cfg)
            s.synchronize()
            t = time.perf_counter()
            for _ in range(5):
                dec.generate_ids(prefix, [50256], cfg)
            s.synchronize()
            res[mx] = (time.perf_counter() - t) / 5
    return (res[24] - res[1]) / 23 * 1e6


def enc_time(s):
    with torch.cuda.stream(s):
        enc.encode(video, pre)
        s.synchronize()
        t = time.perf_counter()
        for _ in range(3):
            enc.encode(video, pre)
        s.synchronize()
    return (time.perf_counter() - t) / 3 * 1e3


layouts = []
for k in (1, 2, 3):
    layouts.append((f"xcd{k}", [i for i in range(NCU) if i % 8 < k]))
for R in (32, 64, 96):
    layouts.append((f"spread{R}", list(range(R))))
for name, dbits in layouts:
    ebits = [i for i in range(NCU) if i not in set(dbits)]
    s_dec, s_enc = stream_of(dbits), stream_of(ebits)
    alone = step_us(s_dec, 2 * len(dbits))
    e_alone = enc_time(s_enc)
    stop = False

    def loop():
        with torch.cuda.stream(s_enc):
            while not stop:
                enc.encode(video, pre)
                s_enc.synchronize()
    th = threading.Thread(target=loop)
    th.start()
    time.sleep(0.05)
    busy = step_us(s_dec, 2 * len(dbits))
    stop = True
    th.join()
    torch.cuda.synchronize()
    print(f"{name:9s} decode CUs {len(dbits):3d}: step alone {alone:6.1f} us, beside encode {busy:6.1f} us | "
          f"encode alone on {len(ebits)} CUs {e_alone:5.2f} ms", flush=True)
