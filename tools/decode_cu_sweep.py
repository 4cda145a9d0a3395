"""Decode step time (B rows, env B=8 default, hipGraph) when the decode stream may use only R CUs (CU-masked stream),
with the GPU otherwise idle, and with an encode loop running on the complementary CUs.
Separates 'fewer CUs' from 'contention' in the overlapped pipeline."""
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
import os
B = int(os.environ.get("B", "8"))
prefix = torch.randn(B, 4, 768, device=dev) * 0.1
lib = N.lib()


def masked(exclude):
    h = C.c_void_p()
    N.check(lib.vcap_stream_create_cu_reserved(int(exclude), C.byref(h)), "stream")
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
    return (res[24] - res[1]) / 23 * 1e6, res[24] * 1e3


for R in [int(x) for x in os.environ.get("RS", "256,128,64,48,32").split(",")]:
    for cap in [int(c) * R if c != "0" else 0 for c in os.environ.get("CAPS", "0,2").split(",")]:
        s_dec = masked(256 - R) if R < 256 else torch.cuda.Stream(dev)
        alone = step_us(s_dec, cap)
        # the same with an encode loop on the other CUs
        stop = False
        s_enc = masked(R) if R < 256 else torch.cuda.Stream(dev)

        def enc_loop():
            with torch.cuda.stream(s_enc):
                while not stop:
                    enc.encode(video, pre)
                    s_enc.synchronize()
        th = threading.Thread(target=enc_loop)
        th.start()
        time.sleep(0.05)
        busy = step_us(s_dec, cap)
        stop = True
        th.join()
        torch.cuda.synchronize()
        print(f"R={R:3d} cap={cap:3d}: alone step {alone[0]:6.1f} us (decode {alone[1]:5.2f} ms) | "
              f"beside encode step {busy[0]:6.1f} us (decode {busy[1]:5.2f} ms)", flush=True)
