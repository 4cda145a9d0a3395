"""Why a decode confined to its own CUs slows down beside the encode: decode token-step time (B rows,
greedy graph, decode stream CU-masked to R CUs) alone and beside background loads that run on the
other CUs only (a CU-masked stream):
  gemm_1round : 256x256-tile GEMM with exactly one tile per CU and a long K (every workgroup placed
                at once: no pending workgroups, MFMA-bound)
  gemm_fc1    : the ViT fc1 GEMM at 16 videos (10+ rounds of workgroups waiting for CUs)
  copy        : a 1 GiB device copy (HBM-bound, many workgroups)
  encode      : the ViT-B/16 encode of 16 videos
"""
import ctypes as C
import os
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
B = int(os.environ.get("B", "16"))
R = int(os.environ.get("R", "32"))
va, ga = configs.vit_arch("vit_base_patch16_224"), configs.gpt2_arch("gpt2")
sd = weights.synthetic_state_dict(1, va, ga)
enc = HipViTEncoder(sd, va, "bf16", dev)
pre = HipPrefix(sd, ga.n_embd, device=dev)
dec = HipGPT2Decoder(sd, ga, "bf16", dev)
video = torch.from_numpy(prng.imagenet_frames(1000, (16, 16, 3, 224, 224))).to(dev)
prefix = torch.randn(B, 4, 768, device=dev) * 0.1
lib = N.lib()
ncu = torch.cuda.get_device_properties(dev).multi_processor_count


def masked(lo, hi):
    words = (ncu + 31) // 32
    m = (C.c_uint32 * words)()
    for c in range(lo, hi):
        m[c // 32] |= 1 << (c % 32)
    h = C.c_void_p()
    N.check(lib.vcap_stream_create_cu_mask(m, words, C.byref(h)), "stream")
    return torch.cuda.ExternalStream(h.value, device=dev)


s_dec = masked(ncu - R, ncu) if R < ncu else torch.cuda.Stream(dev)
s_bg = masked(0, ncu - R) if R < ncu else torch.cuda.Stream(dev)
bg_cus = ncu - R if R < ncu else ncu


def step_us(cap):
    res = {}
    with torch.cuda.stream(s_dec):
        for mx in (1, 24):
            cfg = GenConfig(mx, 8, 3, 1.1, 50256, 50256, True, cap)
            for _ in range(2):
                dec.generate_ids(prefix, [50256], cfg)
            s_dec.synchronize()
            t = time.perf_counter()
            for _ in range(4):
                dec.generate_ids(prefix, [50256], cfg)
            s_dec.synchronize()
            res[mx] = (time.perf_counter() - t) / 4
    return (res[24] - res[1]) / 23 * 1e6


g = torch.Generator(device=dev).manual_seed(0)
K1 = 16384
A1 = (torch.rand(bg_cus * 256, K1, generator=g, device=dev) - 0.5).to(torch.bfloat16)
W1 = (torch.rand(256, K1, generator=g, device=dev) - 0.5).to(torch.bfloat16)
C1 = torch.empty(bg_cus * 256, 256, device=dev, dtype=torch.bfloat16)
A2 = (torch.rand(50432, 768, generator=g, device=dev) - 0.5).to(torch.bfloat16)
W2 = (torch.rand(3072, 768, generator=g, device=dev) - 0.5).to(torch.bfloat16)
b2 = torch.zeros(3072, device=dev)
C2 = torch.empty(50432, 3072, device=dev, dtype=torch.bfloat16)
src = torch.empty(1 << 28, device=dev)
dst = torch.empty_like(src)


def gemm(A, W, Cm, bias, act):
    M, K = A.shape
    n = W.shape[0]
    N.check(lib.vcap_gemm(N.DT_BF16, N.DT_BF16, A.data_ptr(), K, W.data_ptr(), K, Cm.data_ptr(), n, M, n, K,
                          bias.data_ptr() if bias is not None else None, act, None, 0, 0, 0, 0, 0, 0,
                          s_bg.cuda_stream), "gemm")


loads = {
    "gemm_1round": lambda: gemm(A1, W1, C1, None, 0),
    "gemm_fc1": lambda: gemm(A2, W2, C2, b2, 1),
    "copy": lambda: dst.copy_(src),
    "encode": lambda: enc.encode(video, pre),
}
lib.vcap_set_gemm_policy(2)
for cap in [int(c) for c in os.environ.get("CAPS", "32,96").split(",")]:
    print(f"R={R} B={B} cap={cap}: alone {step_us(cap):7.1f} us/step", flush=True)
    for name, fn in loads.items():
        stop = False

        def loop(fn=fn):
            with torch.cuda.stream(s_bg):
                while not stop:
                    for _ in range(4):
                        fn()
                    s_bg.synchronize()
        th = threading.Thread(target=loop)
        th.start()
        time.sleep(0.1)
        # background rate while the decode runs
        us = step_us(cap)
        stop = True
        th.join()
        torch.cuda.synchronize()
        print(f"   beside {name:12s} {us:7.1f} us/step", flush=True)
lib.vcap_set_gemm_policy(0)
