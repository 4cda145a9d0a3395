"""Fused QKV projection + attention (vcap_vit_qkv_attention) against the unfused pair (vcap_gemm with
bias into a qkv buffer, then vcap_vit_attention) at the ViT-B/16 frame shape: bit-identity of the
outputs (all rows, and the class-token-only form) and the median time per launch of each.
Environment: BT (frames, default 256 = one 16-video encode), NT / H (tokens / heads: 197 / 12 = ViT-B/16,
257 / 16 = ViT-L/14), REPS."""
import os
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "video-caption-algorithm_amd"))
import torch  # noqa: E402

from vcap import _native as N  # noqa: E402

BT, NT, H = int(os.environ.get("BT", "256")), int(os.environ.get("NT", "197")), int(os.environ.get("H", "12"))
D = H * 64
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
xn = torch.randn(BT * NT, D, generator=g, device=dev).to(torch.bfloat16)
w = (0.02 * torch.randn(3 * D, D, generator=g, device=dev)).to(torch.bfloat16)
b = 0.02 * torch.randn(3 * D, generator=g, device=dev)
qkv = torch.empty(BT * NT, 3 * D, device=dev, dtype=torch.bfloat16)
ref = torch.empty(BT * NT, D, device=dev, dtype=torch.bfloat16)
out = torch.empty(BT * NT, D, device=dev, dtype=torch.bfloat16)
s = torch.cuda.current_stream().cuda_stream
lib = N.lib()


def unfused(cls_only=0):
    N.check(lib.vcap_gemm(N.DT_BF16, N.DT_BF16, xn.data_ptr(), D, w.data_ptr(), D, qkv.data_ptr(), 3 * D, BT * NT,
                          3 * D, D, b.data_ptr(), 0, None, 0, 0, 0, 0, 0, 0, s), "qkv gemm")
    if cls_only:
        N.check(lib.vcap_vit_attention(N.DT_BF16, qkv.data_ptr(), ref.data_ptr(), BT, NT, H, s), "attn")
    else:
        N.check(lib.vcap_vit_attention(N.DT_BF16, qkv.data_ptr(), ref.data_ptr(), BT, NT, H, s), "attn")


def fused(cls_only=0):
    N.check(lib.vcap_vit_qkv_attention(xn.data_ptr(), w.data_ptr(), b.data_ptr(), out.data_ptr(), BT, NT, H,
                                       cls_only, s), "qkv_attention")


unfused()
fused()
torch.cuda.synchronize()
same = torch.equal(out.view(torch.int16), ref.view(torch.int16))
diff = (out.float() - ref.float()).abs()
print(f"all rows: bit-identical {same}  max |diff| {float(diff.max()):.3e}  rows differing "
      f"{int((diff.amax(1) > 0).sum())} of {BT * NT}", flush=True)
fused(1)
torch.cuda.synchronize()
cls_ref = ref.view(BT, NT, D)[:, 0]
same_cls = torch.equal(out[:BT].view(torch.int16), cls_ref.contiguous().view(torch.int16))
print(f"class-token rows: bit-identical {same_cls}", flush=True)


def timed(fn, reps):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            fn()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) / 10 * 1e3)
    return statistics.median(ts)


reps = int(os.environ.get("REPS", "7"))
tg = timed(lambda: lib.vcap_gemm(N.DT_BF16, N.DT_BF16, xn.data_ptr(), D, w.data_ptr(), D, qkv.data_ptr(), 3 * D,
                                 BT * NT, 3 * D, D, b.data_ptr(), 0, None, 0, 0, 0, 0, 0, 0, s), reps)
ta = timed(lambda: lib.vcap_vit_attention(N.DT_BF16, qkv.data_ptr(), ref.data_ptr(), BT, NT, H, s), reps)
tf = timed(fused, reps)
fl_g = 2.0 * BT * NT * D * 3 * D
fl_a = 4.0 * BT * H * NT * NT * 64
print(f"BT={BT}: qkv gemm {tg:.1f} us + attention {ta:.1f} us = {tg + ta:.1f} us | fused {tf:.1f} us "
      f"({(tg + ta) / tf:.3f}x)  fused {(fl_g + fl_a) / tf / 1e6:.0f} TF/s = {(fl_g + fl_a) / tf / 1e6 / 2500:.3f} "
      f"of the bf16 dense peak", flush=True)
