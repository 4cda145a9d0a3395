"""ViT attention at the benchmark shape (B*T = 128 frames, 197 tokens, 12 heads, bf16) through
vcap_vit_attention: median kernel time over rounds and achieved TFLOP/s (4*BT*H*N^2*64)."""
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "video-caption-algorithm_amd"))
import torch  # noqa: E402

from vcap import _native as N  # noqa: E402

import os
BT, NT, H = int(os.environ.get("BT", "128")), 197, 12
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
qkv = torch.randn(BT * NT, 3 * H * 64, generator=g, device=dev).to(torch.bfloat16)
out = torch.empty(BT * NT, H * 64, device=dev, dtype=torch.bfloat16)
s = torch.cuda.current_stream().cuda_stream
lib = N.lib()
for _ in range(5):
    N.check(lib.vcap_vit_attention(N.DT_BF16, qkv.data_ptr(), out.data_ptr(), BT, NT, H, s), "attn")
ts = []
for _ in range(7):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        lib.vcap_vit_attention(N.DT_BF16, qkv.data_ptr(), out.data_ptr(), BT, NT, H, s)
    e1.record()
    e1.synchronize()
    ts.append(e0.elapsed_time(e1) / 20)
ms = statistics.median(ts)
fl = 4.0 * BT * H * NT * NT * 64
print(f"attention BT={BT} N={NT} H={H}: {ms * 1e3:.1f} us  {fl / ms / 1e9:.1f} TF", flush=True)
q, k, v = qkv.float().view(BT, NT, 3, H, 64).permute(2, 0, 3, 1, 4)
ref = torch.nn.functional.scaled_dot_product_attention(q, k, v).permute(0, 2, 1, 3).reshape(BT * NT, H * 64)
err = (out.float() - ref).abs()
print(f"max |out - fp32 SDPA| {float(err.max()):.3e}  mean {float(err.mean()):.3e}  "
      f"variant {os.environ.get('VCAP_ATTN_VARIANT', 'shipped')}", flush=True)
if os.environ.get("DUMP"):
    torch.save(out.cpu(), os.environ["DUMP"])
