"""ViT LayerNorm launches alone (vcap_layernorm, f32 rows -> bf16 with gamma / beta, and
vcap_layernorm_mx -> MXFP8): 50432 x 768 (16 ViT-B/16 videos) and 65792 x 1024 (8 ViT-L/14 videos
of 32 frames).  Prints us per launch and GB/s of algorithmic bytes (x read once, y written once);
with an output path, saves the outputs for a bit-exactness A/B of two builds
(`python tools/gemm_dump.py --compare a.pt b.pt` reads the file)."""
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "video-caption-algorithm_amd"))
import torch  # noqa: E402

from vcap import _native as N  # noqa: E402

dev = torch.device("cuda:0")
lib = N.lib()
s = torch.cuda.current_stream().cuda_stream
g = torch.Generator(device=dev).manual_seed(0)
out = {}
for rows, D in ((50432, 768), (65792, 1024), (1000, 640)):
    x = torch.randn(rows, D, generator=g, device=dev) * 3 + 1
    gm = torch.rand(D, generator=g, device=dev) + 0.5
    bt = torch.randn(D, generator=g, device=dev) * 0.1
    y = torch.empty(rows, D, dtype=torch.bfloat16, device=dev)
    q = torch.empty(rows, D, dtype=torch.uint8, device=dev)
    sc = torch.zeros(int(lib.vcap_mx_scale_bytes(rows, D)) if D % 256 == 0 else 1, dtype=torch.uint8, device=dev)

    def ln():
        N.check(lib.vcap_layernorm(N.DT_BF16, x.data_ptr(), D, y.data_ptr(), D, gm.data_ptr(), bt.data_ptr(), rows, D,
                                   1e-6, s), "ln")

    def lnmx():
        N.check(lib.vcap_layernorm_mx(x.data_ptr(), D, q.data_ptr(), sc.data_ptr(), gm.data_ptr(), bt.data_ptr(),
                                      rows, D, 1e-6, s), "ln_mx")

    fns = {"ln_bf16": (ln, rows * D * 6)}
    if D % 256 == 0:
        fns["ln_mx"] = (lnmx, rows * D * 5 + rows * D // 32)
    for name, (fn, nbytes) in fns.items():
        for _ in range(3):
            fn()
        ts = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                fn()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) / 20 * 1e3)
        t = statistics.median(ts)
        print(f"{name:8s} {rows} x {D}: {t:7.2f} us  {nbytes / t / 1e3:7.0f} GB/s", flush=True)
    torch.cuda.synchronize()
    out[f"y{rows}"] = y.cpu()
    if D % 256 == 0:
        out[f"q{rows}"] = q.cpu()
        out[f"s{rows}"] = sc.cpu()
if len(sys.argv) > 1:
    torch.save(out, sys.argv[1])
