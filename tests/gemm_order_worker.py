"""Child process of test_gpu_gemm_order.py: one fc1-shaped GEMM (bias + GELU, bf16 out) through
vcap_gemm on seeded operands, the output's sha256 printed.  The parent sets VCAP_GEMM_COLGROUP
(read once per process by the 256x256 kernel's dispatcher) differently for each child."""
import hashlib
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "video-caption-algorithm_amd"))

import torch  # noqa: E402

from vcap import _native as N  # noqa: E402


def main():
    M, n, k = int(sys.argv[1]), 3072, 768
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(5)
    A = ((torch.rand(M, k, generator=g, device=dev) * 2 - 1)).to(torch.bfloat16)
    W = ((torch.rand(n, k, generator=g, device=dev) * 2 - 1) * 0.05).to(torch.bfloat16)
    b = (torch.rand(n, generator=g, device=dev) * 0.2 - 0.1).float()
    C = torch.zeros(M, n, device=dev, dtype=torch.bfloat16)
    lib = N.lib()
    lib.vcap_set_gemm_policy(2)   # the 256x256 kernel for every row (no 128x128 remainder split)
    s = torch.cuda.current_stream().cuda_stream
    N.check(lib.vcap_gemm(N.DT_BF16, N.DT_BF16, A.data_ptr(), k, W.data_ptr(), k, C.data_ptr(), n, M, n, k,
                          b.data_ptr(), 1, None, 0, 0, 0, 0, 0, 0, s), "gemm")
    torch.cuda.synchronize()
    print(hashlib.sha256(C.view(torch.int16).cpu().numpy().tobytes()).hexdigest(), flush=True)


if __name__ == "__main__":
    main()
