"""Diagnostic build of libvcap_hip.so whose decode kernels stamp the 100 MHz real-time clock
(s_memrealtime) at fixed points: workgroup entry, activation operand ready (after the LayerNorm /
A-fragment barrier), MFMAs retired (split-K partials written), reduction barrier passed, epilogue
issued.  The product sources are not touched: this script patches a copy under /tmp and builds
video-caption-algorithm_amd/vcap/_lib/libvcap_stamps.so (use it with VCAP_LIB=..., read with
tools/decode_stamps.py).  Stamps go to a __device__ buffer that nothing else reads.
"""
import os
import re
import shutil
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
SRC = ROOT / "video-caption-algorithm_amd" / "csrc"
OUT = ROOT / "video-caption-algorithm_amd" / "vcap" / "_lib" / "libvcap_stamps.so"

HEADER_T = r'''
__device__ unsigned long long g_vcap_stamps[8 << 18];
__device__ unsigned int g_vcap_stamp_n;
#ifndef VCAP_RT
#define VCAP_RT() ({ asm volatile("" ::: "memory"); unsigned long long _t = __builtin_amdgcn_s_memrealtime(); asm volatile("" ::: "memory"); _t; })
#endif
__device__ __forceinline__ void vcap_stamp_rec(unsigned long long tag, unsigned long long t0, unsigned long long t1,
                                               unsigned long long t2, unsigned long long t3, unsigned long long t4,
                                               unsigned long long t5 = 0) {
  const unsigned i = atomicAdd(&g_vcap_stamp_n, 1u);
  if (i < (1u << 18)) {
    unsigned long long* r = g_vcap_stamps + 8ull * i;
    r[0] = tag; r[1] = blockIdx.x | ((unsigned long long)gridDim.x << 20) | ((unsigned long long)blockIdx.y << 40);
    r[2] = t0; r[3] = t1; r[4] = t2; r[5] = t3; r[6] = t4; r[7] = t5;
  }
}
extern "C" __attribute__((visibility("default"))) int vcap_diag_stamps(void* host, int max_rec) {
  unsigned n = 0;
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(&n, HIP_SYMBOL(g_vcap_stamp_n), sizeof(n)) != hipSuccess) return -1;
  if (n > (1u << 18)) n = 1u << 18;
  if (host && max_rec > 0) {
    const unsigned k = n < (unsigned)max_rec ? n : (unsigned)max_rec;
    if (hipMemcpyFromSymbol(host, HIP_SYMBOL(g_vcap_stamps), 64ull * k) != hipSuccess) return -1;
  }
  const unsigned z = 0;
  if (hipMemcpyToSymbol(HIP_SYMBOL(g_vcap_stamp_n), &z, sizeof(z)) != hipSuccess) return -1;
  return (int)n;
}
'''


def header(sfx: str) -> str:
    # one buffer + reader per translation unit (device globals are per code object)
    return (HEADER_T.replace("g_vcap_stamps", "g_vcap_stamps" + sfx).replace("g_vcap_stamp_n", "g_vcap_stamp_n" + sfx)
            .replace("vcap_stamp_rec", "vcap_stamp_rec" + sfx).replace("vcap_diag_stamps", "vcap_diag_stamps" + sfx))


def patch_decode(s: str) -> str:
    s = s.replace('#include "vcap_kernels.h"\n', '#include "vcap_kernels.h"\n' + header(""), 1)
    # GEMV kernel: entry | activation landed (PRO_LN: LayerNorm tile written + barrier; PRO_DIRECT: the
    # last A fragment's load waited for) | weight stream landed (the last weight fragment waited for:
    # loads retire in issue order) | MFMAs retired (partials in LDS) | reduction barrier | epilogue issued
    k0 = s.index("__global__ __launch_bounds__(256) void vcap_rows_gemv_kernel(RowsGemmArgs a) {")
    k1 = s.index("// Residual GEMV (PRO_DIRECT + EPI_RESID", k0)
    body = s[k0:k1]
    body = body.replace("  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;\n",
                        "  const unsigned long long t0 = VCAP_RT();\n  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;\n", 1)
    body = body.replace("  if constexpr (PRO == PRO_LN || EPI == EPI_LOGITS) __syncthreads();\n",
                        "  if constexpr (PRO == PRO_LN || EPI == EPI_LOGITS) __syncthreads();\n"
                        "  if constexpr (PRO == PRO_DIRECT) asm volatile(\"\" :: \"v\"(af[MTA - 1][NSL - 1].x));\n"
                        "  const unsigned long long t1 = VCAP_RT();\n"
                        "  asm volatile(\"\" :: \"v\"(wf[NSL - 1][NTB - 1].x));\n"
                        "  const unsigned long long tw = VCAP_RT();\n", 1)
    body = body.replace("  if constexpr (EPI == EPI_LOGITS) toks.template mark<NTB>(a, m0, n0, s_rep, s_ban);\n  __syncthreads();\n",
                        "  const unsigned long long t2 = VCAP_RT();\n  if constexpr (EPI == EPI_LOGITS) toks.template mark<NTB>(a, m0, n0, s_rep, s_ban);\n  __syncthreads();\n  const unsigned long long t3 = VCAP_RT();\n", 1)
    body = body.replace("  rows_epilogue<T, MT, NTB, EPI>(a, m0, red, pre_bias, pre_res, lg, s_rep, s_ban, n0, hsel);\n}",
                        "  rows_epilogue<T, MT, NTB, EPI>(a, m0, red, pre_bias, pre_res, lg, s_rep, s_ban, n0, hsel);\n"
                        "  if (threadIdx.x == 0) vcap_stamp_rec((unsigned long long)((NSL << 12) | (EPI << 8) | (PRO << 4) | NTB) | ((unsigned long long)MT << 20) | ((unsigned long long)(hsel >= 0) << 24), t0, t1, tw, t2, t3, VCAP_RT());\n}", 1)
    assert body.count("VCAP_RT()") == 6, body.count("VCAP_RT()")
    s = s[:k0] + body + s[k1:]
    # decode attention (c64): entry | every load landed | output stored (issued)
    a0 = s.index("void vcap_decode_attention_c64_kernel(")
    a1 = s.index("__global__ __launch_bounds__(64) void vcap_decode_attention_c64f_kernel", a0)
    att = s[a0:a1]
    att = att.replace("  __shared__ float s_p[64];\n", "  __shared__ float s_p[64];\n  const unsigned long long t0 = VCAP_RT();\n", 1)
    att = att.replace("  c64_issue(L, q, kc, vc, maxp, m, h, H, seq, ctx);\n",
                      "  c64_issue(L, q, kc, vc, maxp, m, h, H, seq, ctx);\n  asm volatile(\"\" :: \"v\"(L.vv[7].x));\n"
                      "  const unsigned long long t1 = VCAP_RT();\n", 1)
    att = att[:att.rindex("}")] + "  if (threadIdx.x == 0) vcap_stamp_rec(0xA000ull, t0, t1, t1, t1, t1, VCAP_RT());\n}\n\n"
    assert att.count("VCAP_RT()") == 3, att.count("VCAP_RT()")
    s = s[:a0] + att + s[a1:]
    # lm_head stream kernel (greedy / screen): entry | ln_f tile in LDS (+ flags) | first column group
    # done | second group done | last group done | argmax partials written  (tag 0xC000)
    l0 = s.index("__global__ __launch_bounds__(256) void vcap_lm_head_stream_kernel(RowsGemmArgs a, int tpw) {")
    l1 = s.index("template <typename T, int NSL>\nstatic bool launch_lm_stream", l0)
    lm = s[l0:l1]
    lm = lm.replace("  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;\n",
                    "  const unsigned long long st0 = VCAP_RT();\n  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;\n", 1)
    lm = lm.replace("  __syncthreads();  // flags zeroed, A tile written\n",
                    "  __syncthreads();  // flags zeroed, A tile written\n  const unsigned long long st1 = VCAP_RT();\n"
                    "  unsigned long long st2 = 0, st3 = 0;\n", 1)
    lm = lm.replace("    group(wA, gi);\n", "    group(wA, gi);\n    if (gi == 0) st2 = VCAP_RT();\n", 1)
    lm = lm.replace("      group(wB, gi + 1);\n", "      group(wB, gi + 1);\n      if (gi == 0) st3 = VCAP_RT();\n", 1)
    lm = lm.replace("  argmax_take(bv_run, bi_run, dpp_f<DPP_XOR1>(bv_run), dpp_i<DPP_XOR1>(bi_run));\n",
                    "  const unsigned long long st4 = VCAP_RT();\n  argmax_take(bv_run, bi_run, dpp_f<DPP_XOR1>(bv_run), dpp_i<DPP_XOR1>(bi_run));\n", 1)
    lm = lm[:lm.rindex("}")] + "  if (threadIdx.x == 0) vcap_stamp_rec(0xC000ull, st0, st1, st2, st3 ? st3 : st2, st4, VCAP_RT());\n}\n\n"
    assert lm.count("VCAP_RT()") == 6, lm.count("VCAP_RT()")
    s = s[:l0] + lm + s[l1:]
    return s


def patch_attention(s: str) -> str:
    s = s.replace('#include "vcap_kernels.h"\n', '#include "vcap_kernels.h"\n' + header("_attn"), 1)
    k0 = s.index("void vcap_vit_attention_bf16_kernel(")
    ends = [s.find(m, k0) for m in ("// Persistent walk over", "template <int KT, int KE, int WAVES, bool MXO>\nstatic hipError_t launch_attn_bf16")]
    k1 = min(e for e in ends if e > 0)
    b = s[k0:k1]
    b = b.replace("  const int fr = lane & 15, fg = lane >> 4;\n", "  const int fr = lane & 15, fg = lane >> 4;\n  const unsigned long long t0 = VCAP_RT();\n", 1)
    b = b.replace('  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");\n  __syncthreads();\n',
                  '  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");\n  __syncthreads();\n  const unsigned long long t1 = VCAP_RT();\n', 1)
    b = b[:b.rindex("}")] + "  __syncthreads();\n  if (threadIdx.x == 0) vcap_stamp_rec_attn(0xB000ull | KT, t0, t1, VCAP_RT(), 0, 0, 0);\n}\n\n"
    assert b.count("VCAP_RT()") == 3
    return s[:k0] + b + s[k1:]


def main():
    tmp = Path("/tmp/vcap_stamps_build")
    shutil.rmtree(tmp, ignore_errors=True)
    src = tmp / "pkg" / "csrc"  # runtime.hip includes ../../include/vcap.h
    src.mkdir(parents=True)
    (tmp / "obj").mkdir()
    shutil.copytree(ROOT / "include", tmp / "include")
    for f in SRC.iterdir():
        shutil.copy(f, src / f.name)
    p = src / "decode.hip"
    p.write_text(patch_decode(p.read_text()))
    p = src / "vit_attention.hip"
    p.write_text(patch_attention(p.read_text()))
    flags = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-munsafe-fp-atomics", "-Wno-unused-result",
             f"-I{src}", f"-I{ROOT / 'include'}"]
    procs = []
    for f in sorted(src.glob("*.hip")):
        extra = ["-fno-honor-nans"] if f.name == "vit_attention.hip" else []
        procs.append(subprocess.Popen(["/opt/rocm/bin/hipcc", *flags, *extra, "-c", str(f), "-o",
                                       str(tmp / "obj" / (f.stem + ".o"))]))
    if any(p.wait() for p in procs):
        sys.exit("compile failed")
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", str(OUT),
                           *map(str, sorted((tmp / "obj").glob("*.o")))])
    print(OUT)


if __name__ == "__main__":
    main()
