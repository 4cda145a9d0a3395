// Tiled MFMA GEMM for the ViT hot loop (patch-embed, QKV, attn-proj, fc1, fc2) and the
// prefix mapper:  C[M,N] = epilogue( A[M,K] . W[N,K]^T ).
//
// Replaces the reference's Linear layers inside timm Block/Attention/Mlp
// (src/models/video_encoder.py:162-172 patched forward; GELU forced to tanh at :123-134)
// and the CuPy `linear_bias_f32/_f16` kernels (core/operators/cupy_linear_mapper.py:14-70):
// W keeps torch Linear's [out, in] row-major layout, so both operands are K-contiguous.
//
// Tile 128x128, 256 threads = 4 waves in 2x2, each wave 64x64 = 4x4 MFMA 16x16 tiles.
// K step = 128 bytes per row (64 bf16 or 32 f32).  Operands stream global->LDS with
// global_load_lds_dwordx4 (1 KiB per wave instruction, lane-linear LDS image); the
// st_8x16B XOR swizzle (chunk ^ (row & 7)) is applied on the global SOURCE address and on
// the ds_read address, making the ds_read_b128 fragment reads conflict-free.
// bf16 uses mfma_f32_16x16x32_bf16; the fp32 parity mode uses mfma_f32_16x16x4f32 with the
// SAME byte layout (one 16-byte chunk = 4 f32 = one group of four 16x16x4 MFMAs).
#include "vcap_common.h"
#include "vcap_kernels.h"

namespace {

constexpr int BM = 128, BN = 128, ROWB = 128;  // ROWB: bytes of K per tile row
constexpr int TILE_BYTES = BM * ROWB;          // 16 KiB per operand per stage
constexpr int STAGE_BYTES = 2 * TILE_BYTES;

VCAP_DEV void glds16(const void* g, char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
}

template <typename T>
VCAP_DEV void stage_tile(const T* __restrict__ P, long ld, int row0, int rows, int k0, char* lds_tile,
                         int wave, int lane) {
  constexpr int E = Frag<T>::kElems;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int rb = wave * 4 + i;              // 8-row block written by this wave instruction
    const int r = rb * 8 + (lane >> 3);
    const int s = lane & 7;                   // LDS slot within the 128-byte row
    const int c = s ^ (r & 7);                // global chunk stored in that slot
    int gr = row0 + r;
    gr = gr < rows ? gr : rows - 1;
    const T* src = P + (long)gr * ld + k0 + c * E;
    glds16(src, lds_tile + rb * 1024);
  }
}

VCAP_DEV u32x4 lds_frag(const char* tile, int row, int chunk) {
  return *reinterpret_cast<const u32x4*>(tile + row * ROWB + ((chunk ^ (row & 7)) << 4));
}

}  // namespace

// EPI (compile time, so each ViT GEMM role is its own kernel symbol in a profile):
//   0 bias (QKV)   1 bias+gelu_tanh (fc1)   2 bias+residual in place (attn-proj, fc2)
//   3 general: runtime act / residual mode / row remap (patch-embed, vcap_gemm ABI)
template <typename TIn, typename TOut, int EPI>
__global__ __launch_bounds__(256) void vcap_gemm_kernel(const TIn* __restrict__ A, long lda,
                                                        const TIn* __restrict__ W, long ldw,
                                                        TOut* C, long ldc, int M, int N, int K, GemmEpi epi) {
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE_BYTES];
  constexpr int E = Frag<TIn>::kElems;
  constexpr int BK = ROWB / sizeof(TIn);

  const int tiles_n = (N + BN - 1) / BN;
  const int tiles_m = (M + BM - 1) / BM;
  const int nwg = tiles_m * tiles_n;
  // XCD-aware bijective remap: blocks b, b+8, ... share an XCD; give each XCD a contiguous run
  // of tile ids so its L2 sees the same A row-panel across consecutive N tiles.
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q = nwg >> 3, r8 = nwg & 7;
  const int wgid = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + (bid >> 3);
  const int tm = wgid / tiles_n, tn = wgid % tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // split-K (gridDim.y > 1): this workgroup sums K-tiles [kt0, kt0 + nk) and stores its partial
  // tile into slab blockIdx.y of epi.splitk_ws; vcap_splitk_reduce_kernel adds the slabs in split
  // order (deterministic: the same sum on every run and on every stream's CU mask)
  const int nk = K / BK / (int)gridDim.y;
  const int kt0 = (int)blockIdx.y * nk;
  const bool split = gridDim.y > 1;
  stage_tile(A, lda, m0, M, kt0 * BK, smem, wave, lane);
  stage_tile(W, ldw, n0, N, kt0 * BK, smem + TILE_BYTES, wave, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  const int fr = lane & 15, fg = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    char* cur = smem + (kt & 1) * STAGE_BYTES;
    if (kt + 1 < nk) {
      char* nxt = smem + ((kt + 1) & 1) * STAGE_BYTES;
      stage_tile(A, lda, m0, M, (kt0 + kt + 1) * BK, nxt, wave, lane);
      stage_tile(W, ldw, n0, N, (kt0 + kt + 1) * BK, nxt + TILE_BYTES, wave, lane);
    }
    const char* ta = cur;
    const char* tb = cur + TILE_BYTES;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      u32x4 af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = lds_frag(ta, wm * 64 + i * 16 + fr, s * 4 + fg);
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[j] = lds_frag(tb, wn * 64 + j * 16 + fr, s * 4 + fg);
      // weight fragment as the MFMA A operand: a lane ends up with 4 consecutive COLUMNS of
      // one row, so the epilogue stores vectors
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma_frag(bfr[j], af[i], acc[i][j], (TIn*)nullptr);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  (void)E;

  // epilogue: lane holds row fr, columns 4*fg .. 4*fg+3 of each 16x16 tile
  const bool vec = (N & 3) == 0 && (ldc & 3) == 0 && (!epi.res || (epi.ldr & 3) == 0);
  // in-place residual (EPI 2): every residual row of the wave is loaded before the first store
  // (load / add / store per element serialised 16 HBM round trips: the loads cannot pass the
  // previous store to the same pointer, and the in-order vmcnt waits for that store too)
  f32x4 rpre[4][4];
  const bool pre = EPI == 2 && vec && !split;
  if constexpr (EPI == 2) {
    if (pre) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int m = min(m0 + wm * 64 + i * 16 + fr, M - 1);
          const int nb = min(n0 + wn * 64 + j * 16 + 4 * fg, N - 4);
          rpre[i][j] = *reinterpret_cast<const f32x4*>(epi.res + (long)m * epi.ldr + nb);
        }
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int nb = n0 + wn * 64 + j * 16 + 4 * fg;
    if (nb >= N) continue;
    float bias[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) bias[e] = (epi.bias && nb + e < N && !split) ? epi.bias[nb + e] : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = m0 + wm * 64 + i * 16 + fr;
      if (m >= M) continue;
      long orow = m;
      if constexpr (EPI == 3) orow = epi.G ? (long)(m / epi.G) * epi.Gs + epi.goff + (m % epi.G) : (long)m;
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = acc[i][j][e] + bias[e];
      if (split) {  // raw partial sums (N % 4 == 0: dispatcher)
        *reinterpret_cast<f32x4*>(epi.splitk_ws + ((long)blockIdx.y * M + m) * N + nb) = (f32x4){v[0], v[1], v[2], v[3]};
        continue;
      }
      if constexpr (EPI == 1) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = gelu_tanh(v[e]);
      } else if constexpr (EPI == 3) {
        if (epi.act == 1)
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = gelu_tanh(v[e]);
      }
      const float* rr = nullptr;
      if constexpr (EPI == 2) rr = epi.res + orow * epi.ldr + nb;
      if constexpr (EPI == 3) {
        if (epi.res_mode == 1) rr = epi.res + orow * epi.ldr + nb;
        else if (epi.res_mode == 2) rr = epi.res + (long)((m % epi.G) + epi.roff) * epi.ldr + nb;
      }
      if (vec && nb + 3 < N) {
        if (pre) {
          const f32x4 r = rpre[i][j];
          v[0] += r.x; v[1] += r.y; v[2] += r.z; v[3] += r.w;
        } else if (rr) {
          const f32x4 r = *reinterpret_cast<const f32x4*>(rr);
          v[0] += r.x; v[1] += r.y; v[2] += r.z; v[3] += r.w;
        }
        if constexpr (sizeof(TOut) == 2) {
          *reinterpret_cast<u32x2*>(C + orow * ldc + nb) = (u32x2){pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3])};
        } else {
          *reinterpret_cast<f32x4*>(C + orow * ldc + nb) = (f32x4){v[0], v[1], v[2], v[3]};
        }
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          if (nb + e >= N) continue;
          C[orow * ldc + nb + e] = Num<TOut>::from_f(v[e] + (rr ? rr[e] : 0.f));
        }
      }
    }
  }
}

// C[orow(m)][n] = (sum over splits s = 0.. of ws[s][m][n] + bias[n]) + C[orow(m)][n]: the split-K
// partials of an in-place residual GEMM, summed in a fixed order.
__global__ __launch_bounds__(256) void vcap_splitk_reduce_kernel(const float* __restrict__ ws, int splits, float* C,
                                                                 long ldc, int M, int N, GemmEpi epi) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;  // f32x4 index
  const int nq = N >> 2;
  if (i >= (long)M * nq) return;
  const int m = (int)(i / nq), n = (int)(i - (long)m * nq) * 4;
  f32x4 v = *reinterpret_cast<const f32x4*>(ws + (long)m * N + n);
  for (int sp = 1; sp < splits; ++sp) v += *reinterpret_cast<const f32x4*>(ws + ((long)sp * M + m) * N + n);
  if (epi.bias) v += *reinterpret_cast<const f32x4*>(epi.bias + n);
  const long orow = epi.G ? (long)(m / epi.G) * epi.Gs + epi.goff + (m % epi.G) : (long)m;
  float* c = C + orow * ldc + n;
  *reinterpret_cast<f32x4*>(c) = v + *reinterpret_cast<const f32x4*>(c);
}

template <typename TIn, typename TOut, int EPI>
static hipError_t launch_gemm_epi(const void* A, long lda, const void* W, long ldw, void* C, long ldc, int M, int N,
                                  int K, const GemmEpi& epi, hipStream_t s) {
  const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  // Few tiles (the CLS-only last block: M = B*T rows) leave most CUs idle through a long K
  // loop: split K over several workgroups per tile when C is f32 and already holds the
  // residual (attn-proj / fc2 in place) and the caller gave a partials workspace (bf16 operands
  // only: the fp32 parity mode keeps one summation chain).  The split count depends on K alone
  // (the largest divisor c <= 8 of the K-tile count leaving >= 3 K-tiles per workgroup), never on
  // M or the stream's CU mask, so a row sums the same way whichever batch it is encoded in and a
  // CU-masked pipelined encode sums exactly like a serial one.  (No CU-count gate: a large encode
  // batch takes more rounds of split workgroups instead of switching the summation order.  The
  // encoder's partials workspace holds 16 splits of its B*T CLS rows, so the size check below
  // only refuses a caller-supplied workspace that is too small.)
  int splits = 1;
  if constexpr (sizeof(TIn) == 2 && sizeof(TOut) == 4) {
    const bool in_place = epi.bias != nullptr && epi.res == (const float*)C && epi.ldr == ldc &&
                          (EPI == 2 || (EPI == 3 && epi.res_mode == 1 && epi.act == 0)) && epi.splitk_ws &&
                          (N & 3) == 0 && (ldc & 3) == 0 && ((uintptr_t)C & 15) == 0;
    const int nkt = K / (ROWB / (int)sizeof(TIn));
    int c = 1;
    for (int d = 8; d >= 2; --d)
      if (nkt % d == 0 && nkt / d >= 3) {
        c = d;
        break;
      }
    if (in_place && c > 1 && (size_t)c * M * N * sizeof(float) <= epi.splitk_bytes)
      splits = c;
  }
  hipLaunchKernelGGL((vcap_gemm_kernel<TIn, TOut, EPI>), dim3(tiles, splits), dim3(256), 0, s, (const TIn*)A, lda,
                     (const TIn*)W, ldw, (TOut*)C, ldc, M, N, K, epi);
  if (splits > 1) {
    if (hipError_t e = hipGetLastError()) return e;
    const long nvec = (long)M * (N / 4);
    hipLaunchKernelGGL(vcap_splitk_reduce_kernel, dim3((unsigned)((nvec + 255) / 256)), dim3(256), 0, s,
                       (const float*)epi.splitk_ws, splits, (float*)C, ldc, M, N, epi);
  }
  return hipGetLastError();
}

template <typename TIn, typename TOut>
static hipError_t launch_gemm(const void* A, long lda, const void* W, long ldw, void* C, long ldc, int M, int N,
                              int K, const GemmEpi& epi, hipStream_t s) {
  const bool plain_rows = epi.G == 0;
  if (plain_rows && epi.res_mode == 0 && epi.act == 0)
    return launch_gemm_epi<TIn, TOut, 0>(A, lda, W, ldw, C, ldc, M, N, K, epi, s);
  if constexpr (sizeof(TOut) == sizeof(TIn)) {
    if (plain_rows && epi.res_mode == 0 && epi.act == 1)
      return launch_gemm_epi<TIn, TOut, 1>(A, lda, W, ldw, C, ldc, M, N, K, epi, s);
  }
  if constexpr (sizeof(TOut) == 4) {
    if (plain_rows && epi.res_mode == 1 && epi.act == 0 && epi.res == (const float*)C && epi.ldr == ldc)
      return launch_gemm_epi<TIn, TOut, 2>(A, lda, W, ldw, C, ldc, M, N, K, epi, s);
  }
  return launch_gemm_epi<TIn, TOut, 3>(A, lda, W, ldw, C, ldc, M, N, K, epi, s);
}

static int g_gemm_policy = 0;  // 0 auto, 1 always the 128x128 kernel, 2 the 256x256 kernel where it applies
void vcap_gemm_set_policy(int p) { g_gemm_policy = p; }

int vcap_device_cus() {
  int dev = 0, ncu = 256;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  return ncu;
}

// CUs the stream's kernels may use (hipExtStreamGetCUMask; the encode stream of the overlapped
// pipeline is CU-masked), so the round arithmetic below matches what the stream really gets.
int vcap_stream_cus(hipStream_t s) {
  int dev = 0, ncu = 256;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  uint32_t mask[16] = {0};
  if (hipExtStreamGetCUMask(s, 16, mask) != hipSuccess) return ncu;
  int n = 0;
  for (int i = 0; i < 16; ++i) n += __builtin_popcount(mask[i]);
  return n > 0 && n < ncu ? n : ncu;
}

// in_dt: operand dtype; out_dt: C dtype (the residual stream is f32)
hipError_t vcap_gemm_dispatch(int in_dt, int out_dt, const void* A, long lda, const void* W, long ldw, void* C,
                              long ldc, int M, int N, int K, const GemmEpi& epi, hipStream_t s) {
  if (in_dt == VCAP_DT_MXFP8) {  // block-scaled fp8: the 256x256 kernel only
    if (!vcap_gemm256_ok(in_dt, out_dt, lda, ldw, ldc, M, N, K, epi)) return hipErrorInvalidValue;
    return vcap_gemm256_dispatch(in_dt, out_dt, A, lda, W, ldw, C, ldc, M, N, K, epi, s);
  }
  if (g_gemm_policy != 1 && vcap_gemm256_ok(in_dt, out_dt, lda, ldw, ldc, M, N, K, epi)) {
    // 256x256 tiles run one workgroup per CU: they need enough tiles to fill the chip, and a
    // last round that is mostly empty costs a whole tile time.  Rows of the full rounds go to
    // the 256x256 kernel, a small remainder to the 128x128 kernel (2 per CU, one short round).
    const int tn = (N + 255) / 256;
    const long tiles256 = (long)((M + 255) / 256) * tn;
    if (g_gemm_policy == 2) return vcap_gemm256_dispatch(in_dt, out_dt, A, lda, W, ldw, C, ldc, M, N, K, epi, s);
    const int ncu = vcap_stream_cus(s);
    if (tiles256 >= ncu) {
      const long rounds = tiles256 / ncu;
      const long rem = tiles256 - rounds * ncu;
      const bool plain = epi.G == 0 && (epi.res_mode == 0 || epi.res == (const float*)C);
      const int m_full = (int)((rounds * ncu / tn) * 256);  // rows covered by whole 256-tile rounds
      if (plain && rem > 0 && rem * 4 < ncu && m_full > 0 && m_full < M) {
        if (hipError_t e = vcap_gemm256_dispatch(in_dt, out_dt, A, lda, W, ldw, C, ldc, m_full, N, K, epi, s))
          return e;
        const size_t ein = in_dt == VCAP_DT_BF16 ? 2 : 4, eout = out_dt == VCAP_DT_BF16 ? 2 : 4;
        GemmEpi e2 = epi;
        if (epi.res) e2.res = epi.res + (long)m_full * epi.ldr;
        const void* A2 = (const char*)A + (size_t)m_full * lda * ein;
        void* C2 = (char*)C + (size_t)m_full * ldc * eout;
        if (in_dt == VCAP_DT_BF16 && out_dt == VCAP_DT_BF16)
          return launch_gemm<bf16_t, bf16_t>(A2, lda, W, ldw, C2, ldc, M - m_full, N, K, e2, s);
        if (in_dt == VCAP_DT_BF16 && out_dt == VCAP_DT_F32)
          return launch_gemm<bf16_t, float>(A2, lda, W, ldw, C2, ldc, M - m_full, N, K, e2, s);
        return launch_gemm<float, float>(A2, lda, W, ldw, C2, ldc, M - m_full, N, K, e2, s);
      }
      return vcap_gemm256_dispatch(in_dt, out_dt, A, lda, W, ldw, C, ldc, M, N, K, epi, s);
    }
  }
  if (in_dt == VCAP_DT_BF16 && out_dt == VCAP_DT_BF16)
    return launch_gemm<bf16_t, bf16_t>(A, lda, W, ldw, C, ldc, M, N, K, epi, s);
  if (in_dt == VCAP_DT_BF16 && out_dt == VCAP_DT_F32)
    return launch_gemm<bf16_t, float>(A, lda, W, ldw, C, ldc, M, N, K, epi, s);
  if (in_dt == VCAP_DT_F32 && out_dt == VCAP_DT_F32)
    return launch_gemm<float, float>(A, lda, W, ldw, C, ldc, M, N, K, epi, s);
  return hipErrorInvalidValue;
}

int vcap_gemm_k_align(int in_dt) { return in_dt == VCAP_DT_MXFP8 ? 256 : in_dt == VCAP_DT_BF16 ? 64 : 32; }
