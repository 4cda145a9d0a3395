// 256x256-tile MFMA GEMM for the ViT projections (QKV, attn-proj, fc1, fc2, patch-embed):
//   C[M,N] = epilogue( A[M,K] . W[N,K]^T )     (torch Linear layout, both operands K-contiguous)
// Replaces the timm Linear layers the reference drives (src/models/video_encoder.py:162-172).
//
// Structure (CDNA4 8-phase software pipeline, one workgroup of 8 waves per CU):
//  * tile 256x256, K step 64 bf16 (128 B per row), waves 2 (M) x 4 (N), 128x64 outputs per wave
//    held as four 64x32 quadrants of 16x16 MFMA accumulators;
//  * LDS (128 KiB, one dynamic array) = 2 K-tile buffers x {A-h0, A-h1, B-h0, B-h1}; a "half"
//    holds the 128 rows that feed one quadrant row / column of every wave:
//      A-hX local row l -> tile row (l>>6)*128 + X*64 + (l&63)
//      B-hY local row l -> tile col (l>>5)*64  + Y*32 + (l&31)
//    so each half is read in exactly ONE phase of its K-tile and can be restaged right after;
//  * per K-tile 4 phases, each = ds_read one register subtile, issue one half-tile of a future
//    K-tile (2 global_load_lds_dwordx4 per thread), barrier, 16 MFMAs on one quadrant, barrier:
//        phase 1: read A-h0 + B-h0 -> quadrant (0,0)     phase 2: read B-h1 -> (0,1)
//        phase 3: read A-h1        -> (1,1)              phase 4: (registers only) -> (1,0)
//  * the two wave groups (wr = 0 / 1, one wave of each per SIMD) run staggered by one barrier:
//    while one group issues its MFMAs the other issues its ds_reads and LDS-DMA.  Each phase
//    retires its ds_reads (lgkmcnt(0)) before its first barrier, so a half can be restaged in
//    the phase right after its last read, and the staging order over an iteration (K-tiles t,
//    t+1; buffers even/odd) keeps 3 half-tiles in flight across every barrier:
//        p1 A-h1(t+1)  p2 A-h0(t+2)  p3 B-h0(t+2)  p4 B-h1(t+2) | vmcnt(6): t+1 landed
//        p5 A-h1(t+2)  p6 A-h0(t+3)  p7 B-h0(t+3)  p8 B-h1(t+3) | vmcnt(6): t+2 landed
//    a staged buffer is read only in a phase after the counted wait and the barrier that
//    follow it in both groups;
//  * the MFMA takes the weight fragment as its A operand, so each lane ends up holding 4
//    consecutive output COLUMNS of one row: vectorised bias / residual / store epilogue.
#include <cstdlib>

#include "vcap_common.h"
#include "vcap_kernels.h"

namespace {

constexpr int TM = 256, TN = 256, ROWB = 128;
constexpr int HALF = 128 * ROWB;  // 16 KiB
constexpr int BUF = 4 * HALF;     // one K-tile: A-h0 A-h1 B-h0 B-h1
constexpr int LDS_BYTES = 2 * BUF;
// MXFP8: 4 scale buffers (K-tile kt in buffer kt & 3), each = the A block then the W block
// (1 KiB each, the global mx_scale_index layout of vcap_common.h)
constexpr int SBUF = 2048;
constexpr int LDS_BYTES_MX = LDS_BYTES + 4 * SBUF;

VCAP_DEV void glds16(const void* g, char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
}

// Per-thread source byte offsets of one half (128 rows x 128 B) of a K-tile: wave w writes LDS
// 1 KiB blocks 2w, 2w+1 (8 rows each, lane-linear) and the XOR swizzle (chunk ^ (row & 7)) is
// applied on the source.  GS: log2 of the rows per wave-group (6 for A: 64 rows of each of 2
// M-waves; 5 for B: 32 rows of each of 4 N-waves).  32-bit offsets from a uniform base keep
// every global_load_lds in the SGPR-base + VGPR-offset form.
template <typename T, int GS>
VCAP_DEV void half_offsets(uint32_t (&off)[2], long ld, int rows, int base, int X, int wave, int lane) {
  constexpr int E = Frag<T>::kElems;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int lr = (wave * 2 + i) * 8 + (lane >> 3);
    const int c = (lane & 7) ^ (lr & 7);
    int gr = base + (lr >> GS) * (2 << GS) + X * (1 << GS) + (lr & ((1 << GS) - 1));
    gr = gr < rows ? gr : rows - 1;
    off[i] = (uint32_t)(((long)gr * ld + c * E) * (long)sizeof(T));
  }
}

VCAP_DEV void glds4(const void* g, char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)lds_wave_base, 4, 0, 0);
}

VCAP_DEV void stage_half(const char* base_k, const uint32_t (&off)[2], char* lds_half, int wave) {
#pragma unroll
  for (int i = 0; i < 2; ++i) glds16(base_k + off[i], lds_half + (wave * 2 + i) * 1024);
}

VCAP_DEV u32x4 frag(const char* half, int row, int chunk) {
  return *reinterpret_cast<const u32x4*>(half + row * ROWB + ((chunk ^ (row & 7)) << 4));
}

// bf16 / MXFP8 output stores are streaming (nontemporal): a round's 128 KiB-per-CU write-back then
// does not evict the A row panels / W tiles the next round re-reads from L2 (fc1 135.7 -> 127.5 us,
// QKV 100 -> 97 us alone).  The in-place f32 residual stores stay plain (the LayerNorm reads them
// next: 1097 -> 1102 captions/s).  profiles/r02_gemm_nt_store_ab.txt.
template <typename V>
VCAP_DEV void out_store(V* p, const V& v) {
  if constexpr (__is_same(V, f32x4)) *p = v;
  else __builtin_nontemporal_store(v, p);
}

VCAP_DEV void lds_fence() { asm volatile("" ::: "memory"); }

}  // namespace


// Epilogue of a 256-row tile: wave (wr, wc) holds the 128 x 64 block at rows m0 + wr*128, columns
// n0 + wc*64 as four 64 x 32 quadrants; lane holds C[m][n .. n+3] of each 16x16 MFMA tile
// (m = .. + fr, n = .. + 4*fg).
template <typename TIn, typename TOut, int EPI>
VCAP_DEV void epilogue256(const f32x4 (&acc)[2][2][4][2], int m0, int n0, int wr, int wc, int lane, int M, int N,
                          TOut* C, long ldc, const GemmEpi& epi) {
  const int fr = lane & 15, fg = lane >> 4;
  if constexpr (EPI == 4) {
    // bias + GELU, re-quantised to MXFP8 for the next GEMM: the 32-column block
    // n0 + wc*64 + qn*32 of row m lives in this lane (j = 0, 1) and the lanes fg = 0..3 of the
    // same fr, so its max |x| is a 2-step permlane reduction.  The scale bytes of one lane's 8 row
    // blocks (qm, i + h) of a column block are adjacent in the mx_scale_index layout (row bits
    // 4..7 are its fastest index): they are collected in a register and stored as one u64 per
    // (lane, qn) instead of 8 scattered byte stores.
    // Stores (r06): both 32-column blocks of a row pair are quantised before the lane-group transpose,
    // so each 16-byte store instruction writes 64 contiguous bytes of a row (4 lanes) instead of 32:
    // the 32-byte row pieces of the earlier layout cost this launch 238 -> 166 us alone at 50432 rows
    // (fc1 shape; the same bytes: tools/mx_epi_check.py; profiles/r06_mx_fc1_epilogue_ab.txt).
    uint64_t sc[2] = {0, 0};
    f32x4 biasq[2][2];
#pragma unroll
    for (int qn = 0; qn < 2; ++qn)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        biasq[qn][j] = *reinterpret_cast<const f32x4*>(epi.bias + min(n0 + wc * 64 + qn * 32 + j * 16 + fg * 4, N - 4));
#pragma unroll
    for (int qm = 0; qm < 2; ++qm)
#pragma unroll
      for (int i = 0; i < 4; i += 2) {
        uint32_t x[2][4];   // [qn][h * 2 + j]
#pragma unroll
        for (int qn = 0; qn < 2; ++qn)
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            f32x4 v[2];
            float amax = 0.f;
#pragma unroll
            for (int j = 0; j < 2; ++j) {
              v[j] = gelu_tanh4(acc[qm][qn][i + h][j] + biasq[qn][j]);
#pragma unroll
              for (int e = 0; e < 4; ++e) amax = fmaxf(amax, fabsf(v[j][e]));
            }
            amax = rows_max(amax);
            const int sbyte = mx_scale_byte(amax);
            const float inv = mx_inv_scale(sbyte);
            const f32x4 q0 = v[0] * inv, q1 = v[1] * inv;
            x[qn][2 * h] = pack_fp8x4(q0.x, q0.y, q0.z, q0.w);
            x[qn][2 * h + 1] = pack_fp8x4(q1.x, q1.y, q1.z, q1.w);
            sc[qn] |= (uint64_t)(uint32_t)sbyte << (8 * (qm * 4 + i + h));
          }
        const int nb0 = n0 + wc * 64;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          uint32_t y[4] = {x[0][2 * h], x[0][2 * h + 1], x[1][2 * h], x[1][2 * h + 1]};
          transpose4_groups(y);
          const int ms = m0 + wr * 128 + qm * 64 + (i + h) * 16 + fr;
          if (ms < M && nb0 < N)
            out_store(reinterpret_cast<u32x4*>((uint8_t*)C + (long)ms * ldc + nb0 + fg * 16),
                      (u32x4){y[0], y[1], y[2], y[3]});
        }
      }
#pragma unroll
    for (int qn = 0; qn < 2; ++qn) {
      const int nb = n0 + wc * 64 + qn * 32;
      // rows m0 + wr*128 + fr + 16 * (qm * 4 + i + h): byte (qm * 4 + i + h) of sc[qn]; rows past M
      // land in the scale buffer's padding of the last 256-row group
      if (fg == 0 && nb < N)
        *reinterpret_cast<uint64_t*>(epi.c_scale + mx_scale_index(m0 + wr * 128 + fr, nb, (M + 255) >> 8)) = sc[qn];
    }
  } else if (sizeof(TOut) == 2 && (EPI == 0 || EPI == 1) && (N & 31) == 0 && (ldc & 7) == 0 &&
             ((uintptr_t)C & 15) == 0) {
    // bf16 out, 16-byte stores: lanes fg and fg ^ 1 (lane ^ 16) trade halves so the even lane
    // holds columns [8k, 8k+8) of the j = 0 tile and the odd lane [16+8k, +8) of the j = 1 tile
    // (k = fg >> 1); one dwordx4 store per row instead of two dwordx2 (the epilogue's store
    // issue, not HBM bandwidth, is what the row-per-lane dwordx2 pattern pays for)
    const bool odd = (lane & 16) != 0;
#pragma unroll
    for (int qm = 0; qm < 2; ++qm)
#pragma unroll
      for (int qn = 0; qn < 2; ++qn) {
        const int nb = n0 + wc * 64 + qn * 32;
        f32x4 bias[2];
#pragma unroll
        for (int j = 0; j < 2; ++j)
          bias[j] = epi.bias ? *reinterpret_cast<const f32x4*>(epi.bias + min(nb + j * 16 + fg * 4, N - 4))
                             : (f32x4){0.f, 0.f, 0.f, 0.f};
        const int col = nb + (odd ? 12 + 4 * fg : 4 * fg);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int m = m0 + wr * 128 + qm * 64 + i * 16 + fr;
          uint32_t p[2][2];
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            f32x4 v = acc[qm][qn][i][j] + bias[j];
            if constexpr (EPI == 1) v = gelu_tanh4(v);
            p[j][0] = pack_bf2(v.x, v.y);
            p[j][1] = pack_bf2(v.z, v.w);
          }
          const uint32_t r0 = (uint32_t)xor16_i((int)(odd ? p[0][0] : p[1][0]));
          const uint32_t r1 = (uint32_t)xor16_i((int)(odd ? p[0][1] : p[1][1]));
          const u32x4 o = odd ? (u32x4){r0, r1, p[1][0], p[1][1]} : (u32x4){p[0][0], p[0][1], r0, r1};
          if (m < M && nb < N) out_store(reinterpret_cast<u32x4*>(C + (long)m * ldc + col), o);
        }
      }
  } else if constexpr (EPI == 2) {
    // In-place f32 residual: C (== epi.res) += acc + bias.  Each residual load is issued a
    // quadrant ahead of the stores that follow it in program order: written as load / add / store
    // per element, the loads could not move above the previous element's store (same pointer),
    // and the in-order vmcnt made every load wait for that store too - 32 serialised HBM round
    // trips per wave, 17.6 us of a 38 us proj tile (r02 per-workgroup stamps, profiles/r02_gemm_stamps.txt).  Rows past M load row
    // M - 1 and store nothing.
    f32x4 bias[2][2];
#pragma unroll
    for (int qn = 0; qn < 2; ++qn)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int n = min(n0 + wc * 64 + qn * 32 + j * 16 + fg * 4, N - 4);
        bias[qn][j] = epi.bias ? *reinterpret_cast<const f32x4*>(epi.bias + n) : (f32x4){0.f, 0.f, 0.f, 0.f};
      }
    auto res_load = [&](f32x4 (&r)[4][2], int qm, int qn) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int m = min(m0 + wr * 128 + qm * 64 + i * 16 + fr, M - 1);
          const int n = min(n0 + wc * 64 + qn * 32 + j * 16 + fg * 4, N - 4);
          r[i][j] = *reinterpret_cast<const f32x4*>(epi.res + (long)m * epi.ldr + n);
        }
    };
    auto res_store = [&](const f32x4 (&r)[4][2], int qm, int qn) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int m = m0 + wr * 128 + qm * 64 + i * 16 + fr;
          const int n = n0 + wc * 64 + qn * 32 + j * 16 + fg * 4;
          const f32x4 v = acc[qm][qn][i][j] + bias[qn][j] + r[i][j];
          if (m < M && n < N) out_store(reinterpret_cast<f32x4*>(C + (long)m * ldc + n), v);
        }
    };
    f32x4 r0[4][2], r1[4][2];
    res_load(r0, 0, 0);
    res_load(r1, 0, 1);
    res_store(r0, 0, 0);
    res_load(r0, 1, 0);
    res_store(r1, 0, 1);
    res_load(r1, 1, 1);
    res_store(r0, 1, 0);
    res_store(r1, 1, 1);
  } else {
#pragma unroll
  for (int qm = 0; qm < 2; ++qm)
#pragma unroll
    for (int qn = 0; qn < 2; ++qn)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int n = n0 + wc * 64 + qn * 32 + j * 16 + fg * 4;
        if (n >= N) continue;
        const f32x4 bias = epi.bias ? *reinterpret_cast<const f32x4*>(epi.bias + n) : (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int m = m0 + wr * 128 + qm * 64 + i * 16 + fr;
          if (m >= M) continue;
          f32x4 v = acc[qm][qn][i][j] + bias;
          long orow = m;
          if constexpr (EPI == 1) {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = gelu_tanh(v[e]);
          } else if constexpr (EPI == 2) {
            v += *reinterpret_cast<const f32x4*>(epi.res + orow * epi.ldr + n);
          } else if constexpr (EPI == 3) {
            if (epi.act == 1)
#pragma unroll
              for (int e = 0; e < 4; ++e) v[e] = gelu_tanh(v[e]);
            orow = epi.G ? (long)(m / epi.G) * epi.Gs + epi.goff + (m % epi.G) : (long)m;
            if (epi.res_mode == 1) v += *reinterpret_cast<const f32x4*>(epi.res + orow * epi.ldr + n);
            else if (epi.res_mode == 2)
              v += *reinterpret_cast<const f32x4*>(epi.res + (long)((m % epi.G) + epi.roff) * epi.ldr + n);
          }
          if constexpr (sizeof(TOut) == 2) {
            out_store(reinterpret_cast<u32x2*>(C + orow * ldc + n), (u32x2){pack_bf2(v.x, v.y), pack_bf2(v.z, v.w)});
          } else {
            out_store(reinterpret_cast<f32x4*>(C + orow * ldc + n), v);
          }
        }
      }
  }
}

template <typename TIn, typename TOut, int EPI>
__global__ __launch_bounds__(512) void vcap_gemm256_kernel(const TIn* __restrict__ A, long lda,
                                                           const TIn* __restrict__ W, long ldw, TOut* C, long ldc,
                                                           int M, int N, int K, GemmEpi epi) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int BK = ROWB / sizeof(TIn);
  constexpr bool MX = sizeof(TIn) == 1;  // MXFP8: one scaled 16x16x128 MFMA per K-tile and fragment

  const int tiles_n = (N + TN - 1) / TN;
  const int tiles_m = (M + TM - 1) / TM;
  const int nwg = tiles_m * tiles_n;
  // XCD-aware bijective remap: consecutive tile ids (same A row panel) land on one XCD's L2
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q = nwg >> 3, r8 = nwg & 7;
  const int wgid = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + (bid >> 3);
  // tile order: row-major (consecutive ids share an A row panel), or column groups of w tile columns
  // (an XCD's run of ids then re-reads only w weight tiles: its L2 keeps them across rounds instead
  // of re-fetching all tiles_n of them every round; A panels are read once per group)
  int mt, nt;
  if (epi.colgroup > 0) {
    const int w = epi.colgroup, per = w * tiles_m;
    const int g = wgid / per, rem = wgid - g * per;
    mt = rem / w;
    nt = g * w + (rem - (rem / w) * w);
  } else {
    mt = wgid / tiles_n;
    nt = wgid - mt * tiles_n;
  }
  const int m0 = mt * TM, n0 = nt * TN;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // uniform: LDS-DMA bases stay scalar
  const int wr = wave >> 2, wc = wave & 3;
  const int fr = lane & 15, fg = lane >> 4;

  f32x4 acc[2][2][4][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[a][b][i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  // fragment pairs: lo = first 16-byte chunk, hi = second (MXFP8: one 8-register MFMA operand)
  u32x8 a0[4], a1[4], b0[2], b1[2];
  int sa[2], sb;  // MXFP8 scales of the current K-tile: A (byte X*4+i -> sa[X] byte i), W (byte Y*2+j)

  uint32_t offA[2][2], offB[2][2];
  half_offsets<TIn, 6>(offA[0], lda, M, m0, 0, wave, lane);
  half_offsets<TIn, 6>(offA[1], lda, M, m0, 1, wave, lane);
  half_offsets<TIn, 5>(offB[0], ldw, N, n0, 0, wave, lane);
  half_offsets<TIn, 5>(offB[1], ldw, N, n0, 1, wave, lane);
  // MXFP8 scales of K-tile kt: waves 0-3 stage the A block of row group m0/256, waves 4-7 the W
  // block of column group n0/256 (256 B per wave), with the A-h0 half of that K-tile.
  const uint8_t* s_src = nullptr;  // wave-uniform; the lane adds lane * 4
  long s_stride = 0;
  if constexpr (MX) {
    const int ga = (M + 255) >> 8, gw = (N + 255) >> 8;
    s_src = wave < 4 ? epi.a_scale + (long)(m0 >> 8) * 1024 : epi.w_scale + (long)(n0 >> 8) * 1024;
    s_src += (wave & 3) * 256;
    s_stride = (long)(wave < 4 ? ga : gw) * 1024;
  }
  char* const sbase = smem + 2 * BUF;
  auto stA = [&](int X, int kt) {
    stage_half((const char*)A + (long)kt * ROWB, offA[X], smem + (kt & 1) * BUF + X * HALF, wave);
    if constexpr (MX) {
      if (X == 0) glds4(s_src + kt * s_stride + lane * 4, sbase + (kt & 3) * SBUF + wave * 256);
    }
  };
  auto stB = [&](int Y, int kt) {
    stage_half((const char*)W + (long)kt * ROWB, offB[Y], smem + (kt & 1) * BUF + (2 + Y) * HALF, wave);
  };
  // Lane group fg reads 16-byte chunks fg and 4 + fg of each row: bf16 / f32 feed them to the two
  // K sub-steps; MXFP8 feeds both to one scaled MFMA, whose operand layout is exactly that
  // (K [16 fg, +16) and [64 + 16 fg, +16), tools/mx_layout_probe.hip) while the scale of lane
  // group b applies to K block [32 b, +32).
  auto rdA = [&](u32x8 (&f)[4], int X, int kt) {
    const char* h = smem + (kt & 1) * BUF + X * HALF;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = wr * 64 + i * 16 + fr;
      f[i] = cat8(frag(h, row, fg), frag(h, row, 4 + fg));
    }
  };
  auto rdB = [&](u32x8 (&f)[2], int Y, int kt) {
    const char* h = smem + (kt & 1) * BUF + (2 + Y) * HALF;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int row = wc * 32 + j * 16 + fr;
      f[j] = cat8(frag(h, row, fg), frag(h, row, 4 + fg));
    }
  };
  // MXFP8: this lane's scales of K-tile kt - A rows wr*128 + X*64 + i*16 + fr (byte i of sa[X]),
  // W rows wc*64 + Y*32 + j*16 + fr (byte Y*2 + j of sb), block fg
  auto rdS = [&](int kt) {
    if constexpr (MX) {
      const char* sb_ = sbase + (kt & 3) * SBUF + fg * 256 + fr * 16;
      const u32x2 a = *reinterpret_cast<const u32x2*>(sb_ + wr * 8);
      sa[0] = (int)a.x;
      sa[1] = (int)a.y;
      sb = (int)*reinterpret_cast<const uint32_t*>(sb_ + 1024 + wc * 4);
    }
  };
  auto mma = [&](f32x4 (&c)[4][2], const u32x8 (&af)[4], int X, const u32x8 (&bf)[2], int Y) {
    __builtin_amdgcn_s_setprio(1);
    if constexpr (MX) {
      const int s_a = sa[X];
      asm volatile("s_nop 1" ::: "memory");  // VALU -> MFMA operand wait states (asm MFMAs)
      // OPSEL must be an immediate: expand (Y, i, j) explicitly
#define VCAP_MX4(YY)                                           \
      mfma_mx<YY * 2 + 0, 0>(bf[0], sb, af[0], s_a, c[0][0]);  \
      mfma_mx<YY * 2 + 1, 0>(bf[1], sb, af[0], s_a, c[0][1]);  \
      mfma_mx<YY * 2 + 0, 1>(bf[0], sb, af[1], s_a, c[1][0]);  \
      mfma_mx<YY * 2 + 1, 1>(bf[1], sb, af[1], s_a, c[1][1]);  \
      mfma_mx<YY * 2 + 0, 2>(bf[0], sb, af[2], s_a, c[2][0]);  \
      mfma_mx<YY * 2 + 1, 2>(bf[1], sb, af[2], s_a, c[2][1]);  \
      mfma_mx<YY * 2 + 0, 3>(bf[0], sb, af[3], s_a, c[3][0]);  \
      mfma_mx<YY * 2 + 1, 3>(bf[1], sb, af[3], s_a, c[3][1]);
      if (Y == 0) {
        VCAP_MX4(0)
      } else {
        VCAP_MX4(1)
      }
#undef VCAP_MX4
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) c[i][j] = mfma_frag(lo4(bf[j]), lo4(af[i]), c[i][j], (TIn*)nullptr);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) c[i][j] = mfma_frag(hi4(bf[j]), hi4(af[i]), c[i][j], (TIn*)nullptr);
    }
    __builtin_amdgcn_s_setprio(0);
  };
  // counted waits: 2 LDS-DMA per thread per staged half, plus the scale row with each A-h0 (MX)
  auto wait_landed = [&]() {
    if constexpr (MX) asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  };
  // The phase's ds_reads are retired BEFORE its first barrier: once any wave is past that
  // barrier, every wave's reads of the phase are done, so a half may be restaged in the very
  // next phase even with the two wave groups staggered by a barrier.
  auto sync_reads = [&]() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    lds_fence();
    __builtin_amdgcn_s_barrier();
  };
  auto end_phase = [&]() {
    lds_fence();
    __builtin_amdgcn_s_barrier();
    lds_fence();
  };

  const int nk = K / BK;  // even, >= 2 (dispatcher)
  // prologue: K-tile 0 complete; K-tile 1 minus its A-h1 in flight
  stA(0, 0);
  stA(1, 0);
  stB(0, 0);
  stB(1, 0);
  stA(0, 1);
  stB(0, 1);
  stB(1, 1);
  wait_landed();
  end_phase();
  // Stagger: the wr == 1 wave group runs one barrier behind, so on every SIMD one wave issues
  // its MFMAs while the other issues ds_reads / LDS-DMA.  (Balanced by wr == 0 after the loop.)
  if (wr == 1) __builtin_amdgcn_s_barrier();

  for (int t = 0; t < nk; t += 2) {
    const bool more = t + 2 < nk;
    // ---- K-tile t (even buffer)
    rdB(b0, 0, t);
    rdA(a0, 0, t);
    rdS(t);
    stA(1, t + 1);
    sync_reads();
    mma(acc[0][0], a0, 0, b0, 0);
    end_phase();

    rdB(b1, 1, t);
    if (more) stA(0, t + 2);
    sync_reads();
    mma(acc[0][1], a0, 0, b1, 1);
    end_phase();

    rdA(a1, 1, t);
    if (more) stB(0, t + 2);
    sync_reads();
    mma(acc[1][1], a1, 1, b1, 1);
    end_phase();

    if (more) {
      stB(1, t + 2);
      wait_landed();  // K-tile t+1 landed (this wave's part)
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    sync_reads();
    mma(acc[1][0], a1, 1, b0, 0);
    end_phase();

    // ---- K-tile t+1 (odd buffer)
    rdB(b0, 0, t + 1);
    rdA(a0, 0, t + 1);
    rdS(t + 1);
    if (more) stA(1, t + 2);
    sync_reads();
    mma(acc[0][0], a0, 0, b0, 0);
    end_phase();

    rdB(b1, 1, t + 1);
    if (more) stA(0, t + 3);
    sync_reads();
    mma(acc[0][1], a0, 0, b1, 1);
    end_phase();

    rdA(a1, 1, t + 1);
    if (more) stB(0, t + 3);
    sync_reads();
    mma(acc[1][1], a1, 1, b1, 1);
    end_phase();

    if (more) {
      stB(1, t + 3);
      wait_landed();  // K-tile t+2 landed
    }
    sync_reads();
    mma(acc[1][0], a1, 1, b0, 0);
    end_phase();
  }
  if (wr == 0) __builtin_amdgcn_s_barrier();
  if constexpr (MX) mfma_mx_drain();

  epilogue256<TIn, TOut, EPI>(acc, m0, n0, wr, wc, lane, M, N, C, ldc, epi);
}

template <typename TIn, typename TOut, int EPI>
static hipError_t launch256_epi(const void* A, long lda, const void* W, long ldw, void* C, long ldc, int M, int N,
                                int K, const GemmEpi& epi, hipStream_t s) {
  constexpr int lds = sizeof(TIn) == 1 ? LDS_BYTES_MX : LDS_BYTES;
  static bool configured = false;
  if (!configured) {
    hipError_t e = hipFuncSetAttribute((const void*)vcap_gemm256_kernel<TIn, TOut, EPI>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    if (e != hipSuccess) return e;
    configured = true;
  }
  const int tiles_n = (N + TN - 1) / TN;
  const int tiles = ((M + TM - 1) / TM) * tiles_n;
  GemmEpi e = epi;
  e.colgroup = 0;
  if (EPI == 1) {
    // column-group tile order for the GELU GEMM (fc1), whose weight tiles do not fit one XCD's 4 MB
    // L2 beside its A panels (ViT-B: 12 x 384 KB): the widest group of whole tile columns dividing
    // tiles_n with <= 2.5 MB of weights, so an XCD keeps its group's tiles across rounds.  Measured
    // (profiles/r04_gemm_colgroup_ab.txt, 16-video fc1): FETCH 426 -> 294 MB per launch, 310 -> 306 us
    // in the pipelined bench, equal alone.
    const long tile_bytes = (long)TN * K * (long)sizeof(TIn);
    int w = 0;
    for (int c = tiles_n - 1; c >= 1; --c)
      if (tiles_n % c == 0 && c * tile_bytes <= 2560L * 1024) {
        w = c;
        break;
      }
    if (w > 0 && w < tiles_n && tiles_n % w == 0) e.colgroup = w;
  }
  hipLaunchKernelGGL((vcap_gemm256_kernel<TIn, TOut, EPI>), dim3(tiles), dim3(512), lds, s, (const TIn*)A, lda,
                     (const TIn*)W, ldw, (TOut*)C, ldc, M, N, K, e);
  return hipGetLastError();
}

template <typename TIn, typename TOut>
static hipError_t launch256(const void* A, long lda, const void* W, long ldw, void* C, long ldc, int M, int N, int K,
                            const GemmEpi& epi, hipStream_t s) {
  if constexpr (sizeof(TOut) == 1) {
    return launch256_epi<TIn, TOut, 4>(A, lda, W, ldw, C, ldc, M, N, K, epi, s);  // MXFP8 out (bias + gelu)
  } else {
    const bool plain_rows = epi.G == 0;
    if (plain_rows && epi.res_mode == 0 && epi.act == 0)
      return launch256_epi<TIn, TOut, 0>(A, lda, W, ldw, C, ldc, M, N, K, epi, s);
    if constexpr (sizeof(TOut) == sizeof(TIn) || sizeof(TOut) == 2) {   // (MXFP8 in -> bf16 GELU out too)
      if (plain_rows && epi.res_mode == 0 && epi.act == 1)
        return launch256_epi<TIn, TOut, 1>(A, lda, W, ldw, C, ldc, M, N, K, epi, s);
    }
    if constexpr (sizeof(TOut) == 4) {
      if (plain_rows && epi.res_mode == 1 && epi.act == 0 && epi.res == (const float*)C && epi.ldr == ldc)
        return launch256_epi<TIn, TOut, 2>(A, lda, W, ldw, C, ldc, M, N, K, epi, s);
    }
    return launch256_epi<TIn, TOut, 3>(A, lda, W, ldw, C, ldc, M, N, K, epi, s);
  }
}

// Shapes this kernel takes: K a multiple of two K-tiles, N and the strides in whole 16-byte
// vectors for the epilogue, 16-byte aligned bias / residual rows.
bool vcap_gemm256_ok(int in_dt, int out_dt, long lda, long ldw, long ldc, int M, int N, int K, const GemmEpi& epi) {
  const int bk = in_dt == VCAP_DT_MXFP8 ? 128 : in_dt == VCAP_DT_BF16 ? 64 : 32;
  if (K % (2 * bk) != 0 || N % 16 != 0 || M <= 0) return false;
  const int ein = in_dt == VCAP_DT_MXFP8 ? 16 : in_dt == VCAP_DT_BF16 ? 8 : 4;
  if (in_dt == VCAP_DT_MXFP8 && (!epi.a_scale || !epi.w_scale)) return false;
  if (out_dt == VCAP_DT_MXFP8 && (in_dt != VCAP_DT_MXFP8 || N % 128 || ldc % 16 || epi.act != 1 || !epi.bias ||
                                  !epi.c_scale || epi.G || epi.res_mode))
    return false;
  if (lda % ein || ldw % ein) return false;
  if (ldc % 4) return false;
  if (epi.bias && ((uintptr_t)epi.bias & 15)) return false;
  if (epi.res && (((uintptr_t)epi.res & 15) || epi.ldr % 4)) return false;
  (void)out_dt;
  return true;
}

hipError_t vcap_gemm256_dispatch(int in_dt, int out_dt, const void* A, long lda, const void* W, long ldw, void* C,
                                 long ldc, int M, int N, int K, const GemmEpi& epi, hipStream_t s) {
  if (in_dt == VCAP_DT_BF16 && out_dt == VCAP_DT_BF16)
    return launch256<bf16_t, bf16_t>(A, lda, W, ldw, C, ldc, M, N, K, epi, s);
  if (in_dt == VCAP_DT_BF16 && out_dt == VCAP_DT_F32)
    return launch256<bf16_t, float>(A, lda, W, ldw, C, ldc, M, N, K, epi, s);
  if (in_dt == VCAP_DT_F32 && out_dt == VCAP_DT_F32)
    return launch256<float, float>(A, lda, W, ldw, C, ldc, M, N, K, epi, s);
  if (in_dt == VCAP_DT_MXFP8 && out_dt == VCAP_DT_BF16)
    return launch256<fp8_t, bf16_t>(A, lda, W, ldw, C, ldc, M, N, K, epi, s);
  if (in_dt == VCAP_DT_MXFP8 && out_dt == VCAP_DT_F32)
    return launch256<fp8_t, float>(A, lda, W, ldw, C, ldc, M, N, K, epi, s);
  if (in_dt == VCAP_DT_MXFP8 && out_dt == VCAP_DT_MXFP8)
    return launch256<fp8_t, fp8_t>(A, lda, W, ldw, C, ldc, M, N, K, epi, s);
  return hipErrorInvalidValue;
}
