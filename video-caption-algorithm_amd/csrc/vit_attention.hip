// ViT multi-head self-attention core: O = softmax(Q K^T / sqrt(64)) V per (frame, head).
// Replaces timm Attention with fused_attn=True -> F.scaled_dot_product_attention
// (src/models/video_encoder.py:112-121; no mask, no causal, scale head_dim^-0.5).
//
// f32 parity path: one workgroup (4 waves) per (frame, head).  K and V of the head are staged in LDS:
// K row-major [NP][64] with an XOR chunk swizzle (conflict-free ds_read_b128 fragment
// reads), V transposed to Vt[64][NP+pad].  Each wave owns 16-query tiles and computes
// S^T = K Q^T on MFMA so a lane ends up holding 4 consecutive keys of ONE query per key
// tile; the whole row (NP <= 288 keys) stays in registers, so softmax is exact (no online
// rescale): row max/sum reduce over the 4 lane groups with two xor-shuffles.  The
// accumulators are then consumed in place as the P^T operand of O^T = Vt P^T (the k
// index permutation is applied identically to the Vt fragment), and a lane writes 4
// consecutive head-dims of one query row.
#include <cstdlib>
#include <cstring>

#include "vcap_common.h"
#include "vcap_kernels.h"

// cls_only: compute the class-token query (q = 0) of each (frame, head) only and write it to
// compact row `frame` of out (the last block of the encoder: only CLS rows are consumed after it).
template <typename T, int KT>
__global__ __launch_bounds__(256) void vcap_vit_attention_kernel(const T* __restrict__ qkv, T* __restrict__ out,
                                                                 int N, int H, int cls_only) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int E = Frag<T>::kElems;     // elements per 16-byte chunk
  constexpr int CH = 64 / E;             // chunks per 64-dim row (8 bf16, 16 f32)
  constexpr int NP = KT * 16;            // padded key count
  constexpr int VS = NP + (sizeof(T) == 2 ? 8 : 4);  // Vt row stride (elements)
  constexpr int NS = 64 / (4 * E);       // 4-chunk k-slabs per 64 dims (2 bf16, 4 f32)
  static_assert(sizeof(T) == 4 || (KT % 2) == 0, "bf16 path consumes 32-key chunks");

  const int bh = blockIdx.x;
  const int bt = bh / H, h = bh % H;
  const int D = H * 64;
  const long ld = 3L * D;
  const T* base = qkv + (long)bt * N * ld + h * 64;

  char* Ks = smem;
  T* Vt = reinterpret_cast<T*>(smem + NP * 64 * sizeof(T));

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // ---- stage K (swizzled) and V^T: every load issued before any use (no predicated loads:
  // a runtime guard around a load makes hipcc wait for each one separately)
  constexpr int ITERS = NP * CH / 256;
  static_assert(NP * CH % 256 == 0, "staging loop assumes whole 256-chunk passes");
  u32x4 kv[ITERS], vv[ITERS];
#pragma unroll
  for (int i = 0; i < ITERS; ++i) {
    const int idx = tid + i * 256;
    const int key = min(idx / CH, N - 1), c = idx % CH;
    kv[i] = *reinterpret_cast<const u32x4*>(base + (long)key * ld + D + c * E);
    vv[i] = *reinterpret_cast<const u32x4*>(base + (long)key * ld + 2 * D + c * E);
  }
#pragma unroll
  for (int i = 0; i < ITERS; ++i) {
    const int idx = tid + i * 256;
    const int key = idx / CH, c = idx % CH;
    const bool live = key < N;
    const u32x4 z = (u32x4){0u, 0u, 0u, 0u};
    *reinterpret_cast<u32x4*>(Ks + key * 64 * sizeof(T) + ((c ^ (key & (CH - 1))) << 4)) = live ? kv[i] : z;
    const u32x4 v = live ? vv[i] : z;
    const T* ve = reinterpret_cast<const T*>(&v);
#pragma unroll
    for (int e = 0; e < E; ++e) Vt[(c * E + e) * VS + key] = ve[e];
  }
  __syncthreads();

  const int fr = lane & 15, fg = lane >> 4;
  const int qtiles = cls_only ? 1 : (N + 15) / 16;
  const float scale = 0.125f;  // 64^-0.5
  for (int qt = wave; qt < qtiles; qt += 4) {
    int q = qt * 16 + fr;
    const int qc = q < N ? q : N - 1;
    u32x4 qf[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) qf[s] = *reinterpret_cast<const u32x4*>(base + (long)qc * ld + (s * 4 + fg) * E);

    f32x4 st[KT];
#pragma unroll
    for (int kt = 0; kt < KT; ++kt) {
      f32x4 acc = (f32x4){0.f, 0.f, 0.f, 0.f};
      const int key = kt * 16 + fr;
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        const int c = s * 4 + fg;
        const u32x4 kf = *reinterpret_cast<const u32x4*>(Ks + key * 64 * sizeof(T) + ((c ^ (key & (CH - 1))) << 4));
        acc = mfma_frag(kf, qf[s], acc, (T*)nullptr);
      }
      st[kt] = acc;  // S^T[key = kt*16 + 4*fg + r][query = fr]
    }
    // ---- exact softmax over the full key row of query fr
    float mx = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < KT; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = kt * 16 + fg * 4 + r;
        if (key >= N) st[kt][r] = -INFINITY;
        mx = fmaxf(mx, st[kt][r]);
      }
    mx = rows_max(mx);
    float sum = 0.f;
#pragma unroll
    for (int kt = 0; kt < KT; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = __expf((st[kt][r] - mx) * scale);
        st[kt][r] = p;
        sum += p;
      }
    sum = rows_sum(sum);
    const float inv = 1.0f / sum;

    // ---- O^T[d][q] = sum_key Vt[d][key] * P^T[key][q]
    f32x4 o[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) o[dt] = (f32x4){0.f, 0.f, 0.f, 0.f};
    if constexpr (sizeof(T) == 2) {
#pragma unroll
      for (int c = 0; c < KT / 2; ++c) {
        const u32x4 pf = (u32x4){pack_bf2(st[2 * c][0], st[2 * c][1]), pack_bf2(st[2 * c][2], st[2 * c][3]),
                                 pack_bf2(st[2 * c + 1][0], st[2 * c + 1][1]),
                                 pack_bf2(st[2 * c + 1][2], st[2 * c + 1][3])};
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
          const T* vrow = Vt + (dt * 16 + fr) * VS + 32 * c + 4 * fg;
          const u32x2 lo = *reinterpret_cast<const u32x2*>(vrow);
          const u32x2 hi = *reinterpret_cast<const u32x2*>(vrow + 16);
          const u32x4 vf = (u32x4){lo.x, lo.y, hi.x, hi.y};
          o[dt] = mfma_frag(vf, pf, o[dt], (T*)nullptr);
        }
      }
    } else {
#pragma unroll
      for (int t = 0; t < KT; ++t) {
        const u32x4 pf = (u32x4){__float_as_uint(st[t][0]), __float_as_uint(st[t][1]), __float_as_uint(st[t][2]),
                                 __float_as_uint(st[t][3])};
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
          const u32x4 vf = *reinterpret_cast<const u32x4*>(Vt + (dt * 16 + fr) * VS + 16 * t + 4 * fg);
          o[dt] = mfma_frag(vf, pf, o[dt], (T*)nullptr);
        }
      }
    }
    if (q < N && (!cls_only || q == 0)) {
      T* orow = out + (cls_only ? (long)bt : (long)bt * N + q) * D + h * 64;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const f32x4 v = o[dt] * inv;  // O^T[d = dt*16 + 4*fg + r][q]
        if constexpr (sizeof(T) == 2) {
          *reinterpret_cast<u32x2*>(orow + dt * 16 + 4 * fg) = (u32x2){pack_bf2(v.x, v.y), pack_bf2(v.z, v.w)};
        } else {
          *reinterpret_cast<f32x4*>(orow + dt * 16 + 4 * fg) = v;
        }
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------
// bf16 path (the benchmark dtype).  Same S^T = K Q^T formulation and exact in-register softmax,
// but nothing passes through VGPRs on the way to LDS and nothing is transposed by stores:
//  * K and V rows arrive by LDS-DMA (global_load_lds_dwordx4, 1 KiB = 8 rows per wave
//    instruction) into [key][64] images with the 16-byte-chunk XOR swizzle slot = c ^ (key & 7)
//    applied on the source address;
//  * the PV MFMA's Vt operand is read straight from the row-major V image with the gfx950
//    transpose read ds_read_b64_tr_b16 (16-lane group: 4 keys x 16 dims -> lane i gets dim i);
//    with the swizzle above the 8 keys a 32-lane half touches land on 64 distinct banks;
//  * Q fragments of all of a wave's query tiles are loaded before the K/V wait;
//  * softmax: exp2 with (1/sqrt(64)) * log2(e) folded into one FMA, P packed to bf16 with
//    v_cvt_pk_bf16_f32.
// max of three as one v_max3_f32: this file is built with -fno-honor-nans (build.py), so maxnum
// needs no operand canonicalisation.  (Not inline asm: the hazard recognizer does not see an asm
// operand that overwrites the source-C registers of an MFMA still in flight.)
VCAP_DEV float max3f(float a, float b, float c) { return fmaxf(fmaxf(a, b), c); }


VCAP_DEV void glds16_attn(const void* g, char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
}

VCAP_DEV uint32_t cvt_pk_bf16(float lo, float hi) { return pack_bf2(lo, hi); }

typedef __attribute__((ext_vector_type(4))) short s16x4;

VCAP_DEV u32x2 tr_read(const char* p) {
  const s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)p);
  return __builtin_bit_cast(u32x2, v);
}

// One 16-query tile of one (frame, head): S^T = K.Q^T over the head's K image, exact softmax in
// registers, O^T = V^T.P^T with V read by transpose reads.  Returns the unnormalised O^T fragments
// and 1 / rowsum (lane (fr, fg) holds dims dt*16 + 4*fg + r of query fr).
// KE: key tiles that can hold real keys (KT or KT - 1: with N <= 16 (KT - 1) the last tile is all
// padding, kept only as the zero half of the last 32-key PV chunk - no S, max or exp for it).
template <int KT, int KE>
VCAP_DEV void attn_bf16_qtile(const char* Ks, const char* Vs, const u32x4 (&qf)[2], int N, f32x4 (&o)[4],
                              float& inv) {
  const int lane = threadIdx.x & 63;
  const int fr = lane & 15, fg = lane >> 4;
  const float c2 = 0.125f * 1.4426950408889634f;  // 64^-0.5 * log2(e)
  // S^T[key][q] = K . Q^T
  f32x4 st[KT];
  if constexpr (KE < KT) st[KT - 1] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int kt = 0; kt < KE; ++kt) {
    f32x4 acc = (f32x4){0.f, 0.f, 0.f, 0.f};
    const int key = kt * 16 + fr;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const u32x4 kf = *reinterpret_cast<const u32x4*>(Ks + key * 128 + (((s * 4 + fg) ^ (key & 7)) << 4));
      acc = mfma_frag(kf, qf[s], acc, (bf16_t*)nullptr);
    }
    st[kt] = acc;  // keys kt*16 + 4*fg + r, query fr
  }
  // padded keys: the dispatcher picks KT with 16 (KT - 2) < N <= 16 KT, so only the last two key
  // tiles can hold them (a compile-time range: a runtime test per tile kept ~60 lane masks live
  // and spilled them through v_writelane / v_readlane)
#pragma unroll
  for (int kt = KT - 2; kt < KE; ++kt) {
    const int lim = N - kt * 16 - fg * 4;
#pragma unroll
    for (int r = 0; r < 4; ++r) st[kt][r] = r < lim ? st[kt][r] : -INFINITY;
  }
  // row max: four independent v_max3 chains (one per accumulator element) instead of one 26-deep
  // dependent chain; the same instruction count
  float mx;
  {
    float m4[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      m4[r] = st[0][r];
#pragma unroll
      for (int kt = 1; kt < KE; kt += 2) m4[r] = kt + 1 < KE ? max3f(m4[r], st[kt][r], st[kt + 1][r]) : fmaxf(m4[r], st[kt][r]);
    }
    mx = fmaxf(max3f(m4[0], m4[1], m4[2]), m4[3]);
  }
  mx = rows_max(mx);
  // the row sum comes out of the PV MFMAs below (a ones operand beside V), so the softmax here
  // is one FMA + one exp per score
  const float mxc = mx * c2;
#pragma unroll
  for (int kt = 0; kt < KE; ++kt)
#pragma unroll
    for (int r = 0; r < 4; ++r) st[kt][r] = __builtin_amdgcn_exp2f(fmaf(st[kt][r], c2, -mxc));

  // O^T[d][q] = sum_key V[key][d] P^T[key][q]; k element j of lane group g <-> key
  // 32c + 4g + j (j < 4) / 32c + 16 + 4g + (j - 4), matching the P^T fragment below
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) o[dt] = (f32x4){0.f, 0.f, 0.f, 0.f};
  // S[q] = sum_key 1 * P^T[key][q]: every output row of this MFMA is the sum of the bf16 P the
  // PV products use (lane (fr, fg) gets query fr's sum in each element)
  f32x4 osum = (f32x4){0.f, 0.f, 0.f, 0.f};
  const u32x4 ones = (u32x4){0x3F803F80u, 0x3F803F80u, 0x3F803F80u, 0x3F803F80u};
  const int qr = fr >> 2, p4 = fr & 3;
#pragma unroll
  for (int c = 0; c < KT / 2; ++c) {
    const u32x4 pf = (u32x4){cvt_pk_bf16(st[2 * c][0], st[2 * c][1]), cvt_pk_bf16(st[2 * c][2], st[2 * c][3]),
                             cvt_pk_bf16(st[2 * c + 1][0], st[2 * c + 1][1]),
                             cvt_pk_bf16(st[2 * c + 1][2], st[2 * c + 1][3])};
    const int r0 = 32 * c + 4 * fg + qr, r1 = r0 + 16;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const int ch = 2 * dt + (p4 >> 1);
      const u32x2 lo = tr_read(Vs + r0 * 128 + ((ch ^ (r0 & 7)) << 4) + 8 * (p4 & 1));
      // keys 16 KE .. 16 KT - 1 are all padding (P = 0): not staged, a zero operand instead
      const u32x2 hi = (KE < KT && c == KT / 2 - 1) ? (u32x2){0u, 0u}
                                                    : tr_read(Vs + r1 * 128 + ((ch ^ (r1 & 7)) << 4) + 8 * (p4 & 1));
      o[dt] = mfma_frag((u32x4){lo.x, lo.y, hi.x, hi.y}, pf, o[dt], (bf16_t*)nullptr);
    }
    osum = mfma_frag(ones, pf, osum, (bf16_t*)nullptr);
  }
  const float sum = osum[0];
  inv = __builtin_amdgcn_rcpf(sum);
}

// A query tile's output, packed for its stores: bf16 -> two dwordx4 per lane (lane pair exchange),
// MXFP8 -> one dwordx4 per lane + the lane group 0 scale bytes.  Built right after the compute;
// `attn_commit` stores it.
struct AttnOut {
  u32x4 w0, w1;
  int sb0, sb1;
  long row;
  bool keep;
};

template <bool MXO>
VCAP_DEV AttnOut attn_pack(const f32x4 (&o)[4], float inv, long row, bool keep) {
  const int lane = threadIdx.x & 63;
  AttnOut r;
  r.row = row;
  r.keep = keep;
  r.sb0 = r.sb1 = 0;
  if constexpr (MXO) {
    // block b = dims [32b, 32b+32) of the row: dt in {2b, 2b+1} of this lane and lanes fg = 0..3;
    // after quantisation a 4x4 lane-group transpose hands every lane 16 contiguous bytes of the
    // head's 64 (lane group g: dims [16g, 16g+16)), one dwordx4 store per lane
    uint32_t x[4];
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const f32x4 v0 = o[2 * b] * inv, v1 = o[2 * b + 1] * inv;
      float amax = 0.f;
#pragma unroll
      for (int e = 0; e < 4; ++e) amax = fmaxf(amax, fmaxf(fabsf(v0[e]), fabsf(v1[e])));
      amax = rows_max(amax);
      const int sb = mx_scale_byte(amax);
      const float is = mx_inv_scale(sb);
      x[2 * b] = pack_fp8x4(v0.x * is, v0.y * is, v0.z * is, v0.w * is);
      x[2 * b + 1] = pack_fp8x4(v1.x * is, v1.y * is, v1.z * is, v1.w * is);
      if (b == 0) r.sb0 = sb; else r.sb1 = sb;
    }
    transpose4_groups(x);
    r.w0 = (u32x4){x[0], x[1], x[2], x[3]};
    r.w1 = r.w0;
  } else {
    // O[q][d = dt*16 + 4*fg + r]; lanes fg, fg ^ 1 (lane ^ 16) trade halves of the dt pair
    // (2k, 2k+1) so each stores 8 contiguous dims with one dwordx4 (the even lane dims
    // [32k + 4fg, +8), the odd lane [32k + 12 + 4fg, +8)); the exchange runs in every lane
    const bool odd = (lane & 16) != 0;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const f32x4 va = o[2 * k] * inv, vb = o[2 * k + 1] * inv;
      const uint32_t a0 = cvt_pk_bf16(va.x, va.y), a1 = cvt_pk_bf16(va.z, va.w);
      const uint32_t b0 = cvt_pk_bf16(vb.x, vb.y), b1 = cvt_pk_bf16(vb.z, vb.w);
      const uint32_t r0 = (uint32_t)xor16_i((int)(odd ? a0 : b0));
      const uint32_t r1 = (uint32_t)xor16_i((int)(odd ? a1 : b1));
      const u32x4 w = odd ? (u32x4){r0, r1, b0, b1} : (u32x4){a0, a1, r0, r1};
      if (k == 0) r.w0 = w; else r.w1 = w;
    }
  }
  return r;
}

template <bool MXO>
VCAP_DEV void attn_commit(const AttnOut& r, void* out, int D, int h, uint8_t* oscale, int groups) {
  if (!r.keep) return;
  const int lane = threadIdx.x & 63, fg = lane >> 4;
  if constexpr (MXO) {
    if (fg == 0) {
      oscale[mx_scale_index((int)r.row, h * 64, groups)] = (uint8_t)r.sb0;
      oscale[mx_scale_index((int)r.row, h * 64 + 32, groups)] = (uint8_t)r.sb1;
    }
    *reinterpret_cast<u32x4*>((uint8_t*)out + r.row * D + h * 64 + 16 * fg) = r.w0;
  } else {
    const bool odd = (lane & 16) != 0;
    bf16_t* orow = (bf16_t*)out + r.row * D + h * 64;
    *reinterpret_cast<u32x4*>(orow + (odd ? 12 + 4 * fg : 4 * fg)) = r.w0;
    *reinterpret_cast<u32x4*>(orow + 32 + (odd ? 12 + 4 * fg : 4 * fg)) = r.w1;
  }
}

// One workgroup per (frame, head) pair; two of them share a CU (56 KiB of LDS, <= 128 VGPRs
// for 4 waves per SIMD), so one pair's DMA overlaps the other's MFMA / softmax.  (A persistent
// double-buffered walk over pairs measured equal alone and slower in the bench, r02: removed.
// Issuing K, Q, then V and running the first query tile's S + softmax before the V wait measured
// 39.1-39.7 vs 37.8-38.6 us at 128 frames, r03 (profiles/r03_attention_v_overlap_ab.txt): reverted.)
// MXO: write the output as MXFP8 (e4m3 + E8M0 per 32 of the head's 64 dims) for an MXFP8 attn-proj
// GEMM; oscale in the vcap_common.h layout over `groups` 256-row groups.
template <int KT, int KE, int WAVES, bool MXO>
__global__ __launch_bounds__(WAVES * 64) void vcap_vit_attention_bf16_kernel(const bf16_t* __restrict__ qkv,
                                                                             void* __restrict__ out, int N, int H,
                                                                             uint8_t* __restrict__ oscale,
                                                                             int groups, int cls_only) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int NP = KT * 16;
  constexpr int NS = KE * 16;  // staged key rows (the all-padding last tile is never read)
  constexpr int QT_MAX = (KT + WAVES - 1) / WAVES;  // query tiles per wave (N <= NP)
  static_assert(KT % 2 == 0, "PV consumes 32-key chunks");
  char* Ks = smem;
  char* Vs = smem + NS * 128;

  const int bh = blockIdx.x;
  const int bt = bh / H, h = bh - bt * H;
  const int D = H * 64;
  const long ld = 3L * D;
  const bf16_t* base = qkv + (long)bt * N * ld + h * 64;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fg = lane >> 4;

  // ---- K, V -> LDS by DMA (rows past N re-read row N-1: finite, masked out of the softmax)
  for (int blk = wave; blk < NS / 8; blk += WAVES) {
    const int r = blk * 8 + (lane >> 3);
    const int c = (lane & 7) ^ (r & 7);
    const bf16_t* src = base + (long)min(r, N - 1) * ld + c * 8;
    glds16_attn(src + D, Ks + blk * 1024);
    glds16_attn(src + 2 * D, Vs + blk * 1024);
  }
  (void)NP;
  // ---- this wave's Q fragments
  const int qtiles = cls_only ? 1 : (N + 15) / 16;
  u32x4 qf[QT_MAX][2];
#pragma unroll
  for (int i = 0; i < QT_MAX; ++i) {
    const int q = min((wave + i * WAVES) * 16 + fr, N - 1);
#pragma unroll
    for (int s = 0; s < 2; ++s) qf[i][s] = *reinterpret_cast<const u32x4*>(base + (long)q * ld + s * 32 + fg * 8);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

#pragma unroll
  for (int i = 0; i < QT_MAX; ++i) {
    const int qt = wave + i * WAVES;
    if (qt >= qtiles) break;
    f32x4 o[4];
    float inv;
    attn_bf16_qtile<KT, KE>(Ks, Vs, qf[i], N, o, inv);
    const int q = qt * 16 + fr;
    const bool keep = q < N && (!cls_only || q == 0);
    const long row = cls_only ? (long)bt : (long)bt * N + q;
    attn_commit<MXO>(attn_pack<MXO>(o, inv, row, keep), out, D, h, oscale, groups);
  }
}

template <int KT, int KE, int WAVES, bool MXO>
static hipError_t launch_attn_bf16(const void* qkv, void* out, int BT, int N, int H, uint8_t* oscale, int cls_only,
                                   hipStream_t s) {
  const size_t lds = (size_t)KE * 16 * 128 * 2;  // 53 KiB at KE = 13: three workgroups per CU
  static bool configured = false;
  if (!configured) {
    hipError_t e = hipFuncSetAttribute((const void*)vcap_vit_attention_bf16_kernel<KT, KE, WAVES, MXO>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    configured = true;
  }
  const int groups = ((cls_only ? BT : BT * N) + 255) / 256;  // scale rows = output rows
  hipLaunchKernelGGL((vcap_vit_attention_bf16_kernel<KT, KE, WAVES, MXO>), dim3(BT * H), dim3(WAVES * 64), lds, s,
                     (const bf16_t*)qkv, out, N, H, oscale, groups, cls_only);
  return hipGetLastError();
}

template <typename T, int KT>
static hipError_t launch_attn(const void* qkv, void* out, int BT, int N, int H, int cls_only, hipStream_t s) {
  constexpr int NP = KT * 16;
  constexpr int VS = NP + (sizeof(T) == 2 ? 8 : 4);
  const size_t lds = (size_t)NP * 64 * sizeof(T) + (size_t)64 * VS * sizeof(T);
  static bool configured = false;  // dynamic LDS above 64 KiB needs the explicit opt-in
  if (!configured) {
    hipError_t e = hipFuncSetAttribute((const void*)vcap_vit_attention_kernel<T, KT>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    configured = true;
  }
  hipLaunchKernelGGL((vcap_vit_attention_kernel<T, KT>), dim3(BT * H), dim3(256), lds, s, (const T*)qkv, (T*)out, N,
                     H, cls_only);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
// Fused QKV projection + attention (bf16, ViT-B/16 frame: 197 tokens, head_dim 64).  One workgroup
// (8 waves) per (frame, head): it computes the head's 192 q / k / v features of the frame's 208
// (padded) tokens from the LayerNorm output and the head's 192 weight rows, writes them as bf16
// straight into the attention's LDS images and runs the attention above on them - q / k / v never
// leave the CU (the unfused pair writes 3 x 768 bf16 per token to HBM and reads them back).
//  * GEMM: C^T[feature][token] with the weight fragment as the MFMA A operand (each lane ends up
//    with 4 consecutive features of one token = 8 contiguous bytes of a [token][64] image) and the
//    K order of vcap_gemm256_kernel (32-wide sub-steps, lane group g = K [8g, 8g + 8)), so every
//    q / k / v value, its bias add and its bf16 rounding are those of the unfused QKV GEMM and the
//    output is bit-identical to QKV GEMM + vcap_vit_attention_bf16_kernel;
//  * waves 4 (feature groups of 3 tiles) x 2 (token groups of 7 / 6 tiles): 21 / 18 16x16
//    accumulators per wave;
//  * K-tiles of 64 (208 token rows + 192 weight rows x 128 B = 50 KiB) stream by LDS-DMA through a
//    3-deep ring (150 KiB: one workgroup per CU), rows XOR-swizzled on the source like the
//    GEMM's; token rows past N re-read row N - 1 (what the unfused attention stages);
//  * the ring's first 78 KiB then hold the K, V and Q images ([token][64], chunk ^ (token & 7)).
// Grid: frames x heads, XCD-aware when frames % 8 == 0 (workgroup b runs on XCD b % 8; the heads
// of one frame go to the same XCD back to back so its LayerNorm rows are re-read from that L2).
namespace qa {
constexpr int TT = 13, FT = 12;                // token tiles (208 tokens), feature tiles (q, k, v)
constexpr int RT = TT * 16, RW = FT * 16;      // 208 token rows, 192 weight rows per K-tile
constexpr int STAGE = (RT + RW) * 128;         // 51200 B
constexpr int NSTAGE = 3;
constexpr int LDS = NSTAGE * STAGE;            // 153600 B
constexpr int BLKS = (RT + RW) / 8;            // 50 LDS-DMA wave instructions (8 rows) per K-tile
constexpr int NB_MAX = (BLKS + 7) / 8;         // 7 (waves 0, 1), 6 (waves 2..7)
}  // namespace qa

// A bare workgroup barrier.  __syncthreads() would also make every wave drain ALL its vector memory
// operations first (s_waitcnt vmcnt(0)), i.e. wait for the K-tile DMA issued one iteration ago and
// cut the ring's look-ahead to one K-tile; the waits this kernel needs are explicit (qa_wait_older
// before, lgkmcnt(0) after the image writes).
VCAP_DEV void qa_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <bool TWO_NB>
VCAP_DEV void qa_wait_older(bool older) {
  // all but this wave's most recent K-tile of LDS-DMA landed
  if (older) {
    if constexpr (TWO_NB) asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
}

__global__ __launch_bounds__(512) void vcap_vit_qkv_attention_kernel(const bf16_t* __restrict__ xn,
                                                                     const bf16_t* __restrict__ wqkv,
                                                                     const float* __restrict__ bqkv,
                                                                     bf16_t* __restrict__ out, int BT, int N, int H,
                                                                     int cls_only) {
  using namespace qa;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int D = H * 64;  // = K of the projection
  const int b = blockIdx.x;
  int bt, h;
  if ((BT & 7) == 0) {
    const int x = b & 7, j = b >> 3;
    bt = (j / H) * 8 + x;
    h = j - (j / H) * H;
  } else {
    bt = b / H;
    h = b - bt * H;
  }
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fg = lane >> 4;
  const int fgrp = wave & 3, tgrp = wave >> 2;
  const int t0 = tgrp * 7, ntt = tgrp ? TT - 7 : 7;

  // The two wave groups (tgrp 0 = waves 0-3, one per SIMD, token tiles 0-6; tgrp 1 = waves 4-7,
  // tiles 7-12) run one barrier apart: while one group issues its 42 MFMAs of a K-tile the other
  // reads its fragments of the K-tile and issues its half of the LDS-DMA of the K-tile two ahead,
  // so every SIMD always has one wave with MFMAs to issue (vcap_gemm256_kernel's stagger).
  // Group g stages LDS-DMA blocks 25 g .. 25 g + 24 of each K-tile (8 rows = 1 KiB each; token rows
  // 0-207 are blocks 0-25, weight rows blocks 26-49): wave wig of the group blocks wig + 4 i.
  const int wig = wave & 3;
  const int npg = wig == 0 ? NB_MAX : NB_MAX - 1;  // 7 / 6 / 6 / 6 = 25 pieces per group
  const char* src[NB_MAX];
#pragma unroll
  for (int i = 0; i < NB_MAX; ++i) {
    const int blk = min(25 * tgrp + wig + 4 * i, BLKS - 1);
    const int lr = blk * 8 + (lane >> 3);
    const int c = (lane & 7) ^ (lr & 7);
    const bf16_t* p;
    if (lr < RT) {
      p = xn + ((long)bt * N + min(lr, N - 1)) * D;
    } else {
      const int f = lr - RT;  // 0..191: q / k / v feature f & 63 of head h
      p = wqkv + ((long)(f >> 6) * D + h * 64 + (f & 63)) * D;
    }
    src[i] = (const char*)(p + c * 8);
  }
  auto stage = [&](int kt) {  // this wave's pieces of K-tile kt
    char* dst = smem + (kt % NSTAGE) * STAGE;
#pragma unroll
    for (int i = 0; i < NB_MAX; ++i)
      if (i < npg) glds16_attn(src[i] + kt * 128, dst + (25 * tgrp + wig + 4 * i) * 1024);
  };
  auto wait_tile = [&](bool older) {  // this wave's pieces of all but its latest staged K-tile
    if (npg == NB_MAX) qa_wait_older<true>(older);
    else qa_wait_older<false>(older);
  };

  f32x4 acc[3][7];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 7; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int nk = D / 64;
  stage(0);
  if (nk > 1) stage(1);
  wait_tile(nk > 1);
  qa_barrier();                      // K-tile 0 landed
  if (tgrp == 1) qa_barrier();       // group 1 runs one barrier behind
  for (int kt = 0; kt < nk; ++kt) {
    // ---- read phase: fragments of K-tile kt, this wave's pieces of K-tile kt + 2 (into the slot
    // of K-tile kt - 1, whose reads both groups finished before the last barrier)
    const char* Tb = smem + (kt % NSTAGE) * STAGE;
    const char* Wb = Tb + RT * 128;
    u32x4 wf[2][3], tf[2][7];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const int row = (fgrp * 3 + i) * 16 + fr;
        wf[s][i] = *reinterpret_cast<const u32x4*>(Wb + row * 128 + (((s * 4 + fg) ^ (row & 7)) << 4));
      }
#pragma unroll
      for (int j = 0; j < 7; ++j) {
        if (j < ntt) {
          const int row = (t0 + j) * 16 + fr;
          tf[s][j] = *reinterpret_cast<const u32x4*>(Tb + row * 128 + (((s * 4 + fg) ^ (row & 7)) << 4));
        }
      }
    }
    if (kt + 2 < nk) stage(kt + 2);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // fragments in registers before the barrier
    wait_tile(kt + 2 < nk);                             // this wave's pieces of K-tile kt + 1 landed
    qa_barrier();
    // ---- MFMA phase
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int j = 0; j < 7; ++j)
#pragma unroll
        for (int i = 0; i < 3; ++i)
          if (j < ntt) acc[i][j] = mfma_frag(wf[s][i], tf[s][j], acc[i][j], (bf16_t*)nullptr);
    __builtin_amdgcn_s_setprio(0);
    qa_barrier();
  }
  if (tgrp == 0) qa_barrier();       // balance group 1's extra barrier
  qa_barrier();                      // every wave's fragment reads done: the ring becomes the images

  char* Ks = smem;
  char* Vs = smem + RT * 128;
  char* Qs = smem + 2 * RT * 128;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int ft = fgrp * 3 + i, part = ft >> 2;        // 0 q, 1 k, 2 v
    const int d0 = (ft & 3) * 16 + 4 * fg;              // this lane's 4 features of the head
    const f32x4 bias = *reinterpret_cast<const f32x4*>(bqkv + part * D + h * 64 + d0);
    char* img = part == 0 ? Qs : (part == 1 ? Ks : Vs);
#pragma unroll
    for (int j = 0; j < 7; ++j) {
      if (j < ntt) {
        const int tok = (t0 + j) * 16 + fr;
        const f32x4 v = acc[i][j] + bias;
        const u32x2 p = (u32x2){pack_bf2(v.x, v.y), pack_bf2(v.z, v.w)};
        *reinterpret_cast<u32x2*>(img + tok * 128 + (((d0 >> 3) ^ (tok & 7)) << 4) + (d0 & 7) * 2) = p;
      }
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the images written before any wave reads them
  qa_barrier();

  constexpr int WAVES = 8, QT_MAX = 2;
  const int qtiles = cls_only ? 1 : (N + 15) / 16;
#pragma unroll
  for (int i = 0; i < QT_MAX; ++i) {
    const int qt = wave + i * WAVES;
    if (qt >= qtiles) break;
    u32x4 qf[2];
    const int qrow = qt * 16 + fr;  // rows past N hold row N - 1's q (clamped staging)
#pragma unroll
    for (int s = 0; s < 2; ++s)
      qf[s] = *reinterpret_cast<const u32x4*>(Qs + qrow * 128 + (((s * 4 + fg) ^ (qrow & 7)) << 4));
    f32x4 o[4];
    float inv;
    attn_bf16_qtile<14, 13>(Ks, Vs, qf, N, o, inv);
    const int q = qt * 16 + fr;
    const bool keep = q < N && (!cls_only || q == 0);
    const long row = cls_only ? (long)bt : (long)bt * N + q;
    attn_commit<false>(attn_pack<false>(o, inv, row, keep), out, D, h, nullptr, 0);
  }
}

// ------------------------------------------------------------------------------------------------
// The same fusion for the ViT-L/14 frame (257 tokens, 17 token tiles = 272 rows; configs[3]).  A
// 64-wide K-tile of 272 token + 192 weight rows is 58 KiB, so three whole slots (174 KiB) do not fit;
// the token rows keep three slots (102 KiB: they stream from the LayerNorm output once per head) and
// the weight rows - L2-resident, shared by every frame of the head - two (48 KiB), 150 KiB in all.
// The weight tile kt + 1 may only be written once both groups have read tile kt - 1 (its slot), i.e.
// from group 0's read phase kt on, and group 1 reads it one barrier after group 0: so group 0 (the
// leading group) stages every weight block, one K-tile ahead, and waits for them at the end of its MFMA
// phase; the token blocks go two K-tiles ahead, 5 of 34 per K-tile from group 0 and 29 from group 1
// (29 pieces per group: 8 / 7 / 7 / 7 per wave).  Arithmetic, K order, bias add and bf16 rounding are
// those of vcap_vit_qkv_attention_kernel, so the output is bit-identical to the unfused QKV GEMM +
// vcap_vit_attention_bf16_kernel<18, 17> pair.
namespace qb {
constexpr int TT = 17, FT = 12;                 // token tiles (272 tokens), feature tiles
constexpr int RT = TT * 16, RW = FT * 16;       // 272 token rows, 192 weight rows
constexpr int TSLOT = RT * 128, WSLOT = RW * 128;
constexpr int NTS = 3, NWS = 2;
constexpr int LDS = NTS * TSLOT + NWS * WSLOT;  // 153600 B
constexpr int TBLK = RT / 8, WBLK = RW / 8;     // 34 token, 24 weight blocks (8 rows = 1 KiB) per K-tile
constexpr int G0_TOK = TBLK - 29;               // token blocks of group 0 (29 .. 33)
constexpr int NB_MAX = 8;                       // pieces per wave: 8 (waves 0, 4), 7 (others)
}  // namespace qb

// s_waitcnt vmcnt(n) for a wave-uniform n in 0..8
VCAP_DEV void qb_vm_wait(int n) {
  switch (n) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    case 7: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
  }
}

__global__ __launch_bounds__(512) void vcap_vit_qkv_attention_l_kernel(const bf16_t* __restrict__ xn,
                                                                       const bf16_t* __restrict__ wqkv,
                                                                       const float* __restrict__ bqkv,
                                                                       bf16_t* __restrict__ out, int BT, int N, int H,
                                                                       int cls_only) {
  using namespace qb;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int D = H * 64;
  const int b = blockIdx.x;
  int bt, h;
  if ((BT & 7) == 0) {
    const int x = b & 7, j = b >> 3;
    bt = (j / H) * 8 + x;
    h = j - (j / H) * H;
  } else {
    bt = b / H;
    h = b - bt * H;
  }
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fg = lane >> 4;
  const int fgrp = wave & 3, tgrp = wave >> 2;
  const int t0 = tgrp * 9, ntt = tgrp ? TT - 9 : 9;
  char* const Tsl = smem;                     // token slots
  char* const Wsl = smem + NTS * TSLOT;       // weight slots

  // this wave's pieces: group-local block list 0..28, wave wig takes wig + 4 i; group 0's list is the
  // 24 weight blocks then token blocks 29..33, group 1's the token blocks 0..28
  const int wig = wave & 3;
  const int npc = wig == 0 ? NB_MAX : NB_MAX - 1;
  const int nw = tgrp == 0 ? WBLK / 4 : 0;  // weight pieces: group 0's list entries wig + 4 i < 24
  const int nt = npc - nw;
  const char* src[NB_MAX];
  int dsto[NB_MAX];  // byte offset within the token / weight slot
#pragma unroll
  for (int i = 0; i < NB_MAX; ++i) {
    const int li = min(wig + 4 * i, 28);
    const bool wblk = tgrp == 0 && li < WBLK;
    const int blk = wblk ? li : (tgrp == 0 ? (TBLK - G0_TOK) + (li - WBLK) : li);  // group 0: tokens 29..33
    const int lr = blk * 8 + (lane >> 3);       // row within its region
    const int c = (lane & 7) ^ (lr & 7);
    const bf16_t* p;
    if (!wblk) {
      p = xn + ((long)bt * N + min(lr, N - 1)) * D;
    } else {
      const int f = lr;  // 0..191: q / k / v feature f & 63 of head h
      p = wqkv + ((long)(f >> 6) * D + h * 64 + (f & 63)) * D;
    }
    src[i] = (const char*)(p + c * 8);
    dsto[i] = blk * 1024;
  }
  auto stage_w = [&](int kt) {  // group 0: this wave's weight pieces of K-tile kt
    char* dst = Wsl + (kt % NWS) * WSLOT;
#pragma unroll
    for (int i = 0; i < NB_MAX; ++i)
      if (i < nw) glds16_attn(src[i] + kt * 128, dst + dsto[i]);
  };
  auto stage_t = [&](int kt) {  // this wave's token pieces of K-tile kt
    char* dst = Tsl + (kt % NTS) * TSLOT;
#pragma unroll
    for (int i = 0; i < NB_MAX; ++i)
      if (i >= nw && i < npc) glds16_attn(src[i] + kt * 128, dst + dsto[i]);
  };

  f32x4 acc[3][9];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 9; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int nk = D / 64;
  stage_w(0);
  stage_t(0);
  if (nk > 1) stage_t(1);
  qb_vm_wait(nk > 1 ? nt : 0);       // K-tile 0 landed (tile 1's token pieces may still fly)
  qa_barrier();
  if (tgrp == 1) qa_barrier();       // group 1 runs one barrier behind
  for (int kt = 0; kt < nk; ++kt) {
    // ---- read phase: fragments of K-tile kt; group 0 stages the weights of kt + 1 (the slot of
    // kt - 1, read by both groups before the last barrier), every wave its token pieces of kt + 2
    const char* Tb = Tsl + (kt % NTS) * TSLOT;
    const char* Wb = Wsl + (kt % NWS) * WSLOT;
    u32x4 wf[2][3], tf[2][9];
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const int row = (fgrp * 3 + i) * 16 + fr;
        wf[s2][i] = *reinterpret_cast<const u32x4*>(Wb + row * 128 + (((s2 * 4 + fg) ^ (row & 7)) << 4));
      }
#pragma unroll
      for (int j = 0; j < 9; ++j) {
        if (j < ntt) {
          const int row = (t0 + j) * 16 + fr;
          tf[s2][j] = *reinterpret_cast<const u32x4*>(Tb + row * 128 + (((s2 * 4 + fg) ^ (row & 7)) << 4));
        }
      }
    }
    const int w_now = kt + 1 < nk ? nw : 0, t_now = kt + 2 < nk ? nt : 0;
    if (w_now) stage_w(kt + 1);
    if (t_now) stage_t(kt + 2);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // fragments in registers before the barrier
    qb_vm_wait(w_now + t_now);                          // all but this phase's pieces: tokens of kt + 1
    qa_barrier();
    // ---- MFMA phase
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int j = 0; j < 9; ++j)
#pragma unroll
        for (int i = 0; i < 3; ++i)
          if (j < ntt) acc[i][j] = mfma_frag(wf[s2][i], tf[s2][j], acc[i][j], (bf16_t*)nullptr);
    __builtin_amdgcn_s_setprio(0);
    if (w_now) qb_vm_wait(t_now);  // group 0: the weights of kt + 1 landed before group 1 reads them
    qa_barrier();
  }
  if (tgrp == 0) qa_barrier();       // balance group 1's extra barrier
  qa_barrier();                      // every wave's fragment reads done: the token slots become the images

  char* Ks = smem;
  char* Vs = smem + RT * 128;
  char* Qs = smem + 2 * RT * 128;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int ft = fgrp * 3 + i, part = ft >> 2;        // 0 q, 1 k, 2 v
    const int d0 = (ft & 3) * 16 + 4 * fg;
    const f32x4 bias = *reinterpret_cast<const f32x4*>(bqkv + part * D + h * 64 + d0);
    char* img = part == 0 ? Qs : (part == 1 ? Ks : Vs);
#pragma unroll
    for (int j = 0; j < 9; ++j) {
      if (j < ntt) {
        const int tok = (t0 + j) * 16 + fr;
        const f32x4 v = acc[i][j] + bias;
        const u32x2 pk = (u32x2){pack_bf2(v.x, v.y), pack_bf2(v.z, v.w)};
        *reinterpret_cast<u32x2*>(img + tok * 128 + (((d0 >> 3) ^ (tok & 7)) << 4) + (d0 & 7) * 2) = pk;
      }
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  qa_barrier();

  constexpr int WAVES = 8, QT_MAX = 3;
  const int qtiles = cls_only ? 1 : (N + 15) / 16;
#pragma unroll
  for (int i = 0; i < QT_MAX; ++i) {
    const int qt = wave + i * WAVES;
    if (qt >= qtiles) break;
    u32x4 qf[2];
    const int qrow = qt * 16 + fr;
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
      qf[s2] = *reinterpret_cast<const u32x4*>(Qs + qrow * 128 + (((s2 * 4 + fg) ^ (qrow & 7)) << 4));
    f32x4 o[4];
    float inv;
    attn_bf16_qtile<18, 17>(Ks, Vs, qf, N, o, inv);
    const int q = qt * 16 + fr;
    const bool keep = q < N && (!cls_only || q == 0);
    const long row = cls_only ? (long)bt : (long)bt * N + q;
    attn_commit<false>(attn_pack<false>(o, inv, row, keep), out, D, h, nullptr, 0);
  }
}

bool vcap_vit_qkv_attention_supported(int dt, int N, int H) {
  return dt == VCAP_DT_BF16 && ((N > 12 * 16 && N <= 13 * 16) || (N > 16 * 16 && N <= 17 * 16)) && H > 0 &&
         H * 64 <= 4096;
}

hipError_t vcap_vit_qkv_attention_dispatch(const void* xn, const void* wqkv, const float* bqkv, void* out, int BT,
                                           int N, int H, int cls_only, hipStream_t s) {
  if (!vcap_vit_qkv_attention_supported(VCAP_DT_BF16, N, H) || BT <= 0 || !bqkv) return hipErrorInvalidValue;
  if (N > 13 * 16) {  // ViT-L/14: 17 token tiles
    static bool configured_l = false;
    if (!configured_l) {
      hipError_t e = hipFuncSetAttribute((const void*)vcap_vit_qkv_attention_l_kernel,
                                         hipFuncAttributeMaxDynamicSharedMemorySize, qb::LDS);
      if (e != hipSuccess) return e;
      configured_l = true;
    }
    hipLaunchKernelGGL(vcap_vit_qkv_attention_l_kernel, dim3(BT * H), dim3(512), qb::LDS, s, (const bf16_t*)xn,
                       (const bf16_t*)wqkv, bqkv, (bf16_t*)out, BT, N, H, cls_only);
    return hipGetLastError();
  }
  static bool configured = false;
  if (!configured) {
    hipError_t e = hipFuncSetAttribute((const void*)vcap_vit_qkv_attention_kernel,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, qa::LDS);
    if (e != hipSuccess) return e;
    configured = true;
  }
  hipLaunchKernelGGL(vcap_vit_qkv_attention_kernel, dim3(BT * H), dim3(512), qa::LDS, s, (const bf16_t*)xn,
                     (const bf16_t*)wqkv, bqkv, (bf16_t*)out, BT, N, H, cls_only);
  return hipGetLastError();
}

// bf16 kernel choice by padded key count; KE = key tiles that can hold real keys
template <bool MXO>
static hipError_t attn_bf16_dispatch(const void* qkv, void* out, uint8_t* oscale, int BT, int N, int H,
                                     int cls_only, hipStream_t s) {
  switch (((N + 31) / 32) * 2) {  // keys padded to a multiple of 32
    case 2: return launch_attn_bf16<2, 2, 4, MXO>(qkv, out, BT, N, H, oscale, cls_only, s);
    case 14:
      if (N <= 13 * 16) return launch_attn_bf16<14, 13, 8, MXO>(qkv, out, BT, N, H, oscale, cls_only, s);
      return launch_attn_bf16<14, 14, 8, MXO>(qkv, out, BT, N, H, oscale, cls_only, s);
    case 18:
      if (N <= 17 * 16) return launch_attn_bf16<18, 17, 8, MXO>(qkv, out, BT, N, H, oscale, cls_only, s);
      return launch_attn_bf16<18, 18, 8, MXO>(qkv, out, BT, N, H, oscale, cls_only, s);
    default: return hipErrorInvalidValue;
  }
}

hipError_t vcap_vit_attention_dispatch(int dt, const void* qkv, void* out, int BT, int N, int H, hipStream_t s,
                                       int cls_only) {
  if (N <= 0 || N > 288) return hipErrorInvalidValue;
  if (dt == VCAP_DT_BF16) return attn_bf16_dispatch<false>(qkv, out, nullptr, BT, N, H, cls_only, s);
  switch (((N + 31) / 32) * 2) {
    case 2: return launch_attn<float, 2>(qkv, out, BT, N, H, cls_only, s);
    case 14: return launch_attn<float, 14>(qkv, out, BT, N, H, cls_only, s);
    case 18: return launch_attn<float, 18>(qkv, out, BT, N, H, cls_only, s);
    default: return hipErrorInvalidValue;
  }
}

// bf16 q/k/v -> MXFP8 attention output (+ scales) for the MXFP8 attn-proj GEMM
hipError_t vcap_vit_attention_mx_dispatch(const void* qkv, void* out, uint8_t* oscale, int BT, int N, int H,
                                          hipStream_t s, int cls_only) {
  if (N <= 0 || N > 288 || !oscale) return hipErrorInvalidValue;
  return attn_bf16_dispatch<true>(qkv, out, oscale, BT, N, H, cls_only, s);
}
