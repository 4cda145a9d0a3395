// Shared device helpers for the vcap HIP kernels (gfx950 / CDNA4, wave64).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define VCAP_DEV __device__ __forceinline__

typedef uint16_t bf16_t;
typedef __attribute__((ext_vector_type(8))) short bf16x8;   // MFMA 16x16x32 bf16 A/B fragment
typedef __attribute__((ext_vector_type(4))) float f32x4;    // MFMA 16x16 accumulator / f32 fragment
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
typedef __attribute__((ext_vector_type(2))) unsigned int u32x2;

VCAP_DEV float bf2f(bf16_t h) { return __uint_as_float(((uint32_t)h) << 16); }

VCAP_DEV bf16_t f2bf(float f) {
  // round-to-nearest-even; inputs here are finite activations/weights
  uint32_t u = __float_as_uint(f);
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (bf16_t)(u >> 16);
}

// two f32 -> packed bf16x2 (round-to-nearest-even): the vector conversion selects one
// v_cvt_pk_bf16_f32 on gfx950.  (Not inline asm: the hazard recognizer does not check an asm's
// VGPR operands against MFMAs in flight, so an asm def could land on an MFMA's source-C registers.)
typedef __attribute__((ext_vector_type(2))) float f32x2_;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;
VCAP_DEV uint32_t pack_bf2(float lo, float hi) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_){lo, hi}, bf16x2_t));
}

template <typename T> struct Num;
template <> struct Num<float> {
  static VCAP_DEV float to_f(float v) { return v; }
  static VCAP_DEV float from_f(float v) { return v; }
};
template <> struct Num<bf16_t> {
  static VCAP_DEV float to_f(bf16_t v) { return bf2f(v); }
  static VCAP_DEV bf16_t from_f(float v) { return f2bf(v); }
};

// LayerNorm arithmetic of the decode kernels in ONE fixed operation order.  Left to
// -ffp-contract, `a*a + b*b` may become fma(a, a, b*b) in one kernel and fma(b, b, a*a) in another,
// so kernels normalising the same rows (the launch chain's GEMV prologues, the lm_head stream
// kernel, the persistent decode) could differ by an ulp of rstd - enough to flip a bf16 rounding
// now and then.  Written with explicit fmas, no multiply is left feeding an add, so there is
// nothing for contraction to choose (a `#pragma clang fp contract(off)` form measured 4 us per
// decode step slower: it also kept the affine step from packed f32 math).
VCAP_DEV float sumsq4(f32x4 d) { return fmaf(d.x, d.x, d.y * d.y) + fmaf(d.z, d.z, d.w * d.w); }
VCAP_DEV f32x4 ln_affine4(f32x4 x, float mean, float rstd, f32x4 g, f32x4 b) {
  return __builtin_elementwise_fma((x - mean) * rstd, g, b);
}

// tanh-approximate GELU, the form both torch's GELU(approximate="tanh")
// (ViT MLP, src/models/video_encoder.py:123-134) and HF gelu_new (GPT-2 MLP) compute.
// 0.5 x (1 + tanh(u)) == x * sigmoid(2u): one v_exp_f32 + one reciprocal instead of the
// device-library tanhf (|error| ~1e-7 relative, far below the bf16 output rounding and the
// fp32-mode tolerances).  exp overflow for very negative u gives x / inf = -0, the exact limit.
// Raw v_exp_f32 (2^x) and v_rcp_f32 (1 ulp each), with -2*log2(e)*sqrt(2/pi) folded into the
// cubic: 7 VALU ops per element instead of a tanhf call or an IEEE divide sequence.
VCAP_DEV float gelu_tanh(float x) {
  const float a0 = -2.0f * 1.4426950408889634f * 0.7978845608028654f;  // -2 log2(e) sqrt(2/pi)
  const float a1 = a0 * 0.044715f;
  const float e = __builtin_amdgcn_exp2f(x * fmaf(a1, x * x, a0));  // exp(-2u)
  return x * __builtin_amdgcn_rcpf(1.0f + e);
}

// The same GELU on 4 lanes' worth of a GEMM epilogue vector: the polynomial, the +1 and the
// final product as packed-f32 VALU ops (v_pk_mul_f32 / v_pk_fma_f32 / v_pk_add_f32, two
// elements per instruction), only v_exp_f32 / v_rcp_f32 per element.  Same operations in the
// same order per element as gelu_tanh (fma contraction included), so the results are identical.
typedef __attribute__((ext_vector_type(2))) float f32x2;
VCAP_DEV f32x2 pk_fma(f32x2 a, f32x2 b, f32x2 c) { return __builtin_elementwise_fma(a, b, c); }
VCAP_DEV f32x4 gelu_tanh4(f32x4 v) {
  const float a0 = -2.0f * 1.4426950408889634f * 0.7978845608028654f;
  const float a1 = a0 * 0.044715f;
  f32x4 out;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const f32x2 x = h ? (f32x2){v.z, v.w} : (f32x2){v.x, v.y};
    const f32x2 t = pk_fma((f32x2){a1, a1}, x * x, (f32x2){a0, a0});
    const f32x2 y = x * t;
    const f32x2 d = (f32x2){1.0f, 1.0f} + (f32x2){__builtin_amdgcn_exp2f(y.x), __builtin_amdgcn_exp2f(y.y)};
    const f32x2 r = x * (f32x2){__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
    if (h) {
      out.z = r.x;
      out.w = r.y;
    } else {
      out.x = r.x;
      out.y = r.y;
    }
  }
  return out;
}

// Cross-lane reductions on the VALU: DPP within 16-lane rows, then the gfx950 permlane16/32
// swaps across rows.  (__shfl_xor lowers to ds_bpermute, an LDS round trip of ~100+ cycles per
// step; a 6-step butterfly of those serialises ~700 cycles per reduction.)
template <int CTRL>
VCAP_DEV float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
template <int CTRL>
VCAP_DEV int dpp_i(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false);
}
constexpr int DPP_XOR1 = 0xB1, DPP_XOR2 = 0x4E, DPP_HALF_MIRROR = 0x141, DPP_MIRROR = 0x140;

// partner value across 16-lane rows (lane ^ 16) and across wave halves (lane ^ 32)
VCAP_DEV float xor16_f(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float((threadIdx.x & 16) ? r[0] : r[1]);
}
VCAP_DEV float xor32_f(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float((threadIdx.x & 32) ? r[0] : r[1]);
}
VCAP_DEV int xor16_i(int v) {
  const auto r = __builtin_amdgcn_permlane16_swap((unsigned)v, (unsigned)v, false, false);
  return (int)((threadIdx.x & 16) ? r[0] : r[1]);
}
VCAP_DEV int xor32_i(int v) {
  const auto r = __builtin_amdgcn_permlane32_swap((unsigned)v, (unsigned)v, false, false);
  return (int)((threadIdx.x & 32) ? r[0] : r[1]);
}

// 4x4 transpose of dwords across the lane groups {l, l^16, l^32, l^48} (same position in every
// 16-lane row): on return, lane group g holds (x[0], x[1], x[2], x[3]) of groups 0, 1, 2, 3 as
// they were in slot g.  Two butterfly stages, each lane exchanging its "receive" slot of every
// slot pair with the partner group (v_permlane16_swap, then v_permlane32_swap).
VCAP_DEV void transpose4_groups(uint32_t (&x)[4]) {
  const int g = (threadIdx.x >> 4) & 3;
#pragma unroll
  for (int base = 0; base < 4; base += 2) {  // stage 1: pairs (0,1), (2,3) with group g ^ 1
    const bool lo = g & 1;                   // receive slot: the one whose bit 0 differs from g's
    const uint32_t r = (uint32_t)xor16_i((int)(lo ? x[base] : x[base + 1]));
    if (lo) x[base] = r; else x[base + 1] = r;
  }
#pragma unroll
  for (int k = 0; k < 2; ++k) {  // stage 2: pairs (0,2), (1,3) with group g ^ 2
    const bool lo = g & 2;
    const uint32_t r = (uint32_t)xor32_i((int)(lo ? x[k] : x[k + 2]));
    if (lo) x[k] = r; else x[k + 2] = r;
  }
}

VCAP_DEV float row16_sum(float v) {
  v += dpp_f<DPP_XOR1>(v);
  v += dpp_f<DPP_XOR2>(v);
  v += dpp_f<DPP_HALF_MIRROR>(v);
  v += dpp_f<DPP_MIRROR>(v);
  return v;
}
VCAP_DEV float row16_max(float v) {
  v = fmaxf(v, dpp_f<DPP_XOR1>(v));
  v = fmaxf(v, dpp_f<DPP_XOR2>(v));
  v = fmaxf(v, dpp_f<DPP_HALF_MIRROR>(v));
  v = fmaxf(v, dpp_f<DPP_MIRROR>(v));
  return v;
}
// sum / max over the 4 lanes {l, l^16, l^32, l^48} (same position in every row)
VCAP_DEV float rows_sum(float v) {
  v += xor16_f(v);
  return v + xor32_f(v);
}
VCAP_DEV float rows_max(float v) {
  v = fmaxf(v, xor16_f(v));
  return fmaxf(v, xor32_f(v));
}
VCAP_DEV float wave_sum(float v) { return rows_sum(row16_sum(v)); }
VCAP_DEV float wave_max(float v) { return rows_max(row16_max(v)); }

// (value, index) argmax over the wave; ties resolve to the smallest index (torch.argmax order)
VCAP_DEV void argmax_take(float& bv, int& bi, float ov, int oi) {
  // bitwise, not short-circuit: `||` / `&&` here compiled to exec-mask branches (~14 scalar and
  // vector instructions per take instead of 3 compares + 2 selects)
  const bool t = (ov > bv) | ((ov == bv) & (oi < bi));
  bv = t ? ov : bv;
  bi = t ? oi : bi;
}
VCAP_DEV void wave_argmax(float& bv, int& bi) {
  argmax_take(bv, bi, dpp_f<DPP_XOR1>(bv), dpp_i<DPP_XOR1>(bi));
  argmax_take(bv, bi, dpp_f<DPP_XOR2>(bv), dpp_i<DPP_XOR2>(bi));
  argmax_take(bv, bi, dpp_f<DPP_HALF_MIRROR>(bv), dpp_i<DPP_HALF_MIRROR>(bi));
  argmax_take(bv, bi, dpp_f<DPP_MIRROR>(bv), dpp_i<DPP_MIRROR>(bi));
  argmax_take(bv, bi, xor16_f(bv), xor16_i(bi));
  argmax_take(bv, bi, xor32_f(bv), xor32_i(bi));
}

// MFMA wrappers. Both consume one 16-byte fragment per lane per call group:
//  bf16: lane l holds A[l&15][8(l>>4)+j], B[8(l>>4)+j][l&15], j=0..7 (one 16x16x32)
//  f32 : lane l holds A[l&15][4(l>>4)+i], B[4(l>>4)+i][l&15], i=0..3 as FOUR 16x16x4
//        calls (call i uses element i: k index 4g+i for lane group g; the k order is a
//        permutation applied identically to A and B, so the sum is exact f32 FMA chain).
VCAP_DEV f32x4 mfma_frag(const u32x4& a, const u32x4& b, f32x4 c, bf16_t*) {
  bf16x8 av = __builtin_bit_cast(bf16x8, a);
  bf16x8 bv = __builtin_bit_cast(bf16x8, b);
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, c, 0, 0, 0);
}
VCAP_DEV f32x4 mfma_frag(const u32x4& a, const u32x4& b, f32x4 c, float*) {
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.x), __uint_as_float(b.x), c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.y), __uint_as_float(b.y), c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.z), __uint_as_float(b.z), c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.w), __uint_as_float(b.w), c, 0, 0, 0);
  return c;
}

// ---- MXFP8: OCP e4m3fn elements with one E8M0 (power-of-two) scale per 32 consecutive K
// elements of a row, the gfx950-native block-scaled format the v_mfma_scale_f32_16x16x128_f8f6f4
// instruction consumes at twice the bf16 MFMA rate.  Element value = fp8 * 2^(scale - 127).
// Scales are stored in the order the 256x256 GEMM consumes them: per (128-wide K-tile, group of
// 256 rows) one contiguous 1 KiB block laid out [k-block 0..3][row % 16][row / 16 (0..15)], so a
// workgroup stages a K-tile's scales for its 256 rows with one 4-byte LDS-DMA per thread and a
// lane reads the scales of its 4 row sub-tiles (one per MFMA, picked by OPSEL) in one ds_read.
VCAP_DEV long mx_scale_index(int row, int k, int groups) {
  return ((long)((k >> 7) * groups + (row >> 8)) * 4 + ((k >> 5) & 3)) * 256 + (row & 15) * 16 + ((row >> 4) & 15);
}
typedef uint8_t fp8_t;
typedef __attribute__((ext_vector_type(8))) int i32x8;
typedef __attribute__((ext_vector_type(8))) unsigned int u32x8;

VCAP_DEV u32x8 cat8(const u32x4& lo, const u32x4& hi) {
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}
VCAP_DEV u32x4 lo4(const u32x8& v) { return __builtin_shufflevector(v, v, 0, 1, 2, 3); }
VCAP_DEV u32x4 hi4(const u32x8& v) { return __builtin_shufflevector(v, v, 4, 5, 6, 7); }

// E8M0 scale of a 32-block from its max |x|: 2^(floor(log2 amax) - 7), so every scaled element
// lies in (-256, 256) - inside e4m3's 448 range, no saturation - and the block max keeps e4m3's
// full 3-bit mantissa.  amax == 0 (or subnormal) gives the smallest scale.
VCAP_DEV int mx_scale_byte(float amax) {
  const int e = (int)((__float_as_uint(amax) >> 23) & 0xFF) - 7;
  return e < 0 ? 0 : e;  // finite amax: e <= 247
}
// 2^-(scale - 127) as an f32 multiplier (exact power of two; exponent field 254 - byte >= 7)
VCAP_DEV float mx_inv_scale(int byte) { return __uint_as_float((uint32_t)(254 - byte) << 23); }

// four f32 (already multiplied by the inverse scale) -> four e4m3 bytes, round-to-nearest-even
VCAP_DEV uint32_t pack_fp8x4(float a, float b, float c, float d) {
  int r = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
  r = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, r, true);
  return (uint32_t)r;
}

// D += (A * 2^(sa-127)) . (B * 2^(sb-127)) over K = 128.  Operand layout (measured on gfx950,
// tools/mx_layout_probe.hip): lane l holds row / column (l & 15), K elements [16 g, +16) in its
// bytes 0-15 and [64 + 16 g, +16) in bytes 16-31 (g = l >> 4); the scale in byte SA / SB of
// lane l's sa / sb applies to K block [32 g, +32) of row / column (l & 15).
//
// Issued as inline asm with the accumulator tied ("+v"): the builtin's register allocation does
// not keep D == C for this instruction, and in the 256x256 GEMM (128 accumulator registers)
// that turns into hundreds of spills.  The compiler's hazard recognizer cannot see inside the
// asm, so callers put >= 2 wait states between VALU writes of the operands and the MFMA and
// >= 18 between the last MFMA and VALU reads of its result (mfma_mx_drain()).
template <int SA, int SB>
VCAP_DEV void mfma_mx(const u32x8& a, int sa, const u32x8& b, int sb, f32x4& c);
#define VCAP_MX_SPEC(SA, SB, A0, A1, B0, B1)                                                         \
  template <>                                                                                       \
  VCAP_DEV void mfma_mx<SA, SB>(const u32x8& a, int sa, const u32x8& b, int sb, f32x4& c) {         \
    asm volatile("v_mfma_scale_f32_16x16x128_f8f6f4 %0, %1, %2, %0, %3, %4 op_sel:[" #A0 "," #B0     \
                 ",0] op_sel_hi:[" #A1 "," #B1 ",0]"                                                \
                 : "+v"(c)                                                                          \
                 : "v"(a), "v"(b), "v"(sa), "v"(sb));                                               \
  }
#define VCAP_MX_ROW(SA, A0, A1)             \
  VCAP_MX_SPEC(SA, 0, A0, A1, 0, 0)         \
  VCAP_MX_SPEC(SA, 1, A0, A1, 1, 0)         \
  VCAP_MX_SPEC(SA, 2, A0, A1, 0, 1)         \
  VCAP_MX_SPEC(SA, 3, A0, A1, 1, 1)
VCAP_MX_ROW(0, 0, 0)
VCAP_MX_ROW(1, 1, 0)
VCAP_MX_ROW(2, 0, 1)
VCAP_MX_ROW(3, 1, 1)
#undef VCAP_MX_ROW
#undef VCAP_MX_SPEC
// Quantise 4 consecutive f32 (columns c..c+3 of `row`) held by lanes in groups of 8 (one 32-block
// per 8 lanes, lane-contiguous): block max |x| by DPP within the 8 lanes, E8M0 scale, 4 e4m3 bytes.
// Every lane of the wave must be active.
VCAP_DEV void mx_quant_store4(f32x4 o, int row, int c, fp8_t* yrow, uint8_t* scales, int groups) {
  float amax = fmaxf(fmaxf(fabsf(o.x), fabsf(o.y)), fmaxf(fabsf(o.z), fabsf(o.w)));
  amax = fmaxf(amax, dpp_f<DPP_XOR1>(amax));
  amax = fmaxf(amax, dpp_f<DPP_XOR2>(amax));
  amax = fmaxf(amax, dpp_f<DPP_HALF_MIRROR>(amax));
  const int sb = mx_scale_byte(amax);
  const float inv = mx_inv_scale(sb);
  *reinterpret_cast<uint32_t*>(yrow + c) = pack_fp8x4(o.x * inv, o.y * inv, o.z * inv, o.w * inv);
  if ((threadIdx.x & 7) == 0) scales[mx_scale_index(row, c, groups)] = (uint8_t)sb;
}

VCAP_DEV void mfma_mx_drain() { asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory"); }

// elements of T per 16-byte fragment chunk
template <typename T> struct Frag { static constexpr int kElems = 16 / sizeof(T); };

#ifndef VCAP_H_
enum { VCAP_DT_F32 = 0, VCAP_DT_BF16 = 1, VCAP_DT_MXFP8 = 2 };  // mirrors include/vcap.h
#endif
