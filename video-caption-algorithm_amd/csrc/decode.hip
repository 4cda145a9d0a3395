// GPT-2 decoder step kernels with a paged KV cache and on-device greedy logits processing.
//
// Replaces the arithmetic of HF GPT2LMHeadModel.generate as the reference calls it
// (src/models/text_decoder.py:131-144) and the benchmark's raw greedy loop
// (core/scripts/benchmark_baseline.py:160-240):
//   per layer: h += c_proj(attn(ln_1(h)));  h += mlp_c_proj(gelu_new(c_fc(ln_2(h))))
//   then logits = ln_f(h) . wte^T, RepetitionPenalty -> NoRepeatNGram -> MinNewTokens -> argmax.
//
// Rows: M = B*S_new rows per step (S_new = prefix+prompt length at prefill, 1 while decoding).
// Every projection is a skinny MFMA GEMM: a workgroup of 4 waves owns NTB 16-column tiles for
// all M rows and splits K over its waves; partial tiles are summed through LDS.  LayerNorm is
// fused into the A-operand prologue (each workgroup recomputes the M row statistics from the
// L2-resident residual stream instead of paying a launch + round trip).
//
// Weights are stored "rows-packed" (vcap_rows_pack): for n-tile t (16 output features) and K
// slab g (one MFMA K step: 32 bf16 / 16 f32), the 64 lanes' B fragments are 1 KiB contiguous,
//   packed[(t * (K/KS) + g) * 64 + lane] (16 B) = W[16t + (lane & 15)][KS*g + E*(lane >> 4) ...+E)
// so every weight load is one fully coalesced 1 KiB wave instruction and a wave's whole K range
// of a tile is one contiguous run (rows >= N are zero).
#include "vcap_common.h"
// Weight fragments, nontemporal: nt keeps the decode's 247 MB per token step from evicting the
// concurrently running encode's operand tiles (plain loads: encode stage +2 %, bench -2 %,
// profiles/r02_decode_experiments.txt).  Two address forms, chosen per kernel by measurement
// (profiles/r03_decode_load_form_ab.txt): flat global loads for the one-row-tile GEMV (MT = 1:
// GPT-2-medium step 644 -> 564 us at 8 rows, beam 4 x 4 731 -> 651 us; GPT-2 small unchanged) and
// buffer loads (SGPR base + one 32-bit VGPR offset) for the 32-row GEMV and the prefill kernel
// (medium beam 8 x 4 930 vs 950 us flat, prefill 20-60 us faster).  Buffer-load policy bits on
// gfx950: 1 = sc0, 2 = nt, 16 = sc1.
template <int AUX = 0>
__device__ __forceinline__ u32x4 vcap_buf_load16(const void* base, long off_bytes) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0x7FFFFFFF, 0x00020000);
  return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)off_bytes, 0, AUX));
}
template <bool FLAT>
__device__ __forceinline__ u32x4 vcap_dec_wload(const void* base, const void* p) {
  if constexpr (FLAT) return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
  else return vcap_buf_load16<2>(base, (const char*)p - (const char*)base);
}
// The GEMV's activation / LayerNorm operands: buffer loads, default policy (flat: GPT-2 small
// 260 -> 263 us per step).
__device__ __forceinline__ u32x4 vcap_dec_aload(const void* base, long off_bytes) {
  return vcap_buf_load16(base, off_bytes);
}
#include "vcap_kernels.h"

#include <algorithm>
#include <cstdlib>

// ------------------------------------------------------------------------------------------------
// Weight packing (one-time, at model load).
template <typename T>
__global__ __launch_bounds__(256) void vcap_rows_pack_kernel(const T* __restrict__ w, long ldw, int N, int K,
                                                             u32x4* __restrict__ packed) {
  constexpr int E = Frag<T>::kElems, KS = 4 * E;
  const int nslab = K / KS;
  const long total = (long)((N + 15) / 16) * nslab * 64;
  for (long c = blockIdx.x * 256L + threadIdx.x; c < total; c += (long)gridDim.x * 256L) {
    const int lane = (int)(c & 63);
    const long tg = c >> 6;
    const int g = (int)(tg % nslab);
    const long row = (tg / nslab) * 16 + (lane & 15);
    u32x4 v = (u32x4){0u, 0u, 0u, 0u};
    if (row < N) v = *reinterpret_cast<const u32x4*>(w + row * ldw + g * KS + (lane >> 4) * E);
    packed[c] = v;
  }
}

VCAP_DEV const u32x4* packed_frag(const void* w, int tile, int nslab, int slab, int lane) {
  return reinterpret_cast<const u32x4*>(w) + ((long)tile * nslab + slab) * 64 + lane;
}

// ------------------------------------------------------------------------------------------------
// Shared epilogue of the rows kernels: split-K partial tiles (red[wave]) -> role output.
// pre_bias/pre_res were loaded at kernel start; s_rep/s_ban flag the processors' tokens that fall
// in this workgroup's column range.
template <typename T, int MT, int NTB, int EPI>
VCAP_DEV void rows_epilogue(const RowsGemmArgs& a, int m0, const float (*red)[MT * NTB * 256], const float* pre_bias,
                            const float* pre_res, float (*lg)[NTB * 16], const unsigned char (*s_rep)[NTB * 16],
                            const unsigned char (*s_ban)[NTB * 16], int n0, int hsel = -1) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int M = a.M, N = a.N;
  const int row = tid >> 4, col = tid & 15;
  // half-tile workgroup (hsel 0 / 1): only the 8 columns it computed are real
  const bool mine = hsel < 0 || (col >> 3) == hsel;
#pragma unroll
  for (int q = 0; q < MT * NTB; ++q) {
    const int e = tid + q * 256;
    const int i = q / NTB, j = q % NTB;
    const int ml = i * 16 + row, m = m0 + ml, n = n0 + j * 16 + col;
    const bool ok = (m < M) && (n < N);
    const float v = (red[0][e] + red[1][e]) + (red[2][e] + red[3][e]) + pre_bias[q];
    if constexpr (EPI == EPI_QKV) {
      if (ok) {
        const int Ed = N / 3;
        const int which = n / Ed, within_e = n - which * Ed;
        if (which == 0) {
          ((T*)a.q_out)[(long)m * Ed + within_e] = Num<T>::from_f(v);
        } else {
          const int head = within_e >> 6, d = within_e & 63;
          const int seq = m / a.S_new, pos = a.past + (m - seq * a.S_new);
          // contiguous per-sequence pages (identity table) unless an explicit table is given
          const int page = a.page_table ? a.page_table[seq * a.maxp + (pos >> 4)] : seq * a.maxp + (pos >> 4);
          T* pool = (T*)(which == 1 ? a.kc : a.vc);
          pool[(((long)page * a.H + head) * 16 + (pos & 15)) * 64 + d] = Num<T>::from_f(v);
        }
      }
    } else if constexpr (EPI == EPI_RESID) {
      if (ok && mine) ((float*)a.out)[(long)m * a.ldo + n] = pre_res[q] + v;
    } else if constexpr (EPI == EPI_GELU) {
      if (ok) ((T*)a.out)[(long)m * a.ldo + n] = Num<T>::from_f(gelu_tanh(v));
    } else if constexpr (EPI == EPI_STORE) {
      if (ok) ((T*)a.out)[(long)m * a.ldo + n] = Num<T>::from_f(v);
    } else if constexpr (EPI == EPI_LSE) {
      if (m < M) {
        if (n < N) a.logits_raw[(long)m * N + n] = v;
        lg[ml][j * 16 + col] = n < N ? v : -INFINITY;
      }
    } else {  // EPI_LOGITS: RepetitionPenalty -> NoRepeatNGram -> MinNewTokens (HF processor order)
      if (m < M) {
        float sv = -INFINITY;
        if (n < N) {
          if (a.logits_raw) a.logits_raw[(long)m * N + n] = v;
          sv = v;
          if (s_rep[ml][j * 16 + col]) sv = sv < 0.f ? sv * a.rep_penalty : sv / a.rep_penalty;
          if (s_ban[ml][j * 16 + col]) sv = -INFINITY;
          if (n == a.eos && a.gen_len < a.min_new) sv = -INFINITY;
          if (a.proc_out) a.proc_out[(long)m * N + n] = sv;
        }
        lg[ml][j * 16 + col] = sv;
      }
    }
  }
  if constexpr (EPI == EPI_LSE) {
    // log_softmax statistics of this workgroup's columns: (max, sum exp(x - max)) per row
    __syncthreads();
    for (int ml = wave; ml < MT * 16 && m0 + ml < M; ml += 4) {
      float mx = -INFINITY;
      for (int c = lane; c < NTB * 16; c += 64) mx = fmaxf(mx, lg[ml][c]);
      mx = wave_max(mx);
      float sm = 0.f;
      for (int c = lane; c < NTB * 16; c += 64) sm += expf(lg[ml][c] - mx);
      sm = wave_sum(sm);
      if (lane == 0) {
        a.part_val[(long)(m0 + ml) * a.nblk + blockIdx.x] = mx;
        a.part_sum[(long)(m0 + ml) * a.nblk + blockIdx.x] = sm;
      }
    }
  }
  if constexpr (EPI == EPI_LOGITS) {
    __syncthreads();
    for (int ml = wave; ml < MT * 16 && m0 + ml < M; ml += 4) {
      float bv = -INFINITY;
      int bi = 0x7fffffff;
      for (int c = lane; c < NTB * 16; c += 64) argmax_take(bv, bi, lg[ml][c], n0 + c);
      wave_argmax(bv, bi);
      if (lane == 0) {
        a.part_val[(long)(m0 + ml) * a.nblk + blockIdx.x] = bv;
        a.part_idx[(long)(m0 + ml) * a.nblk + blockIdx.x] = bi;
      }
    }
  }
}

// Processor token flags for the logits epilogue: zero (kernel start), then mark after the loads.
template <int MP, int NTB>
VCAP_DEV void proc_flags_zero(unsigned char (*s_rep)[NTB * 16], unsigned char (*s_ban)[NTB * 16]) {
  for (int i = threadIdx.x; i < MP * NTB * 16; i += 256) {
    (&s_rep[0][0])[i] = 0;
    (&s_ban[0][0])[i] = 0;
  }
}

// History / ban-list tokens of the (m, t) pairs this thread owns (t < 64), loaded early.
template <int MT>
struct ProcToks {
  int h[MT * 4], b[MT * 4], nb[MT * 4];
  VCAP_DEV void load(const RowsGemmArgs& a, int m0) {
#pragma unroll
    for (int q = 0; q < MT * 4; ++q) {
      const int i = threadIdx.x + q * 256;
      const int m = min(m0 + (i >> 6), a.M - 1), t = min(i & 63, a.hist_ld - 1);
      h[q] = a.hist[m * a.hist_ld + t];
      b[q] = a.banned[m * a.hist_ld + t];
      nb[q] = a.nbanned[m];
    }
  }
  template <int NTB>
  VCAP_DEV void mark(const RowsGemmArgs& a, int m0, int n0, unsigned char (*s_rep)[NTB * 16],
                     unsigned char (*s_ban)[NTB * 16]) const {
#pragma unroll
    for (int q = 0; q < MT * 4; ++q) {
      const int i = threadIdx.x + q * 256;
      const int m = i >> 6, t = i & 63;  // m: row within the chunk
      if (m0 + m >= a.M) continue;
      const unsigned hc = (unsigned)(h[q] - n0), bc = (unsigned)(b[q] - n0);
      if (a.rep_penalty != 1.0f && t < a.gen_len && hc < (unsigned)(NTB * 16)) s_rep[m][hc] = 1;
      if (t < nb[q] && bc < (unsigned)(NTB * 16)) s_ban[m][bc] = 1;
    }
  }
};

// A 32-row PRO_DIRECT GEMV (two 16-row tiles) whose A fragments of both tiles would not fit beside
// its weight fragments (> 64 x 16 B per lane) keeps one row tile of A live at a time.
template <typename T, int MT, int NTB, int PRO, int NSL>
constexpr bool gemv_stream_a() {
  return PRO == PRO_DIRECT && MT == 2 && NSL * (NTB + MT) > 64;
}

// ------------------------------------------------------------------------------------------------
// One (row m, head h) item of causal decode attention over <= 64 cached positions in the
// contiguous page layout the runtime allocates (page of position j of sequence `seq` =
// seq * maxp + j / 16: page ids are computed, not loaded), on ONE wave: scores with lane = key,
// P.V with lane = (key group kg of 8, 8 consecutive dims d8), partial sums reduced over the 8 key
// groups by DPP + permlane swaps.  c64_issue issues every load of the item at once (q, the lane's
// K row, its 8 V rows: one memory round trip); c64_finish is the arithmetic, the ONE operation
// order of vcap_decode_attention_c64_kernel.
struct C64Loads {
  u32x4 q;      // 8 of the head's 64 query dims: chunk (lane & 7)
  u32x4 kv[8];  // K row of key min(lane, ctx - 1)
  u32x4 vv[8];  // V rows of keys it * 8 + kg (clamped), dims [d8, d8 + 8)
};

VCAP_DEV u32x4 c64_ld16(const bf16_t* base, long elem) { return *reinterpret_cast<const u32x4*>(base + elem); }

VCAP_DEV void c64_issue(C64Loads& L, const bf16_t* q, const bf16_t* kc, const bf16_t* vc, int maxp, int m, int h,
                        int H, int seq, int ctx) {
  const int lane = threadIdx.x & 63, kg = lane >> 3, d8 = (lane & 7) * 8;
  auto row_of = [&](int j) { return (((long)(seq * maxp + (j >> 4)) * H + h) * 16 + (j & 15)) * 64; };
  L.q = c64_ld16(q, (long)m * H * 64 + h * 64 + (lane & 7) * 8);
  const long kr = row_of(min(lane, ctx - 1));
#pragma unroll
  for (int c = 0; c < 8; ++c) L.kv[c] = c64_ld16(kc, kr + c * 8);
#pragma unroll
  for (int it = 0; it < 8; ++it) L.vv[it] = c64_ld16(vc, row_of(min(it * 8 + kg, ctx - 1)) + d8);
}

// s_q / s_p: this wave's 64 floats each of LDS; orow = out + m * E + h * 64
VCAP_DEV void c64_finish(const C64Loads& L, float* s_q, float* s_p, int ctx, bf16_t* orow) {
  const int lane = threadIdx.x & 63, kg = lane >> 3, d8 = (lane & 7) * 8;
  if (lane < 8) {
    const unsigned w4[4] = {L.q.x, L.q.y, L.q.z, L.q.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      s_q[lane * 8 + 2 * e] = bf2f((bf16_t)(w4[e] & 0xffff));
      s_q[lane * 8 + 2 * e + 1] = bf2f((bf16_t)(w4[e] >> 16));
    }
  }
  __builtin_amdgcn_wave_barrier();
  float sc = 0.f;
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    const bf16_t* ke = reinterpret_cast<const bf16_t*>(&L.kv[c]);
#pragma unroll
    for (int e = 0; e < 8; ++e) sc += s_q[c * 8 + e] * bf2f(ke[e]);
  }
  sc *= 0.125f;
  const bool live = lane < ctx;
  const float mx = wave_max(live ? sc : -INFINITY);
  const float p = live ? __expf(sc - mx) : 0.f;
  const float sum = wave_sum(p);
  s_p[lane] = p;
  __builtin_amdgcn_wave_barrier();
  float o[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) o[e] = 0.f;
#pragma unroll
  for (int it = 0; it < 8; ++it) {
    const int jj = it * 8 + kg;
    const float pj = jj < ctx ? s_p[jj] : 0.f;
    const unsigned w4[4] = {L.vv[it].x, L.vv[it].y, L.vv[it].z, L.vv[it].w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      o[2 * e] += pj * bf2f((bf16_t)(w4[e] & 0xffff));
      o[2 * e + 1] += pj * bf2f((bf16_t)(w4[e] >> 16));
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) o[e] = rows_sum(o[e] + dpp_f<0x128>(o[e]));
  if (kg == 0) {
    const float inv = 1.0f / sum;
    *reinterpret_cast<u32x4*>(orow + d8) =
        (u32x4){pack_bf2(o[0] * inv, o[1] * inv), pack_bf2(o[2] * inv, o[3] * inv),
                pack_bf2(o[4] * inv, o[5] * inv), pack_bf2(o[6] * inv, o[7] * inv)};
  }
}

// The f32 form (the f32 decoders): the same item on one wave with every load issued at once; the
// score sums dims 0..63 in order and the P.V sums run over the same key groups and DPP / permlane
// reduction as vcap_decode_attention_kernel<float>.
struct C64LoadsF {
  u32x4 q;       // 4 of the head's 64 query dims: chunk (lane & 15)
  u32x4 kv[16];  // K row of key min(lane, ctx - 1)
  u32x4 vv[8][2];  // V rows of keys it * 8 + kg (clamped), dims [d8, d8 + 8)
};

VCAP_DEV void c64f_issue(C64LoadsF& L, const float* q, const float* kc, const float* vc, int maxp, int m, int h,
                         int H, int seq, int ctx) {
  const int lane = threadIdx.x & 63, kg = lane >> 3, d8 = (lane & 7) * 8;
  auto row_of = [&](int j) { return (((long)(seq * maxp + (j >> 4)) * H + h) * 16 + (j & 15)) * 64; };
  auto ld = [](const float* base, long elem) { return *reinterpret_cast<const u32x4*>(base + elem); };
  L.q = ld(q, (long)m * H * 64 + h * 64 + (lane & 15) * 4);
  const long kr = row_of(min(lane, ctx - 1));
#pragma unroll
  for (int c = 0; c < 16; ++c) L.kv[c] = ld(kc, kr + c * 4);
#pragma unroll
  for (int it = 0; it < 8; ++it) {
    const long vr = row_of(min(it * 8 + kg, ctx - 1)) + d8;
    L.vv[it][0] = ld(vc, vr);
    L.vv[it][1] = ld(vc, vr + 4);
  }
}

VCAP_DEV void c64f_finish(const C64LoadsF& L, float* s_q, float* s_p, int ctx, float* orow) {
  const int lane = threadIdx.x & 63, kg = lane >> 3, d8 = (lane & 7) * 8;
  if (lane < 16) *reinterpret_cast<f32x4*>(s_q + lane * 4) = __builtin_bit_cast(f32x4, L.q);
  __builtin_amdgcn_wave_barrier();
  float sc = 0.f;
#pragma unroll
  for (int c = 0; c < 16; ++c) {
    const f32x4 k4 = __builtin_bit_cast(f32x4, L.kv[c]);
#pragma unroll
    for (int e = 0; e < 4; ++e) sc += s_q[c * 4 + e] * k4[e];
  }
  sc *= 0.125f;
  const bool live = lane < ctx;
  const float mx = wave_max(live ? sc : -INFINITY);
  const float p = live ? __expf(sc - mx) : 0.f;
  const float sum = wave_sum(p);
  s_p[lane] = p;
  __builtin_amdgcn_wave_barrier();
  float o[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) o[e] = 0.f;
#pragma unroll
  for (int it = 0; it < 8; ++it) {
    const int jj = it * 8 + kg;
    const float pj = jj < ctx ? s_p[jj] : 0.f;
    const f32x4 v0 = __builtin_bit_cast(f32x4, L.vv[it][0]), v1 = __builtin_bit_cast(f32x4, L.vv[it][1]);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      o[e] += pj * v0[e];
      o[4 + e] += pj * v1[e];
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) o[e] = rows_sum(o[e] + dpp_f<0x128>(o[e]));
  if (kg == 0) {
    const float inv = 1.0f / sum;
    *reinterpret_cast<f32x4*>(orow + d8) = (f32x4){o[0], o[1], o[2], o[3]} * inv;
    *reinterpret_cast<f32x4*>(orow + d8 + 4) = (f32x4){o[4], o[5], o[6], o[7]} * inv;
  }
}

// ------------------------------------------------------------------------------------------------
// Decode GEMV (M <= 32 rows): everything a workgroup needs from memory is issued at kernel start,
// in the order it is consumed (vmcnt retires in issue order):
//   1. the activation operand - PRO_DIRECT: MFMA A fragments straight to VGPRs; PRO_LN: the f32
//      rows + LayerNorm affine (normalised in registers, written once to an XOR-swizzled LDS tile);
//   2. the wave's whole K range of rows-packed weights: NSL slabs x NTB tiles of 1 KiB loads,
//      nontemporal (each weight byte is read by exactly one CU per step);
//   3. the epilogue inputs (bias, residual, processors' token lists).
// NSL (slabs per wave = K / (4*KS)) is a template parameter, so the loads are fully unrolled with
// no clamped duplicates and the compiler counts vmcnt exactly.
template <typename T, int MT, int NTB, int PRO, int EPI, int NSL>
__global__ __launch_bounds__(256) void vcap_rows_gemv_kernel(RowsGemmArgs a) {
  extern __shared__ __attribute__((aligned(16))) char dyn[];  // PRO_LN: A tile [MT*16][K] T
  constexpr int E = Frag<T>::kElems, KS = 4 * E, MP = MT * 16, NE = MT * NTB;
  constexpr int LGM = (EPI == EPI_LOGITS || EPI == EPI_LSE) ? MP : 1;
  constexpr int KC = NSL * KS * 4 / 256;  // f32x4 chunks per lane of a K-long row (PRO_LN)
  constexpr int RPW = MP / 4;             // LN rows per wave
  __shared__ __attribute__((aligned(16))) float red[4][NE * 256];
  __shared__ float lg[LGM][NTB * 16];
  __shared__ unsigned char s_rep[LGM][NTB * 16], s_ban[LGM][NTB * 16];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  const int M = a.M, N = a.N, K = a.K;
  const int m0 = blockIdx.y * MP;
  // a.half (PRO_DIRECT residual GEMVs of NTB = 1): two workgroups per 16-column tile, each streaming
  // the weights of 8 columns (lanes l and l ^ 8 load the same fragment: column (l & 7) of its half),
  // so a K = 3072 projection spreads its weight stream over twice the CUs; the MFMAs, their order
  // and every stored output are those of the full-tile workgroup
  // a.sk_part (the bf16 mlp c_proj, r06): K split over a workgroup pair per 16-column tile and 16-row
  // chunk, each workgroup one K half of the whole tile - half the activation rows per workgroup, the
  // pair meeting as in vcap_rows_gemv8_kernel<float, NSL, 2, 1>
  constexpr bool CAN_SPLIT = EPI == EPI_RESID && NTB == 1 && MT == 1 && PRO == PRO_DIRECT;
  const bool split = CAN_SPLIT && a.sk_part != nullptr;
  const bool half = EPI == EPI_RESID && NTB == 1 && a.half && !split;
  const int hsel = half ? (int)(blockIdx.x & 1) : -1;
  const int ksel = split ? (int)(blockIdx.x & 1) : 0;
  const int n0 = (half || split) ? (int)(blockIdx.x >> 1) * 16 : blockIdx.x * NTB * 16;
  const int wlane = half ? ((lane & 0x30) | (hsel << 3) | (lane & 7)) : lane;
  const int nslab = (split ? 8 : 4) * NSL;  // = K / KS
  const int g0 = (split ? ksel * 4 * NSL : 0) + wave * NSL;
  const int ntiles = (N + 15) >> 4;

  if constexpr (EPI == EPI_LOGITS) proc_flags_zero<MP, NTB>(s_rep, s_ban);

  // ---- 1) activation operand (STREAM_A: row tile 0 only; tile 1 is loaded into the same registers
  // as the tile-0 MFMAs consume them, so the per-row MFMA order - and every output bit - is that of
  // the all-tiles-live form)
  constexpr bool STREAM_A = gemv_stream_a<T, MT, NTB, PRO, NSL>();
  constexpr int MTA = STREAM_A ? 1 : MT;  // row tiles of A fragments live at once
  u32x4 af[PRO == PRO_DIRECT ? MTA : 1][PRO == PRO_DIRECT ? NSL : 1];
  f32x4 xv[PRO == PRO_LN ? RPW : 1][KC > 0 ? KC : 1], gv[KC > 0 ? KC : 1], bv[KC > 0 ? KC : 1];
  if constexpr (PRO == PRO_DIRECT) {
#pragma unroll
    for (int i = 0; i < MTA; ++i) {
      const long xo = (long)min(m0 + i * 16 + fr, M - 1) * a.ldx + fg * E;
#pragma unroll
      for (int s = 0; s < NSL; ++s) af[i][s] = vcap_dec_aload(a.x, (xo + (g0 + s) * KS) * (long)sizeof(T));
    }
  } else {
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
      const long xo = (long)min(m0 + wave + 4 * r, M - 1) * a.ldx + lane * 4;
#pragma unroll
      for (int c = 0; c < KC; ++c) xv[r][c] = __builtin_bit_cast(f32x4, vcap_dec_aload(a.x, (xo + c * 256) * 4L));
    }
#pragma unroll
    for (int c = 0; c < KC; ++c) {
      gv[c] = __builtin_bit_cast(f32x4, vcap_dec_aload(a.ln_g, (c * 256 + lane * 4) * 4L));
      bv[c] = __builtin_bit_cast(f32x4, vcap_dec_aload(a.ln_b, (c * 256 + lane * 4) * 4L));
    }
  }

  if constexpr (PRO == PRO_LN || NSL * (NTB + MTA) < 64)
    asm volatile("" ::: "memory");  // the activation loads issue (and retire) before the weights
  // ---- 2) weights
  u32x4 wf[NSL][NTB];
#pragma unroll
  for (int j = 0; j < NTB; ++j) {
    const u32x4* wp = packed_frag(a.w, min(n0 / 16 + j, ntiles - 1), nslab, g0, wlane);
#pragma unroll
    for (int s = 0; s < NSL; ++s) wf[s][j] = vcap_dec_wload<MT == 1>(a.w, wp + s * 64);
  }

  // ---- 3) epilogue inputs
  float pre_bias[NE], pre_res[NE];
#pragma unroll
  for (int q = 0; q < NE; ++q) {
    const int m = m0 + (q / NTB) * 16 + (tid >> 4), n = n0 + (q % NTB) * 16 + (tid & 15);
    const int mc = min(m, M - 1), nc = min(n, N - 1);
    // unconditional load (from a valid address when there is no bias), then a select: a load
    // guarded by the runtime `a.bias` test compiled to a branch + vmcnt(0) that waited for the
    // whole weight stream before the LayerNorm / A-fragment work could start
    const float bl = *(a.bias ? a.bias + nc : (const float*)a.x);
    pre_bias[q] = a.bias ? bl : 0.f;
    pre_res[q] = 0.f;
    if constexpr (EPI == EPI_RESID) pre_res[q] = ((const float*)a.out)[(long)mc * a.ldo + nc];
  }
  ProcToks<EPI == EPI_LOGITS ? MT : 1> toks;
  if constexpr (EPI == EPI_LOGITS) toks.load(a, m0);
  // Issue order fence: every load above is issued before any of the work below.  The empty asm
  // statements take the first-consumed operands as in/out registers and clobber memory, so no
  // load sinks below them and no LayerNorm arithmetic / MFMA chain is hoisted above them (the
  // scheduler otherwise sank the weight stream below the LayerNorm, or issued it ~8 loads at a
  // time between the MFMAs); the waits they imply are for the oldest loads only.
  if constexpr (PRO == PRO_LN) {
#pragma unroll
    for (int r = 0; r < RPW; ++r)
#pragma unroll
      for (int c = 0; c < KC; ++c) asm volatile("" : "+v"(xv[r][c])::"memory");
  } else if constexpr (NSL * (NTB + MTA) < 64) {  // (at the 64-fragment budget: let the compiler stream)
    asm volatile("" : "+v"(af[0][0])::"memory");
  }

  // ---- LayerNorm in registers -> swizzled LDS tile (waits only for step 1's loads)
  if constexpr (PRO == PRO_LN) {
    const int rowb = K * (int)sizeof(T);
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
      const int m = wave + 4 * r;  // row within the chunk
      float s = 0.f;
#pragma unroll
      for (int c = 0; c < KC; ++c) s += (xv[r][c].x + xv[r][c].y) + (xv[r][c].z + xv[r][c].w);
      const float mean = wave_sum(s) / (float)K;
      float ss = 0.f;
#pragma unroll
      for (int c = 0; c < KC; ++c) {
        const f32x4 d = xv[r][c] - mean;
        ss += sumsq4(d);
      }
      const float rstd = rsqrtf(wave_sum(ss) / (float)K + a.ln_eps);
      const bool live = m0 + m < M;
#pragma unroll
      for (int c = 0; c < KC; ++c) {
        const f32x4 y = live ? ln_affine4(xv[r][c], mean, rstd, gv[c], bv[c]) : (f32x4){0.f, 0.f, 0.f, 0.f};
        const int byte = (c * 256 + lane * 4) * (int)sizeof(T);
        char* dst = dyn + (long)m * rowb + ((((byte >> 4) ^ (m & 15))) << 4) + (byte & 15);
        if constexpr (sizeof(T) == 2) {
          *reinterpret_cast<u32x2*>(dst) = (u32x2){pack_bf2(y.x, y.y), pack_bf2(y.z, y.w)};
        } else {
          *reinterpret_cast<f32x4*>(dst) = y;
        }
      }
    }
  }
  if constexpr (PRO == PRO_LN || EPI == EPI_LOGITS) __syncthreads();

  // ---- MFMA over the wave's K range
  f32x4 acc[MT][NTB];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NTB; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  if constexpr (STREAM_A) {
    const long xo1 = (long)min(m0 + 16 + fr, M - 1) * a.ldx + fg * E;
#pragma unroll
    for (int s = 0; s < NSL; ++s) {
#pragma unroll
      for (int j = 0; j < NTB; ++j) acc[0][j] = mfma_frag(af[0][s], wf[s][j], acc[0][j], (T*)nullptr);
      af[0][s] = vcap_dec_aload(a.x, (xo1 + (g0 + s) * KS) * (long)sizeof(T));
    }
#pragma unroll
    for (int s = 0; s < NSL; ++s)
#pragma unroll
      for (int j = 0; j < NTB; ++j) acc[MT - 1][j] = mfma_frag(af[0][s], wf[s][j], acc[MT - 1][j], (T*)nullptr);
  } else
#pragma unroll
  for (int s = 0; s < NSL; ++s) {
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      u32x4 A;
      if constexpr (PRO == PRO_DIRECT) {
        A = af[i][s];
      } else {
        const int row = i * 16 + fr, chunk = (g0 + s) * 4 + fg;
        A = *reinterpret_cast<const u32x4*>(dyn + (long)row * K * sizeof(T) + ((chunk ^ (row & 15)) << 4));
      }
#pragma unroll
      for (int j = 0; j < NTB; ++j) acc[i][j] = mfma_frag(A, wf[s][j], acc[i][j], (T*)nullptr);
    }
  }

  // ---- split-K reduction + epilogue
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NTB; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) red[wave][(i * NTB + j) * 256 + (fg * 4 + r) * 16 + fr] = acc[i][j][r];
  if constexpr (EPI == EPI_LOGITS) toks.template mark<NTB>(a, m0, n0, s_rep, s_ban);
  __syncthreads();
  if constexpr (CAN_SPLIT) {
    if (split) {
      // the pair hand-off (MI355X guide Guideline 16 R1): sc1 partial stores drained by every storing
      // wave before the barrier, one agent-scope ticket, the second arriver's sc1 loads; the sum is
      // p(K half 0) + p(K half 1) in that order whichever workgroup arrives second
      __shared__ int s_ticket;
      const long pair = (long)blockIdx.y * (gridDim.x >> 1) + (blockIdx.x >> 1);
      const float part = (red[0][tid] + red[1][tid]) + (red[2][tid] + red[3][tid]);
      __hip_atomic_store(a.sk_part + (pair * 2 + ksel) * 256 + tid, part, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) s_ticket = __hip_atomic_fetch_add(a.sk_cnt + pair, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __syncthreads();
      if ((s_ticket & 1) == 0) return;
      const int m = m0 + (tid >> 4), n = n0 + (tid & 15);
      if (m < M && n < N) {
        const float other =
            __hip_atomic_load(a.sk_part + (pair * 2 + (ksel ^ 1)) * 256 + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const float v = (ksel == 0 ? part + other : other + part) + pre_bias[0];
        ((float*)a.out)[(long)m * a.ldo + n] = pre_res[0] + v;
      }
      return;
    }
  }
  rows_epilogue<T, MT, NTB, EPI>(a, m0, red, pre_bias, pre_res, lg, s_rep, s_ban, n0, hsel);
}

// ------------------------------------------------------------------------------------------------
// Residual GEMV (PRO_DIRECT + EPI_RESID, 16-row chunks over blockIdx.y, one 16-column tile per
// workgroup) whose K range needs more fragments than 4 waves hold: the f32 mlp c_proj (K = 3072 of
// GPT-2 small: 48 slabs of 16 per wave would be 96 16-byte fragments per lane; K = 4096 of
// GPT-2-medium).  8 waves (two per SIMD) of NSL slabs each, every weight load issued up front as in
// vcap_rows_gemv_kernel, split-K partials summed through LDS in a fixed order
// ((w0 + w1) + (w2 + w3)) + ((w4 + w5) + (w6 + w7)).  Up to 24 slabs the A fragments are loaded at
// once too; past that (NSL = 32: 128 weight + 128 A registers would not fit the 256 of a 2-wave
// SIMD) they come in batches of 8 slabs, two batches live, batch b + 2 issued once batch b's
// MFMAs have consumed its registers (the activation rows are L2-resident: every workgroup reads them).
template <typename T, int NSL, int KP, int NT>
__global__ __launch_bounds__(512) void vcap_rows_gemv8_kernel(RowsGemmArgs a) {
  constexpr int E = Frag<T>::kElems, KS = 4 * E;
  constexpr int AB = NSL <= 24 ? NSL : 8, NAB = NSL / AB;
  constexpr bool SPLIT = KP > 1;
  static_assert(NSL % AB == 0, "A batches tile the wave's slabs");
  static_assert(NT == 1 || (KP == 4 && NT == 2), "column-tile pairs only with the 4-way K split");
  __shared__ __attribute__((aligned(16))) float red[8][NT * 256];
  __shared__ int s_ticket;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  const int M = a.M, N = a.N;
  const int m0 = blockIdx.y * 16;
  // a.half: two workgroups per 16-column tile, each streaming 8 columns' weights (as in
  // vcap_rows_gemv_kernel: lanes l and l ^ 8 load the same fragment), the stores of its 8 columns.
  // SPLIT (KP K parts): KP workgroups per group of NT 16-column tiles, each taking one K part for all
  // the group's columns, so each ingests 1/KP of the activation rows (the f32 mlp c_proj's 196 KiB of
  // activations per workgroup was twice its weight slice: profiles/r06_decode_stamps.txt).  KP = 2,
  // NT = 1: 98 KiB of activations + 98 KiB of weights per workgroup; KP = 4, NT = 2 (GPT-2 small, r06
  // late): 49 + 98 KiB, the same workgroup count.  The K parts meet below.
  const bool half = !SPLIT && a.half != 0;
  const int hsel = half ? (int)(blockIdx.x & 1) : -1;
  const int ksel = SPLIT ? (int)(blockIdx.x % KP) : 0;
  const int grp = SPLIT ? (int)(blockIdx.x / KP) : (int)blockIdx.x;
  const int n0 = half ? (int)(blockIdx.x >> 1) * 16 : grp * 16 * NT;
  const int wlane = half ? ((lane & 0x30) | (hsel << 3) | (lane & 7)) : lane;
  const int nslab = KP * 8 * NSL, g0 = ksel * 8 * NSL + wave * NSL;
  const int ntiles = (N + 15) >> 4;
  u32x4 af[NAB > 1 ? 2 : 1][AB];
  const long xo = (long)min(m0 + fr, M - 1) * a.ldx + fg * E;
  auto aload = [&](int b) {
#pragma unroll
    for (int s = 0; s < AB; ++s)
      af[b & 1][s] = vcap_dec_aload(a.x, (xo + (g0 + b * AB + s) * KS) * (long)sizeof(T));
  };
  aload(0);
  asm volatile("" ::: "memory");  // the activation loads issue before the weights
  u32x4 wf[NSL][NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const u32x4* wp = packed_frag(a.w, min(n0 / 16 + j, ntiles - 1), nslab, g0, wlane);
#pragma unroll
    for (int s = 0; s < NSL; ++s) wf[s][j] = vcap_dec_wload<true>(a.w, wp + s * 64);
  }
  if constexpr (NAB > 1) aload(1);
  // this thread's output element: tile tj, row, col (NT = 2: all 512 threads; NT = 1: the first 256)
  const int tj = NT == 2 ? (tid >> 8) : 0, e = tid & 255;
  const int row = e >> 4, col = e & 15;
  const int mc = min(m0 + row, M - 1), nc = min(n0 + tj * 16 + col, N - 1);
  const float bl = *(a.bias ? a.bias + nc : (const float*)a.x);
  const float pre_bias = a.bias ? bl : 0.f;
  const float pre_res = ((const float*)a.out)[(long)mc * a.ldo + nc];
  asm volatile("" : "+v"(af[0][0])::"memory");
  f32x4 acc[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) acc[j] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int b = 0; b < NAB; ++b) {
#pragma unroll
    for (int s = 0; s < AB; ++s)
#pragma unroll
      for (int j = 0; j < NT; ++j) acc[j] = mfma_frag(af[b & 1][s], wf[b * AB + s][j], acc[j], (T*)nullptr);
    if (b + 2 < NAB) {
      // batch b consumed before its registers reload, and the batch's 8 loads issue together (the
      // scheduler otherwise sinks each to its use: 8 serial L2 round trips)
      __builtin_amdgcn_sched_barrier(0);
      aload(b + 2);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
#pragma unroll
  for (int j = 0; j < NT; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) red[wave][j * 256 + (fg * 4 + r) * 16 + fr] = acc[j][r];
  __syncthreads();
  const bool mine = tid < NT * 256;
  const int ei = tj * 256 + e;
  if constexpr (SPLIT) {
    // The K-part partials of a column group meet through global memory, the MI355X guide's valid
    // hand-off form (Guideline 16 R1): every partial store is sc1 (agent-scope relaxed atomic store:
    // write-through) and every storing wave drains (vmcnt(0)) before the workgroup barrier; then one
    // lane takes a ticket (agent-scope atomic add, zeroed per decode by vcap_decode_init; KP per group
    // per launch).  The group's last arriver loads the other parts' partials with sc1 loads and stores
    // the output; the others exit.  No one waits (no spin), and the sum is
    // ((p0 + p1) + (p2 + p3)) (KP = 4) or p0 + p1 (KP = 2) whichever arrives last: deterministic.
    const long g = (long)blockIdx.y * (gridDim.x / KP) + grp;
    float part = 0.f;
    if (mine) {
      part = ((red[0][ei] + red[1][ei]) + (red[2][ei] + red[3][ei])) + ((red[4][ei] + red[5][ei]) + (red[6][ei] + red[7][ei]));
      __hip_atomic_store(a.sk_part + ((g * KP + ksel) * NT) * 256 + ei, part, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its sc1 stores
    __syncthreads();
    if (tid == 0) s_ticket = __hip_atomic_fetch_add(a.sk_cnt + g, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    if ((s_ticket % KP) != KP - 1) return;  // not the last of the group (tickets advance by KP per launch)
    if (mine && m0 + row < M && n0 + tj * 16 + col < N) {
      float p[KP];
#pragma unroll
      for (int k = 0; k < KP; ++k)
        p[k] = k == ksel ? part
                         : __hip_atomic_load(a.sk_part + ((g * KP + k) * NT) * 256 + ei, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
      float v;
      if constexpr (KP == 4) v = (p[0] + p[1]) + (p[2] + p[3]);
      else v = p[0] + p[1];
      ((float*)a.out)[(long)(m0 + row) * a.ldo + n0 + tj * 16 + col] = pre_res + (v + pre_bias);
    }
  } else {
    if (mine && m0 + row < M && n0 + col < N && (hsel < 0 || (col >> 3) == hsel)) {
      const float v = ((red[0][ei] + red[1][ei]) + (red[2][ei] + red[3][ei])) +
                      ((red[4][ei] + red[5][ei]) + (red[6][ei] + red[7][ei])) + pre_bias;
      ((float*)a.out)[(long)(m0 + row) * a.ldo + n0 + col] = pre_res + v;
    }
  }
}

// ------------------------------------------------------------------------------------------------
// General rows kernel (prefill rows, f32 parity mode, shapes outside the GEMV instantiations):
// rows [m0, m0 + MT*16) of a blockIdx.y row chunk; weights streamed in double-buffered chunks of
// U slabs; PRO_DIRECT A fragments ride along with each weight chunk in registers, PRO_LN rows
// are normalised into a swizzled LDS tile first (K <= 1024).
template <typename T, int MT, int NTB, int PRO, int EPI>
__global__ __launch_bounds__(256) void vcap_rows_gemm_lds_kernel(RowsGemmArgs a) {
  extern __shared__ __attribute__((aligned(16))) char dyn[];
  constexpr int E = Frag<T>::kElems;
  constexpr int KS = 4 * E;
  constexpr int U = NTB >= 4 ? 2 : 8 / NTB;  // slabs per chunk: U*NTB weight fragments in flight
  constexpr int MP = MT * 16;
  constexpr int NE = MT * NTB;
  constexpr int LGM = (EPI == EPI_LOGITS || EPI == EPI_LSE) ? MP : 1;
  __shared__ __attribute__((aligned(16))) float red[4][NE * 256];
  __shared__ float lg[LGM][NTB * 16];
  __shared__ unsigned char s_rep[LGM][NTB * 16], s_ban[LGM][NTB * 16];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  const int m0 = blockIdx.y * MP;
  const int M = a.M, N = a.N, K = a.K;
  const int n0 = blockIdx.x * NTB * 16;
  const int nslab = K / KS, nsl = nslab / 4, g0 = wave * nsl;
  const int ntiles = (N + 15) >> 4;
  const int rowb = K * (int)sizeof(T);
  if constexpr (EPI == EPI_LOGITS) proc_flags_zero<MP, NTB>(s_rep, s_ban);

  // ---- PRO_LN: rows -> LayerNorm -> swizzled LDS tile
  if constexpr (PRO == PRO_LN) {
    constexpr int RPW = MP / 4;
    const float* X = (const float*)a.x;
    f32x4 gv[4], bv[4];
#pragma unroll
    for (int ci = 0; ci < 4; ++ci) {
      const int c = min(ci * 256 + lane * 4, K - 4);  // clamped, never predicated
      gv[ci] = *reinterpret_cast<const f32x4*>(a.ln_g + c);
      bv[ci] = *reinterpret_cast<const f32x4*>(a.ln_b + c);
    }
#pragma unroll
    for (int gq = 0; gq < RPW; gq += 4) {
      f32x4 xv[4][4];
#pragma unroll
      for (int ci = 0; ci < 4; ++ci) {
        const int c = min(ci * 256 + lane * 4, K - 4);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = min(m0 + wave + 4 * (gq + r), M - 1);
          xv[r][ci] = *reinterpret_cast<const f32x4*>(X + (long)m * a.ldx + c);
        }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int ml = wave + 4 * (gq + r);
        float s = 0.f;
#pragma unroll
        for (int ci = 0; ci < 4; ++ci)
          if (ci * 256 + lane * 4 < K) s += (xv[r][ci].x + xv[r][ci].y) + (xv[r][ci].z + xv[r][ci].w);
        const float mean = wave_sum(s) / (float)K;
        float ss = 0.f;
#pragma unroll
        for (int ci = 0; ci < 4; ++ci)
          if (ci * 256 + lane * 4 < K) {
            const f32x4 d = xv[r][ci] - mean;
            ss += sumsq4(d);
          }
        const float rstd = rsqrtf(wave_sum(ss) / (float)K + a.ln_eps);
        const bool live = m0 + ml < M;
#pragma unroll
        for (int ci = 0; ci < 4; ++ci) {
          const int c = ci * 256 + lane * 4;
          if (c < K) {
            const f32x4 y = live ? ln_affine4(xv[r][ci], mean, rstd, gv[ci], bv[ci]) : (f32x4){0.f, 0.f, 0.f, 0.f};
            const int byte = c * (int)sizeof(T);
            char* dst = dyn + (long)ml * rowb + ((((byte >> 4) ^ (ml & 15))) << 4) + (byte & 15);
            if constexpr (sizeof(T) == 2) {
              *reinterpret_cast<u32x2*>(dst) = (u32x2){pack_bf2(y.x, y.y), pack_bf2(y.z, y.w)};
            } else {
              *reinterpret_cast<f32x4*>(dst) = y;
            }
          }
        }
      }
    }
  }

  // ---- weight (+ PRO_DIRECT activation) fragments, chunk by chunk.  Loads are never predicated
  // (a guarded load waits vmcnt(0) on its own); slabs past the wave's range re-read its last slab.
  u32x4 wa[U][NTB], wb[U][NTB], xa[PRO == PRO_DIRECT ? U : 1][MT], xb[PRO == PRO_DIRECT ? U : 1][MT];
  auto load_chunk = [&](u32x4 (&wf)[U][NTB], u32x4 (&xf)[PRO == PRO_DIRECT ? U : 1][MT], int c) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int sl = min(c * U + u, nsl - 1);
      if constexpr (PRO == PRO_DIRECT) {
#pragma unroll
        for (int i = 0; i < MT; ++i)
          xf[u][i] = *reinterpret_cast<const u32x4*>((const T*)a.x + (long)min(m0 + i * 16 + fr, M - 1) * a.ldx +
                                                     (g0 + sl) * KS + fg * E);
      }
#pragma unroll
      for (int j = 0; j < NTB; ++j)
        wf[u][j] = vcap_dec_wload<false>(a.w,
            packed_frag(a.w, min(n0 / 16 + j, ntiles - 1), nslab, g0 + sl, lane));
    }
  };
  const int nch = (nsl + U - 1) / U;
  load_chunk(wa, xa, 0);
  if (nch > 1) load_chunk(wb, xb, 1);

  // ---- epilogue inputs
  float pre_bias[NE], pre_res[NE];
#pragma unroll
  for (int q = 0; q < NE; ++q) {
    const int m = m0 + (q / NTB) * 16 + (tid >> 4), n = n0 + (q % NTB) * 16 + (tid & 15);
    const int mc = min(m, M - 1), nc = min(n, N - 1);
    // unconditional load (from a valid address when there is no bias), then a select: a load
    // guarded by the runtime `a.bias` test compiled to a branch + vmcnt(0) that waited for the
    // whole weight stream before the LayerNorm / A-fragment work could start
    const float bl = *(a.bias ? a.bias + nc : (const float*)a.x);
    pre_bias[q] = a.bias ? bl : 0.f;
    pre_res[q] = 0.f;
    if constexpr (EPI == EPI_RESID) pre_res[q] = ((const float*)a.out)[(long)mc * a.ldo + nc];
  }
  ProcToks<EPI == EPI_LOGITS ? MT : 1> toks;
  if constexpr (EPI == EPI_LOGITS) toks.load(a, m0);
  if constexpr (PRO == PRO_LN || EPI == EPI_LOGITS) __syncthreads();

  // ---- MFMA over the wave's K range
  f32x4 acc[MT][NTB];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NTB; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  auto compute_chunk = [&](const u32x4 (&wf)[U][NTB], const u32x4 (&xf)[PRO == PRO_DIRECT ? U : 1][MT], int c) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (c * U + u < nsl) {
        const int chunk = (g0 + c * U + u) * 4 + fg;
#pragma unroll
        for (int i = 0; i < MT; ++i) {
          u32x4 A;
          if constexpr (PRO == PRO_DIRECT) {
            A = xf[u][i];
          } else {
            const int row = i * 16 + fr;
            A = *reinterpret_cast<const u32x4*>(dyn + (long)row * rowb + ((chunk ^ (row & 15)) << 4));
          }
#pragma unroll
          for (int j = 0; j < NTB; ++j) acc[i][j] = mfma_frag(A, wf[u][j], acc[i][j], (T*)nullptr);
        }
      }
    }
  };
  for (int c = 0; c < nch; c += 2) {
    compute_chunk(wa, xa, c);
    if (c + 2 < nch) load_chunk(wa, xa, c + 2);
    if (c + 1 < nch) {
      compute_chunk(wb, xb, c + 1);
      if (c + 3 < nch) load_chunk(wb, xb, c + 3);
    }
  }

#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NTB; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) red[wave][(i * NTB + j) * 256 + (fg * 4 + r) * 16 + fr] = acc[i][j][r];
  if constexpr (EPI == EPI_LOGITS) toks.template mark<NTB>(a, m0, n0, s_rep, s_ban);
  __syncthreads();
  rows_epilogue<T, MT, NTB, EPI>(a, m0, red, pre_bias, pre_res, lg, s_rep, s_ban, n0);
}

// ------------------------------------------------------------------------------------------------
// Causal attention of S_new query rows per sequence over the paged cache (positions 0..past+i).
// One wave per (row, head).  The sequence's page ids are read once (lane p holds page p) and
// broadcast with ds_bpermute, so no K/V load waits on a dependent page-table load.
// Scores: lane j <-> key j (+64 ...), full 64-dim dot.  P.V: lane = (key group kg of 8, 8
// consecutive dims d8), partial sums reduced over the 8 key groups by DPP + permlane swaps.
template <typename T>
__global__ __launch_bounds__(256) void vcap_decode_attention_kernel(const T* __restrict__ q, const T* __restrict__ kc,
                                                                    const T* __restrict__ vc,
                                                                    const int* __restrict__ page_table, int maxp,
                                                                    T* __restrict__ out, int M, int H, int S_new,
                                                                    int past) {
  constexpr int E8 = Frag<T>::kElems;  // elements per 16-byte chunk
  __shared__ float s_q[4][64];
  __shared__ float s_p[4][1024];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int item = blockIdx.x * 4 + wave;
  if (item >= M * H) return;
  const int m = item / H, h = item - m * H;
  const int E = H * 64;
  const int seq = m / S_new, qpos = past + (m - seq * S_new);
  const int ctx = qpos + 1;
  const int my_page = page_table[seq * maxp + min(lane, maxp - 1)];
  s_q[wave][lane] = Num<T>::to_f(q[(long)m * E + h * 64 + lane]);
  __builtin_amdgcn_wave_barrier();
  float mx = -INFINITY;
  for (int j0 = 0; j0 < ctx; j0 += 64) {
    const int j = min(j0 + lane, ctx - 1);
    const int page = __shfl(my_page, j >> 4);
    const T* krow = kc + (((long)page * H + h) * 16 + (j & 15)) * 64;
    u32x4 kv[64 / E8];
#pragma unroll
    for (int c = 0; c < 64 / E8; ++c) kv[c] = *reinterpret_cast<const u32x4*>(krow + c * E8);
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < 64 / E8; ++c) {
      const T* ke = reinterpret_cast<const T*>(&kv[c]);
#pragma unroll
      for (int e = 0; e < E8; ++e) s += s_q[wave][c * E8 + e] * Num<T>::to_f(ke[e]);
    }
    s *= 0.125f;
    if (j0 + lane < ctx) {
      s_p[wave][j0 + lane] = s;
      mx = fmaxf(mx, s);
    }
  }
  mx = wave_max(mx);
  float sum = 0.f;
  for (int j = lane; j < ctx; j += 64) {
    const float p = __expf(s_p[wave][j] - mx);
    s_p[wave][j] = p;
    sum += p;
  }
  sum = wave_sum(sum);
  __builtin_amdgcn_wave_barrier();
  const int kg = lane >> 3, d8 = (lane & 7) * 8;
  float o[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) o[e] = 0.f;
#pragma unroll 4
  for (int j0 = 0; j0 < ctx; j0 += 8) {
    const int jj = j0 + kg;
    const int j = min(jj, ctx - 1);
    const int page = __shfl(my_page, j >> 4);
    const T* vrow = vc + (((long)page * H + h) * 16 + (j & 15)) * 64 + d8;
    const float p = jj < ctx ? s_p[wave][j] : 0.f;
    if constexpr (sizeof(T) == 2) {
      const u32x4 vv = *reinterpret_cast<const u32x4*>(vrow);
      const unsigned w4[4] = {vv.x, vv.y, vv.z, vv.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        o[2 * e] += p * bf2f((bf16_t)(w4[e] & 0xffff));
        o[2 * e + 1] += p * bf2f((bf16_t)(w4[e] >> 16));
      }
    } else {
      const f32x4 v0 = *reinterpret_cast<const f32x4*>(vrow);
      const f32x4 v1 = *reinterpret_cast<const f32x4*>(vrow + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        o[e] += p * v0[e];
        o[4 + e] += p * v1[e];
      }
    }
  }
  // reduce over the 8 key groups: lane ^ 8 (row_ror:8 inside a 16-lane row), then ^16, ^32
#pragma unroll
  for (int e = 0; e < 8; ++e) o[e] = rows_sum(o[e] + dpp_f<0x128>(o[e]));
  if (kg == 0) {
    const float inv = 1.0f / sum;
    T* orow = out + (long)m * E + h * 64 + d8;
    if constexpr (sizeof(T) == 2) {
      *reinterpret_cast<u32x4*>(orow) =
          (u32x4){pack_bf2(o[0] * inv, o[1] * inv), pack_bf2(o[2] * inv, o[3] * inv),
                  pack_bf2(o[4] * inv, o[5] * inv), pack_bf2(o[6] * inv, o[7] * inv)};
    } else {
      *reinterpret_cast<f32x4*>(orow) = (f32x4){o[0], o[1], o[2], o[3]} * inv;
      *reinterpret_cast<f32x4*>(orow + 4) = (f32x4){o[4], o[5], o[6], o[7]} * inv;
    }
  }
}

// ------------------------------------------------------------------------------------------------
// Prefill input rows: h[s*S0+i] = (i < P ? prefix[s][i] : wte[prompt[i-P]]) + wpe[i]
// (text_decoder.py:60-74 _build_inputs + GPT2Model position embeddings).
struct PromptIds {
  int n;
  int ids[64];
};

template <typename T>
__global__ __launch_bounds__(256) void vcap_prefill_embed_kernel(const float* __restrict__ prefix, int P,
                                                                 PromptIds prompt, const T* __restrict__ wte,
                                                                 const float* __restrict__ wpe, float* __restrict__ h,
                                                                 int S0, int E, int pos0, int prefix_rep) {
  const int m = blockIdx.x;
  const int s = m / S0 / prefix_rep, i = m % S0;   // prefix_rep rows (beams) share sequence s's prefix
  for (int c = threadIdx.x; c < E; c += 256) {
    float v = (i < P) ? prefix[((long)s * P + i) * E + c] : Num<T>::to_f(wte[(long)prompt.ids[i - P] * E + c]);
    h[(long)m * E + c] = v + wpe[(long)(pos0 + i) * E + c];
  }
}

// Token-id inputs for an externally driven step (beam search / sampling): h[r] = wte[tok[r]] + wpe[pos].
template <typename T>
__global__ __launch_bounds__(256) void vcap_embed_tokens_kernel(const int* __restrict__ tok,
                                                                const T* __restrict__ wte,
                                                                const float* __restrict__ wpe, float* __restrict__ h,
                                                                int E, int pos) {
  const int r = blockIdx.x;
  const int t = tok[r];
  for (int c = threadIdx.x; c < E; c += 256) h[(long)r * E + c] = Num<T>::to_f(wte[(long)t * E + c]) + wpe[(long)pos * E + c];
}

// KV-cache row permutation for beam search: dst row r <- src row src[r], positions [0, len),
// every layer/head (contiguous [page][H][16][64] pools with identity page tables).
template <typename T>
__global__ __launch_bounds__(256) void vcap_kv_gather_kernel(const T* __restrict__ src_pool, T* __restrict__ dst_pool,
                                                             const int* __restrict__ src_rows, int maxp, int H,
                                                             int len, long layer_elems, int L) {
  const int r = blockIdx.x, l = blockIdx.y;
  const int sr = src_rows[r];
  const long row_elems = (long)maxp * H * 16 * 64;
  const T* s = src_pool + l * layer_elems + (long)sr * row_elems;
  T* d = dst_pool + l * layer_elems + (long)r * row_elems;
  const int pages = (len + 15) / 16;
  const long n = (long)pages * H * 16 * 64 / 8;  // 16-byte chunks for bf16 (8 elems) / 2 for f32
  const int per = 16 / sizeof(T);
  for (long i = threadIdx.x; i < (long)pages * H * 16 * 64 / per; i += 256)
    reinterpret_cast<u32x4*>(d)[i] = reinterpret_cast<const u32x4*>(s)[i];
  (void)n;
}

// Per-step state init: identity page tables, cleared history / flags.
__global__ void vcap_decode_init_kernel(int* page_table, int B, int maxp, int* finished, int* nbanned, int* sk_cnt,
                                        int n_sk) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < B * maxp) page_table[i] = i;
  if (i < n_sk) sk_cnt[i] = 0;
  if (i < B) {
    finished[i] = 0;
    nbanned[i] = 0;
  }
}

// Reduce the per-workgroup argmax partials, apply EOS padding, record the token, precompute the
// n-gram ban list for the next step (one thread per n-gram start, history staged in LDS) and
// write the next input embedding wte[tok] + wpe[pos].
// SCREEN (f32 decoders, greedy): the partials are those of the bf16 screen (ScreenArgs); the token is
// the exact-f32 argmax over the tokens the screen's error bound cannot rule out.
template <typename T, bool SCREEN>
__global__ __launch_bounds__(256) void vcap_decode_finalize_kernel(
    const float* __restrict__ part_val, const int* __restrict__ part_idx, int nblk, int step, int* finished,
    int* hist, int hist_ld, int* banned, int* nbanned, int ngram, int eos, int pad, int* out_ids, int out_ld,
    const T* __restrict__ wte, const float* __restrict__ wpe, float* __restrict__ h, int E, int pos_next, int vocab,
    ScreenArgs sc) {
  __shared__ float sv[4];
  __shared__ int si[4];
  __shared__ int s_h[1024];
  __shared__ int s_tok, s_nb;
  __shared__ __attribute__((aligned(16))) float s_hf[SCREEN ? 1024 : 4];
  __shared__ float s_red[4];
  __shared__ int s_cb[SCREEN ? 64 : 1], s_cv[SCREEN ? 4096 : 1], s_bn[SCREEN ? 256 : 1];
  __shared__ int s_ncb, s_ncv;
  const int m = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // every load of the first phase issued at once (clamped addresses, selects after): the history,
  // the argmax partials (nblk <= 1024) and the row's finished flag
  constexpr int HP = 4, PP = 8;
  int hv[HP], pi[PP];
  float pv[PP];
#pragma unroll
  for (int q = 0; q < HP; ++q) hv[q] = hist[m * hist_ld + min(tid + q * 256, hist_ld - 1)];
#pragma unroll
  for (int q = 0; q < PP; ++q) {
    const int b = min(tid + q * 256, nblk - 1);
    pv[q] = part_val[(long)m * nblk + b];
    pi[q] = part_idx[(long)m * nblk + b];
  }
  const int fin = finished[m];
  // screen: the row's ln_f output, the current ban list and its length, issued with the rest
  f32x4 shv = (f32x4){0.f, 0.f, 0.f, 0.f};
  int bnv = 0, nbc = 0;
  if constexpr (SCREEN) {
    if (tid * 4 < E) shv = *reinterpret_cast<const f32x4*>(sc.sh + (long)m * E + tid * 4);
    bnv = banned[m * hist_ld + min(tid, hist_ld - 1)];
    nbc = nbanned[m];
  }
#pragma unroll
  for (int q = 0; q < HP; ++q)
    if (tid + q * 256 < step) s_h[tid + q * 256] = hv[q];
  if constexpr (SCREEN) {
    if (tid * 4 < E) *reinterpret_cast<f32x4*>(s_hf + tid * 4) = shv;
    if (tid < hist_ld) s_bn[tid] = bnv;
  }
  float bv = -INFINITY;
  int bi = 0x7fffffff;
#pragma unroll
  for (int q = 0; q < PP; ++q)
    if (tid + q * 256 < nblk) argmax_take(bv, bi, pv[q], pi[q]);
  wave_argmax(bv, bi);
  if (lane == 0) {
    sv[wave] = bv;
    si[wave] = bi;
  }
  __syncthreads();
  if constexpr (SCREEN) {
    float pb = sv[0];
    int pbi = si[0];
    for (int w = 1; w < 4; ++w) argmax_take(pb, pbi, sv[w], si[w]);
    if (!fin && pb > -INFINITY) {
      // ||h|| of the row's ln_f output (the f32 rows the screen's bf16 A operand was rounded from)
      float nh = wave_sum(sumsq4(shv));
      if (lane == 0) s_red[wave] = nh;
      __syncthreads();
      nh = (s_red[0] + s_red[1]) + (s_red[2] + s_red[3]);
      const float bmax = sc.coef * sqrtf(nh) * 1.001f;
      const float thr = pb - 2.f * bmax;  // a token below it cannot reach the max's lower bound
      float ev = -INFINITY;
      int ei = 0x7fffffff;
      const long prow = (long)m * vocab;
      // blocks whose approximate maximum reaches the threshold (partials already in registers)
      if (tid == 0) s_ncb = 0;
      __syncthreads();
#pragma unroll
      for (int q = 0; q < PP; ++q)
        if (tid + q * 256 < nblk && pv[q] >= thr) s_cb[min(atomicAdd(&s_ncb, 1), 63)] = tid + q * 256;
      __syncthreads();
      const int ncb = s_ncb;
      // the surviving columns of the candidate blocks into s_cv, 2048 column positions per pass (a
      // candidate block holds tpb * 16 <= 512 columns); past 64 candidate blocks every block is
      // scanned.  Survivors accumulate over the passes and are rescored once at the end (or whenever
      // the next pass could overflow s_cv), so the scan's proc loads and the rescoring's wte-row loads
      // are two memory round trips for the usual handful of survivors, not two per pass.
      const bool all_blocks = ncb > 64;
      const int nsb = all_blocks ? nblk : ncb, span = sc.tpb * 16;
      constexpr int PASS = 2048, CAP = 2 * PASS, CW = 4;
      auto rescore = [&](int ncv) {
        // CW candidates per wave at once (their wte rows' loads issued together); each candidate's dot
        // product is one fma chain over the row in order
        for (int i0 = wave; i0 < ncv; i0 += 4 * CW) {
          int vv[CW];
          f32x4 w4[CW][4];
#pragma unroll
          for (int c = 0; c < CW; ++c) {
            vv[c] = s_cv[min(i0 + 4 * c, ncv - 1)];
#pragma unroll
            for (int r = 0; r < 4; ++r)  // E <= 1024
              w4[c][r] = *reinterpret_cast<const f32x4*>(sc.w32 + (long)vv[c] * E + min(lane * 4 + r * 256, E - 4));
          }
#pragma unroll
          for (int c = 0; c < CW; ++c) {
            float d = 0.f;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              if (lane * 4 + r * 256 >= E) break;
              const f32x4 h4 = *reinterpret_cast<const f32x4*>(s_hf + lane * 4 + r * 256);
              d = fmaf(w4[c][r].w, h4.w, fmaf(w4[c][r].z, h4.z, fmaf(w4[c][r].y, h4.y, fmaf(w4[c][r].x, h4.x, d))));
            }
            float p = wave_sum(d);
            // RepetitionPenalty -> NoRepeatNGram -> MinNewTokens, the lm_head epilogue's order
            if (sc.rep != 1.0f) {
              bool rep_hit = false;
              for (int t = 0; t < step; ++t) rep_hit |= s_h[t] == vv[c];
              if (rep_hit) p = p < 0.f ? p * sc.rep : p / sc.rep;
            }
            bool ban_hit = false;
            for (int t = 0; t < nbc; ++t) ban_hit |= s_bn[t] == vv[c];
            if (ban_hit) p = -INFINITY;
            if (vv[c] == eos && step < sc.min_new) p = -INFINITY;
            if (i0 + 4 * c < ncv) argmax_take(ev, ei, p, vv[c]);
          }
        }
      };
      if (tid == 0) s_ncv = 0;
      __syncthreads();
      for (int from = 0; from < nsb * span; from += PASS) {
        const int lim = min(from + PASS, nsb * span);
        int cv[PASS / 256];
        float cp[PASS / 256];
#pragma unroll
        for (int r = 0; r < PASS / 256; ++r) {  // the pass's loads issued together
          const int i = from + tid + r * 256;
          const int bl = i / span, off = i - bl * span;
          cv[r] = i < lim ? (all_blocks ? bl : s_cb[min(bl, 63)]) * span + off : vocab;
          cp[r] = sc.proc[prow + min(cv[r], vocab - 1)];
        }
#pragma unroll
        for (int r = 0; r < PASS / 256; ++r)
          if (cv[r] < vocab && cp[r] >= thr) s_cv[atomicAdd(&s_ncv, 1)] = cv[r];
        __syncthreads();
        const int ncv = s_ncv;
        if (ncv > CAP - PASS || from + PASS >= nsb * span) {  // the next pass could overflow, or the last
          rescore(ncv);
          __syncthreads();  // s_cv / s_ncv reused
          if (tid == 0) s_ncv = 0;
          __syncthreads();
        }
      }
      __syncthreads();  // s_red reads done
      if (lane == 0) {
        sv[wave] = ev;
        si[wave] = ei;
      }
      __syncthreads();
      bv = sv[0];
      bi = si[0];
    }
  }
  if (tid == 0) {
    for (int w = 1; w < 4; ++w) argmax_take(bv, bi, sv[w], si[w]);
    int tok = bi;
    tok = tok < 0 ? 0 : (tok >= vocab ? vocab - 1 : tok);  // all -inf row (cannot happen with finite logits)
    if (fin) tok = pad;
    out_ids[(long)m * out_ld + step] = tok;
    hist[m * hist_ld + step] = tok;
    s_h[step] = tok;
    if (tok == eos) finished[m] = 1;
    s_tok = tok;
    s_nb = 0;
  }
  __syncthreads();
  // NoRepeatNGram ban list for the next step over the L = step+1 generated tokens
  const int L = step + 1;
  if (ngram > 0 && L + 1 >= ngram) {
    for (int i = tid; i + ngram <= L; i += 256) {
      bool match = true;
      for (int t = 0; t < ngram - 1; ++t) match &= (s_h[i + t] == s_h[L - ngram + 1 + t]);
      if (match) banned[m * hist_ld + atomicAdd(&s_nb, 1)] = s_h[i + ngram - 1];
    }
  }
  __syncthreads();
  if (tid == 0) nbanned[m] = s_nb;
  const int tok = s_tok;
  for (int c = tid; c < E; c += 256)
    h[(long)m * E + c] = Num<T>::to_f(wte[(long)tok * E + c]) + wpe[(long)pos_next * E + c];
}

// ------------------------------------------------------------------------------------------------
constexpr size_t kRowsLdsMax = 160 * 1024;  // LDS per CU (static + dynamic)

template <typename T>
constexpr bool gemv_nsl_ok(int nsl) {
  return sizeof(T) == 2 ? (nsl == 6 || nsl == 8 || nsl == 12 || nsl == 16 || nsl == 24 || nsl == 32)
                        : (nsl == 12 || nsl == 16);
}
// register budget: NSL x (NTB weight + MT activation) 16-byte fragments held at once
// (a 32-row PRO_DIRECT GEMV whose two row tiles of A fragments do not fit beside the weights streams
// them: one row tile live at a time, gemv_stream_a above the kernel)
template <typename T, int MT, int NTB, int PRO, int NSL>
constexpr bool gemv_fits() {
  constexpr int KS = 4 * Frag<T>::kElems;
  constexpr int live_a = PRO != PRO_DIRECT ? 0 : gemv_stream_a<T, MT, NTB, PRO, NSL>() ? 1 : MT;
  return gemv_nsl_ok<T>(NSL) && NSL * (NTB + live_a) <= 64 && (PRO != PRO_LN || NSL * KS * 4 <= 1024);
}

// Raise a kernel's dynamic-LDS limit once to what the CU has left beside its static LDS; returns
// that limit (0 on error).
template <typename Kern>
static int allow_lds(Kern k, int& limit) {
  if (limit > 0) return limit;
  hipFuncAttributes attr;
  if (hipFuncGetAttributes(&attr, (const void*)k) != hipSuccess) return 0;
  const int dyn = (int)kRowsLdsMax - (int)attr.sharedSizeBytes;
  if (dyn <= 0 || hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, dyn) != hipSuccess)
    return 0;
  limit = dyn;
  return limit;
}

template <typename T, int MT, int NTB, int PRO, int EPI, int NSL>
static hipError_t launch_gemv(const RowsGemmArgs& a, hipStream_t s) {
  const int half = EPI == EPI_RESID && NTB == 1 && (a.half || a.sk_part) ? 2 : 1;
  const dim3 grid(half * ((a.N + NTB * 16 - 1) / (NTB * 16)), (a.M + MT * 16 - 1) / (MT * 16));
  const size_t lds = PRO == PRO_LN ? (size_t)MT * 16 * a.K * sizeof(T) : 0;
  static int limit = 0;
  if ((size_t)allow_lds(vcap_rows_gemv_kernel<T, MT, NTB, PRO, EPI, NSL>, limit) < lds) return hipErrorInvalidValue;
  hipLaunchKernelGGL((vcap_rows_gemv_kernel<T, MT, NTB, PRO, EPI, NSL>), grid, dim3(256), lds, s, a);
  return hipGetLastError();
}

template <typename T, int MT, int NTB, int PRO, int EPI>
static hipError_t launch_generic(const RowsGemmArgs& a, hipStream_t s) {
  const dim3 grid((a.N + NTB * 16 - 1) / (NTB * 16), (a.M + MT * 16 - 1) / (MT * 16));
  const size_t lds = PRO == PRO_LN ? (size_t)MT * 16 * a.K * sizeof(T) : 0;
  static int limit = 0;
  if ((size_t)allow_lds(vcap_rows_gemm_lds_kernel<T, MT, NTB, PRO, EPI>, limit) < lds) return hipErrorInvalidValue;
  hipLaunchKernelGGL((vcap_rows_gemm_lds_kernel<T, MT, NTB, PRO, EPI>), grid, dim3(256), lds, s, a);
  return hipGetLastError();
}

template <typename T, int MT, int NTB, int PRO, int EPI, int NSL>
static bool try_gemv(int nsl, const RowsGemmArgs& a, hipStream_t s, hipError_t& err) {
  if constexpr (gemv_fits<T, MT, NTB, PRO, NSL>()) {
    if (nsl == NSL) {
      err = launch_gemv<T, MT, NTB, PRO, EPI, NSL>(a, s);
      return true;
    }
  }
  return false;
}

template <typename T, int MT, int NTB, int PRO, int EPI>
static hipError_t launch_rows(const RowsGemmArgs& a, hipStream_t s) {
  // buffer loads address the packed weights (vcap_dec_wload<false>) and a.x (vcap_dec_aload; f32
  // rows under PRO_LN) with 32-bit byte offsets
  if ((long)(a.N + 63) * a.K * (long)sizeof(T) >= 0x7FFFFFFFL ||
      (long)a.M * a.ldx * (long)(PRO == PRO_LN ? sizeof(float) : sizeof(T)) >= 0x7FFFFFFFL)
    return hipErrorInvalidValue;
  // the bf16 K-split residual GEMV (a.sk_part; the dispatcher sends it in 16-row chunks): each workgroup
  // streams half the slabs
  const bool ksplit = sizeof(T) == 2 && a.sk_part && MT == 1 && NTB == 1 && PRO == PRO_DIRECT && EPI == EPI_RESID;
  const int nsl = a.K / (16 * Frag<T>::kElems) / (ksplit ? 2 : 1);
  hipError_t err = hipSuccess;
  if (try_gemv<T, MT, NTB, PRO, EPI, 6>(nsl, a, s, err) || try_gemv<T, MT, NTB, PRO, EPI, 8>(nsl, a, s, err) ||
      try_gemv<T, MT, NTB, PRO, EPI, 12>(nsl, a, s, err) || try_gemv<T, MT, NTB, PRO, EPI, 16>(nsl, a, s, err) ||
      try_gemv<T, MT, NTB, PRO, EPI, 24>(nsl, a, s, err) || try_gemv<T, MT, NTB, PRO, EPI, 32>(nsl, a, s, err))
    return err;
  if constexpr (sizeof(T) == 4 && NTB == 1 && PRO == PRO_DIRECT && EPI == EPI_RESID) {
    // f32 mlp c_proj (K = 3072 GPT-2 small / 4096 GPT-2-medium): 8 waves x 24 / 32 slabs, 16-row
    // chunks over blockIdx.y (r05: the beam searches' 24-32 rows had taken the 64-workgroup
    // generic kernel, 21 us per launch at K = 4096)
    const bool split = a.sk_part && a.sk_cnt && (nsl == 48 || nsl == 64);   // any M: 16-row chunks
    const dim3 grid((split || a.half ? 2 : 1) * ((a.N + 15) / 16), (a.M + 15) / 16);
    if (split && nsl == 48 && a.N % 32 == 0) {
      // GPT-2 small: 4 K parts x 2-column-tile groups (the same workgroup count as the pairs)
      hipLaunchKernelGGL((vcap_rows_gemv8_kernel<float, 6, 4, 2>), grid, dim3(512), 0, s, a);
      return hipGetLastError();
    }
    if (split) {
      if (nsl == 48) hipLaunchKernelGGL((vcap_rows_gemv8_kernel<float, 12, 2, 1>), grid, dim3(512), 0, s, a);
      else hipLaunchKernelGGL((vcap_rows_gemv8_kernel<float, 16, 2, 1>), grid, dim3(512), 0, s, a);
      return hipGetLastError();
    }
    if (nsl == 48 && a.M <= 64) {
      hipLaunchKernelGGL((vcap_rows_gemv8_kernel<float, 24, 1, 1>), grid, dim3(512), 0, s, a);
      return hipGetLastError();
    }
    if (nsl == 64 && a.M <= 64) {
      hipLaunchKernelGGL((vcap_rows_gemv8_kernel<float, 32, 1, 1>), grid, dim3(512), 0, s, a);
      return hipGetLastError();
    }
  }
  return launch_generic<T, MT, NTB, PRO, EPI>(a, s);
}

// ------------------------------------------------------------------------------------------------
// lm_head (PRO_LN + EPI_LOGITS) at M <= 16 rows as a weight stream: one workgroup per CU walks a
// contiguous range of `tpw` 16-column tiles (ln_f computed once per workgroup instead of once per 4
// tiles), NTB tiles per group with the next group's weight fragments issued before this group's
// MFMAs (two register sets), the processors applied per element and a running argmax per row; one
// (max, index) partial per row per workgroup (nblk = grid).  The 77 MB of a GPT-2 vocab then
// streams on ~250 workgroups that all finish together instead of 786 workgroups at 2 per CU, whose
// last ~third ran after the rest (profiles/r03_decode_stamps.txt: 21 us per step, 14 us of it skew).
// Per-element arithmetic (K split over the 4 waves, MFMA order, (w0 + w1) + (w2 + w3) reduction,
// processors) is that of vcap_rows_gemv_kernel, so logits and ids are bit-identical; the argmax is
// a total order (value, then lowest index), so its grouping does not matter.
template <typename T, int NSL, int NTB>
__global__ __launch_bounds__(256) void vcap_lm_head_stream_kernel(RowsGemmArgs a, int tpw) {
  extern __shared__ __attribute__((aligned(16))) char dyn[];  // A tile [16][K] T, then flags
  constexpr int E8 = Frag<T>::kElems, KS = 4 * E8, K = 4 * NSL * KS;
  constexpr int KC = (K + 255) / 256;
  constexpr int kMaxCols = 32 * 16;  // tpw <= 32
  __shared__ __attribute__((aligned(16))) float red[4][NTB * 256];
  unsigned char* s_rep = reinterpret_cast<unsigned char*>(dyn + 16 * K * sizeof(T));
  unsigned char* s_ban = s_rep + 16 * kMaxCols;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  const int M = a.M, N = a.N;
  const int nslab = 4 * NSL, g0 = wave * NSL;
  const int ntiles = (N + 15) >> 4;
  const int t0 = blockIdx.x * tpw, t1 = min(t0 + tpw, ntiles);
  const int c_begin = t0 * 16, ncols = (t1 - t0) * 16;
  const int ngr = (t1 - t0 + NTB - 1) / NTB;
  auto issue = [&](u32x4 (&wf)[NSL][NTB], int gi) {
#pragma unroll
    for (int j = 0; j < NTB; ++j) {
      const u32x4* wp = packed_frag(a.w, min(t0 + gi * NTB + j, t1 - 1), nslab, g0, lane);
#pragma unroll
      for (int s = 0; s < NSL; ++s) wf[s][j] = vcap_dec_wload<true>(a.w, wp + s * 64);
    }
  };
  // first group's weights + ln_f rows + processor token lists, all issued up front
  u32x4 wA[NSL][NTB], wB[NSL][NTB];
  f32x4 xv[4][KC], gv[KC], bv[KC];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const long xo = (long)min(wave + 4 * r, M - 1) * a.ldx;
#pragma unroll
    for (int c = 0; c < KC; ++c)
      xv[r][c] = __builtin_bit_cast(f32x4, vcap_dec_aload(a.x, (xo + min(c * 256 + lane * 4, K - 4)) * 4L));
  }
#pragma unroll
  for (int c = 0; c < KC; ++c) {
    gv[c] = *reinterpret_cast<const f32x4*>(a.ln_g + min(c * 256 + lane * 4, K - 4));
    bv[c] = *reinterpret_cast<const f32x4*>(a.ln_b + min(c * 256 + lane * 4, K - 4));
  }
  issue(wA, 0);
  int htk[4], btk[4], nbk[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int i = tid + q * 256, m = min(i >> 6, M - 1), t = min(i & 63, a.hist_ld - 1);
    htk[q] = a.hist[m * a.hist_ld + t];
    btk[q] = a.banned[m * a.hist_ld + t];
    nbk[q] = a.nbanned[m];
  }
  for (int i = tid; i < 2 * 16 * kMaxCols / 4; i += 256) reinterpret_cast<unsigned*>(s_rep)[i] = 0u;
  // ln_f (vcap_rows_gemv_kernel PRO_LN arithmetic; the clamped chunks past K do not contribute)
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int m = wave + 4 * r;
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < KC; ++c)
      if (c * 256 + lane * 4 < K) s += (xv[r][c].x + xv[r][c].y) + (xv[r][c].z + xv[r][c].w);
    const float mean = wave_sum(s) / (float)K;
    float ss = 0.f;
#pragma unroll
    for (int c = 0; c < KC; ++c)
      if (c * 256 + lane * 4 < K) {
        const f32x4 d = xv[r][c] - mean;
        ss += sumsq4(d);
      }
    const float rstd = rsqrtf(wave_sum(ss) / (float)K + a.ln_eps);
    const bool live = m < M;
#pragma unroll
    for (int c = 0; c < KC; ++c) {
      if (c * 256 + lane * 4 < K) {
        const f32x4 y = live ? ln_affine4(xv[r][c], mean, rstd, gv[c], bv[c]) : (f32x4){0.f, 0.f, 0.f, 0.f};
        if (a.screen_h && blockIdx.x == 0 && live)
          *reinterpret_cast<f32x4*>(a.screen_h + (long)m * K + c * 256 + lane * 4) = y;
        const int byte = (c * 256 + lane * 4) * (int)sizeof(T);
        char* dst = dyn + (long)m * (K * (int)sizeof(T)) + ((((byte >> 4) ^ (m & 15))) << 4) + (byte & 15);
        if constexpr (sizeof(T) == 2) {
          *reinterpret_cast<u32x2*>(dst) = (u32x2){pack_bf2(y.x, y.y), pack_bf2(y.z, y.w)};
        } else {
          *reinterpret_cast<f32x4*>(dst) = y;
        }
      }
    }
  }
  __syncthreads();  // flags zeroed, A tile written
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int i = tid + q * 256, m = i >> 6, t = i & 63;
    if (m >= M) continue;
    const unsigned hc = (unsigned)(htk[q] - c_begin), bc = (unsigned)(btk[q] - c_begin);
    if (a.rep_penalty != 1.0f && t < a.gen_len && hc < (unsigned)ncols) s_rep[m * kMaxCols + hc] = 1;
    if (t < nbk[q] && bc < (unsigned)ncols) s_ban[m * kMaxCols + bc] = 1;
  }
  __syncthreads();
  const int row = tid >> 4, col = tid & 15;
  float bv_run = -INFINITY;
  int bi_run = 0x7fffffff;
  auto group = [&](const u32x4 (&wf)[NSL][NTB], int gi) {
    f32x4 acc[NTB];
#pragma unroll
    for (int j = 0; j < NTB; ++j) acc[j] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < NSL; ++s) {
      const int chunk = (g0 + s) * 4 + fg;
      const u32x4 A = *reinterpret_cast<const u32x4*>(dyn + (long)fr * K * sizeof(T) + ((chunk ^ fr) << 4));
#pragma unroll
      for (int j = 0; j < NTB; ++j) acc[j] = mfma_frag(A, wf[s][j], acc[j], (T*)nullptr);
    }
#pragma unroll
    for (int j = 0; j < NTB; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) red[wave][j * 256 + (fg * 4 + r) * 16 + fr] = acc[j][r];
    __syncthreads();
    if (row < M) {
#pragma unroll
      for (int j = 0; j < NTB; ++j) {
        const int t = t0 + gi * NTB + j, n = t * 16 + col;
        if (t < t1 && n < N) {
          const int e = j * 256 + row * 16 + col;
          const float v = (red[0][e] + red[1][e]) + (red[2][e] + red[3][e]) + 0.f;
          if (a.logits_raw) a.logits_raw[(long)row * N + n] = v;
          float sv = v;
          const int li = row * kMaxCols + (n - c_begin);
          if (s_rep[li]) sv = sv < 0.f ? sv * a.rep_penalty : sv / a.rep_penalty;
          if (s_ban[li]) sv = -INFINITY;
          if (n == a.eos && a.gen_len < a.min_new) sv = -INFINITY;
          if (a.proc_out) a.proc_out[(long)row * N + n] = sv;
          argmax_take(bv_run, bi_run, sv, n);
        }
      }
    }
    __syncthreads();
  };
  for (int gi = 0; gi < ngr; gi += 2) {
    if (gi + 1 < ngr) issue(wB, gi + 1);
    group(wA, gi);
    if (gi + 1 < ngr) {
      if (gi + 2 < ngr) issue(wA, gi + 2);
      group(wB, gi + 1);
    }
  }
  argmax_take(bv_run, bi_run, dpp_f<DPP_XOR1>(bv_run), dpp_i<DPP_XOR1>(bi_run));
  argmax_take(bv_run, bi_run, dpp_f<DPP_XOR2>(bv_run), dpp_i<DPP_XOR2>(bi_run));
  argmax_take(bv_run, bi_run, dpp_f<DPP_HALF_MIRROR>(bv_run), dpp_i<DPP_HALF_MIRROR>(bi_run));
  argmax_take(bv_run, bi_run, dpp_f<DPP_MIRROR>(bv_run), dpp_i<DPP_MIRROR>(bi_run));
  if (col == 0 && row < M) {
    a.part_val[(long)row * gridDim.x + blockIdx.x] = bv_run;
    a.part_idx[(long)row * gridDim.x + blockIdx.x] = bi_run;
  }
}

template <typename T, int NSL>
static bool launch_lm_stream(const RowsGemmArgs& a, int* nblk_out, hipStream_t s, hipError_t& err,
                             int* tpb_out = nullptr) {
  constexpr int NTB = (NSL <= 8) ? 4 : 2;  // two register sets of NSL x NTB fragments
  const int ntiles = (a.N + 15) / 16;
  const int cus = vcap_device_cus();
  const int tpw = (ntiles + cus - 1) / cus;
  const size_t lds = (size_t)16 * (4 * NSL * 4 * Frag<T>::kElems) * sizeof(T) + 2 * 16 * 32 * 16;
  static int limit = 0;
  // a vocabulary that needs > 32 tiles per CU (a device or partition with few CUs), or a kernel whose
  // LDS limit cannot be raised: not this kernel - the 64-column GEMV blocks take the lm_head
  if (tpw > 32 || (size_t)allow_lds(vcap_lm_head_stream_kernel<T, NSL, NTB>, limit) < lds) return false;
  const int grid = (ntiles + tpw - 1) / tpw;
  hipLaunchKernelGGL((vcap_lm_head_stream_kernel<T, NSL, NTB>), dim3(grid), dim3(256), lds, s, a, tpw);
  if (nblk_out) *nblk_out = grid;
  if (tpb_out) *tpb_out = tpw;
  err = hipGetLastError();
  return true;
}

// M <= 16 lm_head as the weight stream above; returns false where it does not apply
static bool try_lm_stream(int dt, const RowsGemmArgs& a, int* nblk_out, hipStream_t s, hipError_t& err) {
  if (a.M > 16 || a.hist_ld > 64) return false;
  const int nsl = a.K / (16 * (dt == VCAP_DT_BF16 ? 8 : 4));
  if ((long)a.M * a.ldx * 4 >= 0x7FFFFFFFL) return false;
#define VCAP_LMS(TT, NN) \
  if (nsl == NN) return launch_lm_stream<TT, NN>(a, nblk_out, s, err);
  if (dt == VCAP_DT_BF16) {
    VCAP_LMS(bf16_t, 1) VCAP_LMS(bf16_t, 6) VCAP_LMS(bf16_t, 8)
  } else {
    VCAP_LMS(float, 2) VCAP_LMS(float, 12) VCAP_LMS(float, 16)
  }
#undef VCAP_LMS
  return false;
}

hipError_t vcap_lm_head_screen_dispatch(const RowsGemmArgs& a, int* nblk_out, int* tpb_out, hipStream_t s) {
  if (a.M > 16 || a.hist_ld > 64 || (a.K != 768 && a.K != 1024) || !a.screen_h || !a.proc_out)
    return hipErrorNotSupported;
  if ((long)a.M * a.ldx * 4 >= 0x7FFFFFFFL) return hipErrorNotSupported;
  hipError_t err = hipSuccess;
  const bool ok = a.K == 768 ? launch_lm_stream<bf16_t, 6>(a, nblk_out, s, err, tpb_out)
                             : launch_lm_stream<bf16_t, 8>(a, nblk_out, s, err, tpb_out);
  return ok ? err : hipErrorNotSupported;
}

// ------------------------------------------------------------------------------------------------
// Beam-search lm_head (PRO_LN + EPI_LSE) at M <= 32 rows as a weight stream (r05): the structure of
// vcap_lm_head_stream_kernel - one workgroup per CU over a contiguous range of `tpw` 16-column tiles,
// ln_f once per workgroup, the next group's weight fragments in flight during this group's MFMAs -
// with both 16-row halves of a 32-row beam step (8 sequences x 4 beams) in the workgroup, so each
// weight byte is read once per step (the 64-column GEMV blocks take 16-row chunks, and the 32-row
// f32 step read the 206 MB GPT-2-medium vocab twice: 109 us).  Raw logits go to logits_raw,
// bit-identical to the GEMV path's (same K split over the 4 waves, MFMA order and reduction); each
// workgroup leaves one (max, sum exp(x - max)) partial per row, kept online per thread and merged
// over the 16 column lanes - the quantity of the GEMV epilogue's two-pass form (its rounding differs
// at the ulp level), merged by vcap_beam_cand_kernel the same way over nblk = grid partials.
template <typename T, int NSL, int NTB, int MT>
__global__ __launch_bounds__(256) void vcap_lm_head_lse_kernel(RowsGemmArgs a, int tpw) {
  extern __shared__ __attribute__((aligned(16))) char dyn[];  // A tile [MT * 16][K] T
  constexpr int E8 = Frag<T>::kElems, KS = 4 * E8, K = 4 * NSL * KS;
  constexpr int KC = (K + 255) / 256;
  constexpr int RPW = MT * 4;  // ln_f rows per wave
  __shared__ __attribute__((aligned(16))) float red[4][MT * NTB * 256];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  const int M = a.M, N = a.N;
  const int nslab = 4 * NSL, g0 = wave * NSL;
  const int ntiles = (N + 15) >> 4;
  const int t0 = blockIdx.x * tpw, t1 = min(t0 + tpw, ntiles);
  const int ngr = (t1 - t0 + NTB - 1) / NTB;
  auto issue = [&](u32x4 (&wf)[NSL][NTB], int gi) {
#pragma unroll
    for (int j = 0; j < NTB; ++j) {
      const u32x4* wp = packed_frag(a.w, min(t0 + gi * NTB + j, t1 - 1), nslab, g0, lane);
#pragma unroll
      for (int s = 0; s < NSL; ++s) wf[s][j] = vcap_dec_wload<true>(a.w, wp + s * 64);
    }
  };
  // ln_f rows + the first group's weights, issued up front
  u32x4 wA[NSL][NTB], wB[NSL][NTB];
  f32x4 xv[RPW][KC], gv[KC], bv[KC];
#pragma unroll
  for (int r = 0; r < RPW; ++r) {
    const long xo = (long)min(wave + 4 * r, M - 1) * a.ldx;
#pragma unroll
    for (int c = 0; c < KC; ++c)
      xv[r][c] = __builtin_bit_cast(f32x4, vcap_dec_aload(a.x, (xo + min(c * 256 + lane * 4, K - 4)) * 4L));
  }
#pragma unroll
  for (int c = 0; c < KC; ++c) {
    gv[c] = *reinterpret_cast<const f32x4*>(a.ln_g + min(c * 256 + lane * 4, K - 4));
    bv[c] = *reinterpret_cast<const f32x4*>(a.ln_b + min(c * 256 + lane * 4, K - 4));
  }
  issue(wA, 0);
  // ln_f (vcap_rows_gemv_kernel PRO_LN arithmetic; the clamped chunks past K do not contribute)
#pragma unroll
  for (int r = 0; r < RPW; ++r) {
    const int m = wave + 4 * r;
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < KC; ++c)
      if (c * 256 + lane * 4 < K) s += (xv[r][c].x + xv[r][c].y) + (xv[r][c].z + xv[r][c].w);
    const float mean = wave_sum(s) / (float)K;
    float ss = 0.f;
#pragma unroll
    for (int c = 0; c < KC; ++c)
      if (c * 256 + lane * 4 < K) {
        const f32x4 d = xv[r][c] - mean;
        ss += sumsq4(d);
      }
    const float rstd = rsqrtf(wave_sum(ss) / (float)K + a.ln_eps);
    const bool live = m < M;
#pragma unroll
    for (int c = 0; c < KC; ++c) {
      if (c * 256 + lane * 4 < K) {
        const f32x4 y = live ? ln_affine4(xv[r][c], mean, rstd, gv[c], bv[c]) : (f32x4){0.f, 0.f, 0.f, 0.f};
        const int byte = (c * 256 + lane * 4) * (int)sizeof(T);
        char* dst = dyn + (long)m * (K * (int)sizeof(T)) + ((((byte >> 4) ^ (m & 15))) << 4) + (byte & 15);
        if constexpr (sizeof(T) == 2) {
          *reinterpret_cast<u32x2*>(dst) = (u32x2){pack_bf2(y.x, y.y), pack_bf2(y.z, y.w)};
        } else {
          *reinterpret_cast<f32x4*>(dst) = y;
        }
      }
    }
  }
  __syncthreads();  // A tile written
  const int row = tid >> 4, col = tid & 15;
  float rmx[MT], rsm[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    rmx[i] = -INFINITY;
    rsm[i] = 0.f;
  }
  auto group = [&](const u32x4 (&wf)[NSL][NTB], int gi) {
    f32x4 acc[MT][NTB];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NTB; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < NSL; ++s) {
      const int chunk = (g0 + s) * 4 + fg;
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        const int ar = i * 16 + fr;
        const u32x4 A = *reinterpret_cast<const u32x4*>(dyn + (long)ar * K * sizeof(T) + ((chunk ^ fr) << 4));
#pragma unroll
        for (int j = 0; j < NTB; ++j) acc[i][j] = mfma_frag(A, wf[s][j], acc[i][j], (T*)nullptr);
      }
    }
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NTB; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) red[wave][(i * NTB + j) * 256 + (fg * 4 + r) * 16 + fr] = acc[i][j][r];
    __syncthreads();
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      const int m = i * 16 + row;
      if (m < M) {
#pragma unroll
        for (int j = 0; j < NTB; ++j) {
          const int t = t0 + gi * NTB + j, n = t * 16 + col;
          if (t < t1 && n < N) {
            const int e = (i * NTB + j) * 256 + row * 16 + col;
            const float v = (red[0][e] + red[1][e]) + (red[2][e] + red[3][e]) + 0.f;
            a.logits_raw[(long)m * N + n] = v;
            const float nm = fmaxf(rmx[i], v);
            rsm[i] = rsm[i] * expf(rmx[i] - nm) + expf(v - nm);
            rmx[i] = nm;
          }
        }
      }
    }
    __syncthreads();
  };
  for (int gi = 0; gi < ngr; gi += 2) {
    if (gi + 1 < ngr) issue(wB, gi + 1);
    group(wA, gi);
    if (gi + 1 < ngr) {
      if (gi + 2 < ngr) issue(wA, gi + 2);
      group(wB, gi + 1);
    }
  }
  // merge the 16 column lanes' partials of each row (a lane that saw no column holds (-inf, 0))
  auto merge = [](float& m, float& s, float om, float os) {
    const float nm = fmaxf(m, om);
    s = s * (m == nm ? 1.f : expf(m - nm)) + os * (om == nm ? 1.f : expf(om - nm));
    m = nm;
  };
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    merge(rmx[i], rsm[i], dpp_f<DPP_XOR1>(rmx[i]), dpp_f<DPP_XOR1>(rsm[i]));
    merge(rmx[i], rsm[i], dpp_f<DPP_XOR2>(rmx[i]), dpp_f<DPP_XOR2>(rsm[i]));
    merge(rmx[i], rsm[i], dpp_f<DPP_HALF_MIRROR>(rmx[i]), dpp_f<DPP_HALF_MIRROR>(rsm[i]));
    merge(rmx[i], rsm[i], dpp_f<DPP_MIRROR>(rmx[i]), dpp_f<DPP_MIRROR>(rsm[i]));
    const int m = i * 16 + row;
    if (col == 0 && m < M) {
      a.part_val[(long)m * gridDim.x + blockIdx.x] = rmx[i];
      a.part_sum[(long)m * gridDim.x + blockIdx.x] = rsm[i];
    }
  }
}

template <typename T, int NSL, int MT>
static bool launch_lm_lse(const RowsGemmArgs& a, int* nblk_out, hipStream_t s, hipError_t& err) {
  constexpr int NTB = (NSL <= 8) ? 4 : 2;  // two register sets of MT x NSL x NTB fragments
  const int ntiles = (a.N + 15) / 16;
  // one workgroup per CU, or per a.max_blocks (a beam search sharing the GPU with an encode)
  const int cus = a.max_blocks > 0 ? std::min(vcap_device_cus(), a.max_blocks) : vcap_device_cus();
  const int tpw = (ntiles + cus - 1) / cus;
  const int grid = (ntiles + tpw - 1) / tpw;
  const size_t lds = (size_t)MT * 16 * (4 * NSL * 4 * Frag<T>::kElems) * sizeof(T);
  static int limit = 0;
  // more partials than the caller's buffers hold, or an LDS limit that cannot be raised: the
  // 64-column GEMV blocks take the lm_head
  if (grid > a.nblk || (size_t)allow_lds(vcap_lm_head_lse_kernel<T, NSL, NTB, MT>, limit) < lds) return false;
  hipLaunchKernelGGL((vcap_lm_head_lse_kernel<T, NSL, NTB, MT>), dim3(grid), dim3(256), lds, s, a, tpw);
  if (nblk_out) *nblk_out = grid;
  err = hipGetLastError();
  return true;
}

static bool try_lm_lse(int dt, const RowsGemmArgs& a, int* nblk_out, hipStream_t s, hipError_t& err) {
  if (a.M > 32 || !a.logits_raw || !a.part_val || !a.part_sum) return false;
  if ((long)a.M * a.ldx * 4 >= 0x7FFFFFFFL) return false;
  const int nsl = a.K / (16 * (dt == VCAP_DT_BF16 ? 8 : 4));
  const bool two = a.M > 16;
#define VCAP_LSE(TT, NN)                                                                           \
  if (nsl == NN) return two ? launch_lm_lse<TT, NN, 2>(a, nblk_out, s, err) : launch_lm_lse<TT, NN, 1>(a, nblk_out, s, err);
  if (dt == VCAP_DT_BF16) {
    VCAP_LSE(bf16_t, 6) VCAP_LSE(bf16_t, 8)
  } else {
    VCAP_LSE(float, 12) VCAP_LSE(float, 16)
  }
#undef VCAP_LSE
  return false;
}

// 16-column tiles per workgroup: the lm_head always takes 4 (argmax partials per 64 columns; 786
// workgroups at 2 per CU.  r03: 2, 5 or 8 tiles per workgroup (1571 / 629 / 393 workgroups) measured
// +1-2 / +6 / +8 us per token step, and forcing 3 workgroups per CU (<= 168 VGPRs) +22 us);
// the projections take 1 unless a grid cap asks for wider workgroups (2 or 4 tiles).
static int rows_ntb(int epi, int N = 0, int max_blocks = 0) {
  if (epi == EPI_LOGITS || epi == EPI_LSE) return 4;
  const int tiles = (N + 15) / 16;
  if (max_blocks <= 0 || tiles <= max_blocks) return 1;
  return tiles <= 2 * max_blocks ? 2 : 4;
}

int vcap_logit_blocks(int V, int M) {
  (void)M;
  const int ntb = rows_ntb(EPI_LOGITS);
  return (V + ntb * 16 - 1) / (ntb * 16);
}

// Public dispatcher.  Rows go in chunks of MT*16 over blockIdx.y (MT = 1 for M <= 16, else 2).
hipError_t vcap_rows_gemm_dispatch(int dt, int pro, int epi, const RowsGemmArgs& a, int* nblk_out, hipStream_t s) {
  const int ks4 = dt == VCAP_DT_BF16 ? 128 : 64;  // 4 waves x one MFMA K step
  if (a.K % ks4 != 0 || a.M <= 0 || a.K <= 0 || a.N <= 0) return hipErrorInvalidValue;
  if (pro == PRO_LN && a.K > 1024) return hipErrorInvalidValue;
  if (epi == EPI_LOGITS && a.hist_ld > 64) return hipErrorInvalidValue;
  if (pro == PRO_LN && epi == EPI_LOGITS) {
    hipError_t err = hipSuccess;
    if (try_lm_stream(dt, a, nblk_out, s, err)) return err;
  }
  if (pro == PRO_LN && epi == EPI_LSE) {
    hipError_t err = hipSuccess;
    if (try_lm_lse(dt, a, nblk_out, s, err)) return err;
  }
  const int ntb = rows_ntb(epi, a.N, a.max_blocks);
  if (nblk_out) *nblk_out = (a.N + ntb * 16 - 1) / (ntb * 16);
  // residual projections (attn / mlp c_proj: N = E, 48 tiles for GPT-2) on whole tiles use a
  // workgroup per 8 columns instead of 16 when the grid may double: the per-CU weight stream, not
  // the MFMAs, bounds these GEMVs (K = 3072: 98 KB of weights per workgroup)
  RowsGemmArgs ah = a;
  const int tiles = (a.N + 15) / 16;
  ah.half = pro == PRO_DIRECT && epi == EPI_RESID && ntb == 1 && a.M <= 32 &&
            (a.max_blocks <= 0 ? 2 * tiles <= vcap_device_cus() : 2 * tiles <= a.max_blocks);
  // f32 LayerNorm-prologue rows of > 512 features in 32-row chunks would need > 64 KiB of A tile
  // beside the split-K buffers (GPT-2-medium fp32 beam search: 32 x 1024 x 4 B + 32 KiB > 160 KiB):
  // such launches take 16-row chunks (two blockIdx.y chunks per 32 rows)
  // the bf16 mlp c_proj K split (GPT-2 small's K = 3072, whole tiles) runs in 16-row chunks at every row
  // count; elsewhere a bf16 launch ignores sk_part.  (GPT-2-medium's K = 4096 keeps the one-workgroup
  // tile in bf16: its device beam search is priced against the reference's hypotheses under fp32
  // (test_l14_medium_beam4_bf16_priced_against_reference), and a beam search's path moves with any
  // change of bf16 summation order.)
  if (dt == VCAP_DT_BF16 && ah.sk_part &&
      !(pro == PRO_DIRECT && epi == EPI_RESID && ntb == 1 && a.K == 3072)) {
    ah.sk_part = nullptr;
    ah.sk_cnt = nullptr;
  }
  const bool bsplit = dt == VCAP_DT_BF16 && ah.sk_part;
  const bool one = a.M <= 16 || bsplit || (pro == PRO_LN && dt != VCAP_DT_BF16 && a.K > 512);
#define VCAP_ROWS(TT, PP, EE, NT) \
  return one ? launch_rows<TT, 1, NT, PP, EE>(ah, s) : launch_rows<TT, 2, NT, PP, EE>(ah, s);
#define VCAP_ROWS_NT(TT, PP, EE)            \
  if (ntb == 4) { VCAP_ROWS(TT, PP, EE, 4) } \
  if (ntb == 2) { VCAP_ROWS(TT, PP, EE, 2) } \
  VCAP_ROWS(TT, PP, EE, 1)
#define VCAP_ROWS_EPI(TT)                                                                    \
  if (pro == PRO_LN && epi == EPI_QKV) { VCAP_ROWS_NT(TT, PRO_LN, EPI_QKV) }                \
  if (pro == PRO_LN && epi == EPI_GELU) { VCAP_ROWS_NT(TT, PRO_LN, EPI_GELU) }              \
  if (pro == PRO_DIRECT && epi == EPI_RESID) { VCAP_ROWS_NT(TT, PRO_DIRECT, EPI_RESID) }    \
  if (pro == PRO_LN && epi == EPI_LOGITS) { VCAP_ROWS(TT, PRO_LN, EPI_LOGITS, 4) }            \
  if (pro == PRO_LN && epi == EPI_LSE) { VCAP_ROWS(TT, PRO_LN, EPI_LSE, 4) }
  if (dt == VCAP_DT_BF16) {
    VCAP_ROWS_EPI(bf16_t)
  } else {
    VCAP_ROWS_EPI(float)
  }
#undef VCAP_ROWS_EPI
#undef VCAP_ROWS_NT
#undef VCAP_ROWS
  return hipErrorInvalidValue;
}

hipError_t vcap_rows_pack_dispatch(int dt, const void* w, long ldw, int N, int K, void* packed, hipStream_t s) {
  const int ks = dt == VCAP_DT_BF16 ? 32 : 16;
  const size_t esz = dt == VCAP_DT_BF16 ? 2 : 4;
  if (N <= 0 || K <= 0 || K % ks != 0 || (ldw * esz) % 16 != 0 || ((uintptr_t)w & 15) || ((uintptr_t)packed & 15))
    return hipErrorInvalidValue;
  const long chunks = (long)((N + 15) / 16) * (K / ks) * 64;
  const int blocks = (int)std::min<long>((chunks + 255) / 256, 4096);
  if (dt == VCAP_DT_BF16)
    hipLaunchKernelGGL((vcap_rows_pack_kernel<bf16_t>), dim3(blocks), dim3(256), 0, s, (const bf16_t*)w, ldw, N, K,
                       (u32x4*)packed);
  else
    hipLaunchKernelGGL((vcap_rows_pack_kernel<float>), dim3(blocks), dim3(256), 0, s, (const float*)w, ldw, N, K,
                       (u32x4*)packed);
  return hipGetLastError();
}

size_t vcap_rows_packed_size(int dt, int N, int K) {
  const int ks = dt == VCAP_DT_BF16 ? 32 : 16;
  return (size_t)((N + 15) / 16) * (size_t)(K / ks) * 1024;
}

// bf16 fast path for contexts of at most 64 positions with the contiguous page layout the
// runtime allocates (page of position j of sequence `seq` = seq * maxp + j / 16, i.e. the identity
// page table): page ids are computed, not loaded, and q, the lane's K row and all of its V rows
// are issued together, so the wave pays ONE memory round trip instead of three
// (page table -> K -> V).  Arithmetic identical to vcap_decode_attention_kernel.
__global__ __launch_bounds__(64) void vcap_decode_attention_c64_kernel(const bf16_t* __restrict__ q,
                                                                       const bf16_t* __restrict__ kc,
                                                                       const bf16_t* __restrict__ vc, int maxp,
                                                                       bf16_t* __restrict__ out, int M, int H,
                                                                       int S_new, int past) {
  __shared__ float s_q[64];
  __shared__ float s_p[64];
  const int item = blockIdx.x;  // one 64-thread workgroup per (row, head)
  if (item >= M * H) return;
  const int m = item / H, h = item - m * H;
  const int seq = m / S_new, qpos = past + (m - seq * S_new);
  const int ctx = qpos + 1;  // <= 64 (dispatcher)
  C64Loads L;
  c64_issue(L, q, kc, vc, maxp, m, h, H, seq, ctx);
  c64_finish(L, s_q, s_p, ctx, out + (long)m * H * 64 + h * 64);
}

__global__ __launch_bounds__(64) void vcap_decode_attention_c64f_kernel(const float* __restrict__ q,
                                                                        const float* __restrict__ kc,
                                                                        const float* __restrict__ vc, int maxp,
                                                                        float* __restrict__ out, int M, int H,
                                                                        int S_new, int past) {
  __shared__ __attribute__((aligned(16))) float s_q[64];
  __shared__ float s_p[64];
  const int item = blockIdx.x;
  if (item >= M * H) return;
  const int m = item / H, h = item - m * H;
  const int seq = m / S_new, qpos = past + (m - seq * S_new);
  const int ctx = qpos + 1;  // <= 64 (dispatcher)
  C64LoadsF L;
  c64f_issue(L, q, kc, vc, maxp, m, h, H, seq, ctx);
  c64f_finish(L, s_q, s_p, ctx, out + (long)m * H * 64 + h * 64);
}

hipError_t vcap_decode_attention_dispatch(int dt, const void* q, const void* kc, const void* vc, const int* pt,
                                          int maxp, void* out, int M, int H, int S_new, int past, hipStream_t s) {
  if (past + S_new > 1024 || maxp > 64) return hipErrorInvalidValue;
  const dim3 grid((M * H + 3) / 4), block(256);
  if (dt == VCAP_DT_BF16 && !pt && past + S_new <= 64) {
    // one 64-thread workgroup per (row, head): the ~100-200 items of a decode step spread over as
    // many CUs (each item's q / K / V round trip on a CU of its own) instead of 4 per CU
    hipLaunchKernelGGL(vcap_decode_attention_c64_kernel, dim3(M * H), dim3(64), 0, s, (const bf16_t*)q,
                       (const bf16_t*)kc, (const bf16_t*)vc, maxp, (bf16_t*)out, M, H, S_new, past);
    return hipGetLastError();
  }
  if (dt == VCAP_DT_F32 && !pt && past + S_new <= 64) {
    hipLaunchKernelGGL(vcap_decode_attention_c64f_kernel, dim3(M * H), dim3(64), 0, s, (const float*)q,
                       (const float*)kc, (const float*)vc, maxp, (float*)out, M, H, S_new, past);
    return hipGetLastError();
  }
  if (!pt) return hipErrorInvalidValue;  // the general kernels read the page table
  if (dt == VCAP_DT_BF16)
    hipLaunchKernelGGL((vcap_decode_attention_kernel<bf16_t>), grid, block, 0, s, (const bf16_t*)q,
                       (const bf16_t*)kc, (const bf16_t*)vc, pt, maxp, (bf16_t*)out, M, H, S_new, past);
  else
    hipLaunchKernelGGL((vcap_decode_attention_kernel<float>), grid, block, 0, s, (const float*)q, (const float*)kc,
                       (const float*)vc, pt, maxp, (float*)out, M, H, S_new, past);
  return hipGetLastError();
}

hipError_t vcap_prefill_embed_dispatch(int dt, const float* prefix, int P, const int* ids, int nids, const void* wte,
                                       const float* wpe, float* h, int B, int E, hipStream_t s, int pos0,
                                       int prefix_rep) {
  if (nids > 64) return hipErrorInvalidValue;
  PromptIds pr;
  pr.n = nids;
  for (int i = 0; i < 64; ++i) pr.ids[i] = i < nids ? ids[i] : 0;
  const int S0 = P + nids;
  if (dt == VCAP_DT_BF16)
    hipLaunchKernelGGL((vcap_prefill_embed_kernel<bf16_t>), dim3(B * S0), dim3(256), 0, s, prefix, P, pr,
                       (const bf16_t*)wte, wpe, h, S0, E, pos0, prefix_rep);
  else
    hipLaunchKernelGGL((vcap_prefill_embed_kernel<float>), dim3(B * S0), dim3(256), 0, s, prefix, P, pr,
                       (const float*)wte, wpe, h, S0, E, pos0, prefix_rep);
  return hipGetLastError();
}

hipError_t vcap_embed_tokens_dispatch(int dt, const int* tok, int rows, const void* wte, const float* wpe, float* h,
                                      int E, int pos, hipStream_t s) {
  if (dt == VCAP_DT_BF16)
    hipLaunchKernelGGL((vcap_embed_tokens_kernel<bf16_t>), dim3(rows), dim3(256), 0, s, tok, (const bf16_t*)wte, wpe, h,
                       E, pos);
  else
    hipLaunchKernelGGL((vcap_embed_tokens_kernel<float>), dim3(rows), dim3(256), 0, s, tok, (const float*)wte, wpe, h, E,
                       pos);
  return hipGetLastError();
}

hipError_t vcap_kv_gather_dispatch(int dt, const void* src_pool, void* dst_pool, const int* src_rows, int rows, int maxp,
                                   int H, int len, long layer_elems, int L, hipStream_t s) {
  if (dt == VCAP_DT_BF16)
    hipLaunchKernelGGL((vcap_kv_gather_kernel<bf16_t>), dim3(rows, L), dim3(256), 0, s, (const bf16_t*)src_pool,
                       (bf16_t*)dst_pool, src_rows, maxp, H, len, layer_elems, L);
  else
    hipLaunchKernelGGL((vcap_kv_gather_kernel<float>), dim3(rows, L), dim3(256), 0, s, (const float*)src_pool,
                       (float*)dst_pool, src_rows, maxp, H, len, layer_elems, L);
  return hipGetLastError();
}

hipError_t vcap_decode_init_dispatch(int* page_table, int B, int maxp, int* finished, int* nbanned, hipStream_t s,
                                     int* sk_cnt, int n_sk) {
  const int n = std::max(std::max(B * maxp, B), sk_cnt ? n_sk : 0);
  hipLaunchKernelGGL(vcap_decode_init_kernel, dim3((n + 255) / 256), dim3(256), 0, s, page_table, B, maxp, finished,
                     nbanned, sk_cnt, sk_cnt ? n_sk : 0);
  return hipGetLastError();
}

hipError_t vcap_decode_finalize_dispatch(int dt, const float* part_val, const int* part_idx, int nblk, int B,
                                         int step, int* finished, int* hist, int hist_ld, int* banned, int* nbanned,
                                         int ngram, int eos, int pad, int* out_ids, int out_ld, const void* wte,
                                         const float* wpe, float* h, int E, int pos_next, int vocab, hipStream_t s,
                                         const ScreenArgs* screen) {
  if (hist_ld > 1024 || nblk < 1 || nblk > 2048 || step >= hist_ld) return hipErrorInvalidValue;
  ScreenArgs sc{};
  if (screen) {
    if (dt != VCAP_DT_F32 || E > 1024 || E % 4 || hist_ld > 256 || screen->tpb < 1 || !screen->proc || !screen->sh ||
        !screen->w32)
      return hipErrorInvalidValue;
    sc = *screen;
  }
  if (dt == VCAP_DT_BF16)
    hipLaunchKernelGGL((vcap_decode_finalize_kernel<bf16_t, false>), dim3(B), dim3(256), 0, s, part_val, part_idx,
                       nblk, step, finished, hist, hist_ld, banned, nbanned, ngram, eos, pad, out_ids, out_ld,
                       (const bf16_t*)wte, wpe, h, E, pos_next, vocab, sc);
  else if (screen)
    hipLaunchKernelGGL((vcap_decode_finalize_kernel<float, true>), dim3(B), dim3(256), 0, s, part_val, part_idx,
                       nblk, step, finished, hist, hist_ld, banned, nbanned, ngram, eos, pad, out_ids, out_ld,
                       (const float*)wte, wpe, h, E, pos_next, vocab, sc);
  else
    hipLaunchKernelGGL((vcap_decode_finalize_kernel<float, false>), dim3(B), dim3(256), 0, s, part_val, part_idx,
                       nblk, step, finished, hist, hist_ld, banned, nbanned, ngram, eos, pad, out_ids, out_ld,
                       (const float*)wte, wpe, h, E, pos_next, vocab, sc);
  return hipGetLastError();
}
