// GPT-2 decoder step kernels with a paged KV cache and on-device greedy logits processing.
//
// Replaces the arithmetic of HF GPT2LMHeadModel.generate as the reference calls it
// (src/models/text_decoder.py:131-144) and the benchmark's raw greedy loop
// (core/scripts/benchmark_baseline.py:160-240):
//   per layer: h += c_proj(attn(ln_1(h)));  h += mlp_c_proj(gelu_new(c_fc(ln_2(h))))
//   then logits = ln_f(h) . wte^T, RepetitionPenalty -> NoRepeatNGram -> MinNewTokens -> argmax.
//
// Rows: M = B*S_new rows per step (S_new = prefix+prompt length at prefill, 1 while decoding).
// Weights are pre-transposed to [N, K] (K contiguous) so every projection is a skinny MFMA
// GEMM: a workgroup of 4 waves owns NTB 16-column tiles for all M rows and splits K over its
// waves (4 independent HBM streams per workgroup); partial tiles are summed through LDS.
// LayerNorm is fused into the A-operand prologue (each workgroup recomputes the M row
// statistics from the L2-resident residual stream instead of paying a launch + round trip).
#include "vcap_common.h"
#include "vcap_kernels.h"

template <typename T, int MT, int NTB, int PRO, int EPI>
__global__ __launch_bounds__(256) void vcap_rows_gemm_kernel(RowsGemmArgs a) {
  constexpr int E = Frag<T>::kElems;
  constexpr int KS = 4 * E;  // K per MFMA group (32 bf16 / 16 f32)
  constexpr int U = 4;       // k-slabs of W fragments kept in flight
  __shared__ float s_mean[MT * 16], s_rstd[MT * 16];
  __shared__ __attribute__((aligned(16))) float red[4][MT * NTB * 256];
  __shared__ float lg[EPI == EPI_LOGITS ? MT * 16 : 1][NTB * 16];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  const int M = a.M, N = a.N, K = a.K;
  const int n0 = blockIdx.x * NTB * 16;

  if constexpr (PRO == PRO_LN) {
    const float* X = (const float*)a.x;
    for (int m = wave; m < M; m += 4) {
      const float* xr = X + (long)m * a.ldx;
      float s = 0.f;
      for (int c = lane; c < K; c += 64) s += xr[c];
      const float mean = wave_sum(s) / (float)K;
      float ss = 0.f;
      for (int c = lane; c < K; c += 64) {
        const float d = xr[c] - mean;
        ss += d * d;
      }
      const float var = wave_sum(ss) / (float)K;  // whole-wave reduction, outside the lane-0 branch
      if (lane == 0) {
        s_mean[m] = mean;
        s_rstd[m] = rsqrtf(var + a.ln_eps);
      }
    }
    __syncthreads();
  }

  f32x4 acc[MT][NTB];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NTB; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const T* W = (const T*)a.w;
  const int kq = K / 4, kb = wave * kq, nsl = kq / KS;
  int wrow[NTB];
#pragma unroll
  for (int j = 0; j < NTB; ++j) {
    const int n = n0 + j * 16 + fr;
    wrow[j] = n < N ? n : N - 1;
  }
  for (int s0 = 0; s0 < nsl; s0 += U) {
    u32x4 wf[U][NTB];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < NTB; ++j)
        if (s0 + u < nsl)
          wf[u][j] = __builtin_nontemporal_load(
              reinterpret_cast<const u32x4*>(W + (long)wrow[j] * a.ldw + kb + (s0 + u) * KS + fg * E));
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (s0 + u >= nsl) break;
      const int k = kb + (s0 + u) * KS + fg * E;
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        const int m = i * 16 + fr;
        u32x4 af = (u32x4){0u, 0u, 0u, 0u};
        if (m < M) {
          if constexpr (PRO == PRO_LN) {
            const float* xr = (const float*)a.x + (long)m * a.ldx + k;
            const float mu = s_mean[m], rs = s_rstd[m];
            if constexpr (sizeof(T) == 2) {
              const f32x4 x0 = *reinterpret_cast<const f32x4*>(xr);
              const f32x4 x1 = *reinterpret_cast<const f32x4*>(xr + 4);
              const f32x4 g0 = *reinterpret_cast<const f32x4*>(a.ln_g + k);
              const f32x4 g1 = *reinterpret_cast<const f32x4*>(a.ln_g + k + 4);
              const f32x4 b0 = *reinterpret_cast<const f32x4*>(a.ln_b + k);
              const f32x4 b1 = *reinterpret_cast<const f32x4*>(a.ln_b + k + 4);
              const f32x4 y0 = (x0 - mu) * rs * g0 + b0;
              const f32x4 y1 = (x1 - mu) * rs * g1 + b1;
              af = (u32x4){pack_bf2(y0.x, y0.y), pack_bf2(y0.z, y0.w), pack_bf2(y1.x, y1.y), pack_bf2(y1.z, y1.w)};
            } else {
              const f32x4 x0 = *reinterpret_cast<const f32x4*>(xr);
              const f32x4 g0 = *reinterpret_cast<const f32x4*>(a.ln_g + k);
              const f32x4 b0 = *reinterpret_cast<const f32x4*>(a.ln_b + k);
              const f32x4 y0 = (x0 - mu) * rs * g0 + b0;
              af = (u32x4){__float_as_uint(y0.x), __float_as_uint(y0.y), __float_as_uint(y0.z),
                           __float_as_uint(y0.w)};
            }
          } else {
            af = *reinterpret_cast<const u32x4*>((const T*)a.x + (long)m * a.ldx + k);
          }
        }
#pragma unroll
        for (int j = 0; j < NTB; ++j) acc[i][j] = mfma_frag(af, wf[u][j], acc[i][j], (T*)nullptr);
      }
    }
  }

  // split-K reduction over the 4 waves
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NTB; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) red[wave][(i * NTB + j) * 256 + (fg * 4 + r) * 16 + fr] = acc[i][j][r];
  __syncthreads();

  for (int e = tid; e < MT * NTB * 256; e += 256) {
    const int tile = e >> 8, within = e & 255;
    const int i = tile / NTB, j = tile % NTB;
    const int row = within >> 4, col = within & 15;
    const int m = i * 16 + row, n = n0 + j * 16 + col;
    float v = red[0][e] + red[1][e] + red[2][e] + red[3][e];
    const bool ok = (m < M) && (n < N);
    if (ok && a.bias) v += a.bias[n];
    if constexpr (EPI == EPI_QKV) {
      if (ok) {
        const int Ed = N / 3;
        const int which = n / Ed, within_e = n % Ed;
        if (which == 0) {
          ((T*)a.q_out)[(long)m * Ed + within_e] = Num<T>::from_f(v);
        } else {
          const int head = within_e >> 6, d = within_e & 63;
          const int seq = m / a.S_new, pos = a.past + (m % a.S_new);
          const int page = a.page_table[seq * a.maxp + (pos >> 4)];
          T* pool = (T*)(which == 1 ? a.kc : a.vc);
          pool[(((long)page * a.H + head) * 16 + (pos & 15)) * 64 + d] = Num<T>::from_f(v);
        }
      }
    } else if constexpr (EPI == EPI_RESID) {
      if (ok) ((float*)a.out)[(long)m * a.ldo + n] += v;
    } else if constexpr (EPI == EPI_GELU) {
      if (ok) ((T*)a.out)[(long)m * a.ldo + n] = Num<T>::from_f(gelu_tanh(v));
    } else if constexpr (EPI == EPI_STORE) {
      if (ok) ((T*)a.out)[(long)m * a.ldo + n] = Num<T>::from_f(v);
    } else {  // EPI_LOGITS
      if (m < M) {
        float sv = -INFINITY;
        if (n < N) {
          if (a.logits_raw) a.logits_raw[(long)m * N + n] = v;
          sv = v;
          if (a.rep_penalty != 1.0f) {
            bool hit = false;
            for (int t = 0; t < a.gen_len; ++t) hit |= (a.hist[m * a.hist_ld + t] == n);
            if (hit) sv = sv < 0.f ? sv * a.rep_penalty : sv / a.rep_penalty;
          }
          const int nb = a.nbanned ? a.nbanned[m] : 0;
          for (int t = 0; t < nb; ++t)
            if (a.banned[m * a.hist_ld + t] == n) sv = -INFINITY;
          if (n == a.eos && a.gen_len < a.min_new) sv = -INFINITY;
        }
        lg[m][j * 16 + col] = sv;
      }
    }
  }
  if constexpr (EPI == EPI_LOGITS) {
    __syncthreads();
    for (int m = wave; m < M; m += 4) {
      float bv = -INFINITY;
      int bi = 0x7fffffff;
      for (int c = lane; c < NTB * 16; c += 64) {
        const float v = lg[m][c];
        const int n = n0 + c;
        if (v > bv || (v == bv && n < bi)) {
          bv = v;
          bi = n;
        }
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        const float ov = __shfl_xor(bv, o, 64);
        const int oi = __shfl_xor(bi, o, 64);
        if (ov > bv || (ov == bv && oi < bi)) {
          bv = ov;
          bi = oi;
        }
      }
      if (lane == 0) {
        a.part_val[(long)m * a.nblk + blockIdx.x] = bv;
        a.part_idx[(long)m * a.nblk + blockIdx.x] = bi;
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------
// Causal attention of S_new query rows per sequence over the paged cache (positions 0..past+i).
template <typename T>
__global__ __launch_bounds__(256) void vcap_decode_attention_kernel(const T* __restrict__ q, const T* __restrict__ kc,
                                                                    const T* __restrict__ vc,
                                                                    const int* __restrict__ page_table, int maxp,
                                                                    T* __restrict__ out, int M, int H, int S_new,
                                                                    int past) {
  __shared__ float s_q[4][64];
  __shared__ float s_p[4][1024];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int item = blockIdx.x * 4 + wave;
  if (item >= M * H) return;
  const int m = item / H, h = item % H;
  const int E = H * 64;
  const int seq = m / S_new, qpos = past + (m % S_new);
  const int ctx = qpos + 1;
  s_q[wave][lane] = Num<T>::to_f(q[(long)m * E + h * 64 + lane]);
  __builtin_amdgcn_wave_barrier();
  const int* pt = page_table + seq * maxp;
  float mx = -INFINITY;
  for (int j = lane; j < ctx; j += 64) {
    const T* krow = kc + (((long)pt[j >> 4] * H + h) * 16 + (j & 15)) * 64;
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < 64; c += Frag<T>::kElems) {
      const u32x4 kv = *reinterpret_cast<const u32x4*>(krow + c);
      const T* ke = reinterpret_cast<const T*>(&kv);
#pragma unroll
      for (int e = 0; e < Frag<T>::kElems; ++e) s += s_q[wave][c + e] * Num<T>::to_f(ke[e]);
    }
    s *= 0.125f;
    s_p[wave][j] = s;
    mx = fmaxf(mx, s);
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
  float o = 0.f;
  for (int j = 0; j < ctx; ++j) {
    const T* vrow = vc + (((long)pt[j >> 4] * H + h) * 16 + (j & 15)) * 64;
    o += s_p[wave][j] * Num<T>::to_f(vrow[lane]);
  }
  out[(long)m * E + h * 64 + lane] = Num<T>::from_f(o / sum);
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
                                                                 int S0, int E) {
  const int m = blockIdx.x;
  const int s = m / S0, i = m % S0;
  for (int c = threadIdx.x; c < E; c += 256) {
    float v = (i < P) ? prefix[((long)s * P + i) * E + c] : Num<T>::to_f(wte[(long)prompt.ids[i - P] * E + c]);
    h[(long)m * E + c] = v + wpe[(long)i * E + c];
  }
}

// Per-step state init: identity page tables, cleared history / flags.
__global__ void vcap_decode_init_kernel(int* page_table, int B, int maxp, int* finished, int* nbanned) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < B * maxp) page_table[i] = i;
  if (i < B) {
    finished[i] = 0;
    nbanned[i] = 0;
  }
}

// Reduce the per-workgroup argmax partials, apply EOS padding, record the token, precompute the
// n-gram ban list for the next step and write the next input embedding wte[tok] + wpe[pos].
template <typename T>
__global__ __launch_bounds__(256) void vcap_decode_finalize_kernel(
    const float* __restrict__ part_val, const int* __restrict__ part_idx, int nblk, int step, int* finished,
    int* hist, int hist_ld, int* banned, int* nbanned, int ngram, int eos, int pad, int* out_ids, int out_ld,
    const T* __restrict__ wte, const float* __restrict__ wpe, float* __restrict__ h, int E, int pos_next) {
  __shared__ float sv[256];
  __shared__ int si[256];
  __shared__ int s_tok;
  const int m = blockIdx.x, tid = threadIdx.x;
  float bv = -INFINITY;
  int bi = 0x7fffffff;
  for (int b = tid; b < nblk; b += 256) {
    const float v = part_val[(long)m * nblk + b];
    const int i = part_idx[(long)m * nblk + b];
    if (v > bv || (v == bv && i < bi)) {
      bv = v;
      bi = i;
    }
  }
  sv[tid] = bv;
  si[tid] = bi;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (tid < o) {
      const float ov = sv[tid + o];
      const int oi = si[tid + o];
      if (ov > sv[tid] || (ov == sv[tid] && oi < si[tid])) {
        sv[tid] = ov;
        si[tid] = oi;
      }
    }
    __syncthreads();
  }
  if (tid == 0) {
    int tok = si[0];
    if (finished[m]) tok = pad;
    out_ids[(long)m * out_ld + step] = tok;
    hist[m * hist_ld + step] = tok;
    if (tok == eos) finished[m] = 1;
    // NoRepeatNGram ban list for the next step over the L = step+1 generated tokens
    const int L = step + 1;
    int nb = 0;
    if (ngram > 0 && L + 1 >= ngram) {
      const int* hs = hist + m * hist_ld;
      for (int i = 0; i + ngram <= L; ++i) {
        bool match = true;
        for (int t = 0; t < ngram - 1; ++t) match &= (hs[i + t] == hs[L - ngram + 1 + t]);
        if (match) banned[m * hist_ld + nb++] = hs[i + ngram - 1];
      }
    }
    nbanned[m] = nb;
    s_tok = tok;
  }
  __syncthreads();
  const int tok = s_tok;
  for (int c = tid; c < E; c += 256)
    h[(long)m * E + c] = Num<T>::to_f(wte[(long)tok * E + c]) + wpe[(long)pos_next * E + c];
}

// ------------------------------------------------------------------------------------------------
template <typename T, int MT, int NTB, int PRO, int EPI>
static hipError_t launch_rows(const RowsGemmArgs& a, hipStream_t s) {
  const int nblk = (a.N + NTB * 16 - 1) / (NTB * 16);
  hipLaunchKernelGGL((vcap_rows_gemm_kernel<T, MT, NTB, PRO, EPI>), dim3(nblk), dim3(256), 0, s, a);
  return hipGetLastError();
}

template <typename T, int PRO, int EPI, int NTB>
static hipError_t launch_rows_mt(const RowsGemmArgs& a, hipStream_t s) {
  const int mt = (a.M + 15) / 16;
  if (mt <= 1) return launch_rows<T, 1, NTB, PRO, EPI>(a, s);
  if (mt <= 2) return launch_rows<T, 2, NTB, PRO, EPI>(a, s);
  if constexpr (NTB <= 2) {
    if (mt <= 4) return launch_rows<T, 4, NTB, PRO, EPI>(a, s);
  }
  if constexpr (NTB <= 1) {
    if (mt <= 8) return launch_rows<T, 8, NTB, PRO, EPI>(a, s);
  }
  return hipErrorInvalidValue;
}

static int rows_ntb(int epi, int M) {
  const int mt = (M + 15) / 16;
  return (epi == EPI_LOGITS) ? (mt <= 2 ? 4 : (mt <= 4 ? 2 : 1)) : 1;
}

int vcap_logit_blocks(int V, int M) {
  const int ntb = rows_ntb(EPI_LOGITS, M);
  return (V + ntb * 16 - 1) / (ntb * 16);
}

// Public dispatcher: picks NTB so the whole M fits (MT*NTB <= 8); logits prefer wide tiles.
hipError_t vcap_rows_gemm_dispatch(int dt, int pro, int epi, const RowsGemmArgs& a, int* nblk_out, hipStream_t s) {
  if (a.K % 64 != 0 || a.M <= 0 || a.M > 128) return hipErrorInvalidValue;
  const int ntb = rows_ntb(epi, a.M);
  if (nblk_out) *nblk_out = (a.N + ntb * 16 - 1) / (ntb * 16);
#define VCAP_ROWS_CASE(TT, PP, EE)                                          \
  if (ntb == 4) return launch_rows_mt<TT, PP, EE, 4>(a, s);                \
  if (ntb == 2) return launch_rows_mt<TT, PP, EE, 2>(a, s);                \
  return launch_rows_mt<TT, PP, EE, 1>(a, s);
#define VCAP_ROWS_EPI(TT)                                                                   \
  if (pro == PRO_LN && epi == EPI_QKV) { VCAP_ROWS_CASE(TT, PRO_LN, EPI_QKV) }             \
  if (pro == PRO_LN && epi == EPI_GELU) { VCAP_ROWS_CASE(TT, PRO_LN, EPI_GELU) }           \
  if (pro == PRO_DIRECT && epi == EPI_RESID) { VCAP_ROWS_CASE(TT, PRO_DIRECT, EPI_RESID) } \
  if (pro == PRO_DIRECT && epi == EPI_LOGITS) { VCAP_ROWS_CASE(TT, PRO_DIRECT, EPI_LOGITS) } \
  if (pro == PRO_DIRECT && epi == EPI_STORE) { VCAP_ROWS_CASE(TT, PRO_DIRECT, EPI_STORE) } \
  if (pro == PRO_LN && epi == EPI_STORE) { VCAP_ROWS_CASE(TT, PRO_LN, EPI_STORE) }
  if (dt == VCAP_DT_BF16) {
    VCAP_ROWS_EPI(bf16_t)
  } else {
    VCAP_ROWS_EPI(float)
  }
#undef VCAP_ROWS_EPI
#undef VCAP_ROWS_CASE
  return hipErrorInvalidValue;
}

hipError_t vcap_decode_attention_dispatch(int dt, const void* q, const void* kc, const void* vc, const int* pt,
                                          int maxp, void* out, int M, int H, int S_new, int past, hipStream_t s) {
  if (past + S_new > 1024) return hipErrorInvalidValue;
  const dim3 grid((M * H + 3) / 4), block(256);
  if (dt == VCAP_DT_BF16)
    hipLaunchKernelGGL((vcap_decode_attention_kernel<bf16_t>), grid, block, 0, s, (const bf16_t*)q,
                       (const bf16_t*)kc, (const bf16_t*)vc, pt, maxp, (bf16_t*)out, M, H, S_new, past);
  else
    hipLaunchKernelGGL((vcap_decode_attention_kernel<float>), grid, block, 0, s, (const float*)q, (const float*)kc,
                       (const float*)vc, pt, maxp, (float*)out, M, H, S_new, past);
  return hipGetLastError();
}

hipError_t vcap_prefill_embed_dispatch(int dt, const float* prefix, int P, const int* ids, int nids, const void* wte,
                                       const float* wpe, float* h, int B, int E, hipStream_t s) {
  if (nids > 64) return hipErrorInvalidValue;
  PromptIds pr;
  pr.n = nids;
  for (int i = 0; i < 64; ++i) pr.ids[i] = i < nids ? ids[i] : 0;
  const int S0 = P + nids;
  if (dt == VCAP_DT_BF16)
    hipLaunchKernelGGL((vcap_prefill_embed_kernel<bf16_t>), dim3(B * S0), dim3(256), 0, s, prefix, P, pr,
                       (const bf16_t*)wte, wpe, h, S0, E);
  else
    hipLaunchKernelGGL((vcap_prefill_embed_kernel<float>), dim3(B * S0), dim3(256), 0, s, prefix, P, pr,
                       (const float*)wte, wpe, h, S0, E);
  return hipGetLastError();
}

hipError_t vcap_decode_init_dispatch(int* page_table, int B, int maxp, int* finished, int* nbanned, hipStream_t s) {
  const int n = B * maxp > B ? B * maxp : B;
  hipLaunchKernelGGL(vcap_decode_init_kernel, dim3((n + 255) / 256), dim3(256), 0, s, page_table, B, maxp, finished,
                     nbanned);
  return hipGetLastError();
}

hipError_t vcap_decode_finalize_dispatch(int dt, const float* part_val, const int* part_idx, int nblk, int B,
                                         int step, int* finished, int* hist, int hist_ld, int* banned, int* nbanned,
                                         int ngram, int eos, int pad, int* out_ids, int out_ld, const void* wte,
                                         const float* wpe, float* h, int E, int pos_next, hipStream_t s) {
  if (dt == VCAP_DT_BF16)
    hipLaunchKernelGGL((vcap_decode_finalize_kernel<bf16_t>), dim3(B), dim3(256), 0, s, part_val, part_idx, nblk,
                       step, finished, hist, hist_ld, banned, nbanned, ngram, eos, pad, out_ids, out_ld,
                       (const bf16_t*)wte, wpe, h, E, pos_next);
  else
    hipLaunchKernelGGL((vcap_decode_finalize_kernel<float>), dim3(B), dim3(256), 0, s, part_val, part_idx, nblk,
                       step, finished, hist, hist_ld, banned, nbanned, ngram, eos, pad, out_ids, out_ld,
                       (const float*)wte, wpe, h, E, pos_next);
  return hipGetLastError();
}
