// Device beam search: HF `GenerationMixin._beam_search` (transformers 5.15.0, the copy this image
// holds; the reference pins 4.57.1 - SURVEY.md §8c) as the reference reaches it through
// text_decoder.py:131-144 with inputs_embeds (the `precise` / `detailed` presets,
// core/inference.py:8-11: num_beams 3 / 4, length_penalty 1.0, early_stopping False), with every
// step's bookkeeping on the device so the whole search is one captured hipGraph:
//
//   lm_head (EPI_LSE: raw logits + per-workgroup log_softmax partials)
//   -> vcap_beam_cand_kernel   per (row, vocab chunk): log_softmax -> RepetitionPenalty ->
//                              NoRepeatNGram -> MinNewTokens -> + running score -> top-2nb
//   -> vcap_beam_select_kernel one workgroup, one wave per batch: top-2nb over the beams'
//                              candidates, running / finished beam updates, HF's stop rule,
//                              next tokens and the K/V ancestry of every row.
//
// K/V are never copied on a reorder: the forward of step t writes position S0 + t of row r into
// physical row r of the contiguous-page cache (a slot written exactly once), and `anc[r][p]` names
// the physical row that holds row r's position p - the attention kernel reads through it.
#include "vcap_common.h"
#include "vcap_kernels.h"

namespace {

constexpr int kBeamChunk = 2048;  // vocab columns per candidate workgroup
constexpr int kMaxK = 16;         // 2 * num_beams <= 16
constexpr float kNeg = -1.0e9f;   // HF's finished / running masking constant

// top-k insertion into a descending (value, index) list; ties keep the smaller index first
VCAP_DEV bool beats(float v, int i, float bv, int bi) { return v > bv || (v == bv && i < bi); }

}  // namespace

int vcap_beam_chunks(int V) { return (V + kBeamChunk - 1) / kBeamChunk; }

// ---------------------------------------------------------------------------------------------
// State init (search.py beam_search's initial tensors): running scores 0 for beam 0, -1e9 for the
// others; finished beams EOS-filled with score -1e9 and beam indices -1; the prefill wrote every
// row's prompt positions into its own physical row.
__global__ void vcap_beam_init_kernel(BeamState st, int B, int nb, int L, int S0, int anc_ld, int eos) {
  const int rows = B * nb;
  const int tid = blockIdx.x * blockDim.x + threadIdx.x, nthr = gridDim.x * blockDim.x;
  for (int i = tid; i < rows * L; i += nthr) {
    st.run_seq[i] = eos;
    st.seqs[i] = eos;
    st.run_bidx[i] = -1;
    st.beam_idx[i] = -1;
  }
  for (int i = tid; i < rows; i += nthr) {
    st.run_score[i] = (i % nb) ? kNeg : 0.f;
    st.beam_score[i] = kNeg;
    st.fin[i] = 0;
  }
  for (int i = tid; i < B; i += nthr) st.unsat[i] = 1;
  if (tid == 0) st.stopped[0] = 0;
  for (int i = tid; i < rows * anc_ld; i += nthr) st.anc[i] = i / anc_ld;   // own physical row
}

// ---------------------------------------------------------------------------------------------
// Candidates of one (row, vocab chunk): processed log-prob + running score, top-2nb of the chunk.
template <int K>
__global__ __launch_bounds__(256) void vcap_beam_cand_kernel(BeamState st, const float* __restrict__ logits,
                                                             const float* __restrict__ part_max,
                                                             const float* __restrict__ part_sum, int nblk, int V,
                                                             int nb, int L, int cur, float rep, int ngram, int min_new,
                                                             int eos) {
  __shared__ float s_red[8];
  __shared__ int s_hist[64], s_ban[64], s_nban;
  __shared__ unsigned char s_flag[kBeamChunk];  // bit 0: repetition penalty, bit 1: banned
  __shared__ float s_wv[4 * K];
  __shared__ int s_wi[4 * K];
  const int r = blockIdx.y, c = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (st.stopped[0]) return;
  const int n0 = c * kBeamChunk, n1 = min(n0 + kBeamChunk, V);

  // log_softmax statistics of the row: merge the lm_head workgroups' (max, sum) partials
  float mx = -INFINITY;
  for (int b = tid; b < nblk; b += 256) mx = fmaxf(mx, part_max[(long)r * nblk + b]);
  mx = wave_max(mx);
  if (lane == 0) s_red[wave] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(s_red[0], s_red[1]), fmaxf(s_red[2], s_red[3]));
  float sm = 0.f;
  for (int b = tid; b < nblk; b += 256) sm += part_sum[(long)r * nblk + b] * expf(part_max[(long)r * nblk + b] - mx);
  sm = wave_sum(sm);
  __syncthreads();
  if (lane == 0) s_red[4 + wave] = sm;
  // row history (the running hypothesis of this row before this step) and its n-gram bans
  if (tid < cur) s_hist[tid] = st.run_seq[(long)r * L + tid];
  if (tid == 0) s_nban = 0;
  for (int i = tid; i < kBeamChunk; i += 256) s_flag[i] = 0;
  __syncthreads();
  const float logsum = logf((s_red[4] + s_red[5]) + (s_red[6] + s_red[7]));
  if (ngram > 0 && cur >= ngram && tid + ngram <= cur) {
    bool match = true;
    for (int t = 0; t < ngram - 1; ++t) match &= s_hist[tid + t] == s_hist[cur - ngram + 1 + t];
    if (match) s_ban[atomicAdd(&s_nban, 1)] = s_hist[tid + ngram - 1];
  }
  __syncthreads();
  if (rep != 1.0f && tid < cur) {
    const unsigned o = (unsigned)(s_hist[tid] - n0);
    if (o < (unsigned)(n1 - n0)) s_flag[o] = 1;   // duplicates write the same byte
  }
  if (tid < s_nban) {
    const unsigned o = (unsigned)(s_ban[tid] - n0);
    if (o < (unsigned)(n1 - n0)) s_flag[o] |= 2;
  }
  __syncthreads();
  const float run = st.run_score[r];
  // this thread's columns -> its own top-K (descending, ties: smaller token first)
  constexpr int PER = kBeamChunk / 256;   // columns per thread
  float cv[PER];
  int ci[PER];
  bool taken[PER];
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    const int n = n0 + tid + q * 256;
    taken[q] = n >= n1;
    cv[q] = -INFINITY;
    ci[q] = 0x7fffffff;
    if (n < n1) {
      float lp = (logits[(long)r * V + n] - mx) - logsum;   // torch log_softmax: (x - max) - log(sum)
      const int f = s_flag[n - n0];
      if (f & 1) lp = lp < 0.f ? lp * rep : lp / rep;
      if (f & 2) lp = -INFINITY;
      if (n == eos && cur < min_new) lp = -INFINITY;
      cv[q] = lp + run;
      ci[q] = n;
    }
  }
  // top-K of each wave (K rounds of wave argmax, no barrier), then of the 4 waves' 4K (wave 0)
#pragma unroll
  for (int k = 0; k < K; ++k) {
    float bv = -INFINITY;
    int bi = 0x7fffffff;
#pragma unroll
    for (int q = 0; q < PER; ++q)
      if (!taken[q]) argmax_take(bv, bi, cv[q], ci[q]);   // ties: the smaller token
    wave_argmax(bv, bi);
#pragma unroll
    for (int q = 0; q < PER; ++q)
      if (!taken[q] && ci[q] == bi) taken[q] = true;
    if (lane == 0) {
      s_wv[wave * K + k] = bv;
      s_wi[wave * K + k] = bi;
    }
  }
  __syncthreads();
  if (wave == 0) {
    const bool have = lane < 4 * K;
    float v = have ? s_wv[lane] : -INFINITY;
    int i = have ? s_wi[lane] : 0x7fffffff;
    bool gone = !have;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      float bv = gone ? -INFINITY : v;
      int bi = gone ? 0x7fffffff : i;
      wave_argmax(bv, bi);
      if (!gone && i == bi && v == bv) gone = true;
      if (lane == 0) {
        st.cand_val[((long)r * gridDim.x + c) * K + k] = bv;
        st.cand_tok[((long)r * gridDim.x + c) * K + k] = bi;
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// One workgroup, wave b = batch b.  Restates search.py beam_search (itself token-identical to the
// reference's HF beam search, tests/test_gpu_search.py) for one step `cur`.
template <int NB>
__global__ __launch_bounds__(1024) void vcap_beam_select_kernel(BeamState st, int B, int L, int V, int C,
                                                                int cur, int eos, float lpen, int S0, int anc_ld) {
  constexpr int nb = NB;
  __shared__ int s_unsat[16], s_allhits[16];
  __shared__ int s_src[16][8];   // per batch: source beam of each new running beam
  __shared__ int s_anc[16 * 8][72];
  const int lane = threadIdx.x & 63, b = threadIdx.x >> 6;
  if (st.stopped[0]) return;   // HF's loop has ended: no further updates (uniform)
  constexpr int K = 2 * NB;
  const bool live = b < B;
  // ---- top-2nb over the nb beams' chunk candidates (flat index beam * V + token, HF topk order)
  float topv[K];
  int topf[K];
  if (live) {
    const int ncand = nb * C * K;
    float cv[20];
    int cf[20];
    bool taken[20];
    const int per = (ncand + 63) / 64;
#pragma unroll
    for (int q = 0; q < 20; ++q) {
      const int i = lane + q * 64;
      taken[q] = true;
      cv[q] = -INFINITY;
      cf[q] = 0x7fffffff;
      if (q < per && i < ncand) {
        const int beam = i / (C * K), rest = i % (C * K);
        const long src = (long)(b * nb + beam) * C * K + rest;
        const int t = st.cand_tok[src];
        cv[q] = t < V ? st.cand_val[src] : -INFINITY;
        cf[q] = t < V ? beam * V + t : 0x7fffffff;   // (a chunk with fewer than 2nb columns)
        taken[q] = false;
      }
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
      float bv = -INFINITY;
      int bi = 0x7fffffff;
#pragma unroll
      for (int q = 0; q < 20; ++q)
        if (!taken[q]) argmax_take(bv, bi, cv[q], cf[q]);
      wave_argmax(bv, bi);
#pragma unroll
      for (int q = 0; q < 20; ++q)
        if (!taken[q] && cf[q] == bi) taken[q] = true;
      topv[k] = bv;
      topf[k] = bi;
    }
  }
  // ---- HF bookkeeping (wave-uniform scalar work; lanes split the per-position copies)
  int hits_all = 1;
  if (live) {
    int src_beam[K], tok[K], hit[K];
    float run_lp[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      src_beam[k] = topf[k] / V;
      tok[k] = topf[k] - src_beam[k] * V;
      hit[k] = (tok[k] == eos) || (cur + 1 >= L);
      run_lp[k] = topv[k] + (hit[k] ? kNeg : -0.0f);
      hits_all &= hit[k];
    }
    // running beams for the next step: top-nb of run_lp (ties: lower candidate position)
    // (indices select through unrolled compares: no dynamically indexed private arrays)
    int nxt[NB];
    float nxt_lp[NB];
    int nxt_tok[NB], nxt_src[NB];
    {
      unsigned used = 0;
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        int best = -1;
        float bv = 0.f;
#pragma unroll
        for (int k = 0; k < K; ++k)
          if (!(used >> k & 1) && (best < 0 || run_lp[k] > bv)) {
            best = k;
            bv = run_lp[k];
          }
        used |= 1u << best;
        nxt[i] = best;
        nxt_lp[i] = bv;
        int t = 0, sb = 0;
#pragma unroll
        for (int k = 0; k < K; ++k)
          if (k == best) {
            t = tok[k];
            sb = src_beam[k];
          }
        nxt_tok[i] = t;
        nxt_src[i] = sb;
      }
    }
    // finished-hypothesis candidates: score / (cur + 1)^length_penalty, masked as HF masks them
    float sc[K];
    const float denom = powf((float)(cur + 1), lpen);
    const int unsat = st.unsat[b];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const bool did = hit[k] && k < nb;
      float v = topv[k] / denom;
      v = v + -0.0f;                        // full (early_stopping is False): + 0 * -1e9
      v = v + (unsat ? -0.0f : kNeg);       // + (~unsat) * -1e9
      v = v + (did ? -0.0f : kNeg);         // + (~did) * -1e9
      sc[k] = v;
    }
    // merge: [existing finished nb] ++ [2nb candidates] -> top-nb (ties: lower position)
    float msc[NB + K];
#pragma unroll
    for (int i = 0; i < NB; ++i) msc[i] = st.beam_score[b * nb + i];
#pragma unroll
    for (int k = 0; k < K; ++k) msc[nb + k] = sc[k];
    int sel[NB];
    float sel_sc[NB];
    {
      unsigned used = 0;
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        int best = -1;
        float bv = 0.f;
#pragma unroll
        for (int k = 0; k < NB + K; ++k)
          if (!(used >> k & 1) && (best < 0 || msc[k] > bv)) {
            best = k;
            bv = msc[k];
          }
        used |= 1u << best;
        sel[i] = best;
        sel_sc[i] = bv;
      }
    }
    // new finished set: gather rows (old finished entries, or a candidate = its source running
    // row + this step's token / beam index).  Read everything, then write (lanes = positions).
    const long base = (long)b * nb * L;
    const int p = lane;   // lane = position (L <= 64)
    int new_seq[NB], new_bidx[NB], new_fin[NB];
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int e = sel[i];
      // the selected candidate's source row, token and hit flag (unrolled select)
      int ctok = 0, csrc = 0, chit = 0;
#pragma unroll
      for (int k = 0; k < K; ++k)
        if (e == NB + k) {
          ctok = tok[k];
          csrc = src_beam[k];
          chit = hit[k] && k < NB;
        }
      new_seq[i] = eos;
      new_bidx[i] = -1;
      if (p < L) {
        if (e < NB) {
          new_seq[i] = st.seqs[base + (long)e * L + p];
          new_bidx[i] = st.beam_idx[base + (long)e * L + p];
        } else {
          new_seq[i] = p == cur ? ctok : st.run_seq[base + (long)csrc * L + p];
          new_bidx[i] = p == cur ? b * nb + csrc : st.run_bidx[base + (long)csrc * L + p];
        }
      }
      new_fin[i] = e < NB ? st.fin[b * nb + e] : chit;
    }
    float new_bscore[NB];
#pragma unroll
    for (int i = 0; i < NB; ++i) new_bscore[i] = sel_sc[i];
    // new running set
    int nr_seq[NB], nr_bidx[NB];
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      nr_seq[i] = eos;
      nr_bidx[i] = -1;
      if (p < L) {
        nr_seq[i] = p == cur ? nxt_tok[i] : st.run_seq[base + (long)nxt_src[i] * L + p];
        nr_bidx[i] = p == cur ? b * nb + nxt_src[i] : st.run_bidx[base + (long)nxt_src[i] * L + p];
      }
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      if (lane < L) {
        st.seqs[base + (long)i * L + lane] = new_seq[i];
        st.beam_idx[base + (long)i * L + lane] = new_bidx[i];
        st.run_seq[base + (long)i * L + lane] = nr_seq[i];
        st.run_bidx[base + (long)i * L + lane] = nr_bidx[i];
      }
    }
    if (lane == 0) {
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        st.beam_score[b * nb + i] = new_bscore[i];
        st.fin[b * nb + i] = new_fin[i];
        st.run_score[b * nb + i] = nxt_lp[i];
        st.tok_next[b * nb + i] = nxt_tok[i];
        s_src[b][i] = nxt_src[i];
      }
      // unsat update (cur + 1 generated tokens): best running vs worst finished
      const float best_len = powf((float)(cur + 1), lpen);
      const float best_running = nxt_lp[0] / best_len;
      float mn = new_bscore[0];
#pragma unroll
      for (int i = 1; i < NB; ++i) mn = fminf(mn, new_bscore[i]);
      bool any = false;
#pragma unroll
      for (int i = 0; i < NB; ++i) any |= best_running > (new_fin[i] ? mn : kNeg);
      const int u = unsat && any;
      st.unsat[b] = u;
      s_unsat[b] = u;
      s_allhits[b] = hits_all;
    }
  }
  __syncthreads();
  // ---- K/V ancestry: row b*nb+i continues source row b*nb+src; position S0+cur is its own
  const int pos = S0 + cur;   // the next forward writes this position
  for (int idx = threadIdx.x; idx < B * nb * anc_ld; idx += blockDim.x) {
    const int r = idx / anc_ld, p = idx % anc_ld;
    s_anc[r][p] = st.anc[(long)(r / nb * nb + s_src[r / nb][r % nb]) * anc_ld + p];
  }
  __syncthreads();
  for (int idx = threadIdx.x; idx < B * nb * anc_ld; idx += blockDim.x) {
    const int r = idx / anc_ld, p = idx % anc_ld;
    st.anc[(long)r * anc_ld + p] = p < pos ? s_anc[r][p] : r;
  }
  if (threadIdx.x == 0) {
    int any_unsat = 0, all_hits = 1;
    for (int i = 0; i < B; ++i) {
      any_unsat |= s_unsat[i];
      all_hits &= s_allhits[i];
    }
    if (!(any_unsat && !all_hits)) st.stopped[0] = 1;   // HF: go = any(unsat) and not all(hits)
  }
}

// best finished hypothesis per batch + its length (beam_idx of beam 0 not -1)
__global__ void vcap_beam_output_kernel(BeamState st, int B, int nb, int L, int* out_ids, int* out_len) {
  const int b = blockIdx.x, p = threadIdx.x;
  if (p < L) out_ids[b * L + p] = st.seqs[(long)b * nb * L + p];
  if (p == 0) {
    int n = 0;
    for (int t = 0; t < L; ++t) n += st.beam_idx[(long)b * nb * L + t] != -1;
    out_len[b] = n;
  }
}

// ---------------------------------------------------------------------------------------------
// Decode attention through the ancestry table (one query position per row): key j of row m is
// K/V position j of physical row anc[m][j], page (phys * maxp + j / 16) of the contiguous pools.
template <typename T>
__global__ __launch_bounds__(256) void vcap_decode_attention_anc_kernel(const T* __restrict__ q, const T* __restrict__ kc,
                                                                        const T* __restrict__ vc,
                                                                        const int* __restrict__ anc, int anc_ld,
                                                                        int maxp, T* __restrict__ out, int M, int H,
                                                                        int past) {
  constexpr int E8 = Frag<T>::kElems;
  __shared__ float s_q[4][64];
  __shared__ float s_p[4][1024];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int item = blockIdx.x * 4 + wave;
  if (item >= M * H) return;
  const int m = item / H, h = item - m * H;
  const int E = H * 64;
  const int ctx = past + 1;
  const int* arow = anc + (long)m * anc_ld;
  auto row_of = [&](const T* pool, int j, int phys) {
    return pool + (((long)(phys * maxp + (j >> 4)) * H + h) * 16 + (j & 15)) * 64;
  };
  s_q[wave][lane] = Num<T>::to_f(q[(long)m * E + h * 64 + lane]);
  __builtin_amdgcn_wave_barrier();
  float mx = -INFINITY;
  for (int j0 = 0; j0 < ctx; j0 += 64) {
    const int j = min(j0 + lane, ctx - 1);
    const T* krow = row_of(kc, j, arow[j]);
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
  for (int j0 = 0; j0 < ctx; j0 += 8) {
    const int jj = j0 + kg;
    const int j = min(jj, ctx - 1);
    const T* vrow = row_of(vc, j, arow[j]) + d8;
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

// ---------------------------------------------------------------------------------------------
hipError_t vcap_beam_init_dispatch(const BeamState& st, int B, int nb, int L, int S0, int anc_ld, int eos,
                                   hipStream_t s) {
  if (B * nb * anc_ld <= 0) return hipErrorInvalidValue;
  const int n = B * nb * (L > anc_ld ? L : anc_ld);
  hipLaunchKernelGGL(vcap_beam_init_kernel, dim3((n + 255) / 256), dim3(256), 0, s, st, B, nb, L, S0, anc_ld, eos);
  return hipGetLastError();
}

hipError_t vcap_beam_cand_dispatch(const BeamState& st, const float* logits, const float* part_max,
                                   const float* part_sum, int nblk, int rows, int V, int nb, int L, int cur,
                                   float rep, int ngram, int min_new, int eos, int chunks, hipStream_t s) {
  if (2 * nb > kMaxK || cur > 64 || chunks != vcap_beam_chunks(V)) return hipErrorInvalidValue;
  const dim3 grid(chunks, rows);
#define VCAP_CAND(NB)                                                                                          \
  if (nb == NB) {                                                                                              \
    hipLaunchKernelGGL((vcap_beam_cand_kernel<2 * NB>), grid, dim3(256), 0, s, st, logits, part_max, part_sum, \
                       nblk, V, nb, L, cur, rep, ngram, min_new, eos);                                         \
    return hipGetLastError();                                                                                  \
  }
  VCAP_CAND(2) VCAP_CAND(3) VCAP_CAND(4) VCAP_CAND(5) VCAP_CAND(6) VCAP_CAND(7) VCAP_CAND(8)
#undef VCAP_CAND
  return hipErrorInvalidValue;
}

hipError_t vcap_beam_select_dispatch(const BeamState& st, int B, int nb, int L, int V, int chunks, int cur, int eos,
                                     float length_penalty, int S0, int anc_ld, hipStream_t s) {
  if (B > 16 || nb > 8 || 2 * nb > kMaxK || L > 64 || anc_ld > 72 || nb * chunks * 2 * nb > 20 * 64)
    return hipErrorInvalidValue;
#define VCAP_SEL(NB)                                                                                       \
  if (nb == NB) {                                                                                          \
    hipLaunchKernelGGL((vcap_beam_select_kernel<NB>), dim3(1), dim3(64 * B), 0, s, st, B, L, V, chunks, cur, \
                       eos, length_penalty, S0, anc_ld);                                                   \
    return hipGetLastError();                                                                              \
  }
  VCAP_SEL(2) VCAP_SEL(3) VCAP_SEL(4) VCAP_SEL(5) VCAP_SEL(6) VCAP_SEL(7) VCAP_SEL(8)
#undef VCAP_SEL
  return hipErrorInvalidValue;
}

hipError_t vcap_beam_output_dispatch(const BeamState& st, int B, int nb, int L, int* out_ids, int* out_len,
                                     hipStream_t s) {
  hipLaunchKernelGGL(vcap_beam_output_kernel, dim3(B), dim3(64), 0, s, st, B, nb, L, out_ids, out_len);
  return hipGetLastError();
}

hipError_t vcap_decode_attention_anc_dispatch(int dt, const void* q, const void* kc, const void* vc, const int* anc,
                                              int anc_ld, int maxp, void* out, int M, int H, int past,
                                              hipStream_t s) {
  if (past + 1 > 1024 || past + 1 > anc_ld) return hipErrorInvalidValue;
  const dim3 grid((M * H + 3) / 4), block(256);
  if (dt == VCAP_DT_BF16)
    hipLaunchKernelGGL((vcap_decode_attention_anc_kernel<bf16_t>), grid, block, 0, s, (const bf16_t*)q,
                       (const bf16_t*)kc, (const bf16_t*)vc, anc, anc_ld, maxp, (bf16_t*)out, M, H, past);
  else
    hipLaunchKernelGGL((vcap_decode_attention_anc_kernel<float>), grid, block, 0, s, (const float*)q,
                       (const float*)kc, (const float*)vc, anc, anc_ld, maxp, (float*)out, M, H, past);
  return hipGetLastError();
}
