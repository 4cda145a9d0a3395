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
// Every global load (the chunk's logits, the row's log_softmax partials, its history) is issued at
// kernel start: one memory round trip, then LDS / register work.
template <int K>
__global__ __launch_bounds__(256) void vcap_beam_cand_kernel(BeamState st, const float* __restrict__ logits,
                                                             const float* __restrict__ part_max,
                                                             const float* __restrict__ part_sum, int nblk, int V,
                                                             int nb, int L, int cur, float rep, int ngram, int min_new,
                                                             int eos) {
  constexpr int PER = kBeamChunk / 256;   // columns per thread
  constexpr int PP = 4;                   // log_softmax partials per thread (nblk <= 1024)
  __shared__ float s_red[8];
  __shared__ int s_hist[64], s_ban[64], s_nban;
  __shared__ __attribute__((aligned(16))) unsigned char s_flag[kBeamChunk];  // bit 0: repetition penalty, bit 1: banned
  __shared__ float s_wv[4 * K];
  __shared__ int s_wi[4 * K];
  const int r = blockIdx.y, c = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n0 = c * kBeamChunk, n1 = min(n0 + kBeamChunk, V);
  // ---- loads
  const int stopped = st.stopped[0];
  float x[PER];
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    const int n = min(n0 + tid + q * 256, n1 - 1);
    x[q] = logits[(long)r * V + n];
  }
  float pm[PP], ps[PP];
#pragma unroll
  for (int q = 0; q < PP; ++q) {
    const int bb = tid + q * 256;
    pm[q] = bb < nblk ? part_max[(long)r * nblk + bb] : -INFINITY;
    ps[q] = bb < nblk ? part_sum[(long)r * nblk + bb] : 0.f;
  }
  const int hv = tid < cur ? st.run_seq[(long)r * L + tid] : 0;
  const float run = st.run_score[r];
  if (stopped) return;   // uniform
  // ---- log_softmax statistics of the row (merge of the lm_head workgroups' (max, sum))
  float mx = fmaxf(fmaxf(pm[0], pm[1]), fmaxf(pm[2], pm[3]));
  mx = wave_max(mx);
  if (lane == 0) s_red[wave] = mx;
  if (tid < cur) s_hist[tid] = hv;
  if (tid == 0) s_nban = 0;
  for (int i = tid; i < kBeamChunk; i += 256) s_flag[i] = 0;
  __syncthreads();
  mx = fmaxf(fmaxf(s_red[0], s_red[1]), fmaxf(s_red[2], s_red[3]));
  float sm = 0.f;
#pragma unroll
  for (int q = 0; q < PP; ++q) sm += ps[q] * expf(pm[q] - mx);
  sm = wave_sum(sm);
  if (lane == 0) s_red[4 + wave] = sm;
  // n-gram bans of the row history
  if (ngram > 0 && cur >= ngram && tid + ngram <= cur) {
    bool match = true;
    for (int t = 0; t < ngram - 1; ++t) match &= s_hist[tid + t] == s_hist[cur - ngram + 1 + t];
    if (match) s_ban[atomicAdd(&s_nban, 1)] = s_hist[tid + ngram - 1];
  }
  if (rep != 1.0f && tid < cur) {
    const unsigned o = (unsigned)(hv - n0);
    if (o < (unsigned)(n1 - n0)) s_flag[o] = 1;   // duplicates write the same byte
  }
  __syncthreads();
  if (tid < s_nban) {
    const unsigned o = (unsigned)(s_ban[tid] - n0);
    if (o < (unsigned)(n1 - n0)) atomicOr((unsigned*)(s_flag + (o & ~3u)), 2u << (8 * (o & 3)));
  }
  const float logsum = logf((s_red[4] + s_red[5]) + (s_red[6] + s_red[7]));
  __syncthreads();
  // taken / out-of-chunk entries hold (-inf, INT_MAX): they lose every comparison against a live
  // entry (a live -inf keeps its token index), so the top-K rounds run branch-free
  float cv[PER];
  int ci[PER];
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    const int n = n0 + tid + q * 256;
    float lp = (x[q] - mx) - logsum;   // torch log_softmax: (x - max) - log(sum)
    const int f = n < n1 ? s_flag[n - n0] : 0;
    if (f & 1) lp = lp < 0.f ? lp * rep : lp / rep;
    if (f & 2) lp = -INFINITY;
    if (n == eos && cur < min_new) lp = -INFINITY;
    cv[q] = n < n1 ? lp + run : -INFINITY;
    ci[q] = n < n1 ? n : 0x7fffffff;
  }
  // top-K of each wave (K rounds of wave argmax, no barrier), then of the 4 waves' 4K (wave 0)
#pragma unroll
  for (int k = 0; k < K; ++k) {
    float bv = cv[0];
    int bi = ci[0];
#pragma unroll
    for (int q = 1; q < PER; ++q) argmax_take(bv, bi, cv[q], ci[q]);   // ties: the smaller token
    wave_argmax(bv, bi);
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const bool hit = ci[q] == bi;
      cv[q] = hit ? -INFINITY : cv[q];
      ci[q] = hit ? 0x7fffffff : ci[q];
    }
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
#pragma unroll
    for (int k = 0; k < K; ++k) {
      float bv = v;
      int bi = i;
      wave_argmax(bv, bi);
      const bool hit = i == bi && v == bv;
      v = hit ? -INFINITY : v;
      i = hit ? 0x7fffffff : i;
      if (lane == 0) {
        st.cand_val[((long)r * gridDim.x + c) * K + k] = bv;
        st.cand_tok[((long)r * gridDim.x + c) * K + k] = bi;
      }
    }
  }
}

// candidates per lane of the select kernel sized for a GPT-2 vocabulary's 25 chunks of top-2nb per
// beam (NB = 4: 800 -> 13 per lane), at most 20; larger vocabularies take the 20-per-lane form
constexpr int kSelNcMax = 20;
constexpr int select_nc(int nb) {
  const int n = (nb * 25 * 2 * nb + 63) / 64;
  return n < 1 ? 1 : (n > 20 ? 20 : n);
}

// register "gather": a[idx] of a small unrolled array as an OR of masked terms (a compare /
// select chain is canonicalised back into a dynamically indexed private array = scratch memory)
template <int NB>
VCAP_DEV int pick(const int (&a)[NB], int idx) {
  int v = 0;
#pragma unroll
  for (int i = 0; i < NB; ++i) v |= a[i] & -(int)(idx == i);
  return v;
}

// ---------------------------------------------------------------------------------------------
// One workgroup, wave b = batch b (B <= 8: 2 waves per SIMD, a 256-register budget).  Restates search.py beam_search (itself token-identical to the
// reference's HF beam search, tests/test_gpu_search.py) for one step `cur`.  Lane p holds position
// p (and p + 64 of the ancestry rows) of every beam of its batch; all state is loaded up front.
template <int NB, int NC>   // NC: candidates per lane (NB * C * K <= 64 * NC)
__global__ __launch_bounds__(512) void vcap_beam_select_kernel(BeamState st, int B, int L, int V, int C,
                                                                int cur, int eos, float lpen, int S0, int anc_ld) {
  constexpr int K = 2 * NB;
  __shared__ int s_unsat[8], s_allhits[8];
  const int lane = threadIdx.x & 63, b = threadIdx.x >> 6;
  const bool live = b < B;
  const int p = lane;
  const long base = (long)b * NB * L;
  // ---- loads (one round trip): every address clamped into range and every load unconditional
  // (a guarded load is compiled as its own branch + wait: 57 serial round trips before this)
  const int stopped = st.stopped[0];
  int rs[NB], rbx[NB], sq[NB], bix[NB], a0[NB], a1[NB], fn[NB];
  float rsc[NB], bsc[NB];
  float cv[NC];
  int cf[NC];
  const int bl = min(b, B - 1);
  const long basel = (long)bl * NB * L;
  const int pl = min(p, L - 1), pa0 = min(p, anc_ld - 1), pa1 = min(p + 64, anc_ld - 1);
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    rs[i] = st.run_seq[basel + (long)i * L + pl];
    rbx[i] = st.run_bidx[basel + (long)i * L + pl];
    sq[i] = st.seqs[basel + (long)i * L + pl];
    bix[i] = st.beam_idx[basel + (long)i * L + pl];
    const long ar = (long)(bl * NB + i) * anc_ld;
    a0[i] = st.anc[ar + pa0];
    a1[i] = st.anc[ar + pa1];
    rsc[i] = st.run_score[bl * NB + i];
    bsc[i] = st.beam_score[bl * NB + i];
    fn[i] = st.fin[bl * NB + i];
  }
  const int uns = st.unsat[bl];
  const int ncand = NB * C * K;
#pragma unroll
  for (int q = 0; q < NC; ++q) {
    const int i = min(lane + q * 64, ncand - 1);
    int beam = 0;   // i / (C * K) by compares (an integer division is ~30 VALU per candidate)
#pragma unroll
    for (int j = 1; j < NB; ++j) beam += i >= j * C * K;
    const long src = (long)bl * NB * C * K + i;
    const int t = st.cand_tok[src];
    const float v = st.cand_val[src];
    const bool ok = lane + q * 64 < ncand && t < V;   // (a chunk with fewer than 2nb columns)
    cv[q] = ok ? v : -INFINITY;
    cf[q] = ok ? beam * V + t : 0x7fffffff;
  }
#pragma unroll
  for (int i = 0; i < NB; ++i) {   // positions past L read as HF's initial padding
    if (p >= L) {
      rs[i] = eos;
      rbx[i] = -1;
      sq[i] = eos;
      bix[i] = -1;
    }
  }
  if (stopped) return;   // HF's loop has ended: no further updates (uniform)
  int hits_all = 1;
  if (live) {
    // ---- top-2nb over the beams' chunk candidates (flat index beam * V + token, HF topk order).
    // Branch-free: a taken candidate becomes (-inf, INT_MAX), which loses every comparison against a
    // live one (a live -inf keeps its index); absent entries hold the same pair from the loads.
    // (Per-lane `taken` flags and guarded takes compiled to ~7800 instructions with 300 exec-mask
    // branches: 21-24 us per step, r05.)
    float topv[K];
    int topf[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      float bv = cv[0];
      int bi = cf[0];
#pragma unroll
      for (int q = 1; q < NC; ++q) argmax_take(bv, bi, cv[q], cf[q]);
      wave_argmax(bv, bi);
#pragma unroll
      for (int q = 0; q < NC; ++q) {
        const bool h = cf[q] == bi;
        cv[q] = h ? -INFINITY : cv[q];
        cf[q] = h ? 0x7fffffff : cf[q];
      }
      topv[k] = bv;
      topf[k] = bi;
    }
    int src_beam[K], tok[K], hit[K];
    float run_lp[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      int sb = 0;   // topf / V by compares
#pragma unroll
      for (int j = 1; j < NB; ++j) sb += topf[k] >= j * V;
      src_beam[k] = sb;
      tok[k] = topf[k] - sb * V;
      hit[k] = (tok[k] == eos) | (cur + 1 >= L);
      run_lp[k] = topv[k] + (hit[k] ? kNeg : -0.0f);   // topk_lp + hits * -1e9
      hits_all &= hit[k];
    }
    // running beams for the next step: top-nb of run_lp (ties: lower candidate position)
    int nxt_tok[NB], nxt_src[NB];
    float nxt_lp[NB];
    {
      unsigned used = 0;
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        int best = -1;
        float bv = 0.f;
#pragma unroll
        for (int k = 0; k < K; ++k) {
          const bool t = !((used >> k) & 1u) & ((best < 0) | (run_lp[k] > bv));
          best = t ? k : best;
          bv = t ? run_lp[k] : bv;
        }
        used |= 1u << best;
        nxt_lp[i] = bv;
        nxt_tok[i] = pick<K>(tok, best);
        nxt_src[i] = pick<K>(src_beam, best);
      }
    }
    // finished-hypothesis candidates: score / (cur + 1)^length_penalty, masked as HF masks them
    float msc[NB + K];
    const float denom = powf((float)(cur + 1), lpen);
#pragma unroll
    for (int i = 0; i < NB; ++i) msc[i] = bsc[i];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const bool did = hit[k] && k < NB;
      float v = topv[k] / denom;
      v = v + -0.0f;                     // full (early_stopping is False): + 0 * -1e9
      v = v + (uns ? -0.0f : kNeg);      // + (~unsat) * -1e9
      v = v + (did ? -0.0f : kNeg);      // + (~did) * -1e9
      msc[NB + k] = v;
    }
    // merge [existing finished nb] ++ [2nb candidates] -> top-nb (ties: lower position)
    int new_seq[NB], new_bidx[NB], new_fin[NB];
    float new_bsc[NB];
    {
      unsigned used = 0;
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        int e = -1;
        float bv = 0.f;
#pragma unroll
        for (int k = 0; k < NB + K; ++k) {
          const bool t = !((used >> k) & 1u) & ((e < 0) | (msc[k] > bv));
          e = t ? k : e;
          bv = t ? msc[k] : bv;
        }
        used |= 1u << e;
        new_bsc[i] = bv;
        // an existing finished hypothesis (e < NB) or candidate k = e - NB: both formed, one kept
        const int k = e - NB;
        const int cs = pick<K>(src_beam, k);
        const bool old_fin = e < NB;
        new_seq[i] = old_fin ? pick<NB>(sq, e) : (p == cur ? pick<K>(tok, k) : pick<NB>(rs, cs));
        new_bidx[i] = old_fin ? pick<NB>(bix, e) : (p == cur ? b * NB + cs : pick<NB>(rbx, cs));
        new_fin[i] = old_fin ? pick<NB>(fn, e) : (pick<K>(hit, k) & (k < NB));
      }
    }
    // ---- writes
    const int pos = S0 + cur;   // the next forward writes this position (own physical row)
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int src = nxt_src[i];
      if (p < L) {
        st.seqs[base + (long)i * L + p] = new_seq[i];
        st.beam_idx[base + (long)i * L + p] = new_bidx[i];
        st.run_seq[base + (long)i * L + p] = p == cur ? nxt_tok[i] : pick<NB>(rs, src);
        st.run_bidx[base + (long)i * L + p] = p == cur ? b * NB + src : pick<NB>(rbx, src);
      }
      const long ar = (long)(b * NB + i) * anc_ld;
      if (p < anc_ld) st.anc[ar + p] = p < pos ? pick<NB>(a0, src) : b * NB + i;
      if (p + 64 < anc_ld) st.anc[ar + p + 64] = p + 64 < pos ? pick<NB>(a1, src) : b * NB + i;
    }
    if (lane == 0) {
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        st.beam_score[b * NB + i] = new_bsc[i];
        st.fin[b * NB + i] = new_fin[i];
        st.run_score[b * NB + i] = nxt_lp[i];
        st.tok_next[b * NB + i] = nxt_tok[i];
      }
      // unsat update (cur + 1 generated tokens): best running vs worst finished
      const float best_running = nxt_lp[0] / powf((float)(cur + 1), lpen);
      float mn = new_bsc[0];
#pragma unroll
      for (int i = 1; i < NB; ++i) mn = fminf(mn, new_bsc[i]);
      bool any = false;
#pragma unroll
      for (int i = 0; i < NB; ++i) any |= best_running > (new_fin[i] ? mn : kNeg);
      const int u = uns && any;
      st.unsat[b] = u;
      s_unsat[b] = u;
      s_allhits[b] = hits_all;
    }
  }
  __syncthreads();
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

// Short-context variant (ctx = past + 1 <= 64, every configs[3] beam step): two memory round trips
// per wave instead of two per 8-key group - (1) the query element and the ancestry entry of key
// `lane`, (2) that key's K row and all 8 V-row chunks this lane accumulates, issued together.
// Arithmetic in the same order as the general kernel above (bit-identical outputs).
template <typename T>
__global__ __launch_bounds__(256) void vcap_decode_attention_anc64_kernel(const T* __restrict__ q,
                                                                          const T* __restrict__ kc,
                                                                          const T* __restrict__ vc,
                                                                          const int* __restrict__ anc, int anc_ld,
                                                                          int maxp, T* __restrict__ out, int M,
                                                                          int H, int past) {
  constexpr int E8 = Frag<T>::kElems;
  constexpr int VC = sizeof(T) == 2 ? 1 : 2;  // 16-byte V chunks per 8 dims
  __shared__ float s_q[4][64];
  __shared__ float s_p[4][64];
  __shared__ int s_a[4][64];
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
  // ---- round trip 1
  const int jk = min(lane, ctx - 1);
  const float qv = Num<T>::to_f(q[(long)m * E + h * 64 + lane]);
  const int ak = arow[jk];
  s_q[wave][lane] = qv;
  s_a[wave][lane] = ak;
  __builtin_amdgcn_wave_barrier();
  // ---- round trip 2: K row of key `lane`, V chunks of keys kg, kg + 8, ...
  const int kg = lane >> 3, d8 = (lane & 7) * 8;
  const T* krow = row_of(kc, jk, ak);
  u32x4 kv[64 / E8];
#pragma unroll
  for (int c = 0; c < 64 / E8; ++c) kv[c] = *reinterpret_cast<const u32x4*>(krow + c * E8);
  u32x4 vv[8][VC];
#pragma unroll
  for (int it = 0; it < 8; ++it) {
    const int j = min(it * 8 + kg, ctx - 1);
    const T* vrow = row_of(vc, j, s_a[wave][j]) + d8;
#pragma unroll
    for (int c = 0; c < VC; ++c) vv[it][c] = *reinterpret_cast<const u32x4*>(vrow + c * 4);
  }
  float sc = 0.f;
#pragma unroll
  for (int c = 0; c < 64 / E8; ++c) {
    const T* ke = reinterpret_cast<const T*>(&kv[c]);
#pragma unroll
    for (int e = 0; e < E8; ++e) sc += s_q[wave][c * E8 + e] * Num<T>::to_f(ke[e]);
  }
  sc *= 0.125f;
  float mx = -INFINITY;
  if (lane < ctx) {
    s_p[wave][lane] = sc;
    mx = sc;
  }
  mx = wave_max(mx);
  float sum = 0.f;
  if (lane < ctx) {
    const float p = __expf(s_p[wave][lane] - mx);
    s_p[wave][lane] = p;
    sum = p;
  }
  sum = wave_sum(sum);
  __builtin_amdgcn_wave_barrier();
  float o[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) o[e] = 0.f;
#pragma unroll
  for (int it = 0; it < 8; ++it) {
    const int jj = it * 8 + kg;
    const float p = jj < ctx ? s_p[wave][min(jj, ctx - 1)] : 0.f;
    if constexpr (sizeof(T) == 2) {
      const unsigned w4[4] = {vv[it][0].x, vv[it][0].y, vv[it][0].z, vv[it][0].w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        o[2 * e] += p * bf2f((bf16_t)(w4[e] & 0xffff));
        o[2 * e + 1] += p * bf2f((bf16_t)(w4[e] >> 16));
      }
    } else {
      const f32x4 v0 = __builtin_bit_cast(f32x4, vv[it][0]), v1 = __builtin_bit_cast(f32x4, vv[it][1]);
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
  if (2 * nb > kMaxK || cur > 64 || chunks != vcap_beam_chunks(V) || nblk > 1024) return hipErrorInvalidValue;
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
  const int ncand = nb * chunks * 2 * nb;
  if (B > 8 || nb > 8 || 2 * nb > kMaxK || L > 64 || anc_ld > 128 || ncand > kSelNcMax * 64)
    return hipErrorInvalidValue;
#define VCAP_SEL(NB)                                                                                          \
  if (nb == NB) {                                                                                             \
    if (ncand <= select_nc(NB) * 64)                                                                          \
      hipLaunchKernelGGL((vcap_beam_select_kernel<NB, select_nc(NB)>), dim3(1), dim3(64 * B), 0, s, st, B, L, V, \
                         chunks, cur, eos, length_penalty, S0, anc_ld);                                       \
    else                                                                                                      \
      hipLaunchKernelGGL((vcap_beam_select_kernel<NB, kSelNcMax>), dim3(1), dim3(64 * B), 0, s, st, B, L, V,    \
                         chunks, cur, eos, length_penalty, S0, anc_ld);                                       \
    return hipGetLastError();                                                                                 \
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
  if (past + 1 <= 64) {
    if (dt == VCAP_DT_BF16)
      hipLaunchKernelGGL((vcap_decode_attention_anc64_kernel<bf16_t>), grid, block, 0, s, (const bf16_t*)q,
                         (const bf16_t*)kc, (const bf16_t*)vc, anc, anc_ld, maxp, (bf16_t*)out, M, H, past);
    else
      hipLaunchKernelGGL((vcap_decode_attention_anc64_kernel<float>), grid, block, 0, s, (const float*)q,
                         (const float*)kc, (const float*)vc, anc, anc_ld, maxp, (float*)out, M, H, past);
    return hipGetLastError();
  }
  if (dt == VCAP_DT_BF16)
    hipLaunchKernelGGL((vcap_decode_attention_anc_kernel<bf16_t>), grid, block, 0, s, (const bf16_t*)q,
                       (const bf16_t*)kc, (const bf16_t*)vc, anc, anc_ld, maxp, (bf16_t*)out, M, H, past);
  else
    hipLaunchKernelGGL((vcap_decode_attention_anc_kernel<float>), grid, block, 0, s, (const float*)q,
                       (const float*)kc, (const float*)vc, anc, anc_ld, maxp, (float*)out, M, H, past);
  return hipGetLastError();
}
