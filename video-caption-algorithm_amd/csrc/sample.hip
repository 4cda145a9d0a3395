// Sampling presets on the device (core/inference.py:12-15 `natural` / `safe_sample`; HF generate's
// _sample as text_decoder.py:131-144 reaches it with do_sample = (num_beams == 1 and temperature != 1)).
//
// The lm_head epilogue already applies RepetitionPenalty -> NoRepeatNGram -> MinNewTokens and, in
// sampling mode, stores the processed scores row (EPI_LOGITS proc_out).  One workgroup of 1024
// threads per row then applies HF's warpers in HF's order and draws the token:
//   TemperatureLogitsWarper  s / T
//   TopKLogitsWarper(50)     keep s >= the 50th largest (ties kept), the rest -inf
//   TopPLogitsWarper(p)      sort ascending, softmax, cumsum; drop where cumsum <= 1 - p (the
//                            largest always kept)
//   multinomial              one draw from softmax(warped) by inverse CDF with a counter-based
//                            Philox4x32-10 stream keyed on (seed, row, step)
// The 50th largest is found exactly by bisection on an order-preserving 32-bit key (32 block-wide
// counts), the <= 256 survivors are ranked in LDS, and lane 0 of wave 0 runs top-p's cumulative sum
// sequentially (double accumulator, as torch's CPU cumsum).  The token is handed to the greedy
// finalize kernel as its only argmax partial (nblk = 1), which pads finished rows, records the
// token, builds the next n-gram ban list and the next input embedding.  No host sync per token:
// the whole sampled decode is one hipGraph like greedy; the seed lives in device memory so one
// graph serves every seed.
#include "vcap_common.h"
#include "vcap_kernels.h"

namespace {

constexpr int kThreads = 1024;
constexpr int kCand = 256;  // survivors of top-k (k <= kCand - ties)

VCAP_DEV unsigned fkey(float f) {
  const unsigned u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

VCAP_DEV uint4 philox(uint4 c, uint2 k) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const unsigned lo0 = 0xD2511F53u * c.x, hi0 = __umulhi(0xD2511F53u, c.x);
    const unsigned lo1 = 0xCD9E8D57u * c.z, hi1 = __umulhi(0xCD9E8D57u, c.z);
    c = make_uint4(hi1 ^ c.y ^ k.x, lo1, hi0 ^ c.w ^ k.y, lo0);
    k.x += 0x9E3779B9u;
    k.y += 0xBB67AE85u;
  }
  return c;
}

template <int NPT>
__global__ __launch_bounds__(kThreads) void vcap_sample_kernel(SampleArgs a) {
  __shared__ float s_cnt[2][kThreads / 64];
  __shared__ float c_val[kCand], o_val[kCand];
  __shared__ int c_idx[kCand], o_idx[kCand];
  __shared__ int s_nc, s_tok;
  const int row = blockIdx.x, t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const float* pr = a.proc + (long)row * a.ldp;
  const int V = a.V;
  float v[NPT];   // (order keys are recomputed from v: 3 VALU each, half the registers)
#pragma unroll
  for (int i = 0; i < NPT; ++i) {
    const int idx = t + i * kThreads;
    // TemperatureLogitsWarper: a true division, as HF computes it
    v[i] = idx < V ? pr[idx] / a.temperature : -INFINITY;
  }
  if (t == 0) s_nc = 0;
  if (a.warped) {
    float* wr = a.warped + (long)row * a.warped_ld;
#pragma unroll
    for (int i = 0; i < NPT; ++i)
      if (t + i * kThreads < V) wr[t + i * kThreads] = -INFINITY;
  }
  // ---- TopK: T = the k-th largest key (bit by bit from the MSB: the largest T with >= k keys >= T)
  const float k = (float)a.top_k;
  unsigned T = 0;
  for (int b = 31; b >= 0; --b) {
    const unsigned cand = T | (1u << b);
    float c = 0.f;
#pragma unroll
    for (int i = 0; i < NPT; ++i) c += fkey(v[i]) >= cand ? 1.f : 0.f;
    c = wave_sum(c);
    const int buf = b & 1;
    if (lane == 0) s_cnt[buf][wave] = c;
    __syncthreads();
    float tot = 0.f;
#pragma unroll
    for (int w = 0; w < kThreads / 64; ++w) tot += s_cnt[buf][w];
    if (tot >= k) T = cand;
  }
  // ---- survivors (finite, key >= T) -> LDS
#pragma unroll
  for (int i = 0; i < NPT; ++i) {
    if (fkey(v[i]) >= T && v[i] > -INFINITY) {
      const int slot = atomicAdd(&s_nc, 1);
      if (slot < kCand) {
        c_val[slot] = v[i];
        c_idx[slot] = t + i * kThreads;
      }
    }
  }
  __syncthreads();
  const int nc = min(s_nc, kCand);
  // ---- ascending order by rank (ties by vocabulary index)
  if (t < nc) {
    const float x = c_val[t];
    const int xi = c_idx[t];
    int r = 0;
    for (int j = 0; j < nc; ++j) {
      const float y = c_val[j];
      r += (y < x) || (y == x && c_idx[j] < xi);
    }
    o_val[r] = x;
    o_idx[r] = xi;
  }
  __syncthreads();
  if (t == 0 && nc == 0) {
    // no finite processed score in the row (NaN or all -inf logits): a defined token, no draw
    s_nc = 0;
    a.pval[row] = 0.f;
    a.pidx[row] = a.force ? min(max(a.force[(long)row * a.force_ld + a.step], 0), V - 1) : a.eos;
  } else if (t == 0) {
    // ---- TopP over the survivors (every other score is -inf: probability 0)
    const float mx = o_val[nc - 1];
    float sum = 0.f;
    for (int j = 0; j < nc; ++j) sum += expf(o_val[j] - mx);
    const float thr = (float)(1.0 - a.top_p);   // HF: cumsum <= (1 - top_p), the bound rounded to f32
    int j0 = nc - 1;  // first kept position (the largest is always kept)
    if (a.top_p < 1.0) {
      double cum = 0.0;
      for (int j = 0; j < nc - 1; ++j) {
        cum += (double)(expf(o_val[j] - mx) / sum);
        if ((float)cum > thr) {
          j0 = j;
          break;
        }
      }
    } else {
      j0 = 0;
    }
    // ---- multinomial over softmax(kept)
    float ks = 0.f;
    for (int j = j0; j < nc; ++j) ks += expf(o_val[j] - mx);
    const unsigned* sd = a.seed;
    const uint4 r4 = philox(make_uint4((unsigned)a.step, (unsigned)row, 0u, 0u), make_uint2(sd[0], sd[1]));
    const float u = (float)(r4.x >> 8) * (1.0f / 16777216.0f);
    const float target = u * ks;
    float acc = 0.f;
    int tok = o_idx[nc - 1];
    for (int j = j0; j < nc; ++j) {
      acc += expf(o_val[j] - mx);
      if (acc > target) {
        tok = o_idx[j];
        break;
      }
    }
    if (a.force) tok = min(max(a.force[(long)row * a.force_ld + a.step], 0), V - 1);  // finalize indexes wte
    s_tok = tok;
    s_nc = j0;  // reused: first kept survivor
    a.pval[row] = 0.f;
    a.pidx[row] = tok;
  }
  __syncthreads();
  if (a.warped) {
    float* wr = a.warped + (long)row * a.warped_ld;
    for (int j = s_nc + t; j < nc; j += kThreads) wr[o_idx[j]] = o_val[j];
  }
  (void)s_tok;
}

}  // namespace

int vcap_sample_max_top_k() { return kCand / 2; }

hipError_t vcap_sample_dispatch(const SampleArgs& a, int rows, hipStream_t s) {
  if (a.V <= 0 || a.V > 50 * kThreads || a.top_k < 1 || a.top_k > kCand / 2 || !(a.temperature > 0.f) ||
      !(a.top_p > 0.0) || a.top_p > 1.0 || !a.seed)
    return hipErrorInvalidValue;
  const int npt = (a.V + kThreads - 1) / kThreads;
#define VCAP_SAMPLE(N)                                                                        \
  if (npt <= N) {                                                                              \
    hipLaunchKernelGGL((vcap_sample_kernel<N>), dim3(rows), dim3(kThreads), 0, s, a);         \
    return hipGetLastError();                                                                  \
  }
  VCAP_SAMPLE(1)
  VCAP_SAMPLE(8)
  VCAP_SAMPLE(16)
  VCAP_SAMPLE(32)
  VCAP_SAMPLE(50)
#undef VCAP_SAMPLE
  return hipErrorInvalidValue;
}
