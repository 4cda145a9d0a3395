// GPT-2 greedy decode steps 1 .. max_new-1 as ONE persistent launch (bf16, <= 16 rows).
//
// Same arithmetic as the launch chain of decode.hip (HF GPT2LMHeadModel.generate as
// src/models/text_decoder.py:131-144 reaches it; raw greedy of core/scripts/benchmark_baseline.py:
// 160-240), per output element operation for operation, so ids and logits are bit-identical to it
// (tests/test_gpu_persist.py).  What changes is how the ~62 dependent steps of a token step are
// sequenced: the launch chain pays a kernel boundary per step (1.9-3.6 us measured,
// profiles/r03_decode_stamps.txt) and every GEMV waits for its weights after its launch; here G
// resident workgroups (one per CU) run every phase of every token step and meet at a grid barrier
// between phases, and each workgroup issues the NEXT phase's weight fragments into registers
// before it arrives at the barrier, so the weight stream (each byte read once per step by one CU,
// nontemporal) lands while the barrier completes instead of after it.
//
// Phases of a token step (past = S0 + step - 1, one query row per sequence):
//   per layer: P1 ln_1 + c_attn (q -> q buffer, K/V -> paged cache)   [3E/16 column tiles]
//              P2 causal attention, one wave per (row, head)
//              P3 attn c_proj + residual into h                        [E/16 tiles]
//              P4 ln_2 + c_fc + gelu_new                               [4E/16 tiles]
//              P5 mlp c_proj + residual into h                         [E/16 tiles, K = 4E]
//   P6 ln_f + tied lm_head + RepetitionPenalty / NoRepeatNGram / MinNewTokens -> per-workgroup argmax
//   P7 finalize (workgroup m < M): argmax over the G partials, EOS padding, history, next n-gram ban
//      list, next input embedding wte[tok] + wpe[pos].
// A GEMV tile = 16 output columns x all rows, K split over the 4 compute waves exactly as
// vcap_rows_gemv_kernel splits it (wave w: K slabs [w*NSL, (w+1)*NSL), partials summed
// (w0 + w1) + (w2 + w3) + bias through LDS).  Tile t of a phase belongs to workgroup t % G.
//
// Workgroup = 4 compute waves + 1 sync wave.  The sync wave issues no other memory operation, so its
// barrier polls return at load latency; a compute wave's prefetched weights would otherwise sit in
// front of every poll in the in-order vmcnt.
//
// Inter-workgroup hand-offs (MI355X_MICROARCH.md "Valid forms", row 1): every byte one workgroup
// hands to another (h, q, attention out, MLP activations, K/V of the current position, argmax
// partials, history / ban lists) is stored write-through (sc1, 4-16 B) and loaded with sc1 buffer
// loads to registers; each storing wave drains (s_waitcnt vmcnt(0)), the workgroup barriers, then
// the sync wave adds 1 to its shard of an 8-way sharded monotonic arrival counter (agent-scope
// atomic), polls all 8 shards with sc1 loads until they sum to (phase + 1) * G, and the workgroup
// barriers again before any compute wave loads.  The counters are zeroed by a memset node before
// every launch.  Every spin is bounded (0.5 s of s_memrealtime): on timeout the workgroup raises an
// abort word every other workgroup polls, bumps the sticky fault counter vcap_decode_faults()
// reports, and all workgroups return.
#include "vcap_common.h"
#include "vcap_kernels.h"

#include <algorithm>
#include <cstdlib>

namespace {

constexpr int kCompute = 256;                    // 4 compute waves
constexpr int kThreads = kCompute + 64;          // + the sync wave
constexpr int kSC1 = 16;                         // buffer-instruction cache policy bit: sc1
constexpr unsigned long kSpinTicks = 50000000ul; // 0.5 s of the 100 MHz s_memrealtime clock
constexpr int kTpw = 64;                         // lm_head tiles per workgroup (flag bitmaps)
constexpr int kShardStride = 32;                 // words between counter shards (128 B)
constexpr int kAbortWord = 8 * kShardStride;

__device__ unsigned g_persist_faults;
// diagnostic (VCAP_PERSIST_FLAGS & 8): s_memrealtime at each phase's arrival and release, per
// workgroup: [wg][phase][2] (tools/persist_time.py --stamps)
constexpr int kStampPhases = 2048;
__device__ unsigned long g_persist_stamps[256][kStampPhases][2];

// Every handed-off buffer lives in the decoder workspace and is addressed as a byte offset from its
// base through ONE buffer resource (4 SGPRs: a resource per buffer held ~40 SGPRs live across the
// step loop and spilled).
VCAP_DEV __amdgpu_buffer_rsrc_t rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, 0x7FFFFFFF, 0x00020000);
}
VCAP_DEV u32x4 ld16(const void* b, int off) {
  return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rsrc(b), off, 0, kSC1));
}
VCAP_DEV u32x2 ld8(const void* b, int off) {
  return __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(rsrc(b), off, 0, kSC1));
}
VCAP_DEV unsigned ld4(const void* b, int off) { return __builtin_amdgcn_raw_buffer_load_b32(rsrc(b), off, 0, kSC1); }
VCAP_DEV void st4(void* b, int off, unsigned v) { __builtin_amdgcn_raw_buffer_store_b32(v, rsrc(b), off, 0, kSC1); }
VCAP_DEV void st8(void* b, int off, u32x2 v) { __builtin_amdgcn_raw_buffer_store_b64(v, rsrc(b), off, 0, kSC1); }
VCAP_DEV void st16(void* b, int off, u32x4 v) { __builtin_amdgcn_raw_buffer_store_b128(v, rsrc(b), off, 0, kSC1); }
VCAP_DEV float ldf(const void* b, int off) { return __uint_as_float(ld4(b, off)); }

// ---- weights: rows-packed bf16 fragments, tile t / slab g / lane at w[(t * nslab + g) * 64 + lane];
// wq[j * NSL + s] = tile (t0 + j*G)'s fragment of the wave's slab s (tiles past nt re-read nt-1)
// (global, not flat, loads: a flat load retires out of order, so any wait on it is a full drain)
typedef const __attribute__((address_space(1))) u32x4 gu32x4;
template <int NSL, int NTB, int NQ>
VCAP_DEV void issue_w(u32x4 (&wq)[NQ], const void* w, int t0, int G, int nt, int wave, int lane) {
  static_assert(NSL * NTB <= NQ, "register budget");
  const u32x4* base = reinterpret_cast<const u32x4*>(w);
#pragma unroll
  for (int j = 0; j < NTB; ++j) {
    const int t = min(t0 + j * G, nt - 1);
    gu32x4* p = (gu32x4*)(base + ((long)t * (4 * NSL) + wave * NSL) * 64 + lane);
#pragma unroll
    for (int s = 0; s < NSL; ++s) wq[j * NSL + s] = __builtin_nontemporal_load(p + s * 64);
  }
}
// the same fragments of ONE tile into LDS by LDS-DMA (no registers held while they land): wave w's
// slab s at lds_w + (w * NSL + s) * 1 KiB, lane-linear
template <int NSL>
VCAP_DEV void issue_w_lds(const void* w, int t, char* lds_w, int wave, int lane) {
  const u32x4* p = reinterpret_cast<const u32x4*>(w) + ((long)t * (4 * NSL) + wave * NSL) * 64 + lane;
#pragma unroll
  for (int s = 0; s < NSL; ++s)
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(p + s * 64),
                                     (__attribute__((address_space(3))) void*)(lds_w + (wave * NSL + s) * 1024), 16, 0,
                                     2 /* nt */);
}

// ---- LayerNorm of the M (<= 16) f32 rows of x into the swizzled bf16 LDS A tile [16][E]
// (vcap_rows_gemv_kernel PRO_LN: wave w normalises rows w, w+4, w+8, w+12; rows >= M are zeros)
template <int E>
VCAP_DEV void ln_rows(const char* base, int ox, int M, const float* g, const float* b, float eps, char* dyn,
                      int wave, int lane) {
  constexpr int KC = (E + 255) / 256;
  f32x4 xv[4][KC], gv[KC], bv[KC];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int m = min(wave + 4 * r, M - 1);
#pragma unroll
    for (int c = 0; c < KC; ++c) {
      const int cc = min(c * 256 + lane * 4, E - 4);
      xv[r][c] = __builtin_bit_cast(f32x4, ld16(base, ox + (m * E + cc) * 4));
    }
  }
#pragma unroll
  for (int c = 0; c < KC; ++c) {
    const int cc = min(c * 256 + lane * 4, E - 4);
    gv[c] = *reinterpret_cast<const f32x4*>(g + cc);
    bv[c] = *reinterpret_cast<const f32x4*>(b + cc);
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int m = wave + 4 * r;
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < KC; ++c)
      if (c * 256 + lane * 4 < E) s += (xv[r][c].x + xv[r][c].y) + (xv[r][c].z + xv[r][c].w);
    const float mean = wave_sum(s) / (float)E;
    float ss = 0.f;
#pragma unroll
    for (int c = 0; c < KC; ++c)
      if (c * 256 + lane * 4 < E) {
        const f32x4 d = xv[r][c] - mean;
        ss += sumsq4(d);
      }
    const float rstd = rsqrtf(wave_sum(ss) / (float)E + eps);
    const bool live = m < M;
#pragma unroll
    for (int c = 0; c < KC; ++c) {
      if (c * 256 + lane * 4 < E) {
        const f32x4 y = live ? ln_affine4(xv[r][c], mean, rstd, gv[c], bv[c]) : (f32x4){0.f, 0.f, 0.f, 0.f};
        const int byte = (c * 256 + lane * 4) * 2;
        char* dst = dyn + (long)m * (E * 2) + ((((byte >> 4) ^ (m & 15))) << 4) + (byte & 15);
        *reinterpret_cast<u32x2*>(dst) = (u32x2){pack_bf2(y.x, y.y), pack_bf2(y.z, y.w)};
      }
    }
  }
}

// MFMAs of one wave's K range (slabs g0 .. g0 + NSL - 1) against NTB tiles; A from the LDS tile
template <int E, int NSL, int NTB, int NQ>
VCAP_DEV void mma_lds(f32x4 (&acc)[NTB], const u32x4 (&wq)[NQ], const char* dyn, int wave, int lane) {
  const int fr = lane & 15, fg = lane >> 4, g0 = wave * NSL;
#pragma unroll
  for (int j = 0; j < NTB; ++j) acc[j] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < NSL; ++s) {
    const int chunk = (g0 + s) * 4 + fg;
    const u32x4 A = *reinterpret_cast<const u32x4*>(dyn + (long)fr * (E * 2) + ((chunk ^ fr) << 4));
#pragma unroll
    for (int j = 0; j < NTB; ++j) acc[j] = mfma_frag(A, wq[j * NSL + s], acc[j], (bf16_t*)nullptr);
  }
}

// split-K partials -> LDS red[wave][j][16 x 16]
template <int NTB>
VCAP_DEV void to_red(float* red, const f32x4 (&acc)[NTB], int wave, int lane) {
  const int fr = lane & 15, fg = lane >> 4;
#pragma unroll
  for (int j = 0; j < NTB; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) red[(wave * 4 + j) * 256 + (fg * 4 + r) * 16 + fr] = acc[j][r];
}
// the reduced pre-epilogue value of element (row, col) of tile j (decode.hip rows_epilogue order)
VCAP_DEV float red_val(const float* red, int j, int row, int col, float bias) {
  const int e = j * 256 + row * 16 + col;
  return (red[e] + red[1024 + e]) + (red[2048 + e] + red[3072 + e]) + bias;
}

struct PersistArgs {
  int G, M, E, H, L, V, S0, maxp, n_pos;
  int step0, step1;
  float ln_eps;
  const float* lnf_g;
  const float* lnf_b;
  const void* lm_head;
  const bf16_t* wte;
  const float* wpe;
  char* base;  // workspace base: the byte offsets o_* below are relative to it
  int o_h, o_q, o_attn, o_act, o_kc, o_vc, page_bytes;
  int o_hist, o_banned, o_nbanned, o_finished, o_pval, o_pidx;
  int hist_ld;
  int ngram;
  float rep;
  int min_new, eos, pad;
  int* out_ids;
  int out_ld;
  float* logits_out;
  unsigned* bar;
  const PersistLayer* layers;  // device copy (vcap_persist_layers_kernel)
  int flags;                   // diagnostics (VCAP_PERSIST_FLAGS): 1 barriers only, 4 no s_sleep in polls,
                               // 8 stamps, 16 / 32 agent acquire / release fences at every barrier
};

struct PersistLayers {
  PersistLayer l[kPersistMaxLayers];
};
// the layer table into device memory (a kernel node: its argument values are part of the graph)
__global__ void vcap_persist_layers_kernel(PersistLayers src, int n, PersistLayer* dst) {
  const int i = threadIdx.x;
  if (i < n) dst[i] = src.l[i];
}

// ---- P2: one (row, head) of causal attention over the contiguous paged cache (decode.hip
// vcap_decode_attention_c64_kernel for ctx <= 64, vcap_decode_attention_kernel<bf16> otherwise)
VCAP_DEV void attn_item(const PersistArgs& a, int okc, int ovc, int m, int h, int ctx, float* s_q, float* s_p,
                        int lane) {
  const int H = a.H, E = a.E, maxp = a.maxp;
  const int seq = m;
  const char* base = a.base;
  auto row_off = [&](int j) { return (((seq * maxp + (j >> 4)) * H + h) * 16 + (j & 15)) * 64 * 2; };
  const unsigned q2 = ld4(base, a.o_q + (m * E + h * 64 + (lane & ~1)) * 2);
  const float qv = bf2f((bf16_t)((lane & 1) ? (q2 >> 16) : (q2 & 0xffff)));
  const int kg = lane >> 3, d8 = (lane & 7) * 8;
  float o[8];
  float sum;
  if (ctx <= 64) {
    u32x4 kv[8];
    const int ko = okc + row_off(min(lane, ctx - 1));
#pragma unroll
    for (int c = 0; c < 8; ++c) kv[c] = ld16(base, ko + c * 16);
    u32x4 vv[8];
#pragma unroll
    for (int it = 0; it < 8; ++it) vv[it] = ld16(base, ovc + row_off(min(it * 8 + kg, ctx - 1)) + d8 * 2);
    s_q[lane] = qv;
    __builtin_amdgcn_wave_barrier();
    float sc = 0.f;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const bf16_t* ke = reinterpret_cast<const bf16_t*>(&kv[c]);
#pragma unroll
      for (int e = 0; e < 8; ++e) sc += s_q[c * 8 + e] * bf2f(ke[e]);
    }
    sc *= 0.125f;
    const bool live = lane < ctx;
    const float mx = wave_max(live ? sc : -INFINITY);
    const float p = live ? __expf(sc - mx) : 0.f;
    sum = wave_sum(p);
    s_p[lane] = p;
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = 0.f;
#pragma unroll
    for (int it = 0; it < 8; ++it) {
      const int jj = it * 8 + kg;
      const float pj = jj < ctx ? s_p[jj] : 0.f;
      const unsigned w4[4] = {vv[it].x, vv[it].y, vv[it].z, vv[it].w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        o[2 * e] += pj * bf2f((bf16_t)(w4[e] & 0xffff));
        o[2 * e + 1] += pj * bf2f((bf16_t)(w4[e] >> 16));
      }
    }
  } else {
    // general context (vcap_decode_attention_kernel<bf16_t>, identity page table)
    s_q[lane] = qv;
    __builtin_amdgcn_wave_barrier();
    float mx = -INFINITY;
    for (int j0 = 0; j0 < ctx; j0 += 64) {
      const int j = min(j0 + lane, ctx - 1);
      const int ko = okc + row_off(j);
      u32x4 kv[8];
#pragma unroll
      for (int c = 0; c < 8; ++c) kv[c] = ld16(base, ko + c * 16);
      float s = 0.f;
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const bf16_t* ke = reinterpret_cast<const bf16_t*>(&kv[c]);
#pragma unroll
        for (int e = 0; e < 8; ++e) s += s_q[c * 8 + e] * bf2f(ke[e]);
      }
      s *= 0.125f;
      if (j0 + lane < ctx) {
        s_p[j0 + lane] = s;
        mx = fmaxf(mx, s);
      }
    }
    mx = wave_max(mx);
    sum = 0.f;
    for (int j = lane; j < ctx; j += 64) {
      const float p = __expf(s_p[j] - mx);
      s_p[j] = p;
      sum += p;
    }
    sum = wave_sum(sum);
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = 0.f;
#pragma unroll 4
    for (int j0 = 0; j0 < ctx; j0 += 8) {
      const int jj = j0 + kg;
      const int j = min(jj, ctx - 1);
      const float p = jj < ctx ? s_p[j] : 0.f;
      const u32x4 vv = ld16(base, ovc + row_off(j) + d8 * 2);
      const unsigned w4[4] = {vv.x, vv.y, vv.z, vv.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        o[2 * e] += p * bf2f((bf16_t)(w4[e] & 0xffff));
        o[2 * e + 1] += p * bf2f((bf16_t)(w4[e] >> 16));
      }
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) o[e] = rows_sum(o[e] + dpp_f<0x128>(o[e]));
  if (kg == 0) {
    const float inv = 1.0f / sum;
    st16(a.base, a.o_attn + (m * E + h * 64 + d8) * 2,
         (u32x4){pack_bf2(o[0] * inv, o[1] * inv), pack_bf2(o[2] * inv, o[3] * inv),
                 pack_bf2(o[4] * inv, o[5] * inv), pack_bf2(o[6] * inv, o[7] * inv)});
  }
}

// LDS (dynamic), regions reused across phases:
//   A tile [16][E] bf16 (P1 / P4 / P6 LayerNorm output) | red [4 waves][4 tiles][256] f32 |
//   s_q [4][64] f32 + s_p [4][1024] f32 (P2) | rep / ban flag bitmaps [16][kTpw * 16] B (P6) |
//   s_h [1024] int (P7) | scalars
template <int E>
struct Lds {
  // the barrier flag and scalars live OUTSIDE the region P5's weight DMA lands in: that DMA is in
  // flight across the P4 -> P5 barrier, which writes the flag
  static constexpr int kMisc = 0;
  static constexpr int kRed = 128;
  static constexpr int kW5 = kRed + 4 * 4 * 256 * 4;   // P5's weights (LDS-DMA), overlapping the rest
  static constexpr int kA = kW5;
  static constexpr int kSq = kA + 16 * E * 2;
  static constexpr int kSp = kSq + 4 * 64 * 4;
  static constexpr int kRep = kSp + 4 * 1024 * 4;
  static constexpr int kBan = kRep + 16 * kTpw * 16;
  static constexpr int kHist = kBan + 16 * kTpw * 16;
  // > 80 KiB: one workgroup per CU (the grid's co-residency then needs G CUs, and each workgroup's
  // weight stream has a CU's load path to itself)
  static constexpr int kEnd = kHist + 4096 > kW5 + 4 * (E / 32) * 1024 ? kHist + 4096 : kW5 + 4 * (E / 32) * 1024;
  static constexpr int kBytes = kEnd > 82 * 1024 ? kEnd : 82 * 1024;
  static_assert(kBytes <= 160 * 1024, "LDS per CU");
};

// Thread / workgroup ids re-derived inside each phase through an opaque asm: every per-thread
// address is then computed where it is used instead of being hoisted out of the step / layer
// loops by LICM and held in registers across all phases (which spilled ~150 VGPRs).
#define VCAP_PHASE_IDS()                                  \
  int tid = threadIdx.x;                                  \
  asm volatile("" : "+v"(tid));                           \
  const int lane = tid & 63, wave = tid >> 6;             \
  const int fr = lane & 15, fg = lane >> 4;               \
  (void)fr;                                               \
  (void)fg;                                               \
  const bool compute = wave < 4;                          \
  (void)compute;                                          \
  int wg = blockIdx.x;                                    \
  asm volatile("" : "+s"(wg))

template <int E>
__global__ __launch_bounds__(kThreads, 1) void vcap_decode_persist_kernel(PersistArgs a) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  using Ly = Lds<E>;
  constexpr int NSL1 = E / 128, NSL4 = E / 32;  // K slabs per wave (bf16 K step 32 x 4 waves)
  constexpr int LMNTB = 2;                      // lm_head tiles per group (register budget)
  constexpr int NQ = 2 * NSL1;                   // the largest register-held weight set (P1 / P4 / lm_head group)
  char* dyn = lds + Ly::kA;
  float* red = reinterpret_cast<float*>(lds + Ly::kRed);
  unsigned char* s_rep = reinterpret_cast<unsigned char*>(lds + Ly::kRep);
  unsigned char* s_ban = reinterpret_cast<unsigned char*>(lds + Ly::kBan);
  int* s_h = reinterpret_cast<int*>(lds + Ly::kHist);
  int* s_misc = reinterpret_cast<int*>(lds + Ly::kMisc);  // [0] barrier ok, [1] tok, [2] nbanned, [4..9) argmax
  float* s_mv = reinterpret_cast<float*>(lds + Ly::kMisc + 64);

  const int G = a.G, M = a.M, H = a.H, V = a.V;
  const int nt_qkv = 3 * E / 16, nt_e = E / 16, nt_fc = 4 * E / 16, nt_v = (V + 15) / 16;
  unsigned phase = 0;
  // End of a phase: every compute wave drains its stores, issues the next phase's weights (the
  // caller, between the two calls), the workgroup meets, the sync wave arrives + polls, and the
  // workgroup meets again before any load of the next phase.
  auto drain = [&]() {
    if (threadIdx.x < kCompute) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  };
  // raw s_barrier + lgkmcnt(0) (LDS only): __syncthreads() would also wait vmcnt(0), i.e. for the
  // next phase's weights just issued (P5's LDS-DMA counts as a pending LDS write) - the very latency
  // the prefetch is there to hide behind the grid barrier
  auto wg_barrier = [&]() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  auto barrier = [&]() -> bool {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    wg_barrier();
    ++phase;
    if ((a.flags & 32) && lane == 0) {   // diagnostic: agent release by every wave
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    if (a.flags & 32) wg_barrier();
    if (wave == 4) {
      if ((a.flags & 8) && lane == 0 && phase <= kStampPhases)
        g_persist_stamps[blockIdx.x][phase - 1][0] = __builtin_amdgcn_s_memrealtime();
      if (lane == 0)
        __hip_atomic_fetch_add(a.bar + (blockIdx.x & 7) * kShardStride, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned target = phase * (unsigned)G;
      const unsigned long t0 = __builtin_amdgcn_s_memrealtime();
      int ok = 1;
      for (;;) {
        const unsigned v = lane < 8 ? __hip_atomic_load(a.bar + lane * kShardStride, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                           : lane == 8 ? __hip_atomic_load(a.bar + kAbortWord, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                       : 0u;
        unsigned sum = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) sum += __builtin_amdgcn_readlane(v, i);
        if (sum >= target) break;
        if (__builtin_amdgcn_readlane(v, 8)) {
          ok = 0;
          break;
        }
        if (__builtin_amdgcn_s_memrealtime() - t0 > kSpinTicks) {
          if (lane == 0) {
            __hip_atomic_store(a.bar + kAbortWord, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_add(&g_persist_faults, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
          ok = 0;
          break;
        }
        if (!(a.flags & 4)) __builtin_amdgcn_s_sleep(1);
      }
      if (lane == 0) s_misc[0] = ok;
      if ((a.flags & 8) && lane == 0 && phase <= kStampPhases)
        g_persist_stamps[blockIdx.x][phase - 1][1] = __builtin_amdgcn_s_memrealtime();
    }
    if ((a.flags & 16) && lane == 0) {   // diagnostic: agent acquire (L1 invalidate) by every wave
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    wg_barrier();
    return s_misc[0] != 0;
  };

  u32x4 wq[NQ];  // the current phase's prefetched weight fragments
  {
    VCAP_PHASE_IDS();
    if (compute && wg < nt_qkv) issue_w<NSL1, 2>(wq, a.layers[0].attn_w, wg, G, nt_qkv, wave, lane);
  }

  if (a.flags & 1) {   // diagnostic: the step's 5L + 2 grid barriers alone
    for (int i = 0; i < (a.step1 - a.step0) * (5 * a.L + 2); ++i) {
      drain();
      if (!barrier()) return;
    }
    return;
  }
  for (int step = a.step0; step < a.step1; ++step) {
    const int past = a.S0 + step - 1, ctx = past + 1;
    for (int l = 0; l < a.L; ++l) {
      const PersistLayer& ly = a.layers[l];
      const int okc = a.o_kc + l * a.page_bytes, ovc = a.o_vc + l * a.page_bytes;
      // ---------------- P1: ln_1 + c_attn -> q, K/V of position `past`
      {
        VCAP_PHASE_IDS();
        const bool act = wg < nt_qkv;
        if (compute && act) ln_rows<E>(a.base, a.o_h, M, ly.ln1_g, ly.ln1_b, a.ln_eps, dyn, wave, lane);
        wg_barrier();
        if (compute && act) {
          f32x4 acc[2];
          mma_lds<E, NSL1, 2>(acc, wq, dyn, wave, lane);
          to_red<2>(red, acc, wave, lane);
        }
        wg_barrier();
        if (compute && act) {
          const int j = tid >> 7, row = (tid >> 3) & 15, c0 = (tid & 7) * 2;
          const int t = wg + j * G;
          if (t < nt_qkv && row < M) {
            const int n = t * 16 + c0;
            const float v0 = red_val(red, j, row, c0, ly.attn_b[n]);
            const float v1 = red_val(red, j, row, c0 + 1, ly.attn_b[n + 1]);
            const unsigned pk = (unsigned)f2bf(v0) | ((unsigned)f2bf(v1) << 16);
            const int which = n / E, within = n - which * E;
            if (which == 0) {
              st4(a.base, a.o_q + (row * E + within) * 2, pk);
            } else {
              const int head = within >> 6, d = within & 63;
              const int off = (((row * a.maxp + (past >> 4)) * H + head) * 16 + (past & 15)) * 64 * 2 + d * 2;
              st4(a.base, (which == 1 ? okc : ovc) + off, pk);
            }
          }
        }
        drain();
        if (!barrier()) return;
      }
      // ---------------- P2: attention, item i = (row, head) on workgroup i % G, wave i / G
      {
        VCAP_PHASE_IDS();
        if (compute) {
          float* s_q = reinterpret_cast<float*>(lds + Ly::kSq) + wave * 64;
          float* s_p = reinterpret_cast<float*>(lds + Ly::kSp) + wave * 1024;
          for (int i = wg + wave * G; i < M * H; i += 4 * G) attn_item(a, okc, ovc, i / H, i % H, ctx, s_q, s_p, lane);
        }
        drain();
        if (compute && wg < nt_e) issue_w<NSL1, 1>(wq, ly.aproj_w, wg, G, nt_e, wave, lane);
        if (!barrier()) return;
      }
      // ---------------- P3: attn c_proj + residual (PRO_DIRECT A = attention output)
      {
        VCAP_PHASE_IDS();
        const int t = wg;
        const bool act = t < nt_e;
        const int row = tid >> 3, c0 = (tid & 7) * 2, n = t * 16 + c0;
        u32x2 res = (u32x2){0u, 0u};
        if (compute && act) {
          u32x4 af[NSL1];
          const int xo = min(fr, M - 1) * E + fg * 8;
#pragma unroll
          for (int s = 0; s < NSL1; ++s) af[s] = ld16(a.base, a.o_attn + (xo + (wave * NSL1 + s) * 32) * 2);
          if (tid < 128 && row < M) res = ld8(a.base, a.o_h + (row * E + n) * 4);
          f32x4 acc[1] = {(f32x4){0.f, 0.f, 0.f, 0.f}};
#pragma unroll
          for (int s = 0; s < NSL1; ++s) acc[0] = mfma_frag(af[s], wq[s], acc[0], (bf16_t*)nullptr);
          to_red<1>(red, acc, wave, lane);
        }
        wg_barrier();
        if (compute && act && tid < 128 && row < M) {
          const float v0 = __uint_as_float(res.x) + red_val(red, 0, row, c0, ly.aproj_b[n]);
          const float v1 = __uint_as_float(res.y) + red_val(red, 0, row, c0 + 1, ly.aproj_b[n + 1]);
          st8(a.base, a.o_h + (row * E + n) * 4, (u32x2){__float_as_uint(v0), __float_as_uint(v1)});
        }
        drain();
        if (compute && wg < nt_fc) issue_w<NSL1, 2>(wq, ly.fc_w, wg, G, nt_fc, wave, lane);
        if (!barrier()) return;
      }
      // ---------------- P4: ln_2 + c_fc + gelu_new
      {
        VCAP_PHASE_IDS();
        const bool act = wg < nt_fc;
        if (compute && act) ln_rows<E>(a.base, a.o_h, M, ly.ln2_g, ly.ln2_b, a.ln_eps, dyn, wave, lane);
        wg_barrier();
        if (compute && act) {
          f32x4 acc[2];
          mma_lds<E, NSL1, 2>(acc, wq, dyn, wave, lane);
          to_red<2>(red, acc, wave, lane);
        }
        wg_barrier();
        if (compute && act) {
          const int j = tid >> 7, row = (tid >> 3) & 15, c0 = (tid & 7) * 2;
          const int t = wg + j * G;
          if (t < nt_fc && row < M) {
            const int n = t * 16 + c0;
            const float v0 = gelu_tanh(red_val(red, j, row, c0, ly.fc_b[n]));
            const float v1 = gelu_tanh(red_val(red, j, row, c0 + 1, ly.fc_b[n + 1]));
            st4(a.base, a.o_act + (row * 4 * E + n) * 2, (unsigned)f2bf(v0) | ((unsigned)f2bf(v1) << 16));
          }
        }
        drain();
        // P5's weights: LDS-DMA into the region the A tile used (free: every wave passed the barrier
        // after its MFMAs); red, still read by this epilogue, is not overlapped
        if (compute && wg < nt_e) issue_w_lds<NSL4>(ly.mproj_w, wg, lds + Ly::kW5, wave, lane);
        if (!barrier()) return;
      }
      // ---------------- P5: mlp c_proj + residual (K = 4E, PRO_DIRECT A = activations)
      {
        VCAP_PHASE_IDS();
        const int t = wg;
        const bool act = t < nt_e;
        const int row = tid >> 3, c0 = (tid & 7) * 2, n = t * 16 + c0;
        u32x2 res = (u32x2){0u, 0u};
        if (compute && act) {
          u32x4 af[NSL4];
          const int xo = min(fr, M - 1) * 4 * E + fg * 8;
#pragma unroll
          for (int s = 0; s < NSL4; ++s) af[s] = ld16(a.base, a.o_act + (xo + (wave * NSL4 + s) * 32) * 2);
          if (tid < 128 && row < M) res = ld8(a.base, a.o_h + (row * E + n) * 4);
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's weight DMA has landed
          const char* w5 = lds + Ly::kW5 + wave * NSL4 * 1024 + lane * 16;
          f32x4 acc[1] = {(f32x4){0.f, 0.f, 0.f, 0.f}};
#pragma unroll
          for (int s = 0; s < NSL4; ++s)
            acc[0] = mfma_frag(af[s], *reinterpret_cast<const u32x4*>(w5 + s * 1024), acc[0], (bf16_t*)nullptr);
          to_red<1>(red, acc, wave, lane);
        }
        wg_barrier();
        if (compute && act && tid < 128 && row < M) {
          const float v0 = __uint_as_float(res.x) + red_val(red, 0, row, c0, ly.mproj_b[n]);
          const float v1 = __uint_as_float(res.y) + red_val(red, 0, row, c0 + 1, ly.mproj_b[n + 1]);
          st8(a.base, a.o_h + (row * E + n) * 4, (u32x2){__float_as_uint(v0), __float_as_uint(v1)});
        }
        drain();
        if (compute) {
          if (l + 1 < a.L) {
            if (wg < nt_qkv) issue_w<NSL1, 2>(wq, a.layers[l + 1].attn_w, wg, G, nt_qkv, wave, lane);
          } else if (wg < nt_v) {
            issue_w<NSL1, LMNTB>(wq, a.lm_head, wg, G, nt_v, wave, lane);
          }
        }
        if (!barrier()) return;
      }
    }
    // ---------------- P6: ln_f + lm_head + processors -> this workgroup's argmax per row
    {
      VCAP_PHASE_IDS();
      const int ntl = wg < nt_v ? (nt_v - wg + G - 1) / G : 0;  // tiles wg, wg + G, ...
      const int gen_len = step;
      // processor flags of this workgroup's columns: local column (k * 16 + c) <-> tile wg + k*G
      for (int i = tid; i < 16 * kTpw * 16 / 4; i += kThreads) {
        reinterpret_cast<unsigned*>(s_rep)[i] = 0u;
        reinterpret_cast<unsigned*>(s_ban)[i] = 0u;
      }
      wg_barrier();
      if (compute) {
        for (int i = tid; i < M * a.hist_ld; i += kCompute) {
          const int m = i / a.hist_ld, tt = i - m * a.hist_ld;
          const int nb = (int)ld4(a.base, a.o_nbanned + m * 4);
          const int th = (int)ld4(a.base, a.o_hist + i * 4);
          const int tb = (int)ld4(a.base, a.o_banned + i * 4);
          if (a.rep != 1.0f && tt < gen_len && th >= 0 && (th >> 4) % G == wg)
            s_rep[m * kTpw * 16 + ((th >> 4) / G) * 16 + (th & 15)] = 1;
          if (tt < nb && tb >= 0 && (tb >> 4) % G == wg) s_ban[m * kTpw * 16 + ((tb >> 4) / G) * 16 + (tb & 15)] = 1;
        }
        if (ntl > 0) ln_rows<E>(a.base, a.o_h, M, a.lnf_g, a.lnf_b, a.ln_eps, dyn, wave, lane);
      }
      wg_barrier();
      float bv = -INFINITY;
      int bi = 0x7fffffff;
      const int row = tid >> 4, col = tid & 15;
      float* lout = a.logits_out ? a.logits_out + (long)step * M * V : nullptr;
      const int ngr = (ntl + LMNTB - 1) / LMNTB;
      auto group = [&](const u32x4 (&w)[NQ], int gi) {
        if (compute) {
          f32x4 acc[LMNTB];
          mma_lds<E, NSL1, LMNTB>(acc, w, dyn, wave, lane);
          to_red<LMNTB>(red, acc, wave, lane);
        }
        wg_barrier();
        if (compute && row < M) {
#pragma unroll
          for (int j = 0; j < LMNTB; ++j) {
            const int k = gi * LMNTB + j, t = wg + k * G;
            const int n = t * 16 + col;
            if (k < ntl && n < V) {
              const float v = red_val(red, j, row, col, 0.f);
              if (lout) lout[(long)row * V + n] = v;
              float sv = v;
              const int li = row * kTpw * 16 + k * 16 + col;
              if (s_rep[li]) sv = sv < 0.f ? sv * a.rep : sv / a.rep;
              if (s_ban[li]) sv = -INFINITY;
              if (n == a.eos && gen_len < a.min_new) sv = -INFINITY;
              argmax_take(bv, bi, sv, n);
            }
          }
        }
        wg_barrier();
      };
      u32x4 wB[NQ];
      for (int gi = 0; gi < ngr; gi += 2) {
        if (compute && gi + 1 < ngr) issue_w<NSL1, LMNTB>(wB, a.lm_head, wg + (gi + 1) * LMNTB * G, G, nt_v, wave, lane);
        group(wq, gi);
        if (gi + 1 < ngr) {
          if (compute && gi + 2 < ngr) issue_w<NSL1, LMNTB>(wq, a.lm_head, wg + (gi + 2) * LMNTB * G, G, nt_v, wave, lane);
          group(wB, gi + 1);
        }
      }
      // per row: the 16 lanes of the row (one DPP row) -> this workgroup's partial
      argmax_take(bv, bi, dpp_f<DPP_XOR1>(bv), dpp_i<DPP_XOR1>(bi));
      argmax_take(bv, bi, dpp_f<DPP_XOR2>(bv), dpp_i<DPP_XOR2>(bi));
      argmax_take(bv, bi, dpp_f<DPP_HALF_MIRROR>(bv), dpp_i<DPP_HALF_MIRROR>(bi));
      argmax_take(bv, bi, dpp_f<DPP_MIRROR>(bv), dpp_i<DPP_MIRROR>(bi));
      if (compute && col == 0 && row < M) {
        st4(a.base, a.o_pval + (row * G + wg) * 4, __float_as_uint(bv));
        st4(a.base, a.o_pidx + (row * G + wg) * 4, (unsigned)bi);
      }
      drain();
      if (!barrier()) return;
    }
    // ---------------- P7: finalize row m on workgroup m
    {
      VCAP_PHASE_IDS();
      const int m = wg;
      if (m < M) {
        const int hl = a.hist_ld;
        float pv = -INFINITY;
        int pi = 0x7fffffff;
        if (tid < G) {
          pv = ldf(a.base, a.o_pval + (m * G + tid) * 4);
          pi = (int)ld4(a.base, a.o_pidx + (m * G + tid) * 4);
        }
        for (int i = tid; i < step; i += kThreads) s_h[i] = (int)ld4(a.base, a.o_hist + (m * hl + i) * 4);
        const int fin = (int)ld4(a.base, a.o_finished + m * 4);
        float bv = -INFINITY;
        int bi = 0x7fffffff;
        argmax_take(bv, bi, pv, pi);
        wave_argmax(bv, bi);
        if (lane == 0) {
          s_mv[wave] = bv;
          s_misc[4 + wave] = bi;
        }
        wg_barrier();
        if (tid == 0) {
          for (int w = 1; w < kThreads / 64; ++w) argmax_take(bv, bi, s_mv[w], s_misc[4 + w]);
          int tok = bi;
          tok = tok < 0 ? 0 : (tok >= V ? V - 1 : tok);
          if (fin) tok = a.pad;
          a.out_ids[(long)m * a.out_ld + step] = tok;   // read by the host only, after the launch
          st4(a.base, a.o_hist + (m * hl + step) * 4, (unsigned)tok);
          s_h[step] = tok;
          if (tok == a.eos) st4(a.base, a.o_finished + m * 4, 1u);
          s_misc[1] = tok;
          s_misc[2] = 0;
        }
        wg_barrier();
        const int Lh = step + 1, ng = a.ngram;
        if (ng > 0 && Lh + 1 >= ng) {
          for (int i = tid; i + ng <= Lh; i += kThreads) {
            bool match = true;
            for (int t = 0; t < ng - 1; ++t) match &= (s_h[i + t] == s_h[Lh - ng + 1 + t]);
            if (match) st4(a.base, a.o_banned + (m * hl + atomicAdd(&s_misc[2], 1)) * 4, (unsigned)s_h[i + ng - 1]);
          }
        }
        wg_barrier();
        if (tid == 0) st4(a.base, a.o_nbanned + m * 4, (unsigned)s_misc[2]);
        const int tok = s_misc[1];
        const int pos = min(a.S0 + step, a.n_pos - 1);
        for (int c = tid * 4; c < E; c += kThreads * 4) {
          const float* wp = a.wpe + (long)pos * E + c;
          const bf16_t* we = a.wte + (long)tok * E + c;
          st16(a.base, a.o_h + (m * E + c) * 4,
               (u32x4){__float_as_uint(bf2f(we[0]) + wp[0]), __float_as_uint(bf2f(we[1]) + wp[1]),
                       __float_as_uint(bf2f(we[2]) + wp[2]), __float_as_uint(bf2f(we[3]) + wp[3])});
        }
      }
      if (tid < kThreads) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every wave stored here
      if (compute && step + 1 < a.step1 && wg < nt_qkv) issue_w<NSL1, 2>(wq, a.layers[0].attn_w, wg, G, nt_qkv, wave, lane);
      if (!barrier()) return;
    }
  }
}

template <int E>
hipError_t launch_persist(const PersistArgs& a, hipStream_t s) {
  static int configured = 0;
  if (!configured) {
    if (hipFuncSetAttribute((const void*)vcap_decode_persist_kernel<E>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            Lds<E>::kBytes) != hipSuccess)
      return hipErrorInvalidValue;
    configured = 1;
  }
  hipLaunchKernelGGL((vcap_decode_persist_kernel<E>), dim3(a.G), dim3(kThreads), Lds<E>::kBytes, s, a);
  return hipGetLastError();
}

}  // namespace

int vcap_persist_min_wgs(int E) { return E / 8 > 64 ? E / 8 : 64; }

size_t vcap_persist_bar_bytes() { return 2048; }
// barrier words + the device layer table
size_t vcap_persist_ws_bytes() { return vcap_persist_bar_bytes() + sizeof(PersistLayer) * kPersistMaxLayers; }

hipError_t vcap_decode_persist_dispatch(const PersistDesc& d, hipStream_t s) {
  const int E = d.E;
  if ((E != 128 && E != 768 && E != 1024) || d.G < vcap_persist_min_wgs(E) || d.G > 256 || d.M < 1 || d.M > 16 ||
      d.L < 1 || d.L > kPersistMaxLayers || d.H * 64 != E || (d.V + 15) / 16 > kTpw * d.G || d.hist_ld > 1024 ||
      d.M * d.H > 4 * d.G || d.S0 + d.step1 - 1 > 1024 || d.step0 < 1 || d.step1 < d.step0 || d.step1 > d.hist_ld ||
      !d.bar)
    return hipErrorInvalidValue;
  if (d.step1 == d.step0) return hipSuccess;
  PersistArgs a;
  a.G = d.G; a.M = d.M; a.E = E; a.H = d.H; a.L = d.L; a.V = d.V; a.S0 = d.S0; a.maxp = d.maxp; a.n_pos = d.n_pos;
  a.step0 = d.step0; a.step1 = d.step1; a.ln_eps = d.ln_eps;
  a.lnf_g = d.lnf_g; a.lnf_b = d.lnf_b; a.lm_head = d.lm_head; a.wte = (const bf16_t*)d.wte; a.wpe = d.wpe;
  // one buffer resource over the workspace: every handed-off buffer as a byte offset from the lowest
  const void* bufs[12] = {d.h, d.q, d.attn, d.act, d.kc, d.vc, d.hist, d.banned, d.nbanned, d.finished, d.pval, d.pidx};
  const char* lo = (const char*)bufs[0];
  for (const void* b : bufs) lo = std::min(lo, (const char*)b);
  int offs[12];
  const long page_bytes = d.page_elems * 2;
  for (int i = 0; i < 12; ++i) {
    const long o = (const char*)bufs[i] - lo;
    if (o < 0 || o + page_bytes * d.L > 0x70000000L) return hipErrorInvalidValue;
    offs[i] = (int)o;
  }
  a.base = const_cast<char*>(lo);
  a.o_h = offs[0]; a.o_q = offs[1]; a.o_attn = offs[2]; a.o_act = offs[3]; a.o_kc = offs[4]; a.o_vc = offs[5];
  a.page_bytes = (int)page_bytes;
  a.o_hist = offs[6]; a.o_banned = offs[7]; a.o_nbanned = offs[8]; a.o_finished = offs[9];
  a.o_pval = offs[10]; a.o_pidx = offs[11];
  a.hist_ld = d.hist_ld;
  a.ngram = d.ngram; a.rep = d.rep; a.min_new = d.min_new; a.eos = d.eos; a.pad = d.pad;
  a.out_ids = d.out_ids; a.out_ld = d.out_ld; a.logits_out = d.logits_out;
  static const int flags = [] {
    const char* e = std::getenv("VCAP_PERSIST_FLAGS");
    return e ? (int)std::strtol(e, nullptr, 10) : 0;
  }();
  a.flags = flags;
  a.bar = d.bar;
  a.layers = reinterpret_cast<const PersistLayer*>(d.bar + vcap_persist_bar_bytes() / 4);
  PersistLayers pl;
  for (int l = 0; l < d.L; ++l) pl.l[l] = d.layers[l];
  if (hipError_t e = hipMemsetAsync(d.bar, 0, vcap_persist_bar_bytes(), s)) return e;
  hipLaunchKernelGGL(vcap_persist_layers_kernel, dim3(1), dim3(64), 0, s, pl, d.L,
                     const_cast<PersistLayer*>(a.layers));
  if (hipError_t e = hipGetLastError()) return e;
  if (E == 768) return launch_persist<768>(a, s);
  if (E == 1024) return launch_persist<1024>(a, s);
  return launch_persist<128>(a, s);
}

// diagnostic read-back of the stamps (not part of include/vcap.h): n values of [wg][phase][2]
extern "C" int vcap_persist_stamps_read(unsigned long* dst, size_t n) {
  const size_t cap = sizeof(g_persist_stamps) / sizeof(unsigned long);
  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_persist_stamps), (n < cap ? n : cap) * sizeof(unsigned long), 0,
                             hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}

unsigned vcap_decode_persist_faults() {
  unsigned v = 0;
  if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_persist_faults), sizeof(v), 0, hipMemcpyDeviceToHost) != hipSuccess)
    return 0xFFFFFFFFu;
  return v;
}
