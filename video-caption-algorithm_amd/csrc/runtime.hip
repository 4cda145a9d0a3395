// Host runtime behind the C ABI (include/vcap.h): argument checking, workspace carving, the
// ViT forward schedule, the GPT-2 decode schedule and its hipGraph cache.
//
// The reference drives these steps from Python (timm forward_features, HF generate); here the
// whole schedule is native so one ABI call issues the full encode or the full decode, and the
// decode (~60 launches per token) can be captured once into a hipGraph and replayed.
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <list>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/vcap.h"
#include "vcap_common.h"
#include "vcap_kernels.h"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

int hip_fail(hipError_t e, const char* where) {
  if (e == hipSuccess) return 0;
  g_err = std::string(where) + ": " + hipGetErrorString(e);
  return -(int)e;
}

#define VCAP_TRY(expr, where)                    \
  do {                                           \
    hipError_t _e = (expr);                      \
    if (_e != hipSuccess) return hip_fail(_e, where); \
  } while (0)

size_t esize(int dt) { return dt == VCAP_DT_MXFP8 ? 1 : dt == VCAP_DT_BF16 ? 2 : 4; }
size_t mx_scale_bytes(int rows, int K) { return (size_t)(K / 128) * (size_t)((rows + 255) / 256) * 1024; }
size_t al(size_t x) { return (x + 255) & ~size_t(255); }

struct Carver {
  char* base;
  size_t off = 0;
  explicit Carver(void* b) : base((char*)b) {}
  void* take(size_t bytes) {
    void* p = base ? base + off : nullptr;
    off += al(bytes);
    return p;
  }
};

bool attn_lds_configured = false;

// Decoder rows one call may carry (B * (prefix + prompt) at the prefill, rows of a step).  Rows go
// through the GEMV kernels in 16 / 32-row chunks (blockIdx.y), so this bounds workspace sizes only.
constexpr int kMaxDecodeRows = 512;

// ----------------------------------------------------------------------------------- kernel probes
// Live per-site timing for bench.py's roofline: HIP events recorded around every launch of a
// probed site on the caller's stream (no synchronisation; read back after the timed region).
struct Probe {
  std::vector<hipEvent_t> start, stop;
  std::vector<int> rows;   // work size of each launch (GEMM / attention rows), for per-launch pricing
  int used = 0;
  bool on = false;
};
std::mutex g_probe_mu;
std::unordered_map<std::string, Probe> g_probes;

Probe* probe_for(const char* site) {
  std::lock_guard<std::mutex> lk(g_probe_mu);
  auto it = g_probes.find(site);
  if (it == g_probes.end() || !it->second.on || it->second.used >= (int)it->second.start.size()) return nullptr;
  return &it->second;
}

struct ProbeScope {
  Probe* p;
  hipStream_t s;
  int idx;
  ProbeScope(const char* site, hipStream_t st, int rows) : p(probe_for(site)), s(st), idx(-1) {
    if (p) {
      idx = p->used++;
      p->rows[idx] = rows;
      (void)hipEventRecord(p->start[idx], s);
    }
  }
  ~ProbeScope() {
    if (p) (void)hipEventRecord(p->stop[idx], s);
  }
};


// ----------------------------------------------------------------------------------- ViT
struct VitBufs {
  float* x;
  void* xn;
  void* qkv;
  void* attn;
  void* act;
  uint8_t* xn_s;   // MXFP8 scales of xn / act
  uint8_t* act_s;
  float* splitk;   // split-K partial slabs of the CLS-tail attn-proj / fc2 (deterministic reduce)
  size_t splitk_bytes;
};

// operand dtype of patch-embed / qkv output / attention / attn-proj: bf16 in the MXFP8 mode
int vit_adt(int dt) { return dt == VCAP_DT_MXFP8 ? VCAP_DT_BF16 : dt; }

VitBufs carve_vit(Carver& c, const vcap_vit_desc* d, int B, int T) {
  const int tokens = (d->image / d->patch) * (d->image / d->patch) + 1;
  const size_t M = (size_t)B * T * tokens;
  const size_t es = esize(d->dtype), ea = esize(vit_adt(d->dtype));
  const size_t npatch = (size_t)B * T * (tokens - 1);
  VitBufs v;
  // MXFP8 mode: any GEMM of a layer may stay bf16 (its weight scales NULL), so the LayerNorm and
  // fc1 outputs are sized for bf16 elements
  const size_t en = es > ea ? es : ea;
  v.x = (float*)c.take(M * d->dim * 4);
  v.xn = c.take(M * d->dim * en);
  v.qkv = c.take(M * 3 * d->dim * ea);
  v.attn = c.take(M * d->dim * ea);
  size_t act = M * d->mlp * en;
  const size_t patches = npatch * d->kpad * ea;
  v.act = c.take(act > patches ? act : patches);
  v.xn_s = v.act_s = nullptr;
  v.splitk_bytes = (size_t)16 * B * T * d->dim * 4;   // <= 16 splits of the [B*T, dim] CLS rows
  v.splitk = (float*)c.take(v.splitk_bytes);
  if (d->dtype == VCAP_DT_MXFP8) {
    v.xn_s = (uint8_t*)c.take(mx_scale_bytes((int)M, d->dim));
    v.act_s = (uint8_t*)c.take(mx_scale_bytes((int)M, d->mlp));
  }
  return v;
}

int check_vit(const vcap_vit_desc* d) {
  if (!d || !d->layers) return fail(VCAP_E_ARG, "vit desc is null");
  if (d->dtype != VCAP_DT_F32 && d->dtype != VCAP_DT_BF16 && d->dtype != VCAP_DT_MXFP8)
    return fail(VCAP_E_ARG, "vit dtype");
  if (d->heads * 64 != d->dim) return fail(VCAP_E_UNSUPPORTED, "vit head_dim must be 64");
  const int ka = vcap_gemm_k_align(d->dtype);
  if (d->dim % ka || d->mlp % ka || d->kpad % vcap_gemm_k_align(vit_adt(d->dtype)) || d->kpad < 3 * d->patch * d->patch)
    return fail(VCAP_E_UNSUPPORTED, "vit dims must be multiples of the GEMM K step");
  if (d->dtype == VCAP_DT_MXFP8) {
    // per GEMM: weight scales present = MXFP8 block GEMM, NULL = that GEMM's weights are bf16
    if (d->dim > 1024) return fail(VCAP_E_UNSUPPORTED, "MXFP8 LayerNorm holds rows of <= 1024 in registers");
    if (d->dim % 256 || d->mlp % 256) return fail(VCAP_E_UNSUPPORTED, "MXFP8 dims must be multiples of 256");
  }
  if (d->image % d->patch) return fail(VCAP_E_ARG, "image not divisible by patch");
  const int tokens = (d->image / d->patch) * (d->image / d->patch) + 1;
  if (tokens > 288) return fail(VCAP_E_UNSUPPORTED, "more than 288 tokens");
  return 0;
}

// ----------------------------------------------------------------------------------- GPT-2
struct DecBufs {
  float* h;
  float* sh;  // [B][E] f32 ln_f rows of the bf16 lm_head screen (f32 greedy)
  void* q;
  void* attn;
  void* act;
  void* kc;
  void* vc;
  int* pt;
  float* pval;
  int* pidx;
  int* hist;
  int* banned;
  int* nbanned;
  int* finished;
  float* proc;        // [B][V] processed scores (sampling mode)
  unsigned* seed;     // [2] Philox key of the sampling draws
  // f32 mlp c_proj K split (RowsGemmArgs.sk_*): pair partials + tickets, zeroed by vcap_decode_init at
  // the start of every decode, prefill and forward_embeds sequence (all f32 paths run the same split,
  // so a teacher-forced forward reproduces the free-running graph's logits bit for bit)
  float* skp;
  int* skc;
  int n_skc;
};

int max_logit_blocks(int V, int B) { return vcap_logit_blocks(V, B); }

DecBufs carve_dec(Carver& c, const vcap_gpt2_desc* d, int B, int S0, int max_new, int* maxp_out, size_t* page_elems) {
  const int E = d->n_embd;
  const size_t es = esize(d->dtype);
  const size_t Mmax = (size_t)B * S0 > (size_t)B ? (size_t)B * S0 : B;
  const int maxp = (S0 + max_new + 15) / 16;
  *maxp_out = maxp;
  const size_t pages = (size_t)B * maxp;
  const size_t per_layer = pages * d->n_head * 16 * 64;  // elements
  *page_elems = per_layer;
  DecBufs b;
  b.h = (float*)c.take(Mmax * E * 4);
  b.q = c.take(Mmax * E * es);
  b.attn = c.take(Mmax * E * es);
  b.act = c.take(Mmax * 4 * E * es);
  b.kc = c.take(per_layer * d->n_layer * es);
  b.vc = c.take(per_layer * d->n_layer * es);
  b.pt = (int*)c.take(pages * 4);
  // argmax partials: the lm_head's 64-column GEMV blocks or its stream kernel's grid (<= CUs)
  const int nb = std::max({max_logit_blocks(d->vocab, B), vcap_device_cus(), 256});
  b.pval = (float*)c.take((size_t)B * nb * 4);
  b.pidx = (int*)c.take((size_t)B * nb * 4);
  b.hist = (int*)c.take((size_t)B * max_new * 4);
  b.banned = (int*)c.take((size_t)B * max_new * 4);
  b.nbanned = (int*)c.take((size_t)B * 4);
  b.finished = (int*)c.take((size_t)B * 4);
  b.proc = (float*)c.take((size_t)B * d->vocab * 4);
  b.sh = (float*)c.take((size_t)B * E * 4);
  b.seed = (unsigned*)c.take(8);
  // K split: every 16-row chunk of the largest launch (Mmax rows) x E / 16 tiles x 256 partials x 4
  // (the pairs: 2 halves per tile; the f32 4-way split: E / 32 groups x 4 parts x 2 tiles); the
  // tickets, one per tile or group
  b.n_skc = (int)((Mmax + 15) / 16) * ((E + 15) / 16);
  b.skp = (float*)c.take((size_t)b.n_skc * 4 * 256 * 4);
  b.skc = (int*)c.take((size_t)b.n_skc * 4);
  return b;
}

int check_gpt2(const vcap_gpt2_desc* d) {
  if (!d || !d->layers) return fail(VCAP_E_ARG, "gpt2 desc is null");
  if (d->dtype != VCAP_DT_F32 && d->dtype != VCAP_DT_BF16) return fail(VCAP_E_ARG, "gpt2 dtype");
  if (d->n_head * 64 != d->n_embd) return fail(VCAP_E_UNSUPPORTED, "gpt2 head_dim must be 64");
  if (d->n_embd % 128) return fail(VCAP_E_UNSUPPORTED, "n_embd must be a multiple of 128");
  if (d->n_embd > 1024) return fail(VCAP_E_UNSUPPORTED, "n_embd > 1024 (LayerNorm rows are held in registers)");
  return 0;
}

// shape checks + the weight pointers a launch dereferences
int check_gpt2_launch(const vcap_gpt2_desc* d) {
  if (int rc = check_gpt2(d)) return rc;
  if (!d->lm_head || !d->wte || !d->wpe || !d->lnf_g || !d->lnf_b)
    return fail(VCAP_E_ARG, "gpt2 wte / lm_head / wpe / ln_f pointer is null");
  return 0;
}

int run_layers(const vcap_gpt2_desc* d, const DecBufs& w, int maxp, size_t page_elems, int M, int S_new, int past,
               int max_blocks, hipStream_t s, const int* anc = nullptr, int anc_ld = 0) {
  const int E = d->n_embd, H = d->n_head, L = d->n_layer;
  const int dt = d->dtype;
  const size_t es = esize(dt);
  for (int l = 0; l < L; ++l) {
    const vcap_gpt2_layer& ly = d->layers[l];
    RowsGemmArgs a;
    memset(&a, 0, sizeof(a));
    a.M = M;
    a.ln_eps = d->ln_eps;
    // 1) ln_1 + c_attn -> q, paged K/V
    a.x = w.h; a.ldx = E; a.ln_g = ly.ln1_g; a.ln_b = ly.ln1_b;
    a.w = ly.attn_w; a.bias = ly.attn_b; a.N = 3 * E; a.K = E;
    a.q_out = w.q;
    a.kc = (char*)w.kc + (size_t)l * page_elems * es;
    a.vc = (char*)w.vc + (size_t)l * page_elems * es;
    // pages are allocated contiguously per sequence (identity table written by vcap_decode_init):
    // the scatter computes page ids instead of loading them (nullptr table)
    a.page_table = nullptr; a.maxp = maxp; a.H = H; a.S_new = S_new; a.past = past; a.max_blocks = max_blocks;
    VCAP_TRY(vcap_rows_gemm_dispatch(dt, PRO_LN, EPI_QKV, a, nullptr, s), "c_attn");
    // 2) causal attention over the paged cache
    // pages are allocated contiguously per sequence (vcap_decode_init: identity table), so the
    // short-context kernels (bf16 and f32) compute page ids instead of loading them (nullptr table)
    const int* pt_arg = past + S_new <= 64 ? nullptr : w.pt;
    if (anc)   // beam search: keys through the ancestry table (one query row per sequence)
      VCAP_TRY(vcap_decode_attention_anc_dispatch(dt, w.q, a.kc, a.vc, anc, anc_ld, maxp, w.attn, M, H, past, s),
               "decode_attention_anc");
    else
      VCAP_TRY(vcap_decode_attention_dispatch(dt, w.q, a.kc, a.vc, pt_arg, maxp, w.attn, M, H, S_new, past, s),
               "decode_attention");
    // 3) attn c_proj + residual
    RowsGemmArgs b;
    memset(&b, 0, sizeof(b));
    b.M = M; b.x = w.attn; b.ldx = E; b.w = ly.aproj_w; b.bias = ly.aproj_b; b.N = E; b.K = E;
    b.out = w.h; b.ldo = E; b.max_blocks = max_blocks;
    VCAP_TRY(vcap_rows_gemm_dispatch(dt, PRO_DIRECT, EPI_RESID, b, nullptr, s), "attn_c_proj");
    // 4) ln_2 + c_fc + gelu_new
    RowsGemmArgs c;
    memset(&c, 0, sizeof(c));
    c.M = M; c.x = w.h; c.ldx = E; c.ln_g = ly.ln2_g; c.ln_b = ly.ln2_b; c.ln_eps = d->ln_eps;
    c.w = ly.fc_w; c.bias = ly.fc_b; c.N = 4 * E; c.K = E; c.out = w.act; c.ldo = 4 * E; c.max_blocks = max_blocks;
    VCAP_TRY(vcap_rows_gemm_dispatch(dt, PRO_LN, EPI_GELU, c, nullptr, s), "c_fc");
    // 5) mlp c_proj + residual
    RowsGemmArgs e;
    memset(&e, 0, sizeof(e));
    e.M = M; e.x = w.act; e.ldx = 4 * E; e.w = ly.mproj_w; e.bias = ly.mproj_b; e.N = E;
    e.K = 4 * E; e.out = w.h; e.ldo = E; e.max_blocks = max_blocks;
    {  // every row count: the arithmetic may not depend on the launch's M (the dispatcher drops the split where
       // it does not apply)
      e.sk_part = w.skp;
      e.sk_cnt = w.skc;
    }
    VCAP_TRY(vcap_rows_gemm_dispatch(dt, PRO_DIRECT, EPI_RESID, e, nullptr, s), "mlp_c_proj");
  }
  return 0;
}

// ln_f on each sequence's last row (fused into the lm_head's A prologue) + tied lm_head with the
// fused processors and argmax partials.
int run_lm_head(const vcap_gpt2_desc* d, const DecBufs& w, int rows, int S_new, float* logits_raw, int hist_ld,
                int gen_len, float rep, int min_new, int eos, int* nblk, hipStream_t s, float* proc_out = nullptr) {
  const int E = d->n_embd;
  RowsGemmArgs g;
  memset(&g, 0, sizeof(g));
  g.M = rows; g.x = w.h + (size_t)(S_new - 1) * E; g.ldx = (long)S_new * E;
  g.ln_g = d->lnf_g; g.ln_b = d->lnf_b; g.ln_eps = d->ln_eps;
  g.w = d->lm_head; g.bias = nullptr; g.N = d->vocab; g.K = E;
  g.logits_raw = logits_raw;
  g.part_val = w.pval; g.part_idx = w.pidx;
  g.nblk = max_logit_blocks(d->vocab, rows);
  g.hist = w.hist; g.hist_ld = hist_ld; g.gen_len = gen_len; g.banned = w.banned; g.nbanned = w.nbanned;
  g.rep_penalty = rep; g.min_new = min_new; g.eos = eos;
  g.proc_out = proc_out;
  VCAP_TRY(vcap_rows_gemm_dispatch(d->dtype, PRO_LN, EPI_LOGITS, g, nblk, s), "lm_head");
  return 0;
}

// sp != nullptr: sampling mode (HF _sample): the lm_head also stores the processed scores, the
// sample kernel warps them and draws (or takes force_ids), and hands the token to the finalize kernel
int issue_decode(const vcap_gpt2_desc* d, const vcap_gen_params* gp, const float* prefix, const int* ids, int nids,
                 int B, int* out_ids, float* logits_out, const DecBufs& w0, int maxp, size_t page_elems,
                 hipStream_t s, const vcap_sample_params* sp = nullptr, float* warped_out = nullptr,
                 const int* force_ids = nullptr) {
  const int E = d->n_embd, V = d->vocab;
  const int P = d->prefix_len, S0 = P + nids, max_new = gp->max_new_tokens;
  const int dt = d->dtype;
  const DecBufs& w = w0;
  VCAP_TRY(vcap_decode_init_dispatch(w.pt, B, maxp, w.finished, w.nbanned, s, w.skc, w.n_skc), "decode_init");
  VCAP_TRY(vcap_prefill_embed_dispatch(dt, prefix, P, ids, nids, d->wte, d->wpe, w.h, B, E, s), "prefill_embed");
  for (int step = 0; step < max_new; ++step) {
    const int S_new = step == 0 ? S0 : 1;
    const int past = step == 0 ? 0 : S0 + step - 1;
    if (int rc = run_layers(d, w, maxp, page_elems, B * S_new, S_new, past, gp->max_blocks, s)) return rc;
    int nblk = 0;
    // f32 greedy: the bf16 lm_head screens, the finalize rescores the survivors in f32 (exact argmax);
    // requested raw logits or sampling need every f32 score - the f32 lm_head then
    ScreenArgs sc{};
    bool screen = false;
    if (dt == VCAP_DT_F32 && d->lm_head_screen && d->screen_bound > 0.f && !logits_out && !sp) {
      RowsGemmArgs g;
      memset(&g, 0, sizeof(g));
      g.M = B; g.x = w.h + (size_t)(S_new - 1) * E; g.ldx = (long)S_new * E;
      g.ln_g = d->lnf_g; g.ln_b = d->lnf_b; g.ln_eps = d->ln_eps;
      g.w = d->lm_head_screen; g.N = V; g.K = E;
      g.part_val = w.pval; g.part_idx = w.pidx;
      g.hist = w.hist; g.hist_ld = max_new; g.gen_len = step; g.banned = w.banned; g.nbanned = w.nbanned;
      g.rep_penalty = gp->repetition_penalty; g.min_new = gp->min_new_tokens; g.eos = gp->eos_token_id;
      g.proc_out = w.proc; g.screen_h = w.sh;
      int tpb = 0;
      const hipError_t e = vcap_lm_head_screen_dispatch(g, &nblk, &tpb, s);
      if (e == hipSuccess) {
        const float rep = gp->repetition_penalty;
        const float pfac = rep >= 1.f ? rep : 1.f / rep;
        sc = ScreenArgs{w.proc, w.sh, (const float*)d->wte, d->screen_bound * pfac, tpb, rep, gp->min_new_tokens};
        screen = true;
      } else if (e != hipErrorNotSupported) {
        return hip_fail(e, "lm_head_screen");
      }
    }
    if (!screen) {
      if (int rc = run_lm_head(d, w, B, S_new, logits_out ? logits_out + (size_t)step * B * V : nullptr, max_new,
                               step, gp->repetition_penalty, gp->min_new_tokens, gp->eos_token_id, &nblk, s,
                               sp ? w.proc : nullptr))
        return rc;
    }
    if (sp) {
      SampleArgs sa{w.proc, V, V, sp->temperature, sp->top_k, sp->top_p, w.seed, step, force_ids, max_new,
                    warped_out ? warped_out + (size_t)step * B * V : nullptr, V, w.pval, w.pidx,
                    gp->eos_token_id};
      VCAP_TRY(vcap_sample_dispatch(sa, B, s), "sample");
      nblk = 1;
    }
    VCAP_TRY(vcap_decode_finalize_dispatch(dt, w.pval, w.pidx, nblk, B, step, w.finished, w.hist, max_new, w.banned,
                                           w.nbanned, gp->no_repeat_ngram_size, gp->eos_token_id, gp->pad_token_id,
                                           out_ids, max_new, d->wte, d->wpe, w.h, E,
                                           (S0 + step) < d->n_positions ? S0 + step : d->n_positions - 1, V, s,
                                           screen ? &sc : nullptr),
             "finalize");
  }
  return 0;
}

// ----------------------------------------------------------------------------------- graph cache
// Instantiated decode graphs, keyed on everything a replay bakes in (descriptor, parameters,
// buffer addresses, device).  A bounded LRU: a long-running server that hands the decoder new
// buffer addresses cannot grow it without limit.  Each entry remembers an event recorded after
// its latest launch, so an evicted graph is destroyed only once its last replay has finished.
struct GraphEntry {
  hipGraphExec_t exec = nullptr;
  hipEvent_t done = nullptr;
  std::list<std::string>::iterator lru;
};
std::mutex g_graph_mu;
std::unordered_map<std::string, GraphEntry> g_graphs;
std::list<std::string> g_graph_lru;  // front = most recently used
std::unordered_map<int, hipStream_t> g_capture_streams;

size_t graph_cache_cap() {
  static size_t cap = [] {
    const char* e = std::getenv("VCAP_GRAPH_CACHE_MAX");
    // serving sees one greedy + one beam graph per (batch size, prompt, workspace): 64 entries keep a
    // service whose coalesced batch sizes vary over 1..8 from re-capturing on every call
    long v = e ? std::strtol(e, nullptr, 10) : 64;
    return (size_t)(v < 1 ? 1 : v);
  }();
  return cap;
}

void graph_entry_destroy(GraphEntry& ge) {
  if (ge.done) {
    (void)hipEventSynchronize(ge.done);
    (void)hipEventDestroy(ge.done);
  }
  if (ge.exec) (void)hipGraphExecDestroy(ge.exec);
  ge.exec = nullptr;
  ge.done = nullptr;
}

// caller holds g_graph_mu: unlink the least recently used entries down to n and hand them back, so
// the caller destroys them (waiting for their last replay) after releasing the mutex - a wait under
// the lock would stall every decode on other threads / streams
std::vector<GraphEntry> graph_cache_evict_to(size_t n) {
  std::vector<GraphEntry> out;
  while (g_graphs.size() > n && !g_graph_lru.empty()) {
    auto it = g_graphs.find(g_graph_lru.back());
    g_graph_lru.pop_back();
    if (it == g_graphs.end()) continue;
    out.push_back(it->second);
    g_graphs.erase(it);
  }
  return out;
}

void graph_entries_destroy(std::vector<GraphEntry>& v) {
  for (auto& ge : v) graph_entry_destroy(ge);
  v.clear();
}

// evicted entries, destroyed when this goes out of scope (declared before the lock_guard, so
// after the mutex is released)
struct Evicted {
  std::vector<GraphEntry> v;
  ~Evicted() { graph_entries_destroy(v); }
};

// The descriptor's bytes up to its last field: vcap_gpt2_desc ends in a pointer + a float, so its
// 4 bytes of tail padding (whatever a C caller's stack held) stay out of the key; the int / float
// head is 8 x 4 bytes, so no interior padding precedes the pointers.
static_assert(offsetof(vcap_gpt2_desc, wte) == 8 * sizeof(int), "vcap_gpt2_desc: interior padding");
static_assert(sizeof(vcap_gpt2_layer) == 12 * sizeof(void*), "vcap_gpt2_layer: padding");
static_assert(sizeof(vcap_gen_params) == 8 * sizeof(int) && sizeof(vcap_beam_params) == 10 * sizeof(int),
              "vcap_gen_params / vcap_beam_params: padding");
static void put_gpt2_desc(std::string& k, const vcap_gpt2_desc* d) {
  k.append((const char*)d, offsetof(vcap_gpt2_desc, screen_bound) + sizeof(d->screen_bound));
  for (int l = 0; l < d->n_layer; ++l) k.append((const char*)&d->layers[l], sizeof(vcap_gpt2_layer));
}

std::string graph_key(const vcap_gpt2_desc* d, const vcap_gen_params* gp, const float* prefix, const int* ids,
                      int nids, int B, const int* out_ids, const float* logits, const void* ws) {
  std::string k;
  auto put = [&](const void* p, size_t n) { k.append((const char*)p, n); };
  put_gpt2_desc(k, d);
  put(gp, sizeof(*gp));
  put(&prefix, sizeof(prefix));
  put(ids, sizeof(int) * (size_t)nids);
  put(&nids, sizeof(nids));
  put(&B, sizeof(B));
  put(&out_ids, sizeof(out_ids));
  put(&logits, sizeof(logits));
  put(&ws, sizeof(ws));
  int dev = 0;
  (void)hipGetDevice(&dev);
  put(&dev, sizeof(dev));
  return k;
}

// Replay the graph cached under `key`, capturing `issue(capture_stream)` into it first if absent.
template <typename Issue>
int launch_cached(const std::string& key, hipStream_t s, Issue issue) {
  Evicted evicted;   // destroyed after the lock is released (declared first)
  std::lock_guard<std::mutex> lk(g_graph_mu);
  auto it = g_graphs.find(key);
  if (it == g_graphs.end()) {
    int dev = 0;
    VCAP_TRY(hipGetDevice(&dev), "hipGetDevice");
    hipStream_t cs = g_capture_streams[dev];
    if (!cs) {
      VCAP_TRY(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking), "hipStreamCreate");
      g_capture_streams[dev] = cs;
    }
    VCAP_TRY(hipStreamBeginCapture(cs, hipStreamCaptureModeThreadLocal), "hipStreamBeginCapture");
    int rc = issue(cs);
    hipGraph_t graph = nullptr;
    hipError_t ec = hipStreamEndCapture(cs, &graph);
    if (rc) {
      if (graph) (void)hipGraphDestroy(graph);
      return rc;
    }
    VCAP_TRY(ec, "hipStreamEndCapture");
    GraphEntry ge;
    hipError_t ei = hipGraphInstantiate(&ge.exec, graph, nullptr, nullptr, 0);
    (void)hipGraphDestroy(graph);
    VCAP_TRY(ei, "hipGraphInstantiate");
    if (hipError_t ee = hipEventCreateWithFlags(&ge.done, hipEventDisableTiming)) {
      (void)hipGraphExecDestroy(ge.exec);
      return hip_fail(ee, "hipEventCreate");
    }
    evicted.v = graph_cache_evict_to(graph_cache_cap() - 1);
    g_graph_lru.push_front(key);
    ge.lru = g_graph_lru.begin();
    it = g_graphs.emplace(key, ge).first;
  } else {
    g_graph_lru.splice(g_graph_lru.begin(), g_graph_lru, it->second.lru);
  }
  VCAP_TRY(hipGraphLaunch(it->second.exec, s), "hipGraphLaunch");
  VCAP_TRY(hipEventRecord(it->second.done, s), "hipEventRecord");
  return 0;
}

// ----------------------------------------------------------------------------------- beam search
struct BeamBufs {
  DecBufs w;
  int maxp;
  size_t page_elems;
  float* logits;
  float* part_max;
  float* part_sum;
  BeamState st;
  int nblk, chunks, anc_ld;
};

BeamBufs carve_beam(Carver& c, const vcap_gpt2_desc* d, int B, int nb, int S0, int L) {
  BeamBufs b;
  const int R = B * nb;
  b.w = carve_dec(c, d, R, S0, L, &b.maxp, &b.page_elems);
  b.nblk = max_logit_blocks(d->vocab, R);
  b.chunks = vcap_beam_chunks(d->vocab);
  b.anc_ld = S0 + L;
  b.logits = (float*)c.take((size_t)R * d->vocab * 4);
  b.part_max = (float*)c.take((size_t)R * b.nblk * 4);
  b.part_sum = (float*)c.take((size_t)R * b.nblk * 4);
  BeamState& st = b.st;
  const size_t RL = (size_t)R * L * 4;
  st.run_seq = (int*)c.take(RL);
  st.run_bidx = (int*)c.take(RL);
  st.seqs = (int*)c.take(RL);
  st.beam_idx = (int*)c.take(RL);
  st.run_score = (float*)c.take((size_t)R * 4);
  st.beam_score = (float*)c.take((size_t)R * 4);
  st.fin = (int*)c.take((size_t)R * 4);
  st.unsat = (int*)c.take((size_t)B * 4);
  st.stopped = (int*)c.take(4);
  st.tok_next = (int*)c.take((size_t)R * 4);
  st.anc = (int*)c.take((size_t)R * b.anc_ld * 4);
  st.cand_val = (float*)c.take((size_t)R * b.chunks * 2 * nb * 4);
  st.cand_tok = (int*)c.take((size_t)R * b.chunks * 2 * nb * 4);
  return b;
}

int issue_beam(const vcap_gpt2_desc* d, const vcap_beam_params* bp, const float* prefix, const int* ids, int nids,
               int B, int* out_ids, int* out_len, const BeamBufs& bb, hipStream_t s) {
  const int E = d->n_embd, nb = bp->num_beams, L = bp->max_new_tokens, R = B * nb;
  const int S0 = d->prefix_len + nids;
  const DecBufs& w = bb.w;
  int nblk = bb.nblk;  // log_softmax partials per row the lm_head leaves (<= bb.nblk)
  auto lm_head = [&](int S_new) -> int {
    RowsGemmArgs g;
    memset(&g, 0, sizeof(g));
    g.M = R; g.x = w.h + (size_t)(S_new - 1) * E; g.ldx = (long)S_new * E;
    g.ln_g = d->lnf_g; g.ln_b = d->lnf_b; g.ln_eps = d->ln_eps;
    g.w = d->lm_head; g.N = d->vocab; g.K = E;
    g.logits_raw = bb.logits; g.part_val = bb.part_max; g.part_sum = bb.part_sum; g.nblk = bb.nblk;
    g.max_blocks = bp->max_blocks;  // the streamed lm_head's grid (<= one workgroup per CU)
    nblk = bb.nblk;
    VCAP_TRY(vcap_rows_gemm_dispatch(d->dtype, PRO_LN, EPI_LSE, g, &nblk, s), "lm_head_lse");
    return 0;
  };
  VCAP_TRY(vcap_decode_init_dispatch(w.pt, R, bb.maxp, w.finished, w.nbanned, s, w.skc, w.n_skc), "decode_init");
  // prefill: every beam row gets its sequence's prompt (HF expands the input to B * num_beams)
  VCAP_TRY(vcap_prefill_embed_dispatch(d->dtype, prefix, d->prefix_len, ids, nids, d->wte, d->wpe, w.h, R, E, s, 0, nb),
           "prefill_embed");
  if (int rc = run_layers(d, w, bb.maxp, bb.page_elems, R * S0, S0, 0, 0, s)) return rc;
  if (int rc = lm_head(S0)) return rc;
  VCAP_TRY(vcap_beam_init_dispatch(bb.st, B, nb, L, S0, bb.anc_ld, bp->eos_token_id, s), "beam_init");
  for (int cur = 0; cur < L; ++cur) {
    if (cur > 0) {
      const int pos = S0 + cur - 1;
      VCAP_TRY(vcap_embed_tokens_dispatch(d->dtype, bb.st.tok_next, R, d->wte, d->wpe, w.h, E, pos, s), "embed");
      if (int rc = run_layers(d, w, bb.maxp, bb.page_elems, R, 1, pos, bp->max_blocks, s, bb.st.anc, bb.anc_ld))
        return rc;
      if (int rc = lm_head(1)) return rc;
    }
    VCAP_TRY(vcap_beam_cand_dispatch(bb.st, bb.logits, bb.part_max, bb.part_sum, nblk, R, d->vocab, nb, L, cur,
                                     bp->repetition_penalty, bp->no_repeat_ngram_size, bp->min_new_tokens,
                                     bp->eos_token_id, bb.chunks, s),
             "beam_cand");
    VCAP_TRY(vcap_beam_select_dispatch(bb.st, B, nb, L, d->vocab, bb.chunks, cur, bp->eos_token_id,
                                       bp->length_penalty, S0, bb.anc_ld, s),
             "beam_select");
  }
  VCAP_TRY(vcap_beam_output_dispatch(bb.st, B, nb, L, out_ids, out_len, s), "beam_output");
  return 0;
}

}  // namespace

// =====================================================================================================
extern "C" {

const char* vcap_last_error(void) { return g_err.c_str(); }
int vcap_abi_version(void) { return VCAP_ABI_VERSION; }

int vcap_stream_create_cu_reserved(int reserve_cus, void** stream) {
  if (!stream || reserve_cus < 0) return fail(VCAP_E_ARG, "vcap_stream_create_cu_reserved: bad arguments");
  int dev = 0;
  VCAP_TRY(hipGetDevice(&dev), "hipGetDevice");
  int ncu = 0;
  VCAP_TRY(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev), "cu count");
  if (reserve_cus >= ncu) return fail(VCAP_E_ARG, "cannot reserve every CU");
  // Clearing the first `reserve_cus` mask bits: with 32 cleared, the stream's workgroups still land on
  // all 8 XCCs and block id % 8 still picks one XCC, so the GEMMs' XCD-aware tile remap
  // holds (r02 per-workgroup stamps with 32 CUs reserved, profiles/r02_encode_alone.txt).
  std::vector<uint32_t> mask((ncu + 31) / 32, 0u);
  for (int c = reserve_cus; c < ncu; ++c) mask[c / 32] |= 1u << (c % 32);
  hipStream_t s = nullptr;
  VCAP_TRY(hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()), "hipExtStreamCreateWithCUMask");
  *stream = (void*)s;
  return 0;
}

int vcap_stream_create_cu_mask(const uint32_t* mask, int words, void** stream) {
  if (!stream || !mask || words <= 0) return fail(VCAP_E_ARG, "vcap_stream_create_cu_mask: bad arguments");
  hipStream_t s = nullptr;
  VCAP_TRY(hipExtStreamCreateWithCUMask(&s, (uint32_t)words, mask), "hipExtStreamCreateWithCUMask");
  *stream = (void*)s;
  return 0;
}

int vcap_stream_destroy(void* stream) {
  VCAP_TRY(hipStreamDestroy((hipStream_t)stream), "hipStreamDestroy");
  return 0;
}

int vcap_set_gemm_policy(int policy) {
  if (policy < 0 || policy > 2) return fail(VCAP_E_ARG, "gemm policy must be 0 (auto), 1 (128x128) or 2 (256x256)");
  vcap_gemm_set_policy(policy);
  return 0;
}

int vcap_gemm(int in_dtype, int out_dtype, const void* A, int64_t lda, const void* W, int64_t ldw, void* C,
              int64_t ldc, int M, int N, int K, const float* bias, int act, const float* res, int64_t ldr,
              int res_mode, int G, int Gs, int goff, int roff, void* stream) {
  if (!A || !W || !C || M <= 0 || N <= 0 || K <= 0) return fail(VCAP_E_ARG, "vcap_gemm: bad arguments");
  if (K % vcap_gemm_k_align(in_dtype)) return fail(VCAP_E_UNSUPPORTED, "vcap_gemm: K must be a multiple of the K step");
  if (res_mode && !res) return fail(VCAP_E_ARG, "vcap_gemm: residual pointer missing");
  if ((res_mode == 2 || G) && G <= 0) return fail(VCAP_E_ARG, "vcap_gemm: row group G must be > 0");
  if (res_mode && out_dtype != VCAP_DT_F32) return fail(VCAP_E_UNSUPPORTED, "vcap_gemm: residual needs f32 output");
  GemmEpi e{bias, res, (long)ldr, act, res_mode, G, Gs, goff, roff};
  g_err.clear();
  VCAP_TRY(vcap_gemm_dispatch(in_dtype, out_dtype, A, lda, W, ldw, C, ldc, M, N, K, e, (hipStream_t)stream),
           "vcap_gemm");
  return 0;
}

int vcap_linear_bias(int dtype, const void* x, const void* w, const float* b, void* y, int rows, int in_features,
                     int out_features, void* stream) {
  return vcap_gemm(dtype, dtype, x, in_features, w, in_features, y, out_features, rows, out_features, in_features, b,
                   0, nullptr, 0, 0, 0, 0, 0, 0, stream);
}

int vcap_layernorm(int out_dtype, const float* x, int64_t ldx, void* y, int64_t ldy, const float* gamma,
                   const float* beta, int rows, int dim, float eps, void* stream) {
  if (!x || !y || rows < 0 || dim <= 0) return fail(VCAP_E_ARG, "vcap_layernorm: bad arguments");
  if ((gamma == nullptr) != (beta == nullptr)) return fail(VCAP_E_ARG, "vcap_layernorm: gamma/beta mismatch");
  VCAP_TRY(vcap_layernorm_dispatch(out_dtype, x, (long)ldx, y, (long)ldy, gamma, beta, rows, dim, eps,
                                   (hipStream_t)stream),
           "vcap_layernorm");
  return 0;
}

size_t vcap_mx_scale_bytes(int rows, int K) {
  if (rows <= 0 || K <= 0 || K % 128) return 0;
  return mx_scale_bytes(rows, K);
}

int vcap_mx_quantize(int in_dtype, const void* x, int64_t ldx, int rows, int K, void* q, uint8_t* scales,
                     void* stream) {
  if (!x || !q || !scales || rows <= 0 || K <= 0 || ldx < K) return fail(VCAP_E_ARG, "vcap_mx_quantize: bad arguments");
  if (in_dtype != VCAP_DT_F32 && in_dtype != VCAP_DT_BF16) return fail(VCAP_E_ARG, "vcap_mx_quantize: in_dtype");
  if (K % 256) return fail(VCAP_E_UNSUPPORTED, "vcap_mx_quantize: K must be a multiple of 256");
  VCAP_TRY(vcap_mx_quantize_dispatch(in_dtype, x, (long)ldx, rows, K, (uint8_t*)q, scales, rows, (hipStream_t)stream),
           "vcap_mx_quantize");
  return 0;
}

int vcap_layernorm_mx(const float* x, int64_t ldx, void* q, uint8_t* scales, const float* gamma, const float* beta,
                      int rows, int dim, float eps, void* stream) {
  if (!x || !q || !scales || rows <= 0 || dim <= 0 || ldx < dim) return fail(VCAP_E_ARG, "vcap_layernorm_mx: bad arguments");
  if ((gamma == nullptr) != (beta == nullptr)) return fail(VCAP_E_ARG, "vcap_layernorm_mx: gamma/beta mismatch");
  if (dim % 256 || dim > 1024) return fail(VCAP_E_UNSUPPORTED, "vcap_layernorm_mx: dim must be 256, 512, 768 or 1024");
  VCAP_TRY(vcap_layernorm_mx_dispatch(x, (long)ldx, (uint8_t*)q, scales, rows, gamma, beta, rows, dim, eps,
                                      (hipStream_t)stream),
           "vcap_layernorm_mx");
  return 0;
}

int vcap_gemm_mx(const void* A, const uint8_t* a_scales, const void* W, const uint8_t* w_scales, int out_dtype,
                 void* C, int64_t ldc, uint8_t* c_scales, int M, int N, int K, const float* bias, int act,
                 const float* res, void* stream) {
  if (!A || !a_scales || !W || !w_scales || !C || M <= 0 || N <= 0 || K <= 0)
    return fail(VCAP_E_ARG, "vcap_gemm_mx: bad arguments");
  if (K % 256) return fail(VCAP_E_UNSUPPORTED, "vcap_gemm_mx: K must be a multiple of 256");
  if (N % 16 || ldc < N || ldc % 16) return fail(VCAP_E_UNSUPPORTED, "vcap_gemm_mx: N and ldc must be multiples of 16");
  if (out_dtype == VCAP_DT_MXFP8) {
    if (act != 1 || !bias || !c_scales || res || N % 128)
      return fail(VCAP_E_UNSUPPORTED, "vcap_gemm_mx: MXFP8 output needs bias + gelu (act=1), c_scales, N % 128 == 0");
    if (reinterpret_cast<uintptr_t>(c_scales) % 8)
      return fail(VCAP_E_ARG, "vcap_gemm_mx: c_scales must be 8-byte aligned");
  } else if (out_dtype != VCAP_DT_BF16 && out_dtype != VCAP_DT_F32) {
    return fail(VCAP_E_ARG, "vcap_gemm_mx: out_dtype");
  }
  if (res && out_dtype != VCAP_DT_F32) return fail(VCAP_E_UNSUPPORTED, "vcap_gemm_mx: residual needs f32 output");
  if (act < 0 || act > 1) return fail(VCAP_E_ARG, "vcap_gemm_mx: act must be 0 or 1");
  GemmEpi e{bias, res, (long)ldc, act, res ? 1 : 0, 0, 0, 0, 0, a_scales, w_scales, c_scales};
  g_err.clear();
  VCAP_TRY(vcap_gemm_dispatch(VCAP_DT_MXFP8, out_dtype, A, K, W, K, C, ldc, M, N, K, e, (hipStream_t)stream),
           "vcap_gemm_mx");
  return 0;
}

size_t vcap_frames_workspace_bytes(int n, int in_h, int in_w, int out_h, int out_w) {
  if (n <= 0 || in_h <= 0 || in_w <= 0 || out_h <= 0 || out_w <= 0) return 0;
  return vcap_frames_ws_bytes(n, in_h, in_w, out_h, out_w);
}

int vcap_frames_preprocess(const uint8_t* frames, int n, int in_h, int in_w, int out_h, int out_w, const float* mean3,
                           const float* std3, float* out, uint8_t* out_u8, void* workspace, size_t ws_bytes,
                           void* stream) {
  if (!frames || n <= 0 || in_h <= 0 || in_w <= 0 || out_h <= 0 || out_w <= 0 || !mean3 || !std3 || (!out && !out_u8))
    return fail(VCAP_E_ARG, "vcap_frames_preprocess: bad arguments");
  if (in_w > 31 * out_w || in_h > 31 * out_h)
    return fail(VCAP_E_UNSUPPORTED, "vcap_frames_preprocess: downscale factor above 31");
  if (ws_bytes < vcap_frames_ws_bytes(n, in_h, in_w, out_h, out_w))
    return fail(VCAP_E_WORKSPACE, "vcap_frames_preprocess: workspace too small");
  VCAP_TRY(vcap_frames_preprocess_dispatch(frames, n, in_h, in_w, out_h, out_w, mean3, std3, out, out_u8, workspace,
                                           (hipStream_t)stream),
           "vcap_frames_preprocess");
  return 0;
}

int vcap_jpeg_probe(const uint8_t* data, size_t len, int* width, int* height, int* comps) {
  if (!data || !len) return fail(VCAP_E_ARG, "vcap_jpeg_probe: bad arguments");
  JpegInfo f;
  std::string e;
  if (int rc = vcap_jpeg_header(data, len, &f, &e)) return fail(rc, "vcap_jpeg_probe: " + e);
  if (width) *width = f.width;
  if (height) *height = f.height;
  if (comps) *comps = f.ncomp;
  return 0;
}

size_t vcap_jpeg_workspace_bytes(const uint8_t* data, size_t len, int n) {
  JpegInfo f;
  std::string e;
  if (!data || !len || n <= 0 || vcap_jpeg_header(data, len, &f, &e)) return 0;
  return vcap_jpeg_ws_bytes(f, n);
}

int vcap_jpeg_decode_batch(const uint8_t* const* data, const size_t* lens, int n, uint8_t* out, void* workspace,
                           size_t ws_bytes, void* stream) {
  if (!data || !lens || n <= 0 || !out || !workspace) return fail(VCAP_E_ARG, "vcap_jpeg_decode_batch: bad arguments");
  for (int i = 0; i < n; ++i)
    if (!data[i] || !lens[i]) return fail(VCAP_E_ARG, "vcap_jpeg_decode_batch: empty image buffer");
  std::string e;
  if (int rc = vcap_jpeg_decode(data, lens, n, out, workspace, ws_bytes, (hipStream_t)stream, &e))
    return fail(rc, "vcap_jpeg_decode_batch: " + e);
  g_err.clear();
  return 0;
}

static int ensure_attn_lds() {
  if (attn_lds_configured) return 0;
  attn_lds_configured = true;
  return 0;
}

int vcap_vit_attention(int dtype, const void* qkv, void* out, int frames, int tokens, int heads, void* stream) {
  if (!qkv || !out || frames <= 0 || tokens <= 0 || heads <= 0) return fail(VCAP_E_ARG, "vcap_vit_attention: bad arguments");
  if (tokens > 288) return fail(VCAP_E_UNSUPPORTED, "vcap_vit_attention: tokens > 288");
  ensure_attn_lds();
  VCAP_TRY(vcap_vit_attention_dispatch(dtype, qkv, out, frames, tokens, heads, (hipStream_t)stream),
           "vcap_vit_attention");
  return 0;
}

int vcap_vit_qkv_attention(const void* xn, const void* wqkv, const float* bqkv, void* out, int frames, int tokens,
                           int heads, int cls_only, void* stream) {
  if (!xn || !wqkv || !bqkv || !out || frames <= 0 || tokens <= 0 || heads <= 0)
    return fail(VCAP_E_ARG, "vcap_vit_qkv_attention: bad arguments");
  if (!vcap_vit_qkv_attention_supported(VCAP_DT_BF16, tokens, heads))
    return fail(VCAP_E_UNSUPPORTED, "vcap_vit_qkv_attention: needs 192 < tokens <= 208 (ViT-B/16) or 256 < tokens <= 272 (ViT-L/14) "
                "and heads*64 <= 4096");
  VCAP_TRY(vcap_vit_qkv_attention_dispatch(xn, wqkv, bqkv, out, frames, tokens, heads, cls_only ? 1 : 0,
                                           (hipStream_t)stream),
           "vcap_vit_qkv_attention");
  return 0;
}

int vcap_vit_attention_mx(const void* qkv, void* out, uint8_t* out_scales, int frames, int tokens, int heads,
                          void* stream) {
  if (!qkv || !out || !out_scales || frames <= 0 || tokens <= 0 || heads <= 0)
    return fail(VCAP_E_ARG, "vcap_vit_attention_mx: bad arguments");
  if (tokens > 288) return fail(VCAP_E_UNSUPPORTED, "vcap_vit_attention_mx: tokens > 288");
  if ((heads * 64) % 256) return fail(VCAP_E_UNSUPPORTED, "vcap_vit_attention_mx: heads*64 must be a multiple of 256");
  VCAP_TRY(vcap_vit_attention_mx_dispatch(qkv, out, out_scales, frames, tokens, heads, (hipStream_t)stream),
           "vcap_vit_attention_mx");
  return 0;
}

int vcap_vit_pool_temporal(int dtype, const void* feat, void* out, int bsz, int timesteps, int tokens, int channels,
                           int pool_gap, void* stream) {
  if (!feat || !out || bsz <= 0 || timesteps <= 0 || tokens <= 0 || channels <= 0)
    return fail(VCAP_E_ARG, "vcap_vit_pool_temporal: bad arguments");
  if (pool_gap && tokens <= 1) return fail(VCAP_E_ARG, "vcap_vit_pool_temporal: gap needs tokens > 1");
  VCAP_TRY(vcap_vit_pool_dispatch(dtype, feat, out, bsz, timesteps, tokens, channels, pool_gap, (hipStream_t)stream),
           "vcap_vit_pool_temporal");
  return 0;
}

int vcap_prefix_project(const float* emb, int B, int video_dim, const vcap_prefix_desc* pd, float* prefix_out,
                        void* stream) {
  if (!emb || !pd || !prefix_out || !pd->mapper_w || B <= 0) return fail(VCAP_E_ARG, "vcap_prefix_project: bad arguments");
  if (video_dim > 1024) return fail(VCAP_E_UNSUPPORTED, "video_dim > 1024");
  VCAP_TRY(vcap_vit_head_prefix_dispatch(nullptr, B, 1, 1, 1, nullptr, nullptr, 0.f, nullptr, nullptr, video_dim,
                                         pd->ln_scale, pd->in_weight, pd->mapper_w, pd->mapper_b,
                                         pd->prefix_len * pd->n_embd, nullptr, prefix_out, emb, nullptr,
                                         (hipStream_t)stream),
           "vcap_prefix_project");
  return 0;
}

size_t vcap_vit_workspace_bytes(const vcap_vit_desc* d, int B, int T) {
  if (check_vit(d)) return 0;
  Carver c(nullptr);
  carve_vit(c, d, B, T);
  return c.off;
}

// block `ly` runs QKV + attention as one kernel: bf16 operands (neither QKV nor attn-proj in MXFP8) at a
// token count the fused kernel takes
static bool vit_layer_fused(const vcap_vit_desc* d, const vcap_vit_layer& ly) {
  const bool mx = d->dtype == VCAP_DT_MXFP8;
  const int g = d->image / d->patch;
  return !(mx && ly.qkv_ws) && !(mx && ly.proj_ws) && vcap_vit_qkv_attention_supported(vit_adt(d->dtype), g * g + 1, d->heads);
}

int vcap_vit_layer_fuses_qkv_attention(const vcap_vit_desc* d, int layer) {
  if (int rc = check_vit(d)) return rc;
  if (layer < 0 || layer >= d->depth) return fail(VCAP_E_ARG, "vcap_vit_layer_fuses_qkv_attention: layer out of range");
  return vit_layer_fused(d, d->layers[layer]) ? 1 : 0;
}

int vcap_vit_encode(const vcap_vit_desc* d, const vcap_prefix_desc* pd, const float* frames, int B, int T,
                    float* enc_out, float* prefix_out, void* workspace, size_t ws_bytes, void* stream) {
  if (int rc = check_vit(d)) return rc;
  if (!frames || !enc_out || B <= 0 || T <= 0) return fail(VCAP_E_ARG, "vcap_vit_encode: bad arguments");
  if (prefix_out && (!pd || !pd->mapper_w)) return fail(VCAP_E_ARG, "vcap_vit_encode: prefix desc missing");
  if (ws_bytes < vcap_vit_workspace_bytes(d, B, T)) return fail(VCAP_E_WORKSPACE, "vcap_vit_encode: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  Carver c(workspace);
  VitBufs w = carve_vit(c, d, B, T);
  const int dt = d->dtype, D = d->dim, g = d->image / d->patch, P = g * g, N = P + 1, BT = B * T;
  const int adt = vit_adt(dt);
  const bool mx = dt == VCAP_DT_MXFP8;
  const int M = BT * N;
  // patch embedding: im2col + GEMM whose epilogue adds bias + pos[1+p] and scatters row bt*N+1+p
  VCAP_TRY(vcap_patchify_dispatch(adt, frames, w.act, w.x, d->cls, d->pos, BT, d->image, d->patch, d->kpad, N, D, s),
           "patchify");
  GemmEpi pe{d->patch_b, d->pos, D, 0, 2, P, N, 1, 1};
  VCAP_TRY(vcap_gemm_dispatch(adt, VCAP_DT_F32, w.act, d->kpad, d->patch_w, d->kpad, w.x, D, BT * P, D, d->kpad, pe, s),
           "patch_gemm");
  for (int l = 0; l < d->depth; ++l) {
    const vcap_vit_layer& ly = d->layers[l];
    // The last block feeds only the class-token rows (final LN on CLS rows, CLS temporal pool:
    // video_encoder.py:256-258, pool="cls" at caption_model.py:45), so after its QKV projection
    // (K/V of every token are needed) it runs on the BT CLS rows only: CLS-query attention into a
    // compact [BT, D] buffer, then attn-proj / LN2 / fc1 / fc2 on BT rows with the residual rows
    // remapped to x[bt*N] (GemmEpi G = 1, Gs = N).  Outputs are identical; 6 % fewer FLOPs.
    const bool last = l == d->depth - 1;
    const int Mt = last ? BT : M;                       // rows after the QKV projection
    const char* probe_attn = last ? "vit.attention.cls" : "vit.attention";
    // MXFP8 mode, per GEMM (weight scales present): the producer of its A operand emits MXFP8
    const bool mq = mx && ly.qkv_ws, mp = mx && ly.proj_ws, m1 = mx && ly.fc1_ws, m2 = mx && ly.fc2_ws;
    const int dq = mq ? VCAP_DT_MXFP8 : adt, dp = mp ? VCAP_DT_MXFP8 : adt;
    const int d1 = m1 ? VCAP_DT_MXFP8 : adt, d2 = m2 ? VCAP_DT_MXFP8 : adt;
    if (mq)
      VCAP_TRY(vcap_layernorm_mx_dispatch(w.x, D, (uint8_t*)w.xn, w.xn_s, M, ly.ln1_g, ly.ln1_b, M, D, d->ln_eps, s),
               "norm1");
    else
      VCAP_TRY(vcap_layernorm_dispatch(adt, w.x, D, w.xn, D, ly.ln1_g, ly.ln1_b, M, D, d->ln_eps, s), "norm1");
    GemmEpi e1{ly.qkv_b, nullptr, 0, 0, 0, 0, 0, 0, 0, mq ? w.xn_s : nullptr, mq ? ly.qkv_ws : nullptr, nullptr};
    if (vit_layer_fused(d, ly)) {
      // QKV projection + attention in one kernel: q / k / v stay on chip
      ProbeScope ps(probe_attn, s, M);
      VCAP_TRY(vcap_vit_qkv_attention_dispatch(w.xn, ly.qkv_w, ly.qkv_b, w.attn, BT, N, d->heads, last, s),
               "qkv_attention");
    } else {
      {
        ProbeScope ps("vit.qkv", s, M);
        VCAP_TRY(vcap_gemm_dispatch(dq, adt, w.xn, D, ly.qkv_w, D, w.qkv, 3 * D, M, 3 * D, D, e1, s), "qkv");
      }
      ProbeScope ps(probe_attn, s, M);
      if (mp)
        VCAP_TRY(vcap_vit_attention_mx_dispatch(w.qkv, w.attn, w.xn_s, BT, N, d->heads, s, last), "attention");
      else
        VCAP_TRY(vcap_vit_attention_dispatch(adt, w.qkv, w.attn, BT, N, d->heads, s, last), "attention");
    }
    // MXFP8: the attention output arrives as MXFP8 (its scales reuse xn_s, free until norm2)
    GemmEpi e2{ly.proj_b, w.x, D, 0, 1, last ? 1 : 0, last ? N : 0, 0, 0, mp ? w.xn_s : nullptr,
               mp ? ly.proj_ws : nullptr, nullptr, last ? w.splitk : nullptr, w.splitk_bytes};
    {
      ProbeScope ps(last ? "vit.proj.cls" : "vit.proj", s, Mt);
      VCAP_TRY(vcap_gemm_dispatch(dp, VCAP_DT_F32, w.attn, D, ly.proj_w, D, w.x, D, Mt, D, D, e2, s), "attn_proj");
    }
    const long ldx2 = last ? (long)N * D : D;            // CLS rows of x are N*D apart
    if (m1)
      VCAP_TRY(vcap_layernorm_mx_dispatch(w.x, ldx2, (uint8_t*)w.xn, w.xn_s, Mt, ly.ln2_g, ly.ln2_b, Mt, D,
                                          d->ln_eps, s),
               "norm2");
    else
      VCAP_TRY(vcap_layernorm_dispatch(adt, w.x, ldx2, w.xn, D, ly.ln2_g, ly.ln2_b, Mt, D, d->ln_eps, s), "norm2");
    // fc1 emits MXFP8 straight from its epilogue when both MLP GEMMs are MXFP8; an MXFP8 fc2 after
    // a bf16 fc1 quantises the bf16 activation (vcap_mx_quantize) into the free qkv buffer
    const bool fused_q = m1 && m2;
    GemmEpi e3{ly.fc1_b, nullptr, 0, 1, 0, 0, 0, 0, 0, m1 ? w.xn_s : nullptr, m1 ? ly.fc1_ws : nullptr,
               fused_q ? w.act_s : nullptr};
    {
      ProbeScope ps(last ? "vit.fc1.cls" : "vit.fc1", s, Mt);
      VCAP_TRY(vcap_gemm_dispatch(d1, fused_q ? VCAP_DT_MXFP8 : adt, w.xn, D, ly.fc1_w, D, w.act, d->mlp, Mt, d->mlp,
                                  D, e3, s),
               "fc1");
    }
    const void* a2 = w.act;
    if (m2 && !fused_q) {
      VCAP_TRY(vcap_mx_quantize_dispatch(adt, w.act, d->mlp, Mt, d->mlp, (uint8_t*)w.qkv, w.act_s, Mt, s), "fc1 quant");
      a2 = w.qkv;
    }
    GemmEpi e4{ly.fc2_b, w.x, D, 0, 1, last ? 1 : 0, last ? N : 0, 0, 0, m2 ? w.act_s : nullptr,
               m2 ? ly.fc2_ws : nullptr, nullptr, last ? w.splitk : nullptr, w.splitk_bytes};
    {
      ProbeScope ps(last ? "vit.fc2.cls" : "vit.fc2", s, Mt);
      VCAP_TRY(vcap_gemm_dispatch(d2, VCAP_DT_F32, a2, d->mlp, ly.fc2_w, d->mlp, w.x, D, Mt, D, d->mlp, e4, s),
               "fc2");
    }
  }
  const float ls = pd ? pd->ln_scale : 0.f, iw = pd ? pd->in_weight : 0.f;
  const int MO = pd ? pd->prefix_len * pd->n_embd : 0;
  VCAP_TRY(vcap_vit_head_prefix_dispatch(w.x, B, T, N, D, d->norm_g, d->norm_b, d->ln_eps, d->proj_w, d->proj_b,
                                         d->video_dim, ls, iw, pd ? pd->mapper_w : nullptr,
                                         pd ? pd->mapper_b : nullptr, MO, enc_out, prefix_out, nullptr,
                                         (float*)w.xn, s),
           "head_prefix");
  return 0;
}

size_t vcap_rows_packed_bytes(int dtype, int N, int K) {
  if (dtype != VCAP_DT_F32 && dtype != VCAP_DT_BF16) return 0;
  if (N <= 0 || K <= 0 || K % (dtype == VCAP_DT_BF16 ? 32 : 16)) return 0;
  return vcap_rows_packed_size(dtype, N, K);
}

int vcap_rows_pack(int dtype, const void* w, int64_t ldw, int N, int K, void* packed, void* stream) {
  if (dtype != VCAP_DT_F32 && dtype != VCAP_DT_BF16) return fail(VCAP_E_ARG, "rows_pack dtype");
  if (!w || !packed || ldw < K) return fail(VCAP_E_ARG, "rows_pack: null pointer or ldw < K");
  VCAP_TRY(vcap_rows_pack_dispatch(dtype, w, (long)ldw, N, K, packed, (hipStream_t)stream),
           "rows_pack (K % 32/16, 16-byte aligned rows and pointers)");
  return 0;
}

size_t vcap_gpt2_workspace_bytes(const vcap_gpt2_desc* d, int B, int S0, int max_new_tokens) {
  if (check_gpt2(d)) return 0;
  Carver c(nullptr);
  int maxp;
  size_t pe;
  carve_dec(c, d, B, S0, max_new_tokens, &maxp, &pe);
  return c.off;
}

int vcap_gpt2_generate(const vcap_gpt2_desc* d, const vcap_gen_params* gp, const float* prefix, const int* prompt_ids,
                       int prompt_len, int B, int* out_ids, float* logits_out, void* workspace, size_t ws_bytes,
                       void* stream) {
  if (int rc = check_gpt2_launch(d)) return rc;
  if (!gp || !prefix || !out_ids || B <= 0 || prompt_len < 0 || prompt_len > 64 || (prompt_len && !prompt_ids))
    return fail(VCAP_E_ARG, "vcap_gpt2_generate: bad arguments");
  if (gp->max_new_tokens <= 0) return fail(VCAP_E_ARG, "max_new_tokens must be > 0");
  if (gp->max_new_tokens > 64)
    return fail(VCAP_E_UNSUPPORTED, "max_new_tokens > 64 (the lm_head stages the processors' history in LDS)");
  const int S0 = d->prefix_len + prompt_len;
  if (S0 <= 0 || B * S0 > kMaxDecodeRows)
    return fail(VCAP_E_UNSUPPORTED, "B*(prefix+prompt) exceeds vcap_gpt2_max_rows()");
  if (S0 + gp->max_new_tokens > d->n_positions || S0 + gp->max_new_tokens > 1024)
    return fail(VCAP_E_UNSUPPORTED, "context exceeds n_positions");
  for (int i = 0; i < prompt_len; ++i)
    if (prompt_ids[i] < 0 || prompt_ids[i] >= d->vocab) return fail(VCAP_E_ARG, "prompt id out of range");
  if (ws_bytes < vcap_gpt2_workspace_bytes(d, B, S0, gp->max_new_tokens))
    return fail(VCAP_E_WORKSPACE, "vcap_gpt2_generate: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  Carver c(workspace);
  int maxp;
  size_t page_elems;
  DecBufs w = carve_dec(c, d, B, S0, gp->max_new_tokens, &maxp, &page_elems);
  if (!gp->use_graph)
    return issue_decode(d, gp, prefix, prompt_ids, prompt_len, B, out_ids, logits_out, w, maxp, page_elems, s);

  const std::string key = graph_key(d, gp, prefix, prompt_ids, prompt_len, B, out_ids, logits_out, workspace);
  return launch_cached(key, s, [&](hipStream_t cs) {
    return issue_decode(d, gp, prefix, prompt_ids, prompt_len, B, out_ids, logits_out, w, maxp, page_elems, cs);
  });
}

int vcap_gpt2_sample(const vcap_gpt2_desc* d, const vcap_gen_params* gp, const vcap_sample_params* sp,
                     const float* prefix, const int* prompt_ids, int prompt_len, int B, int* out_ids,
                     float* logits_out, float* warped_out, const int* force_ids, void* workspace, size_t ws_bytes,
                     void* stream) {
  if (int rc = check_gpt2_launch(d)) return rc;
  if (!gp || !sp || !prefix || !out_ids || B <= 0 || prompt_len < 0 || prompt_len > 64 || (prompt_len && !prompt_ids))
    return fail(VCAP_E_ARG, "vcap_gpt2_sample: bad arguments");
  if (!(sp->temperature > 0.f) || !(sp->top_p > 0.0) || sp->top_p > 1.0 || sp->top_k < 1)
    return fail(VCAP_E_ARG, "vcap_gpt2_sample: needs temperature > 0, 0 < top_p <= 1, top_k >= 1");
  if (sp->top_k > vcap_sample_max_top_k() || d->vocab > 50 * 1024)
    return fail(VCAP_E_UNSUPPORTED, "vcap_gpt2_sample: top_k <= 128 and vocab <= 51200");
  if (gp->max_new_tokens <= 0 || gp->max_new_tokens > 64)
    return fail(VCAP_E_UNSUPPORTED, "max_new_tokens must be in 1..64");
  const int S0 = d->prefix_len + prompt_len;
  if (B * S0 > kMaxDecodeRows) return fail(VCAP_E_UNSUPPORTED, "B*(prefix+prompt) exceeds vcap_gpt2_max_rows()");
  if (S0 + gp->max_new_tokens > d->n_positions) return fail(VCAP_E_UNSUPPORTED, "context exceeds n_positions");
  for (int i = 0; i < prompt_len; ++i)
    if (prompt_ids[i] < 0 || prompt_ids[i] >= d->vocab) return fail(VCAP_E_ARG, "prompt id out of range");
  if (ws_bytes < vcap_gpt2_workspace_bytes(d, B, S0, gp->max_new_tokens))
    return fail(VCAP_E_WORKSPACE, "vcap_gpt2_sample: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  Carver c(workspace);
  int maxp;
  size_t page_elems;
  DecBufs w = carve_dec(c, d, B, S0, gp->max_new_tokens, &maxp, &page_elems);
  // the Philox key goes to device memory outside the graph: one captured graph serves every seed
  VCAP_TRY(hipMemsetD32Async((hipDeviceptr_t)w.seed, (int)(uint32_t)sp->seed, 1, s), "seed lo");
  VCAP_TRY(hipMemsetD32Async((hipDeviceptr_t)(w.seed + 1), (int)(uint32_t)(sp->seed >> 32), 1, s), "seed hi");
  if (!gp->use_graph)
    return issue_decode(d, gp, prefix, prompt_ids, prompt_len, B, out_ids, logits_out, w, maxp, page_elems, s, sp,
                        warped_out, force_ids);
  std::string key = graph_key(d, gp, prefix, prompt_ids, prompt_len, B, out_ids, logits_out, workspace);
  vcap_sample_params ks = *sp;
  ks.seed = 0;
  key.append("sample");
  key.append((const char*)&ks, sizeof(ks));
  key.append((const char*)&warped_out, sizeof(warped_out));
  key.append((const char*)&force_ids, sizeof(force_ids));
  return launch_cached(key, s, [&](hipStream_t cs) {
    return issue_decode(d, gp, prefix, prompt_ids, prompt_len, B, out_ids, logits_out, w, maxp, page_elems, cs, sp,
                        warped_out, force_ids);
  });
}

int vcap_probe_enable(const char* site, int max_launches) {
  if (!site || max_launches <= 0) return fail(VCAP_E_ARG, "vcap_probe_enable: bad arguments");
  std::lock_guard<std::mutex> lk(g_probe_mu);
  Probe& p = g_probes[site];
  while ((int)p.start.size() < max_launches) {
    hipEvent_t a, b;
    VCAP_TRY(hipEventCreate(&a), "hipEventCreate");
    VCAP_TRY(hipEventCreate(&b), "hipEventCreate");
    p.start.push_back(a);
    p.stop.push_back(b);
    p.rows.push_back(0);
  }
  p.used = 0;
  p.on = true;
  return 0;
}

int vcap_probe_read_launches(const char* site, float* ms, int* rows, int cap, int* launches) {
  if (!site || !launches || cap < 0 || (cap > 0 && (!ms || !rows)))
    return fail(VCAP_E_ARG, "vcap_probe_read_launches: bad arguments");
  std::lock_guard<std::mutex> lk(g_probe_mu);
  auto it = g_probes.find(site);
  *launches = 0;
  if (it == g_probes.end()) return 0;
  Probe& p = it->second;
  if (p.used > cap) return fail(VCAP_E_ARG, "vcap_probe_read_launches: more launches than cap");
  for (int i = 0; i < p.used; ++i) {
    VCAP_TRY(hipEventSynchronize(p.stop[i]), "hipEventSynchronize");
    VCAP_TRY(hipEventElapsedTime(&ms[i], p.start[i], p.stop[i]), "hipEventElapsedTime");
    rows[i] = p.rows[i];
  }
  *launches = p.used;
  p.on = false;
  p.used = 0;
  return 0;
}

int vcap_probe_read(const char* site, float* total_ms, int* launches) {
  if (!site || !total_ms || !launches) return fail(VCAP_E_ARG, "vcap_probe_read: bad arguments");
  std::lock_guard<std::mutex> lk(g_probe_mu);
  auto it = g_probes.find(site);
  *total_ms = 0.f;
  *launches = 0;
  if (it == g_probes.end()) return 0;
  Probe& p = it->second;
  for (int i = 0; i < p.used; ++i) {
    VCAP_TRY(hipEventSynchronize(p.stop[i]), "hipEventSynchronize");
    float ms = 0.f;
    VCAP_TRY(hipEventElapsedTime(&ms, p.start[i], p.stop[i]), "hipEventElapsedTime");
    *total_ms += ms;
  }
  *launches = p.used;
  p.on = false;
  p.used = 0;
  return 0;
}

size_t vcap_gpt2_beam_workspace_bytes(const vcap_gpt2_desc* d, int rows, int S0, int max_new_tokens) {
  if (check_gpt2(d)) return 0;
  Carver c(nullptr);
  int maxp;
  size_t pe;
  carve_dec(c, d, rows, S0, max_new_tokens, &maxp, &pe);
  c.take(pe * d->n_layer * esize(d->dtype));  // reorder scratch (one pool at a time)
  return c.off;
}

static int step_setup(const vcap_gpt2_desc* d, int rows, int S0, int max_new, void* ws, size_t ws_bytes, DecBufs* w,
                      int* maxp, size_t* pe, void** scratch) {
  if (int rc = check_gpt2_launch(d)) return rc;
  if (rows <= 0 || rows > kMaxDecodeRows || S0 <= 0 || max_new <= 0 || S0 + max_new > d->n_positions)
    return fail(VCAP_E_ARG, "gpt2 step: bad rows / lengths");
  if (ws_bytes < vcap_gpt2_beam_workspace_bytes(d, rows, S0, max_new))
    return fail(VCAP_E_WORKSPACE, "gpt2 step: workspace too small (vcap_gpt2_beam_workspace_bytes)");
  Carver c(ws);
  *w = carve_dec(c, d, rows, S0, max_new, maxp, pe);
  *scratch = c.take(*pe * d->n_layer * esize(d->dtype));
  return 0;
}

int vcap_gpt2_prefill(const vcap_gpt2_desc* d, const float* prefix, const int* prompt_ids, int prompt_len, int B,
                      int rows, int max_new_tokens, float* logits_out, void* workspace, size_t ws_bytes,
                      void* stream) {
  const int S0 = d ? d->prefix_len + prompt_len : 0;
  if (!prefix || !logits_out || B <= 0 || B > rows || prompt_len < 0 || prompt_len > 64 || (prompt_len && !prompt_ids))
    return fail(VCAP_E_ARG, "vcap_gpt2_prefill: bad arguments");
  if (B * S0 > kMaxDecodeRows) return fail(VCAP_E_UNSUPPORTED, "B*(prefix+prompt) exceeds vcap_gpt2_max_rows()");
  DecBufs w;
  int maxp;
  size_t pe;
  void* scratch;
  if (int rc = step_setup(d, rows, S0, max_new_tokens, workspace, ws_bytes, &w, &maxp, &pe, &scratch)) return rc;
  hipStream_t s = (hipStream_t)stream;
  VCAP_TRY(vcap_decode_init_dispatch(w.pt, rows, maxp, w.finished, w.nbanned, s, w.skc, w.n_skc), "decode_init");
  VCAP_TRY(vcap_prefill_embed_dispatch(d->dtype, prefix, d->prefix_len, prompt_ids, prompt_len, d->wte, d->wpe, w.h, B,
                                       d->n_embd, s),
           "prefill_embed");
  if (int rc = run_layers(d, w, maxp, pe, B * S0, S0, 0, 0, s)) return rc;
  int nblk;
  return run_lm_head(d, w, B, S0, logits_out, 1, 0, 1.0f, 0, -1, &nblk, s);
}

int vcap_gpt2_step(const vcap_gpt2_desc* d, const int* tokens, int rows, int S0, int max_new_tokens, int pos,
                   float* logits_out, void* workspace, size_t ws_bytes, void* stream) {
  if (!tokens || !logits_out || pos < S0 || pos >= S0 + max_new_tokens)
    return fail(VCAP_E_ARG, "vcap_gpt2_step: bad arguments (S0 <= pos < S0 + max_new_tokens)");
  DecBufs w;
  int maxp;
  size_t pe;
  void* scratch;
  if (int rc = step_setup(d, rows, S0, max_new_tokens, workspace, ws_bytes, &w, &maxp, &pe, &scratch)) return rc;
  hipStream_t s = (hipStream_t)stream;
  VCAP_TRY(vcap_embed_tokens_dispatch(d->dtype, tokens, rows, d->wte, d->wpe, w.h, d->n_embd, pos, s), "embed_tokens");
  if (int rc = run_layers(d, w, maxp, pe, rows, 1, pos, 0, s)) return rc;
  int nblk;
  return run_lm_head(d, w, rows, 1, logits_out, 1, 0, 1.0f, 0, -1, &nblk, s);
}

int vcap_gpt2_forward_embeds(const vcap_gpt2_desc* d, const float* embeds, int rows, int n_tok, int past_len, int S0,
                             int max_new_tokens, float* logits_out, void* workspace, size_t ws_bytes, void* stream) {
  if (!embeds || !logits_out || rows <= 0) return fail(VCAP_E_ARG, "vcap_gpt2_forward_embeds: bad arguments");
  if (past_len == 0 ? n_tok != S0 : (n_tok != 1 || past_len < S0 || past_len >= S0 + max_new_tokens))
    return fail(VCAP_E_ARG, "vcap_gpt2_forward_embeds: prefill needs n_tok == S0; a step one token at "
                            "S0 <= past_len < S0 + max_new_tokens");
  if (past_len == 0 && rows * S0 > kMaxDecodeRows)
    return fail(VCAP_E_UNSUPPORTED, "rows*S0 exceeds vcap_gpt2_max_rows() at prefill");
  DecBufs w;
  int maxp;
  size_t pe;
  void* scratch;
  if (int rc = step_setup(d, rows, S0, max_new_tokens, workspace, ws_bytes, &w, &maxp, &pe, &scratch)) return rc;
  hipStream_t s = (hipStream_t)stream;
  if (past_len == 0) VCAP_TRY(vcap_decode_init_dispatch(w.pt, rows, maxp, w.finished, w.nbanned, s, w.skc, w.n_skc), "decode_init");
  // the prefill-embedding kernel with every position taken from `embeds` (P = n_tok, no prompt ids)
  VCAP_TRY(vcap_prefill_embed_dispatch(d->dtype, embeds, n_tok, nullptr, 0, d->wte, d->wpe, w.h, rows, d->n_embd, s,
                                       past_len),
           "embed_inputs");
  if (int rc = run_layers(d, w, maxp, pe, rows * n_tok, n_tok, past_len, 0, s)) return rc;
  int nblk;
  return run_lm_head(d, w, rows, n_tok, logits_out, 1, 0, 1.0f, 0, -1, &nblk, s);
}

int vcap_gpt2_reorder(const vcap_gpt2_desc* d, const int* src_rows, int rows, int S0, int max_new_tokens, int length,
                      void* workspace, size_t ws_bytes, void* stream) {
  if (!src_rows || length <= 0) return fail(VCAP_E_ARG, "vcap_gpt2_reorder: bad arguments");
  DecBufs w;
  int maxp;
  size_t pe;
  void* scratch;
  if (int rc = step_setup(d, rows, S0, max_new_tokens, workspace, ws_bytes, &w, &maxp, &pe, &scratch)) return rc;
  hipStream_t s = (hipStream_t)stream;
  const size_t bytes = pe * d->n_layer * esize(d->dtype);
  for (void* pool : {w.kc, w.vc}) {
    VCAP_TRY(vcap_kv_gather_dispatch(d->dtype, pool, scratch, src_rows, rows, maxp, d->n_head, length, (long)pe,
                                     d->n_layer, s),
             "kv_gather");
    VCAP_TRY(hipMemcpyAsync(pool, scratch, bytes, hipMemcpyDeviceToDevice, s), "kv copy-back");
  }
  return 0;
}

int vcap_decode_attention(int dtype, const void* q, const void* k_pool, const void* v_pool, const int* page_table,
                          int maxp, void* out, int M, int heads, int S_new, int past, void* stream) {
  if (!q || !k_pool || !v_pool || !out || M <= 0 || heads <= 0 || S_new <= 0 || past < 0 || maxp <= 0 ||
      M % S_new)
    return fail(VCAP_E_ARG, "vcap_decode_attention: bad arguments");
  if (dtype != VCAP_DT_F32 && dtype != VCAP_DT_BF16) return fail(VCAP_E_ARG, "vcap_decode_attention: dtype");
  if (past + S_new > 16 * maxp) return fail(VCAP_E_ARG, "vcap_decode_attention: context exceeds the page table");
  if (!page_table && (dtype != VCAP_DT_BF16 || past + S_new > 64))
    return fail(VCAP_E_UNSUPPORTED, "vcap_decode_attention: a NULL page table needs bf16 and context <= 64");
  VCAP_TRY(vcap_decode_attention_dispatch(dtype, q, k_pool, v_pool, page_table, maxp, out, M, heads, S_new, past,
                                          (hipStream_t)stream),
           "vcap_decode_attention");
  return 0;
}


void vcap_graph_cache_clear(void) {
  std::vector<GraphEntry> evicted;
  {
    std::lock_guard<std::mutex> lk(g_graph_mu);
    evicted = graph_cache_evict_to(0);
    g_graphs.clear();
    g_graph_lru.clear();
  }
  graph_entries_destroy(evicted);
}

int vcap_gpt2_max_rows(void) { return kMaxDecodeRows; }

size_t vcap_gpt2_beam_search_workspace_bytes(const vcap_gpt2_desc* d, int B, int num_beams, int S0,
                                             int max_new_tokens) {
  if (check_gpt2(d) || B <= 0 || num_beams <= 0) return 0;
  Carver c(nullptr);
  carve_beam(c, d, B, num_beams, S0, max_new_tokens);
  return c.off;
}

int vcap_gpt2_beam_search(const vcap_gpt2_desc* d, const vcap_beam_params* bp, const float* prefix,
                          const int* prompt_ids, int prompt_len, int B, int* out_ids, int* out_len, void* workspace,
                          size_t ws_bytes, void* stream) {
  if (int rc = check_gpt2_launch(d)) return rc;
  if (!bp || !prefix || !out_ids || !out_len || B <= 0 || prompt_len < 0 || prompt_len > 64 ||
      (prompt_len && !prompt_ids))
    return fail(VCAP_E_ARG, "vcap_gpt2_beam_search: bad arguments");
  const int nb = bp->num_beams, L = bp->max_new_tokens, S0 = d->prefix_len + prompt_len;
  if (nb < 2 || nb > 8 || B > 8 || L <= 0 || L > 64 || S0 + L > 128 || S0 + L > d->n_positions)
    return fail(VCAP_E_UNSUPPORTED, "vcap_gpt2_beam_search: needs 2 <= num_beams <= 8, B <= 8, max_new <= 64, "
                                    "prefix + prompt + max_new <= 128");
  if (B * nb * S0 > kMaxDecodeRows) return fail(VCAP_E_UNSUPPORTED, "B*num_beams*(prefix+prompt) exceeds max rows");
  if (bp->early_stopping != 0) return fail(VCAP_E_UNSUPPORTED, "only early_stopping=False (the reference's presets)");
  if (bp->max_blocks < 0) return fail(VCAP_E_ARG, "vcap_gpt2_beam_search: max_blocks < 0");
  if (nb * vcap_beam_chunks(d->vocab) * 2 * nb > 20 * 64)
    return fail(VCAP_E_UNSUPPORTED, "num_beams too large for the vocabulary (candidate registers)");
  for (int i = 0; i < prompt_len; ++i)
    if (prompt_ids[i] < 0 || prompt_ids[i] >= d->vocab) return fail(VCAP_E_ARG, "prompt id out of range");
  if (ws_bytes < vcap_gpt2_beam_search_workspace_bytes(d, B, nb, S0, L))
    return fail(VCAP_E_WORKSPACE, "vcap_gpt2_beam_search: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  Carver c(workspace);
  BeamBufs bb = carve_beam(c, d, B, nb, S0, L);
  if (!bp->use_graph) return issue_beam(d, bp, prefix, prompt_ids, prompt_len, B, out_ids, out_len, bb, s);
  std::string key = "beam";
  auto put = [&](const void* p, size_t n) { key.append((const char*)p, n); };
  put_gpt2_desc(key, d);
  put(bp, sizeof(*bp));
  put(&prefix, sizeof(prefix));
  put(prompt_ids, sizeof(int) * (size_t)prompt_len);
  put(&prompt_len, sizeof(prompt_len));
  put(&B, sizeof(B));
  put(&out_ids, sizeof(out_ids));
  put(&out_len, sizeof(out_len));
  put(&workspace, sizeof(workspace));
  int dev = 0;
  (void)hipGetDevice(&dev);
  put(&dev, sizeof(dev));
  return launch_cached(key, s, [&](hipStream_t cs) {
    return issue_beam(d, bp, prefix, prompt_ids, prompt_len, B, out_ids, out_len, bb, cs);
  });
}

int vcap_graph_cache_size(void) {
  std::lock_guard<std::mutex> lk(g_graph_mu);
  return (int)g_graphs.size();
}

}  // extern "C"
