// Kernel-side interface shared by the .hip translation units and the host runtime.
#pragma once
#include <hip/hip_runtime.h>

#include <string>

struct GemmEpi {
  const float* bias;  // [N] or nullptr
  const float* res;   // residual source (f32) or nullptr
  long ldr;           // residual row stride (elements)
  int act;            // 0 none, 1 gelu_tanh
  int res_mode;       // 0 none, 1 residual row == output row (may alias C), 2 row (m % G) + roff
  int G, Gs, goff;    // output row remap: G ? (m/G)*Gs + goff + m%G : m
  int roff;
  // MXFP8 operands (in_dt == VCAP_DT_MXFP8): E8M0 block scales of A and W, K-tile-major
  // (vcap_common.h); c_scale receives the scales of an MXFP8 output (act must be gelu).
  const uint8_t* a_scale;
  const uint8_t* w_scale;
  uint8_t* c_scale;
  // deterministic split-K (few-tile in-place residual GEMMs, bf16 operands): f32 partial slabs
  // [split][M][N]; the partials are summed in split order by a second kernel.  nullptr: no split.
  float* splitk_ws;
  size_t splitk_bytes;
  // 256x256 kernel tile order (set by its dispatcher): 0 = row-major over (row panel, column tile);
  // w > 0 = column groups of w tile columns, row-major inside a group
  int colgroup;
};

enum { PRO_LN = 0, PRO_DIRECT = 1 };
// EPI_LSE: raw logits -> logits_raw + per-workgroup (max, sum exp(x - max)) partials per row
// (part_val / part_sum): the log_softmax statistics of beam search
enum { EPI_QKV = 0, EPI_RESID = 1, EPI_GELU = 2, EPI_LOGITS = 3, EPI_STORE = 4, EPI_LSE = 5 };

struct RowsGemmArgs {
  const void* x;  // PRO_LN: f32 residual rows; PRO_DIRECT: T rows
  long ldx;
  const float* ln_g;
  const float* ln_b;
  float ln_eps;
  const void* w;  // rows-packed T weights of a [N, K] matrix (vcap_rows_pack_dispatch)
  const float* bias;
  int M, N, K;
  void* out;  // RESID: f32 [M, ldo] (+=); GELU/STORE: T [M, ldo]
  long ldo;
  // QKV scatter into the paged cache
  void* q_out;            // T [M, E]
  void* kc;               // T pool: [pages][H][16][64] for this layer
  void* vc;
  const int* page_table;  // [seq][maxp]
  int maxp, H, S_new, past;
  // logits: processors + per-workgroup argmax partials
  float* logits_raw;  // optional [M, N] raw logits
  float* part_val;
  int* part_idx;
  float* part_sum;  // EPI_LSE
  int nblk;
  const int* hist;  // [M][hist_ld] generated tokens
  int hist_ld, gen_len;
  const int* banned;  // [M][hist_ld]
  const int* nbanned;
  float rep_penalty;
  int min_new, eos;
  int max_blocks;  // 0: one 16-column tile per workgroup; > 0: widen tiles to stay near this grid
  float* proc_out;  // EPI_LOGITS, optional [M, N]: the processed scores (sampling mode)
  int half;         // set by vcap_rows_gemm_dispatch: residual GEMV tiles split into two 8-column workgroups
  float* screen_h;  // lm_head stream kernel, optional [M, K] f32: workgroup 0 stores the ln_f rows it used
  // f32 K-split residual GEMV (vcap_rows_gemv8_kernel<float, NSL, true>): per (row chunk, tile) two
  // workgroups take one K half each; the pair meets through sk_part (2 x 256 f32 partials) and the
  // arrival ticket sk_cnt (zeroed by vcap_decode_init at the start of every decode)
  float* sk_part;
  int* sk_cnt;
};

// Exact-fp32 greedy token from a bf16 lm_head screen (f32 decoders; vcap_decode_finalize_dispatch):
// the bf16 stream kernel left the processed approximate scores in `proc` [B][vocab], its argmax
// partials per block of `tpb` 16-column tiles, and the f32 ln_f rows in `sh` [B][E].  Every token
// whose exact f32 processed score could reach the approximate maximum's lower bound (|approx - exact|
// <= coef * ||h||, coef = c * max_v ||w_v|| * max(rep, 1 / rep)) is rescored against the f32 `w32`
// rows; the argmax of the exact scores (value, then lowest index) is the token.
struct ScreenArgs {
  const float* proc;
  const float* sh;
  const float* w32;
  float coef;
  int tpb;
  float rep;
  int min_new;
};

// ---- sampling warpers + draw (csrc/sample.hip)
struct SampleArgs {
  const float* proc;  // [rows][ldp] processed scores (processors applied)
  int V, ldp;
  float temperature;
  int top_k;
  double top_p;
  const unsigned* seed;  // device [2]: Philox key
  int step;
  const int* force;      // optional [rows][force_ld]: emit these tokens instead of drawing (tests)
  int force_ld;
  float* warped;         // optional [rows][warped_ld]: the warped scores HF's _sample draws from
  long warped_ld;
  float* pval;           // [rows]: the token as the finalize kernel's only argmax partial
  int* pidx;
  int eos;               // emitted for a row with no finite processed score (NaN / all -inf logits)
};
hipError_t vcap_sample_dispatch(const SampleArgs& a, int rows, hipStream_t s);
int vcap_sample_max_top_k();

hipError_t vcap_gemm_dispatch(int in_dt, int out_dt, const void* A, long lda, const void* W, long ldw, void* C,
                              long ldc, int M, int N, int K, const GemmEpi& epi, hipStream_t s);
int vcap_gemm_k_align(int in_dt);
// CUs a launch on stream s may use (its CU mask, else the device's CU count)
int vcap_stream_cus(hipStream_t s);
// CUs of the current device (launch plans that must not depend on a stream's CU mask)
int vcap_device_cus();
bool vcap_gemm256_ok(int in_dt, int out_dt, long lda, long ldw, long ldc, int M, int N, int K, const GemmEpi& epi);
hipError_t vcap_gemm256_dispatch(int in_dt, int out_dt, const void* A, long lda, const void* W, long ldw, void* C,
                                 long ldc, int M, int N, int K, const GemmEpi& epi, hipStream_t s);
void vcap_gemm_set_policy(int p);
hipError_t vcap_layernorm_mx_dispatch(const float* x, long ldx, uint8_t* q, uint8_t* scales, int srows,
                                      const float* gamma, const float* beta, int rows, int D, float eps,
                                      hipStream_t s);
hipError_t vcap_mx_quantize_dispatch(int in_dt, const void* x, long ldx, int rows, int K, uint8_t* q,
                                     uint8_t* scales, int srows, hipStream_t s);
hipError_t vcap_layernorm_dispatch(int out_dt, const float* x, long ldx, void* y, long ldy, const float* gamma,
                                   const float* beta, int rows, int D, float eps, hipStream_t s);
// cls_only: only the class-token query of each (frame, head), written to compact row `frame`
hipError_t vcap_vit_attention_dispatch(int dt, const void* qkv, void* out, int BT, int N, int H, hipStream_t s,
                                       int cls_only = 0);
// fused QKV projection + attention (bf16, 192 < N <= 208 or 256 < N <= 272): xn [BT*N, H*64] LayerNorm output, wqkv
// [3*H*64, H*64], bqkv [3*H*64] -> out as vcap_vit_attention_dispatch's
bool vcap_vit_qkv_attention_supported(int dt, int N, int H);
hipError_t vcap_vit_qkv_attention_dispatch(const void* xn, const void* wqkv, const float* bqkv, void* out, int BT,
                                           int N, int H, int cls_only, hipStream_t s);
hipError_t vcap_vit_attention_mx_dispatch(const void* qkv, void* out, uint8_t* oscale, int BT, int N, int H,
                                          hipStream_t s, int cls_only = 0);
hipError_t vcap_patchify_dispatch(int dt, const float* frames, void* patches, float* x, const float* cls,
                                  const float* pos, int BT, int img, int p, int Kp, int N, int D, hipStream_t s);
hipError_t vcap_vit_head_prefix_dispatch(const float* x, int B, int T, int N, int D, const float* ng, const float* nb,
                                         float neps, const float* pw, const float* pb, int VD, float ln_scale,
                                         float in_weight, const float* mw, const float* mb, int MO, float* enc_out,
                                         float* prefix, const float* emb_in, float* emb_scratch, hipStream_t s);
hipError_t vcap_vit_pool_dispatch(int dt, const void* x, void* y, int B, int T, int tokens, int C, int gap,
                                  hipStream_t s);
hipError_t vcap_rows_gemm_dispatch(int dt, int pro, int epi, const RowsGemmArgs& a, int* nblk_out, hipStream_t s);
hipError_t vcap_rows_pack_dispatch(int dt, const void* w, long ldw, int N, int K, void* packed, hipStream_t s);
size_t vcap_rows_packed_size(int dt, int N, int K);
int vcap_logit_blocks(int V, int M);
hipError_t vcap_decode_attention_dispatch(int dt, const void* q, const void* kc, const void* vc, const int* pt,
                                          int maxp, void* out, int M, int H, int S_new, int past, hipStream_t s);
hipError_t vcap_prefill_embed_dispatch(int dt, const float* prefix, int P, const int* ids, int nids, const void* wte,
                                       const float* wpe, float* h, int B, int E, hipStream_t s, int pos0 = 0,
                                       int prefix_rep = 1);
hipError_t vcap_decode_init_dispatch(int* page_table, int B, int maxp, int* finished, int* nbanned, hipStream_t s,
                                     int* sk_cnt = nullptr, int n_sk = 0);
hipError_t vcap_decode_finalize_dispatch(int dt, const float* part_val, const int* part_idx, int nblk, int B,
                                         int step, int* finished, int* hist, int hist_ld, int* banned, int* nbanned,
                                         int ngram, int eos, int pad, int* out_ids, int out_ld, const void* wte,
                                         const float* wpe, float* h, int E, int pos_next, int vocab, hipStream_t s,
                                         const ScreenArgs* screen = nullptr);
// The bf16 lm_head as the screen of an f32 greedy step (the stream kernel only: M <= 16); returns
// hipErrorNotSupported, launching nothing, where that kernel does not apply.
hipError_t vcap_lm_head_screen_dispatch(const RowsGemmArgs& a, int* nblk_out, int* tpb_out, hipStream_t s);
hipError_t vcap_embed_tokens_dispatch(int dt, const int* tok, int rows, const void* wte, const float* wpe, float* h,
                                      int E, int pos, hipStream_t s);
// ---- device beam search (csrc/beam.hip) ----
struct BeamState {  // per-call device state, carved from the caller's workspace (B batches, nb beams, L = max_new)
  int* run_seq;      // [B][nb][L] running hypotheses' tokens
  float* run_score;  // [B][nb]
  int* run_bidx;     // [B][nb][L] beam indices (HF running_beam_indices)
  int* seqs;         // [B][nb][L] finished hypotheses (EOS-initialised)
  float* beam_score; // [B][nb] (-1e9 initialised)
  int* beam_idx;     // [B][nb][L] (-1 initialised)
  int* fin;          // [B][nb]
  int* unsat;        // [B]
  int* stopped;      // [1] HF's loop has ended (no further updates)
  int* tok_next;     // [B*nb] next input tokens
  int* anc;          // [B*nb][anc_ld] physical row holding each position's K/V
  float* cand_val;   // [B*nb][C][2nb]
  int* cand_tok;
};
hipError_t vcap_beam_init_dispatch(const BeamState& st, int B, int nb, int L, int S0, int anc_ld, int eos,
                                   hipStream_t s);
hipError_t vcap_beam_cand_dispatch(const BeamState& st, const float* logits, const float* part_max,
                                   const float* part_sum, int nblk, int rows, int V, int nb, int L, int cur,
                                   float rep, int ngram, int min_new, int eos, int chunks, hipStream_t s);
hipError_t vcap_beam_select_dispatch(const BeamState& st, int B, int nb, int L, int V, int chunks, int cur, int eos,
                                     float length_penalty, int S0, int anc_ld, hipStream_t s);
hipError_t vcap_beam_output_dispatch(const BeamState& st, int B, int nb, int L, int* out_ids, int* out_len,
                                     hipStream_t s);
int vcap_beam_chunks(int V);
// causal decode attention (one query row per sequence) whose key j of row m lives in physical
// row anc[m * anc_ld + j] of the contiguous-page pools (beam search: no KV copies on reorder)
hipError_t vcap_decode_attention_anc_dispatch(int dt, const void* q, const void* kc, const void* vc, const int* anc,
                                              int anc_ld, int maxp, void* out, int M, int H, int past,
                                              hipStream_t s);

hipError_t vcap_kv_gather_dispatch(int dt, const void* src_pool, void* dst_pool, const int* src_rows, int rows, int maxp,
                                   int H, int len, long layer_elems, int L, hipStream_t s);
size_t vcap_frames_ws_bytes(int n, int in_h, int in_w, int out_h, int out_w);
hipError_t vcap_frames_preprocess_dispatch(const uint8_t* frames, int n, int in_h, int in_w, int out_h, int out_w,
                                           const float* mean3, const float* std3, float* out, uint8_t* out_u8,
                                           void* ws, hipStream_t s);

// JPEG frame decode (jpeg.hip): header of one baseline image, workspace of n same-shape images,
// host entropy decode + device IDCT / upsampling / colour conversion into uint8 [n, H, W, 3].
struct JpegInfo {
  int width = 0, height = 0, ncomp = 0, hmax = 1, vmax = 1;
  int id[3] = {0, 0, 0}, h[3] = {1, 1, 1}, v[3] = {1, 1, 1};
  int bx[3] = {0, 0, 0}, by[3] = {0, 0, 0};  // block grid per component, padded to whole MCUs
};
int vcap_jpeg_header(const uint8_t* data, size_t len, JpegInfo* info, std::string* err);
size_t vcap_jpeg_ws_bytes(const JpegInfo& f, int n);
int vcap_jpeg_decode(const uint8_t* const* data, const size_t* lens, int n, uint8_t* out, void* ws, size_t ws_bytes,
                     hipStream_t s, std::string* err);
