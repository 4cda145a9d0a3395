/*
 * vcap.h - C ABI of the MI355X-native video-caption hot path (libvcap_hip.so).
 *
 * Plain pointers and sizes only: device pointers are HIP device addresses, `stream` is a
 * hipStream_t passed as void*.  Every entry point returns 0 on success or a negative code
 * (-hipError_t, or VCAP_E_* for argument errors) and sets a thread-local message readable
 * with vcap_last_error().  Nothing allocates device memory behind the caller's back: the
 * caller owns the workspace (size from the *_workspace_bytes queries); nothing synchronises
 * the stream.
 *
 * Reference interfaces each entry point replaces (paths relative to the reference repo):
 *   vcap_linear_bias        core/operators/cupy_linear_mapper.py:14-70 (linear_bias_f32/_f16 CUDA-C)
 *                           and CuPyLinearCompat.forward :137-184 (nn.Linear drop-in)
 *   vcap_vit_pool_temporal  core/operators/cupy_vit_pool.py:23-104 (vit_pool_{cls,gap}_{f32,f16}),
 *                           vit_fused_pool_temporal :127-186
 *   vcap_prefix_project     core/operators/normalization.py:6-13 apply_prefix_norm + the decoder
 *                           mapper (src/models/text_decoder.py:249), i.e. core/engine.py:44-50 -> :60-74
 *   vcap_gemm / vcap_layernorm / vcap_vit_attention / vcap_gemm_mx / vcap_layernorm_mx
 *                           the timm ViT block arithmetic the reference drives through
 *                           src/models/video_encoder.py:112-174 (fused SDPA, tanh-GELU MLP,
 *                           in-place residual) - op-level entry points for the plugin registry
 *                           (core/operators/trt_plugin_hooks.py:7-34)
 *   vcap_frames_preprocess  core/preprocessing/frame_loader.py:34-45 (Resize -> ToTensor -> Normalize)
 *   vcap_vit_encode         ViTFrameEncoder.forward (src/models/video_encoder.py:288-326) fused with
 *                           the engine prefix (core/engine.py:43-50) and the mapper
 *   vcap_gpt2_generate      GPT2TextDecoder.generate (src/models/text_decoder.py:105-146) ->
 *                           GPT2LMHeadModel.generate greedy with RepetitionPenalty / NoRepeatNGram /
 *                           MinNewTokens, and the raw greedy loop of
 *                           core/scripts/benchmark_baseline.py:160-240 (processors disabled)
 */
#ifndef VCAP_H_
#define VCAP_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VCAP_ABI_VERSION 15

/* VCAP_DT_MXFP8: OCP e4m3fn elements + one E8M0 scale per 32 consecutive K elements of a row
 * (the gfx950 block-scaled MFMA format; BASELINE configs[4]).  Scale arrays use the GEMM's
 * staging order: per (128-wide K-tile, group of 256 rows) one 1 KiB block laid out
 * [k-block 0..3][row % 16][row / 16] - byte offset
 *   ((k/128 * ceil(rows/256) + row/256) * 4 + (k%128)/32) * 256 + (row%16) * 16 + (row%256)/16,
 * size vcap_mx_scale_bytes(rows, K).  Element value = e4m3 * 2^(scale - 127). */
enum { VCAP_DT_F32 = 0, VCAP_DT_BF16 = 1, VCAP_DT_MXFP8 = 2 };
enum { VCAP_E_ARG = -1000, VCAP_E_WORKSPACE = -1001, VCAP_E_UNSUPPORTED = -1002 };

typedef struct vcap_vit_layer {
  const float* ln1_g; const float* ln1_b;
  const void* qkv_w; const float* qkv_b;     /* [3D, D] */
  const void* proj_w; const float* proj_b;   /* [D, D]  */
  const float* ln2_g; const float* ln2_b;
  const void* fc1_w; const float* fc1_b;     /* [4D, D] */
  const void* fc2_w; const float* fc2_b;     /* [D, 4D] */
  /* dtype VCAP_DT_MXFP8 only: qkv_w / proj_w / fc1_w / fc2_w are e4m3 and these their E8M0
   * scales (vcap_mx_quantize); the patch-embed weight stays bf16 */
  const uint8_t* qkv_ws; const uint8_t* proj_ws; const uint8_t* fc1_ws; const uint8_t* fc2_ws;
} vcap_vit_layer;

typedef struct vcap_vit_desc {
  int dtype;                 /* operand dtype of the block GEMMs (VCAP_DT_*; MXFP8: QKV / attn-proj /
                                fc1 / fc2 in MXFP8 with LayerNorm, attention and GELU emitting MXFP8
                                operands; patch-embed and the QK^T / PV products in bf16) */
  int dim, depth, heads, patch, image, mlp, video_dim;
  int kpad;                  /* patch K (3*p*p) padded to the GEMM K step */
  float ln_eps;              /* 1e-6 (timm) */
  const void* patch_w;       /* [dim, kpad] */
  const float* patch_b;      /* [dim] */
  const float* cls;          /* [dim] */
  const float* pos;          /* [tokens, dim] */
  const float* norm_g; const float* norm_b;
  const float* proj_w;       /* encoder.proj [video_dim, dim] f32 */
  const float* proj_b;
  const vcap_vit_layer* layers;  /* host array of `depth` entries */
} vcap_vit_desc;

typedef struct vcap_prefix_desc {
  float ln_scale;            /* <=0 disables the layer_norm*ln_scale step (core/engine.py:47) */
  float in_weight;           /* <=0 disables the *in_weight step (core/engine.py:49) */
  int prefix_len, n_embd;
  const float* mapper_w;     /* [prefix_len*n_embd, video_dim] f32 */
  const float* mapper_b;
} vcap_prefix_desc;

/* GPT-2 projection weights are passed ROWS-PACKED: the torch Linear-layout [N, K] matrix
 * (Conv1D weights transposed) rearranged by vcap_rows_pack() into MFMA-fragment order, so each
 * decode weight load is one contiguous 1 KiB wave instruction (layout in csrc/decode.hip). */
typedef struct vcap_gpt2_layer {
  const float* ln1_g; const float* ln1_b;
  const void* attn_w; const float* attn_b;   /* packed [3E, E] (c_attn Conv1D transposed) */
  const void* aproj_w; const float* aproj_b; /* packed [E, E] */
  const float* ln2_g; const float* ln2_b;
  const void* fc_w; const float* fc_b;       /* packed [4E, E] */
  const void* mproj_w; const float* mproj_b; /* packed [E, 4E] */
} vcap_gpt2_layer;

typedef struct vcap_gpt2_desc {
  int dtype;
  int n_embd, n_layer, n_head, vocab, n_positions, prefix_len;
  float ln_eps;              /* 1e-5 */
  const void* wte;           /* [vocab, E] token embedding (plain layout, row gathers) */
  const void* lm_head;       /* packed [vocab, E]: the tied lm_head = vcap_rows_pack(wte) */
  const float* wpe;          /* [n_positions, E] f32 */
  const float* lnf_g; const float* lnf_b;
  const vcap_gpt2_layer* layers; /* host array of n_layer entries */
  /* f32 decoders, optional (NULL / 0 disable): a bf16 rows-packed copy of the lm_head and
   * screen_bound = c * max_v ||w_v||_2 with c >= 2u + u^2 + 4 * 1024 * 2^-24 = 8.07e-3 (u = 2^-8, the
   * bf16 unit roundoff of EACH of h and w; the two f32 dot products over n_embd <= 1024, doubled
   * for a truncating accumulator; vcap/model.py uses c = 0.0082).  The runtime scales the bound by
   * max(rep, 1/rep) while a repetition penalty is active.  A greedy step without requested logits then runs the
   * lm_head in bf16 as a screen and rescores, in f32 against wte, every token whose exact score
   * could reach the screen's maximum: the token is the exact f32 argmax (processors applied, ties
   * to the lowest id) at half the lm_head's weight bytes. */
  const void* lm_head_screen;
  float screen_bound;
} vcap_gpt2_desc;

typedef struct vcap_gen_params {
  int max_new_tokens;
  int min_new_tokens;        /* 0 for raw greedy */
  int no_repeat_ngram_size;  /* 0 disables */
  float repetition_penalty;  /* 1.0 disables */
  int eos_token_id, pad_token_id;
  int use_graph;             /* capture the whole decode into a hipGraph and replay it */
  int max_blocks;            /* 0: whole-chip grids; > 0: cap the projection GEMV grids near this
                                many workgroups (wider tiles per workgroup) - for a decode that
                                shares the GPU with an encode holding most CUs */
} vcap_gen_params;

const char* vcap_last_error(void);
int vcap_abi_version(void);

/* ---- tuning: which ViT GEMM kernel vcap_gemm / vcap_vit_encode use (process-wide):
 *      0 auto (256x256-tile kernel when the shape yields >= 512 tiles), 1 128x128 only,
 *      2 256x256 wherever its shape constraints hold.  Results are identical up to fp32
 *      summation order within a tile (both accumulate K in the same order). ---- */
int vcap_set_gemm_policy(int policy);

/* ---- a stream whose kernels avoid `reserve_cus` CUs (hipExtStreamCreateWithCUMask), so a
 *      latency-bound chain on another stream (the decode graph) always finds free CUs while
 *      the MFMA-bound encode fills the rest.  Destroy with vcap_stream_destroy. ---- */
int vcap_stream_create_cu_reserved(int reserve_cus, void** stream);
int vcap_stream_create_cu_mask(const uint32_t* mask, int words, void** stream);  /* raw CU bit mask */
int vcap_stream_destroy(void* stream);

/* ---- op-level entry points ---- */
int vcap_linear_bias(int dtype, const void* x, const void* w, const float* b, void* y, int rows, int in_features,
                     int out_features, void* stream);
int vcap_gemm(int in_dtype, int out_dtype, const void* A, int64_t lda, const void* W, int64_t ldw, void* C,
              int64_t ldc, int M, int N, int K, const float* bias, int act, const float* res, int64_t ldr,
              int res_mode, int G, int Gs, int goff, int roff, void* stream);
int vcap_layernorm(int out_dtype, const float* x, int64_t ldx, void* y, int64_t ldy, const float* gamma,
                   const float* beta, int rows, int dim, float eps, void* stream);
int vcap_vit_attention(int dtype, const void* qkv, void* out, int frames, int tokens, int heads, void* stream);
/* Fused QKV projection + attention (bf16; 192 < tokens <= 208 or 256 < tokens <= 272, i.e. ViT-B/16
 * and ViT-L/14 frames): xn
 * [frames*tokens, heads*64] bf16 (the LayerNorm output), wqkv [3*heads*64, heads*64] bf16, bqkv
 * [3*heads*64] f32 -> out [frames*tokens, heads*64] bf16 (cls_only: [frames, heads*64], the class
 * token's row).  Bit-identical to vcap_gemm (bias, bf16 out) into a qkv buffer followed by
 * vcap_vit_attention; q / k / v stay on chip.  Replaces timm Attention.qkv + the attention core
 * (src/models/video_encoder.py:112-121).  VCAP_E_UNSUPPORTED outside that shape. */
int vcap_vit_qkv_attention(const void* xn, const void* wqkv, const float* bqkv, void* out, int frames, int tokens,
                           int heads, int cls_only, void* stream);

/* ---- frame preprocessing (core/preprocessing/frame_loader.py:34-45: torchvision Resize((S, S)) on
 *      PIL images -> ToTensor -> Normalize): decoded RGB frames uint8 [n, in_h, in_w, 3] (device)
 *      -> out f32 [n, 3, out_h, out_w] (normalised) and/or out_u8 [n, out_h, out_w, 3] (the resized
 *      pixels), bit-identical to PIL Image.resize(BILINEAR) + the f32 /255, -mean, /std chain.
 *      mean3 / std3 are HOST arrays of 3 floats.  Downscale factors up to 31. ---- */
size_t vcap_frames_workspace_bytes(int n, int in_h, int in_w, int out_h, int out_w);
int vcap_frames_preprocess(const uint8_t* frames, int n, int in_h, int in_w, int out_h, int out_w, const float* mean3,
                           const float* std3, float* out, uint8_t* out_u8, void* workspace, size_t ws_bytes,
                           void* stream);

/* ---- JPEG frame decode (core/preprocessing/frame_loader.py:42-44: PIL Image.open(path).convert("RGB"),
 *      i.e. libjpeg-turbo's default decompression) for baseline sequential Huffman JPEGs: 8-bit, 1 or
 *      3 components in one interleaved scan, 4:4:4 / 4:2:2 / 4:2:0, restart markers.  The host
 *      parses and entropy-decodes (parallel threads, one image each); the device dequantises and runs
 *      jpeg_idct_islow, fancy-upsamples chroma and converts YCbCr -> RGB with libjpeg's fixed-point
 *      arithmetic, bit-identical to Pillow.  Progressive / arithmetic-coded / 12-bit / CMYK images ->
 *      VCAP_E_UNSUPPORTED, and so are RGB-coded JPEGs (libjpeg's colour-space rule: no JFIF marker and
 *      an Adobe transform of 0, or component ids 'R','G','B').  vcap_jpeg_decode_batch: n images (HOST
 *      byte buffers) that share size and chroma sampling (each image keeps its own quantisation and
 *      Huffman tables, as ffmpeg's per-frame MJPEG qscale writes them) -> out uint8 [n, H, W, 3]
 *      (device); returns after the device work of the call has finished, on every path (the host
 *      coefficient staging is released). ---- */
int vcap_jpeg_probe(const uint8_t* data, size_t len, int* width, int* height, int* comps);
size_t vcap_jpeg_workspace_bytes(const uint8_t* data, size_t len, int n);
int vcap_jpeg_decode_batch(const uint8_t* const* data, const size_t* lens, int n, uint8_t* out, void* workspace,
                           size_t ws_bytes, void* stream);

/* ---- MXFP8 (BASELINE configs[4]: fp8 MFMA path for the ViT GEMMs) ----
 * vcap_mx_quantize: rows of f32 / bf16 [rows, K] (row stride ldx) -> e4m3 [rows, K] + scales.
 * vcap_layernorm_mx: LayerNorm (f32 rows) fused with the quantisation of its output.
 * vcap_gemm_mx: C = epi(A . W^T) with A [M, K], W [N, K] MXFP8 (contiguous rows, K % 256 == 0);
 *   out_dtype BF16 / F32 (res != NULL: C += ..., in place, f32) or MXFP8 (act must be 1 = bias +
 *   GELU-tanh, C e4m3 [M, N] + c_scales (8-byte aligned, vcap_mx_scale_bytes(M, N) bytes: the
 *   padding rows of the last 256-row group are written too), N % 128 == 0). */
size_t vcap_mx_scale_bytes(int rows, int K);
/* bf16 qkv [frames*tokens, 3*heads*64] -> attention output in MXFP8 ([frames*tokens, heads*64] e4m3 +
 * scales), the A operand of an MXFP8 attn-proj GEMM */
int vcap_vit_attention_mx(const void* qkv, void* out, uint8_t* out_scales, int frames, int tokens, int heads,
                          void* stream);
int vcap_mx_quantize(int in_dtype, const void* x, int64_t ldx, int rows, int K, void* q, uint8_t* scales,
                     void* stream);
int vcap_layernorm_mx(const float* x, int64_t ldx, void* q, uint8_t* scales, const float* gamma, const float* beta,
                      int rows, int dim, float eps, void* stream);
int vcap_gemm_mx(const void* A, const uint8_t* a_scales, const void* W, const uint8_t* w_scales, int out_dtype,
                 void* C, int64_t ldc, uint8_t* c_scales, int M, int N, int K, const float* bias, int act,
                 const float* res, void* stream);
int vcap_vit_pool_temporal(int dtype, const void* feat, void* out, int bsz, int timesteps, int tokens, int channels,
                           int pool_gap, void* stream);
int vcap_prefix_project(const float* emb, int B, int video_dim, const vcap_prefix_desc* pd, float* prefix_out,
                        void* stream);

/* ---- weight layout for the GPT-2 decoder (one-time, at model load) ----
 * vcap_rows_packed_bytes: bytes of the packed copy of a [N, K] matrix (N rounded up to 16).
 * vcap_rows_pack: w [N, K] row stride ldw (elements, 16-byte aligned rows) -> packed.
 * K must be a multiple of 32 (bf16) / 16 (f32); the decoder needs n_embd % 128 == 0. */
size_t vcap_rows_packed_bytes(int dtype, int N, int K);
int vcap_rows_pack(int dtype, const void* w, int64_t ldw, int N, int K, void* packed, void* stream);

/* ---- fused paths ---- */
size_t vcap_vit_workspace_bytes(const vcap_vit_desc* d, int B, int T);
int vcap_vit_encode(const vcap_vit_desc* d, const vcap_prefix_desc* pd, const float* frames, int B, int T,
                    float* enc_out, float* prefix_out, void* workspace, size_t ws_bytes, void* stream);
/* ABI v15: 1 when vcap_vit_encode runs block `layer`'s QKV projection and attention as the fused
 * vcap_vit_qkv_attention kernel, 0 when as a QKV GEMM + attention kernel (fp32 operands, MXFP8 QKV /
 * attn-proj, other token counts), < 0 on a bad descriptor / layer.  The same predicate the encode
 * uses, for callers that attribute FLOPs and bytes per kernel (bench.py). */
int vcap_vit_layer_fuses_qkv_attention(const vcap_vit_desc* d, int layer);

size_t vcap_gpt2_workspace_bytes(const vcap_gpt2_desc* d, int B, int S0, int max_new_tokens);
int vcap_gpt2_generate(const vcap_gpt2_desc* d, const vcap_gen_params* gp, const float* prefix, const int* prompt_ids,
                       int prompt_len, int B, int* out_ids, float* logits_out, void* workspace, size_t ws_bytes,
                       void* stream);
/* ---- sampling presets (core/inference.py:12-15 natural / safe_sample; HF _sample as
 *      text_decoder.py:131-144 reaches it with do_sample = num_beams == 1 and temperature != 1):
 *      the greedy decode's processors, then TemperatureLogitsWarper -> TopKLogitsWarper(top_k) ->
 *      TopPLogitsWarper(top_p) -> one multinomial draw per row and step from a counter-based
 *      Philox4x32-10 stream keyed on `seed` (csrc/sample.hip).  The same hipGraph serves every seed.
 *      warped_out (optional, [max_new][B][vocab] f32): the warped scores each draw used (-inf where
 *      removed), i.e. HF's output_scores; force_ids (optional, [B][max_new]): emit these tokens
 *      instead of drawing (tests replay a recorded history).  Parity with the reference is
 *      distributional: the RNG streams differ. ---- */
typedef struct vcap_sample_params {
  float temperature;  /* > 0 */
  int top_k;          /* HF generation-config default 50; 1..128 */
  double top_p;       /* (0, 1] */
  uint64_t seed;
} vcap_sample_params;
int vcap_gpt2_sample(const vcap_gpt2_desc* d, const vcap_gen_params* gp, const vcap_sample_params* sp,
                     const float* prefix, const int* prompt_ids, int prompt_len, int B, int* out_ids,
                     float* logits_out, float* warped_out, const int* force_ids, void* workspace, size_t ws_bytes,
                     void* stream);
void vcap_graph_cache_clear(void);
/* number of instantiated decode graphs held by the cache (bounded LRU, VCAP_GRAPH_CACHE_MAX) */
int vcap_graph_cache_size(void);
/* decoder rows one call may carry: B * (prefix + prompt) at the prefill, B * num_beams per step */
int vcap_gpt2_max_rows(void);

/* ---- causal decode attention over the paged KV cache (one GPT-2 layer; HF GPT2Attention's
 *      sdpa path at decode time, text_decoder.py:131-144 -> modeling_gpt2): q [M, H*64] (M = seqs *
 *      S_new rows), pools [pages][H][16][64], page_table [seqs][maxp] or NULL for the contiguous
 *      layout (page of position j of sequence s = s*maxp + j/16), out [M, H*64].  Row m attends
 *      to positions 0 .. past + (m % S_new) of its sequence. ---- */
int vcap_decode_attention(int dtype, const void* q, const void* k_pool, const void* v_pool, const int* page_table,
                          int maxp, void* out, int M, int heads, int S_new, int past, void* stream);

/* ---- device beam search (HF `_beam_search` as text_decoder.py:131-144 reaches it for the
 *      `precise` / `detailed` presets: log_softmax -> RepetitionPenalty -> NoRepeatNGram ->
 *      MinNewTokens -> + beam scores -> top-2*num_beams, length_penalty, early_stopping=False).
 *      The whole search (prefill + max_new steps + bookkeeping) is one call, replayed as one
 *      hipGraph; out_ids [B, max_new] = each sequence's best finished hypothesis (EOS-padded),
 *      out_len [B] = its generated length (HF returns the first max(out_len) columns).
 *      Limits: B <= 8 sequences, 2 <= num_beams <= 8, max_new <= 64, prefix+prompt+max_new <= 128. ---- */
typedef struct vcap_beam_params {
  int num_beams;
  int max_new_tokens;
  int min_new_tokens;
  int no_repeat_ngram_size;
  float repetition_penalty;
  float length_penalty;
  int early_stopping;  /* only 0 (False) */
  int eos_token_id;
  int use_graph;
  int max_blocks;      /* ABI v14: as vcap_gen_params.max_blocks - 0: whole-chip grids; > 0: cap each step's
                          projection GEMV grids and the beam lm_head's grid near this many workgroups */
} vcap_beam_params;
size_t vcap_gpt2_beam_search_workspace_bytes(const vcap_gpt2_desc* d, int B, int num_beams, int S0,
                                             int max_new_tokens);
int vcap_gpt2_beam_search(const vcap_gpt2_desc* d, const vcap_beam_params* bp, const float* prefix,
                          const int* prompt_ids, int prompt_len, int B, int* out_ids, int* out_len, void* workspace,
                          size_t ws_bytes, void* stream);

/* ---- step-wise decode for host-driven search (beam search / sampling).  One state carved for
 *      `rows` decoder rows lives in the caller's workspace across calls:
 *        prefill  B <= rows sequences into rows [0, B), logits of each last position -> [B, vocab]
 *        step     feed one token per row at position `pos` (S0 <= pos < S0+max_new) -> [rows, vocab]
 *        reorder  row r <- row src_rows[r] for cache positions [0, length)   (beam reordering,
 *                 also the B -> B*num_beams expansion after prefill) ---- */
size_t vcap_gpt2_beam_workspace_bytes(const vcap_gpt2_desc* d, int rows, int S0, int max_new_tokens);
int vcap_gpt2_prefill(const vcap_gpt2_desc* d, const float* prefix, const int* prompt_ids, int prompt_len, int B,
                      int rows, int max_new_tokens, float* logits_out, void* workspace, size_t ws_bytes, void* stream);
int vcap_gpt2_step(const vcap_gpt2_desc* d, const int* tokens, int rows, int S0, int max_new_tokens, int pos,
                   float* logits_out, void* workspace, size_t ws_bytes, void* stream);
int vcap_gpt2_reorder(const vcap_gpt2_desc* d, const int* src_rows, int rows, int S0, int max_new_tokens, int length,
                      void* workspace, size_t ws_bytes, void* stream);
/* ---- the same state driven by input EMBEDDINGS (HF `GPT2LMHeadModel(inputs_embeds=...,
 *      past_key_values=..., use_cache=True)` as core/scripts/benchmark_baseline.py:160-240 calls
 *      it through `model.decoder.model`): past_len == 0 -> prefill of n_tok == S0 positions
 *      (rows sequences, embeds [rows, S0, E] f32); past_len > 0 -> one position (n_tok == 1,
 *      embeds [rows, 1, E]) at S0 <= past_len < S0 + max_new_tokens.  h = embeds + wpe[pos];
 *      logits of each row's last position -> [rows, vocab] f32.  Same workspace as above. ---- */
int vcap_gpt2_forward_embeds(const vcap_gpt2_desc* d, const float* embeds, int rows, int n_tok, int past_len, int S0,
                             int max_new_tokens, float* logits_out, void* workspace, size_t ws_bytes, void* stream);

/* ---- live kernel timing for the benchmark's roofline (sites: "vit.qkv", "vit.attention",
 *      "vit.proj", "vit.fc1", "vit.fc2"): events are recorded around each launch of the site on
 *      the caller's stream, without synchronising; vcap_probe_read waits for them. ---- */
int vcap_probe_enable(const char* site, int max_launches);
int vcap_probe_read(const char* site, float* total_ms, int* launches);
/* Per-launch form: ms[i] / rows[i] (the launch's GEMM or attention rows) for each of the *launches
 * (<= cap) recorded launches; like vcap_probe_read it disables the site. */
int vcap_probe_read_launches(const char* site, float* ms, int* rows, int cap, int* launches);

#ifdef __cplusplus
}
#endif
#endif /* VCAP_H_ */
