// ViT prologue/epilogue kernels around the block GEMMs.
//
//  * vcap_patchify: frames [BT,3,H,W] f32 -> im2col patches [BT*P, Kp] (T, zero K-pad) feeding the
//    patch-embed GEMM (timm PatchEmbed Conv2d(3,D,p,stride p), called at
//    src/models/video_encoder.py:195), and the class-token rows x[bt,0,:] = cls + pos[0]
//    (timm _pos_embed).  The GEMM epilogue adds bias + pos[1+p] and scatters rows bt*N+1+p.
//  * vcap_vit_head_prefix: the fused tail of the encoder + engine prefix:
//    final LayerNorm on CLS rows only (the only rows consumed) -> mean over T
//    (video_encoder.py:256-258) -> encoder.proj Linear D->256 (:316) -> optional
//    layer_norm(no affine)*ln_scale*in_weight (core/engine.py:44-50) -> mapper Linear
//    256->P*E (text_decoder.py:249).  fp32 throughout (video_encoder.py:323-324 casts to fp32).
//  * vcap_vit_pool: the reference CuPy pool op (core/operators/cupy_vit_pool.py:23-104):
//    y[b,c] = mean_t x[b*T+t, 0, c] ("cls") or mean_{t,p>=1} x[b*T+t, p, c] ("gap").
#include "vcap_common.h"
#include "vcap_kernels.h"

template <typename T>
__global__ __launch_bounds__(256) void vcap_patchify_kernel(const float* __restrict__ frames, T* __restrict__ patches,
                                                            float* __restrict__ x, const float* __restrict__ cls,
                                                            const float* __restrict__ pos, int BT, int img, int p,
                                                            int Kp, int N, int D) {
  const int g = img / p, P = g * g;
  const int row = blockIdx.x;
  if (row >= BT * P) {  // class-token row
    const int bt = row - BT * P;
    float* xr = x + (long)bt * N * D;
    for (int d = threadIdx.x; d < D; d += 256) xr[d] = cls[d] + pos[d];
    return;
  }
  const int bt = row / P, pp = row % P;
  const int py = pp / g, px = pp % g;
  const float* f = frames + (long)bt * 3 * img * img;
  T* out = patches + (long)row * Kp;
  const int K = 3 * p * p;
  for (int k = threadIdx.x; k < Kp; k += 256) {
    float v = 0.f;
    if (k < K) {
      const int c = k / (p * p), rem = k % (p * p), i = rem / p, j = rem % p;
      v = f[((long)c * img + (py * p + i)) * img + (px * p + j)];
    }
    out[k] = Num<T>::from_f(v);
  }
}

// Vectorised im2col for patch sizes that are multiples of 8 (ViT-B/16): one thread per 8
// consecutive K elements of a patch row (= 8 consecutive pixels of one image row), two 16-byte
// loads and one 16-byte (bf16) / two (f32) stores; K padding is zero-filled.
template <typename T>
__global__ __launch_bounds__(256) void vcap_patchify8_kernel(const float* __restrict__ frames, T* __restrict__ patches,
                                                             int BT, int img, int p, int Kp) {
  const int g = img / p, P = g * g, K = 3 * p * p, cpr = Kp / 8;
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)BT * P * cpr) return;
  const long row = i / cpr;
  const int k = (int)(i % cpr) * 8;
  f32x4 a = {0.f, 0.f, 0.f, 0.f}, b = a;
  if (k < K) {
    const int bt = (int)(row / P), pp = (int)(row % P);
    const int py = pp / g, px = pp % g;
    const int c = k / (p * p), rem = k % (p * p), y = rem / p, x0 = rem % p;
    const float* src = frames + (((long)bt * 3 + c) * img + (py * p + y)) * img + px * p + x0;
    a = *reinterpret_cast<const f32x4*>(src);
    b = *reinterpret_cast<const f32x4*>(src + 4);
  }
  T* dst = patches + row * Kp + k;
  if constexpr (sizeof(T) == 2) {
    *reinterpret_cast<u32x4*>(dst) = (u32x4){pack_bf2(a.x, a.y), pack_bf2(a.z, a.w), pack_bf2(b.x, b.y),
                                             pack_bf2(b.z, b.w)};
  } else {
    *reinterpret_cast<f32x4*>(dst) = a;
    *reinterpret_cast<f32x4*>(dst + 4) = b;
  }
}

__global__ __launch_bounds__(256) void vcap_cls_rows_kernel(float* __restrict__ x, const float* __restrict__ cls,
                                                            const float* __restrict__ pos, int N, int D) {
  float* xr = x + (long)blockIdx.x * N * D;
  for (int d = threadIdx.x; d < D; d += 256) xr[d] = cls[d] + pos[d];
}

hipError_t vcap_patchify_dispatch(int dt, const float* frames, void* patches, float* x, const float* cls,
                                  const float* pos, int BT, int img, int p, int Kp, int N, int D, hipStream_t s) {
  const int g = img / p;
  if (p % 8 == 0 && Kp % 8 == 0 && img % 4 == 0) {
    const long chunks = (long)BT * g * g * (Kp / 8);
    const dim3 grid((unsigned)((chunks + 255) / 256));
    if (dt == VCAP_DT_BF16)
      hipLaunchKernelGGL((vcap_patchify8_kernel<bf16_t>), grid, dim3(256), 0, s, frames, (bf16_t*)patches, BT, img, p,
                         Kp);
    else
      hipLaunchKernelGGL((vcap_patchify8_kernel<float>), grid, dim3(256), 0, s, frames, (float*)patches, BT, img, p,
                         Kp);
    hipLaunchKernelGGL(vcap_cls_rows_kernel, dim3(BT), dim3(256), 0, s, x, cls, pos, N, D);
    return hipGetLastError();
  }
  const dim3 grid(BT * g * g + BT), block(256);
  if (dt == VCAP_DT_BF16)
    hipLaunchKernelGGL((vcap_patchify_kernel<bf16_t>), grid, block, 0, s, frames, (bf16_t*)patches, x, cls, pos, BT,
                       img, p, Kp, N, D);
  else
    hipLaunchKernelGGL((vcap_patchify_kernel<float>), grid, block, 0, s, frames, (float*)patches, x, cls, pos, BT,
                       img, p, Kp, N, D);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// Encoder head + engine prefix, as two wide launches (every weight load of a wave issued before
// its first reduction, so each phase costs ~one memory round trip):
//   head:   pooled = mean_t LN_final(x[b, t, CLS]);  emb = pooled . proj_w^T + proj_b
//           (video_encoder.py:316-326 CLS temporal pool + encoder.proj)      grid (B, VD/16)
//   prefix: e = LN(emb) * ln_scale * in_weight (core/engine.py:44-50);
//           prefix = e . mapper_w^T + mapper_b (text_decoder.py:249)         grid (B, MO/64)
constexpr int HEAD_OUT = 16;    // proj outputs per head block (4 per wave)
constexpr int PREFIX_OUT = 64;  // mapper outputs per prefix block (16 per wave, 4 at a time)

__global__ __launch_bounds__(256) void vcap_vit_head_kernel(const float* __restrict__ x, int T, int N, int D,
                                                            const float* __restrict__ ng, const float* __restrict__ nb,
                                                            float neps, const float* __restrict__ pw,
                                                            const float* __restrict__ pb, int VD,
                                                            float* __restrict__ emb) {
  __shared__ float part[4][1024];
  __shared__ float pooled[1024];
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // 1) final LayerNorm of each frame's CLS row, summed over frames (per-wave partials)
  float accv[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) accv[i] = 0.f;
  for (int t = wave; t < T; t += 4) {
    const float* xr = x + ((long)(b * T + t) * N) * D;
    float xv[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) xv[i] = xr[min(lane + 64 * i, D - 1)];  // clamped, never predicated
    float sm = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) sm += (lane + 64 * i < D) ? xv[i] : 0.f;
    const float mean = wave_sum(sm) / (float)D;
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const float d = xv[i] - mean;
      ss += (lane + 64 * i < D) ? d * d : 0.f;
    }
    const float rstd = rsqrtf(wave_sum(ss) / (float)D + neps);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int c = min(lane + 64 * i, D - 1);
      accv[i] += (xv[i] - mean) * rstd * ng[c] + nb[c];
    }
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int c = lane + 64 * i;
    if (c < D) part[wave][c] = accv[i];
  }
  __syncthreads();
  for (int c = tid; c < D; c += 256) pooled[c] = (part[0][c] + part[1][c] + part[2][c] + part[3][c]) / (float)T;
  __syncthreads();
  // 2) encoder.proj, 4 outputs per wave with all their weight loads in flight
  const int ob = blockIdx.y * HEAD_OUT + wave * 4;
  float sacc[4] = {0.f, 0.f, 0.f, 0.f};
  for (int c0 = 0; c0 < D; c0 += 256) {
    float wv[4][4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        wv[k][i] = pw[(long)min(ob + k, VD - 1) * D + min(c0 + lane + 64 * i, D - 1)];
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int c = c0 + lane + 64 * i;
        if (c < D) sacc[k] += pooled[c] * wv[k][i];
      }
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float v = wave_sum(sacc[k]);
    if (lane == 0 && ob + k < VD) emb[(long)b * VD + ob + k] = v + pb[ob + k];
  }
}

__global__ __launch_bounds__(256) void vcap_prefix_map_kernel(const float* __restrict__ emb_in, int VD, float ln_scale,
                                                              float in_weight, const float* __restrict__ mw,
                                                              const float* __restrict__ mb, int MO,
                                                              float* __restrict__ prefix) {
  __shared__ float emb[1024];
  __shared__ float stat[2];
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int c = tid; c < VD; c += 256) emb[c] = emb_in[(long)b * VD + c];
  __syncthreads();
  // engine prefix normalisation (layer_norm without affine, eps 1e-5) * ln_scale, * in_weight
  if (ln_scale > 0.f || in_weight > 0.f) {
    if (wave == 0) {
      float sm = 0.f;
      for (int c = lane; c < VD; c += 64) sm += emb[c];
      const float mean = wave_sum(sm) / (float)VD;
      float ss = 0.f;
      for (int c = lane; c < VD; c += 64) {
        const float d = emb[c] - mean;
        ss += d * d;
      }
      ss = wave_sum(ss);  // whole-wave reduction, outside the lane-0 branch
      if (lane == 0) {
        stat[0] = mean;
        stat[1] = rsqrtf(ss / (float)VD + 1e-5f);
      }
    }
    __syncthreads();
    const float mean = stat[0], rstd = stat[1];
    for (int c = tid; c < VD; c += 256) {
      float v = emb[c];
      if (ln_scale > 0.f) v = (v - mean) * rstd * ln_scale;
      if (in_weight > 0.f) v = v * in_weight;
      emb[c] = v;
    }
    __syncthreads();
  }
  // mapper: 16 outputs per wave in groups of 4, weight loads of a group in flight together
  for (int g = 0; g < 4; ++g) {
    const int ob = blockIdx.y * PREFIX_OUT + wave * 16 + g * 4;
    if (ob >= MO) break;
    float sacc[4] = {0.f, 0.f, 0.f, 0.f};
    for (int c0 = 0; c0 < VD; c0 += 256) {
      float wv[4][4];
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          wv[k][i] = mw[(long)min(ob + k, MO - 1) * VD + min(c0 + lane + 64 * i, VD - 1)];
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int c = c0 + lane + 64 * i;
          if (c < VD) sacc[k] += emb[c] * wv[k][i];
        }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float v = wave_sum(sacc[k]);
      if (lane == 0 && ob + k < MO) prefix[(long)b * MO + ob + k] = v + mb[ob + k];
    }
  }
}

// x == nullptr: prefix only, from emb_in (vcap_prefix_project).  Otherwise the head writes emb
// to enc_out (or emb_scratch when the caller does not want the encoder output) and the prefix
// launch reads it from there.
hipError_t vcap_vit_head_prefix_dispatch(const float* x, int B, int T, int N, int D, const float* ng, const float* nb,
                                         float neps, const float* pw, const float* pb, int VD, float ln_scale,
                                         float in_weight, const float* mw, const float* mb, int MO, float* enc_out,
                                         float* prefix, const float* emb_in, float* emb_scratch, hipStream_t s) {
  if (D > 1024 || VD > 1024 || B <= 0) return hipErrorInvalidValue;
  const float* emb = emb_in;
  if (x) {
    float* e = enc_out ? enc_out : emb_scratch;
    if (!e) return hipErrorInvalidValue;
    hipLaunchKernelGGL(vcap_vit_head_kernel, dim3(B, (VD + HEAD_OUT - 1) / HEAD_OUT), dim3(256), 0, s, x, T, N, D, ng,
                       nb, neps, pw, pb, VD, e);
    if (hipError_t err = hipGetLastError()) return err;
    emb = e;
  }
  if (!prefix) return hipSuccess;
  if (!emb) return hipErrorInvalidValue;
  hipLaunchKernelGGL(vcap_prefix_map_kernel, dim3(B, (MO + PREFIX_OUT - 1) / PREFIX_OUT), dim3(256), 0, s, emb, VD,
                     ln_scale, in_weight, mw, mb, MO, prefix);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void vcap_vit_pool_kernel(const T* __restrict__ x, T* __restrict__ y, int B, int Tn,
                                                            int tokens, int C, int gap) {
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= B * C) return;
  const int b = idx / C, c = idx % C;
  float acc = 0.f;
  if (!gap) {
    for (int t = 0; t < Tn; ++t) acc += Num<T>::to_f(x[((long)(b * Tn + t) * tokens) * C + c]);
    y[idx] = Num<T>::from_f(acc / (float)Tn);
  } else {
    for (int t = 0; t < Tn; ++t)
      for (int p = 1; p < tokens; ++p) acc += Num<T>::to_f(x[((long)(b * Tn + t) * tokens + p) * C + c]);
    y[idx] = Num<T>::from_f(acc / (float)(Tn * (tokens - 1)));
  }
}

hipError_t vcap_vit_pool_dispatch(int dt, const void* x, void* y, int B, int T, int tokens, int C, int gap,
                                  hipStream_t s) {
  const dim3 grid((B * C + 255) / 256), block(256);
  if (dt == VCAP_DT_BF16)
    hipLaunchKernelGGL((vcap_vit_pool_kernel<bf16_t>), grid, block, 0, s, (const bf16_t*)x, (bf16_t*)y, B, T, tokens,
                       C, gap);
  else
    hipLaunchKernelGGL((vcap_vit_pool_kernel<float>), grid, block, 0, s, (const float*)x, (float*)y, B, T, tokens, C,
                       gap);
  return hipGetLastError();
}
