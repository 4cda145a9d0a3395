// Row LayerNorm: f32 residual stream -> T (bf16 MFMA operand, or f32 in parity mode).
// ViT norm1/norm2 (eps 1e-6, timm Block, src/models/video_encoder.py:168-170) and the
// engine's prefix layer_norm without affine (core/engine.py:47-48, eps 1e-5).
// One wave per row, two-pass mean/variance in fp32 registers, float4 loads.
// Also: the MXFP8 variant (LayerNorm fused with the e4m3 + E8M0 block quantisation of the next
// GEMM's operand) and the standalone MXFP8 quantiser.
#include "vcap_common.h"
#include "vcap_kernels.h"

template <typename TOut, bool VEC4>
__global__ __launch_bounds__(256) void vcap_layernorm_kernel(const float* __restrict__ x, long ldx, TOut* __restrict__ y,
                                                             long ldy, const float* __restrict__ gamma,
                                                             const float* __restrict__ beta, int rows, int D,
                                                             float eps) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const float* xr = x + (long)row * ldx;
  TOut* yr = y + (long)row * ldy;
  constexpr int MAXV = 16;  // D <= 64*4*4 = 1024 on the vector path
  if constexpr (VEC4) {
    const int nv = D / 256;
    f32x4 v[MAXV / 4];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < MAXV / 4; ++i)  // clamped, unpredicated loads (one round trip)
      v[i] = *reinterpret_cast<const f32x4*>(xr + min(i, nv - 1) * 256 + lane * 4);
#pragma unroll
    for (int i = 0; i < MAXV / 4; ++i)
      if (i < nv) s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
    const float mean = wave_sum(s) / (float)D;
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < MAXV / 4; ++i) {
      if (i < nv) {
        f32x4 d = v[i] - mean;
        v[i] = d;
        ss += (d.x * d.x + d.y * d.y) + (d.z * d.z + d.w * d.w);
      }
    }
    const float rstd = rsqrtf(wave_sum(ss) / (float)D + eps);
#pragma unroll
    for (int i = 0; i < MAXV / 4; ++i) {
      if (i < nv) {
        const int c = i * 256 + lane * 4;
        f32x4 o = v[i] * rstd;
        if (gamma) {
          const f32x4 g = *reinterpret_cast<const f32x4*>(gamma + c);
          const f32x4 b = *reinterpret_cast<const f32x4*>(beta + c);
          o = o * g + b;
        }
        if constexpr (sizeof(TOut) == 2) {
          *reinterpret_cast<u32x2*>(yr + c) = (u32x2){pack_bf2(o.x, o.y), pack_bf2(o.z, o.w)};
        } else {
          *reinterpret_cast<f32x4*>(yr + c) = o;
        }
      }
    }
  } else {
    float s = 0.f;
    for (int c = lane; c < D; c += 64) s += xr[c];
    const float mean = wave_sum(s) / (float)D;
    float ss = 0.f;
    for (int c = lane; c < D; c += 64) {
      float d = xr[c] - mean;
      ss += d * d;
    }
    const float rstd = rsqrtf(wave_sum(ss) / (float)D + eps);
    for (int c = lane; c < D; c += 64) {
      float o = (xr[c] - mean) * rstd;
      if (gamma) o = o * gamma[c] + beta[c];
      yr[c] = Num<TOut>::from_f(o);
    }
  }
}

// LayerNorm -> MXFP8 operand of the next GEMM (e4m3 + E8M0 per 32 columns, vcap_common.h layout).
// D % 256 == 0, D <= 1024: lane owns 4 consecutive columns of each 256-column chunk, so one
// 32-block is 8 consecutive lanes.
__global__ __launch_bounds__(256) void vcap_layernorm_mx_kernel(const float* __restrict__ x, long ldx,
                                                                fp8_t* __restrict__ y, uint8_t* __restrict__ scales,
                                                                int groups, const float* __restrict__ gamma,
                                                                const float* __restrict__ beta, int rows, int D,
                                                                float eps) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const float* xr = x + (long)row * ldx;
  const int nv = D / 256;
  f32x4 v[4];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] = *reinterpret_cast<const f32x4*>(xr + min(i, nv - 1) * 256 + lane * 4);
#pragma unroll
  for (int i = 0; i < 4; ++i)
    if (i < nv) s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
  const float mean = wave_sum(s) / (float)D;
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (i < nv) {
      v[i] -= mean;
      ss += (v[i].x * v[i].x + v[i].y * v[i].y) + (v[i].z * v[i].z + v[i].w * v[i].w);
    }
  }
  const float rstd = rsqrtf(wave_sum(ss) / (float)D + eps);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (i < nv) {
      const int c = i * 256 + lane * 4;
      f32x4 o = v[i] * rstd;
      if (gamma) o = o * *reinterpret_cast<const f32x4*>(gamma + c) + *reinterpret_cast<const f32x4*>(beta + c);
      mx_quant_store4(o, row, c, y + (long)row * D, scales, groups);
    }
  }
}

// Rows of f32 / bf16 -> MXFP8 (weights at load time; op-level entry point). K % 256 == 0.
template <typename TIn>
__global__ __launch_bounds__(256) void vcap_mx_quantize_kernel(const TIn* __restrict__ x, long ldx, int rows, int K,
                                                               fp8_t* __restrict__ q, uint8_t* __restrict__ scales,
                                                               int groups) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int c = blockIdx.y * 256 + (threadIdx.x & 63) * 4;
  const TIn* xr = x + (long)row * ldx + c;
  const f32x4 o = {Num<TIn>::to_f(xr[0]), Num<TIn>::to_f(xr[1]), Num<TIn>::to_f(xr[2]), Num<TIn>::to_f(xr[3])};
  mx_quant_store4(o, row, c, q + (long)row * K, scales, groups);
}

hipError_t vcap_layernorm_mx_dispatch(const float* x, long ldx, uint8_t* q, uint8_t* scales, int srows,
                                      const float* gamma, const float* beta, int rows, int D, float eps,
                                      hipStream_t s) {
  if (rows <= 0) return hipSuccess;
  if (D % 256 || D > 1024) return hipErrorInvalidValue;
  hipLaunchKernelGGL(vcap_layernorm_mx_kernel, dim3((rows + 3) / 4), dim3(256), 0, s, x, ldx, q, scales,
                     (srows + 255) / 256, gamma, beta, rows, D, eps);
  return hipGetLastError();
}

hipError_t vcap_mx_quantize_dispatch(int in_dt, const void* x, long ldx, int rows, int K, uint8_t* q,
                                     uint8_t* scales, int srows, hipStream_t s) {
  if (rows <= 0) return hipSuccess;
  if (K % 256) return hipErrorInvalidValue;
  const dim3 grid((rows + 3) / 4, K / 256), block(256);
  const int groups = (srows + 255) / 256;
  if (in_dt == VCAP_DT_F32)
    hipLaunchKernelGGL((vcap_mx_quantize_kernel<float>), grid, block, 0, s, (const float*)x, ldx, rows, K, q, scales,
                       groups);
  else if (in_dt == VCAP_DT_BF16)
    hipLaunchKernelGGL((vcap_mx_quantize_kernel<bf16_t>), grid, block, 0, s, (const bf16_t*)x, ldx, rows, K, q,
                       scales, groups);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t vcap_layernorm_dispatch(int out_dt, const float* x, long ldx, void* y, long ldy, const float* gamma,
                                   const float* beta, int rows, int D, float eps, hipStream_t s) {
  if (rows <= 0) return hipSuccess;
  const dim3 grid((rows + 3) / 4), block(256);
  const bool vec = (D % 256 == 0) && D <= 1024;
  if (out_dt == VCAP_DT_BF16) {
    if (vec)
      hipLaunchKernelGGL((vcap_layernorm_kernel<bf16_t, true>), grid, block, 0, s, x, ldx, (bf16_t*)y, ldy, gamma,
                         beta, rows, D, eps);
    else
      hipLaunchKernelGGL((vcap_layernorm_kernel<bf16_t, false>), grid, block, 0, s, x, ldx, (bf16_t*)y, ldy,
                         gamma, beta, rows, D, eps);
  } else {
    if (vec)
      hipLaunchKernelGGL((vcap_layernorm_kernel<float, true>), grid, block, 0, s, x, ldx, (float*)y, ldy, gamma,
                         beta, rows, D, eps);
    else
      hipLaunchKernelGGL((vcap_layernorm_kernel<float, false>), grid, block, 0, s, x, ldx, (float*)y, ldy, gamma,
                         beta, rows, D, eps);
  }
  return hipGetLastError();
}
