// Frame preprocessing on the GPU: decoded RGB frames (uint8 HWC, as PIL hands them over) ->
// the encoder's normalised f32 [n, 3, out_h, out_w] input, bit-identical to the reference's
// torchvision Resize((S, S)) -> ToTensor -> Normalize chain (core/preprocessing/frame_loader.py:34-45),
// whose Resize on a PIL image is PIL Image.resize(BILINEAR) (Pillow Resample.c, 8 bits per channel):
//   * per output index, double-precision triangle-filter weights over the support widened by the
//     downscale factor, normalised by their left-to-right sum, rounded to 22-bit fixed point;
//   * horizontal pass then vertical pass, each an int32 sum from a 2^21 rounding bias, >> 22,
//     clamped to [0, 255];
//   * / 255 (f32), - mean, / std (f32), channel-planar store.
// The weights are computed on the device with FP contraction off, so every double operation
// rounds exactly as Pillow's C code does on the host (checked bit-exact against PIL in tests).
#include "vcap_common.h"
#include "vcap_kernels.h"

#include <cmath>

namespace {
constexpr int PREC = 22;

struct AxisCoeffs {
  int in_size, out_size, ksize;
  double scale, fscale, support;
};

AxisCoeffs axis_of(int in_size, int out_size) {
  AxisCoeffs a;
  a.in_size = in_size;
  a.out_size = out_size;
  a.scale = (double)in_size / (double)out_size;
  a.fscale = a.scale < 1.0 ? 1.0 : a.scale;
  a.support = 1.0 * a.fscale;
  a.ksize = (int)std::ceil(a.support) * 2 + 1;
  return a;
}
}  // namespace

// one thread per output index of one axis: bounds (xmin, n) + ksize fixed-point weights
__global__ void vcap_resample_coeffs_kernel(int in_size, int out_size, int ksize, double scale, double fscale,
                                            double support, int* __restrict__ bounds, int* __restrict__ kk) {
#pragma clang fp contract(off)
  const int xx = blockIdx.x * blockDim.x + threadIdx.x;
  if (xx >= out_size) return;
  const double center = (xx + 0.5) * scale;
  const double ss = 1.0 / fscale;
  int xmin = (int)(center - support + 0.5);
  if (xmin < 0) xmin = 0;
  int xmax = (int)(center + support + 0.5);
  if (xmax > in_size) xmax = in_size;
  xmax -= xmin;
  double w[64];
  double ww = 0.0;
  for (int x = 0; x < xmax && x < 64; ++x) {
    double t = (x + xmin - center + 0.5) * ss;
    if (t < 0.0) t = -t;
    w[x] = t < 1.0 ? 1.0 - t : 0.0;
    ww += w[x];
  }
  for (int x = 0; x < ksize; ++x) {
    int v = 0;
    if (x < xmax) {
      const double k = ww != 0.0 ? w[x] / ww : w[x];
      v = k < 0 ? (int)(-0.5 + k * (1 << PREC)) : (int)(0.5 + k * (1 << PREC));
    }
    kk[xx * ksize + x] = v;
  }
  bounds[2 * xx] = xmin;
  bounds[2 * xx + 1] = xmax;
}

VCAP_DEV int clip8(int v) {
  v >>= PREC;
  return v < 0 ? 0 : (v > 255 ? 255 : v);
}

// horizontal pass: src [n][h][w][3] -> dst [n][h][out_w][3]
__global__ __launch_bounds__(256) void vcap_resample_h_kernel(const uint8_t* __restrict__ src, int n, int h, int w,
                                                              int out_w, const int* __restrict__ bounds,
                                                              const int* __restrict__ kk, int ksize,
                                                              uint8_t* __restrict__ dst) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)n * h * out_w) return;
  const int xx = (int)(i % out_w);
  const long row = i / out_w;  // frame * h + y
  const int xmin = bounds[2 * xx], xmax = bounds[2 * xx + 1];
  const int* k = kk + xx * ksize;
  const uint8_t* s = src + (row * w + xmin) * 3;
  int s0 = 1 << (PREC - 1), s1 = s0, s2 = s0;
  for (int x = 0; x < xmax; ++x) {
    const int kx = k[x];
    s0 += s[3 * x] * kx;
    s1 += s[3 * x + 1] * kx;
    s2 += s[3 * x + 2] * kx;
  }
  uint8_t* d = dst + i * 3;
  d[0] = (uint8_t)clip8(s0);
  d[1] = (uint8_t)clip8(s1);
  d[2] = (uint8_t)clip8(s2);
}

struct Norm3 {
  float mean[3], std[3];
};

// vertical pass (or a copy when the height is unchanged) + /255, -mean, /std -> [n][3][oh][ow]
__global__ __launch_bounds__(256) void vcap_resample_v_norm_kernel(const uint8_t* __restrict__ src, int n, int h,
                                                                   int ow, int oh, int vertical,
                                                                   const int* __restrict__ bounds,
                                                                   const int* __restrict__ kk, int ksize, Norm3 nm,
                                                                   float* __restrict__ out, uint8_t* __restrict__ out_u8) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)n * oh * ow) return;
  const int xx = (int)(i % ow);
  const int yy = (int)((i / ow) % oh);
  const int f = (int)(i / ((long)ow * oh));
  int v[3];
  if (vertical) {
    const int ymin = bounds[2 * yy], ymax = bounds[2 * yy + 1];
    const int* k = kk + yy * ksize;
    int s0 = 1 << (PREC - 1), s1 = s0, s2 = s0;
    const uint8_t* s = src + (((long)f * h + ymin) * ow + xx) * 3;
    for (int y = 0; y < ymax; ++y) {
      const int ky = k[y];
      const uint8_t* p = s + (long)y * ow * 3;
      s0 += p[0] * ky;
      s1 += p[1] * ky;
      s2 += p[2] * ky;
    }
    v[0] = clip8(s0);
    v[1] = clip8(s1);
    v[2] = clip8(s2);
  } else {
    const uint8_t* p = src + (((long)f * h + yy) * ow + xx) * 3;
    v[0] = p[0];
    v[1] = p[1];
    v[2] = p[2];
  }
  if (out_u8) {
    uint8_t* d = out_u8 + i * 3;
    d[0] = (uint8_t)v[0];
    d[1] = (uint8_t)v[1];
    d[2] = (uint8_t)v[2];
  }
  if (out) {
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const float t = (float)v[c] / 255.0f;
      out[(((long)f * 3 + c) * oh + yy) * ow + xx] = (t - nm.mean[c]) / nm.std[c];
    }
  }
}

size_t vcap_frames_ws_bytes(int n, int in_h, int in_w, int out_h, int out_w) {
  const AxisCoeffs ah = axis_of(in_w, out_w), av = axis_of(in_h, out_h);
  auto al = [](size_t x) { return (x + 255) & ~size_t(255); };
  return al((size_t)out_w * 2 * 4) + al((size_t)out_w * ah.ksize * 4) + al((size_t)out_h * 2 * 4) +
         al((size_t)out_h * av.ksize * 4) + al((size_t)n * in_h * out_w * 3);
}

hipError_t vcap_frames_preprocess_dispatch(const uint8_t* frames, int n, int in_h, int in_w, int out_h, int out_w,
                                           const float* mean3, const float* std3, float* out, uint8_t* out_u8,
                                           void* ws, hipStream_t s) {
  const AxisCoeffs ah = axis_of(in_w, out_w), av = axis_of(in_h, out_h);
  if (ah.ksize > 64 || av.ksize > 64) return hipErrorInvalidValue;  // downscale factor > 31
  auto al = [](size_t x) { return (x + 255) & ~size_t(255); };
  char* p = (char*)ws;
  int* bh = (int*)p;
  p += al((size_t)out_w * 2 * 4);
  int* kh = (int*)p;
  p += al((size_t)out_w * ah.ksize * 4);
  int* bv = (int*)p;
  p += al((size_t)out_h * 2 * 4);
  int* kv = (int*)p;
  p += al((size_t)out_h * av.ksize * 4);
  uint8_t* tmp = (uint8_t*)p;
  const bool horizontal = in_w != out_w, vertical = in_h != out_h;
  if (horizontal) {
    hipLaunchKernelGGL(vcap_resample_coeffs_kernel, dim3((out_w + 63) / 64), dim3(64), 0, s, in_w, out_w, ah.ksize,
                       ah.scale, ah.fscale, ah.support, bh, kh);
    const long tot = (long)n * in_h * out_w;
    hipLaunchKernelGGL(vcap_resample_h_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, frames, n, in_h,
                       in_w, out_w, bh, kh, ah.ksize, tmp);
  }
  if (vertical)
    hipLaunchKernelGGL(vcap_resample_coeffs_kernel, dim3((out_h + 63) / 64), dim3(64), 0, s, in_h, out_h, av.ksize,
                       av.scale, av.fscale, av.support, bv, kv);
  Norm3 nm;
  for (int c = 0; c < 3; ++c) {
    nm.mean[c] = mean3[c];
    nm.std[c] = std3[c];
  }
  const long tot = (long)n * out_h * out_w;
  hipLaunchKernelGGL(vcap_resample_v_norm_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s,
                     horizontal ? tmp : frames, n, in_h, out_w, out_h, vertical ? 1 : 0, bv, kv, av.ksize, nm, out,
                     out_u8);
  return hipGetLastError();
}
