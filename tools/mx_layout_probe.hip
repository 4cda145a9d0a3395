// Probe of v_mfma_scale_f32_16x16x128_f8f6f4 operand layout on gfx950 (run on the GPU box):
// wave w puts a single e4m3 1.0 in lane L = w / 32, byte J = w % 32 of the A operand, 1.0 in
// every byte of B, scale_b = 127 (1.0) in every lane and scale_a = 95 + lane (lane-distinct).
// D[r][c] = 2^(scale of the lane whose scale applied - 127): the nonzero row of D gives the A row
// of (L, J), log2(D) + 32 gives the lane whose scale byte was applied to it.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
typedef __attribute__((ext_vector_type(8))) int i32x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

__global__ void probe(float* out) {
  const int w = blockIdx.x, lane = threadIdx.x;
  const int L = w / 32, J = w % 32;
  unsigned char a[32], b[32];
  for (int j = 0; j < 32; ++j) {
    a[j] = (lane == L && j == J) ? 0x38 : 0;  // e4m3 1.0 = 0 0111 000
    b[j] = 0x38;
  }
  i32x8 av, bv;
  __builtin_memcpy(&av, a, 32);
  __builtin_memcpy(&bv, b, 32);
  f32x4 c = {0.f, 0.f, 0.f, 0.f};
  c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(av, bv, c, 0, 0, 0, 95 + lane, 0, 127);
  for (int i = 0; i < 4; ++i) out[(w * 64 + lane) * 4 + i] = c[i];
}

int main() {
  float* d;
  hipMalloc(&d, 2048 * 64 * 4 * sizeof(float));
  hipLaunchKernelGGL(probe, dim3(2048), dim3(64), 0, 0, d);
  static float h[2048 * 64 * 4];
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  // D layout: lane l, reg i -> row (l >> 4) * 4 + i, col l & 15
  for (int w = 0; w < 2048; ++w) {
    int row = -1, ls = -1, nnz = 0;
    for (int l = 0; l < 64; ++l)
      for (int i = 0; i < 4; ++i) {
        float v = h[(w * 64 + l) * 4 + i];
        if (v != 0.f) {
          ++nnz;
          row = (l >> 4) * 4 + i;
          ls = (int)lrintf(log2f(v)) + 32;
        }
      }
    printf("L=%d J=%d row=%d scale_lane=%d nnz=%d\n", w / 32, w % 32, row, ls, nnz);
  }
  return 0;
}
