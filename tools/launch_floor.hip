// Microbenchmark: per-kernel floor of dependent launches on one stream, eager vs hipGraph replay,
// for an empty kernel and for one that declares 64 KiB of dynamic LDS.  Used to size the decode
// step's kernel budget (DESIGN.md "decode launch floor").
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

__global__ void empty_k(int* p) { if (threadIdx.x == 0 && blockIdx.x == 0 && p[0] == 12345) p[1] = 1; }
__global__ void lds_k(int* p) {
  extern __shared__ int s[];
  s[threadIdx.x] = threadIdx.x;
  __syncthreads();
  if (threadIdx.x == 0 && blockIdx.x == 0 && p[0] == 12345) p[1] = s[5];
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

template <typename F>
double run(hipStream_t s, F launch, int n, bool graph) {
  hipGraphExec_t ge = nullptr;
  if (graph) {
    hipGraph_t g;
    (void)hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
    for (int i = 0; i < n; ++i) launch();
    (void)hipStreamEndCapture(s, &g);
    (void)hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    (void)hipGraphLaunch(ge, s);
  } else {
    for (int i = 0; i < n; ++i) launch();
  }
  (void)hipStreamSynchronize(s);
  hipEvent_t a, b;
  (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  (void)hipEventRecord(a, s);
  const int reps = 5;
  for (int r = 0; r < reps; ++r) {
    if (graph) (void)hipGraphLaunch(ge, s);
    else for (int i = 0; i < n; ++i) launch();
  }
  (void)hipEventRecord(b, s);
  (void)hipEventSynchronize(b);
  float ms; (void)hipEventElapsedTime(&ms, a, b);
  return ms * 1e3 / (reps * n);
}

int main() {
  int* p; CK(hipMalloc(&p, 64)); CK(hipMemset(p, 0, 64));
  hipStream_t s; CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  CK(hipFuncSetAttribute((const void*)lds_k, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024));
  const int n = 500;
  for (int grid : {1, 144, 1024}) {
    auto e = [&] { hipLaunchKernelGGL(empty_k, dim3(grid), dim3(256), 0, s, p); };
    auto l = [&] { hipLaunchKernelGGL(lds_k, dim3(grid), dim3(256), 74 * 1024, s, p); };
    printf("grid %4d: empty eager %.2f us  graph %.2f us | lds74K eager %.2f us graph %.2f us\n", grid,
           run(s, e, n, false), run(s, e, n, true), run(s, l, n, false), run(s, l, n, true));
  }
  return 0;
}
