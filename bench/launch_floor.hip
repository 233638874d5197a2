// Per-kernel cost inside a hipGraph on MI355X: a chain of N dependent kernels (empty,
// 1 block; empty, 256 blocks; 256 blocks touching 1 KB each; and one block doing a
// device-scope atomic ticket) captured once and replayed.  Sizes the fixed cost a
// step pays per launch (the data plane's step is ~22 launches).
#include <hip/hip_runtime.h>
#include <cstdio>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

__global__ void k_empty(int* p) { if (p && threadIdx.x == 1023) p[0] = 1; }
__global__ void k_touch(int* p) { p[blockIdx.x * 256 + threadIdx.x] += 1; }

int run(const char* name, int kind, int blocks, int n) {
  int* buf;
  CK(hipMalloc(&buf, 64 << 20));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  for (int i = 0; i < n; ++i) {
    if (kind == 0) hipLaunchKernelGGL(k_empty, dim3(blocks), dim3(256), 0, s, nullptr);
    else hipLaunchKernelGGL(k_touch, dim3(blocks), dim3(256), 0, s, buf);
  }
  CK(hipStreamEndCapture(s, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int w = 0; w < 5; ++w) CK(hipGraphLaunch(ge, s));
  CK(hipEventRecord(a, s));
  const int reps = 50;
  for (int r = 0; r < reps; ++r) CK(hipGraphLaunch(ge, s));
  CK(hipEventRecord(b, s));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  printf("%-28s blocks %5d: %6.2f us per kernel (chain of %d)\n", name, blocks, 1000.0 * ms / reps / n, n);
  CK(hipFree(buf));
  return 0;
}

int main() {
  run("empty", 0, 1, 20);
  run("empty", 0, 256, 20);
  run("empty", 0, 8192, 20);
  run("touch 1 KB per block", 1, 256, 20);
  run("touch 1 KB per block", 1, 4096, 20);
  return 0;
}
