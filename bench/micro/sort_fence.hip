// Micro-benchmark (run under rocprofv3 --kernel-trace --stats): the radix-sort histogram /
// scatter kernels of the data plane at the pair counts of a step, an empty kernel at
// different wave counts (what a capacity-sized grid costs), and the cost of the
// ticket + __threadfence pattern the data plane uses for "last block" work.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I csrc/kernels bench/micro/sort_fence.hip -o /tmp/sort_fence
#include "dataplane.hip"

#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

__global__ void k_empty(u32* p) { if (p && threadIdx.x == 9999) p[0] = 1; }

// T blocks write 8 KB each, then (fence=1) __threadfence + ticket, the last one reads all
__global__ __launch_bounds__(1024) void k_fence_ticket(u32* buf, u32* ticket, u32 T, int fence) {
  __shared__ u32 s_last;
  const u32 t = blockIdx.x;
  if (t >= T) return;
  for (u32 k = threadIdx.x; k < 2048; k += 1024) buf[t * 2048 + k] = t + k;
  if (fence) __threadfence();
  __syncthreads();
  if (threadIdx.x == 0) s_last = atomicAdd(ticket, 1u) == T - 1;
  __syncthreads();
  if (!s_last) return;
  if (fence) __threadfence();
  if (threadIdx.x == 0) *ticket = 0;
  u32 acc = 0;
  for (u32 i = threadIdx.x; i < T * 2048; i += 1024) acc += buf[i];
  if (acc == 0xdeadbeef) buf[0] = acc;
}

int main() {
  const u32 NMAX = 1u << 20, NT = NMAX / SORT_TILE;
  u32 *k0, *v0, *k1, *v1, *hist, *hscan, *np, *ticket, *buf;
  CK(hipMalloc(&k0, 4ull * NMAX)); CK(hipMalloc(&v0, 4ull * NMAX));
  CK(hipMalloc(&k1, 4ull * NMAX)); CK(hipMalloc(&v1, 4ull * NMAX));
  CK(hipMalloc(&hist, 4ull * 2048 * NT)); CK(hipMalloc(&hscan, 4ull * 2048 * NT));
  CK(hipMalloc(&np, 4)); CK(hipMalloc(&ticket, 4)); CK(hipMalloc(&buf, 4ull * 2048 * 1024));
  CK(hipMemset(ticket, 0, 4));
  std::vector<u32> hk(NMAX), hv(NMAX);
  const u32 sizes[] = {1024, 4096, 15104, 65536};
  for (u32 n : sizes) {
    // phase-B-like keys: 7 source ranks in blocks, 16 queues interleaved
    for (u32 i = 0; i < n; ++i) { const u32 src = i / ((n + 6) / 7); hk[i] = (((i * 7) % 16) << 3) | src; hv[i] = i; }
    CK(hipMemcpy(k0, hk.data(), 4ull * n, hipMemcpyHostToDevice));
    CK(hipMemcpy(v0, hv.data(), 4ull * n, hipMemcpyHostToDevice));
    CK(hipMemcpy(np, &n, 4, hipMemcpyHostToDevice));
    for (int rep = 0; rep < 50; ++rep) {
      hipLaunchKernelGGL(k_rs_hist<11>, dim3(256), dim3(RsNt<11>::v), 0, 0, k0, np, 0u, hist, hscan, ticket, NT);
      hipLaunchKernelGGL(k_rs_scatter<11>, dim3(256), dim3(256), 0, 0, k0, v0, k1, v1, np, 0u, hscan, NT);
      hipLaunchKernelGGL(k_rs_hist<8>, dim3(256), dim3(RsNt<8>::v), 0, 0, k0, np, 0u, hist, hscan, ticket, NT);
    }
    CK(hipDeviceSynchronize());
    // check: sorted by key, stable
    std::vector<u32> ok(n), ov(n);
    CK(hipMemcpy(ok.data(), k1, 4ull * n, hipMemcpyDeviceToHost));
    CK(hipMemcpy(ov.data(), v1, 4ull * n, hipMemcpyDeviceToHost));
    bool good = true;
    for (u32 i = 1; i < n; ++i)
      if (ok[i - 1] > ok[i] || (ok[i - 1] == ok[i] && ov[i - 1] > ov[i])) { good = false; break; }
    printf("{\"n\": %u, \"sorted_stable\": %s}\n", n, good ? "true" : "false");
  }
  for (u32 blocks : {64u, 1024u, 8192u, 32768u})
    for (int rep = 0; rep < 50; ++rep) hipLaunchKernelGGL(k_empty, dim3(blocks), dim3(256), 0, 0, nullptr);
  for (u32 T : {1u, 15u, 64u})
    for (int fence = 0; fence < 2; ++fence)
      for (int rep = 0; rep < 50; ++rep)
        hipLaunchKernelGGL(k_fence_ticket, dim3(T), dim3(1024), 0, 0, buf, ticket, T, fence);
  CK(hipDeviceSynchronize());
  printf("done\n");
  return 0;
}
