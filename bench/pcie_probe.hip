// PCIe transfer probe for the data plane's step IO: how fast do H2D (ingress) and D2H
// (egress) run alone and concurrently, through which engine.  Variants:
//   runtime   hipMemcpyAsync on two streams (runtime picks blit kernel / SDMA)
//   hsa       hsa_amd_memory_async_copy_on_engine, H2D and D2H on distinct SDMA engines
//   kernel    zero-copy kernels on a few workgroups (16-B loads from / stores to mapped
//             pinned host memory)
// Build: hipcc --offload-arch=gfx950 -O3 bench/pcie_probe.hip -o bench/pcie_probe -lhsa-runtime64
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                            \
  do {                                                                                   \
    hipError_t e = (x);                                                                  \
    if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } \
  } while (0)

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

__global__ void k_copy(v4u* dst, const v4u* src, size_t nv) {
  size_t g = blockIdx.x * (size_t)blockDim.x + threadIdx.x, s = (size_t)gridDim.x * blockDim.x;
  for (size_t i = g; i < nv; i += s) dst[i] = __builtin_nontemporal_load(src + i);
}

static double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

struct Agents { std::vector<hsa_agent_t> gpus, cpus; };

int main(int argc, char** argv) {
  size_t n = (argc > 1 ? atol(argv[1]) : 16) << 20;
  int iters = argc > 2 ? atoi(argv[2]) : 20;
  CK(hipSetDevice(0));
  void *h_in, *h_out, *d_in, *d_out, *h_in_m, *h_out_m;
  CK(hipHostMalloc(&h_in, n, hipHostMallocPortable));
  CK(hipHostMalloc(&h_out, n, hipHostMallocPortable));
  CK(hipHostMalloc(&h_in_m, n, hipHostMallocMapped | hipHostMallocPortable));
  CK(hipHostMalloc(&h_out_m, n, hipHostMallocMapped | hipHostMallocPortable));
  memset(h_in, 1, n); memset(h_in_m, 1, n);
  CK(hipMalloc(&d_in, n));
  CK(hipMalloc(&d_out, n));
  CK(hipMemset(d_out, 2, n));
  hipStream_t s1, s2;
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  auto gbps = [&](double t, int dirs) { return dirs * (double)n * iters / t / 1e9; };

  // ---- runtime copies
  for (int mode = 0; mode < 3; ++mode) {
    CK(hipDeviceSynchronize());
    double t0 = now_s();
    for (int i = 0; i < iters; ++i) {
      if (mode != 1) CK(hipMemcpyAsync(d_in, h_in, n, hipMemcpyHostToDevice, s1));
      if (mode != 0) CK(hipMemcpyAsync(h_out, d_out, n, hipMemcpyDeviceToHost, s2));
    }
    CK(hipDeviceSynchronize());
    double t = now_s() - t0;
    printf("runtime %-9s %7.1f GB/s total (%d MiB x %d)\n", mode == 0 ? "H2D" : mode == 1 ? "D2H" : "H2D+D2H",
           gbps(t, mode == 2 ? 2 : 1), (int)(n >> 20), iters);
  }
  // ---- zero-copy kernels on W workgroups
  for (int wgs : {8, 16, 32, 64}) {
    for (int mode = 0; mode < 3; ++mode) {
      CK(hipDeviceSynchronize());
      void *hin_d, *hout_d;
      CK(hipHostGetDevicePointer(&hin_d, h_in_m, 0));
      CK(hipHostGetDevicePointer(&hout_d, h_out_m, 0));
      double t0 = now_s();
      for (int i = 0; i < iters; ++i) {
        if (mode != 1) hipLaunchKernelGGL(k_copy, dim3(wgs), dim3(256), 0, s1, (v4u*)d_in, (const v4u*)hin_d, n / 16);
        if (mode != 0) hipLaunchKernelGGL(k_copy, dim3(wgs), dim3(256), 0, s2, (v4u*)hout_d, (const v4u*)d_out, n / 16);
      }
      CK(hipDeviceSynchronize());
      double t = now_s() - t0;
      printf("kernel%3d %-9s %7.1f GB/s total\n", wgs, mode == 0 ? "H2D" : mode == 1 ? "D2H" : "H2D+D2H",
             gbps(t, mode == 2 ? 2 : 1));
    }
  }
  // ---- HSA SDMA engines
  if (hsa_init() != HSA_STATUS_SUCCESS) { printf("hsa_init failed\n"); return 0; }
  Agents ag;
  hsa_iterate_agents([](hsa_agent_t a, void* data) {
    hsa_device_type_t t;
    hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
    auto* c = (Agents*)data;
    if (t == HSA_DEVICE_TYPE_GPU) c->gpus.push_back(a);
    else if (t == HSA_DEVICE_TYPE_CPU) c->cpus.push_back(a);
    return HSA_STATUS_SUCCESS;
  }, &ag);
  hsa_agent_t gpu = ag.gpus[0], cpu = ag.cpus[0];
  uint32_t m_h2d = 0, m_d2h = 0;
  hsa_amd_memory_copy_engine_status(gpu, cpu, &m_h2d);
  hsa_amd_memory_copy_engine_status(cpu, gpu, &m_d2h);
  printf("sdma engine masks: cpu->gpu 0x%x gpu->cpu 0x%x\n", m_h2d, m_d2h);
  std::vector<int> engines;
  for (int b = 0; b < 32; ++b) if ((m_h2d & m_d2h) & (1u << b)) engines.push_back(b);
  if (engines.size() < 1) return 0;
  hsa_signal_t sg1, sg2;
  hsa_signal_create(0, 0, nullptr, &sg1);
  hsa_signal_create(0, 0, nullptr, &sg2);
  auto run = [&](int e_in, int e_out, int mode) {
    double t0 = now_s();
    for (int i = 0; i < iters; ++i) {
      if (mode != 1) {
        hsa_signal_store_screlease(sg1, 1);
        if (hsa_amd_memory_async_copy_on_engine(d_in, gpu, h_in, cpu, n, 0, nullptr, sg1,
                                                (hsa_amd_sdma_engine_id_t)(1u << e_in), true) != HSA_STATUS_SUCCESS) {
          printf("copy_on_engine H2D %d failed\n", e_in); return;
        }
      }
      if (mode != 0) {
        hsa_signal_store_screlease(sg2, 1);
        if (hsa_amd_memory_async_copy_on_engine(h_out, cpu, d_out, gpu, n, 0, nullptr, sg2,
                                                (hsa_amd_sdma_engine_id_t)(1u << e_out), true) != HSA_STATUS_SUCCESS) {
          printf("copy_on_engine D2H %d failed\n", e_out); return;
        }
      }
      if (mode != 1) hsa_signal_wait_scacquire(sg1, HSA_SIGNAL_CONDITION_EQ, 0, UINT64_MAX, HSA_WAIT_STATE_ACTIVE);
      if (mode != 0) hsa_signal_wait_scacquire(sg2, HSA_SIGNAL_CONDITION_EQ, 0, UINT64_MAX, HSA_WAIT_STATE_ACTIVE);
    }
    double t = now_s() - t0;
    printf("sdma in=%d out=%d %-9s %7.1f GB/s total\n", e_in, e_out, mode == 0 ? "H2D" : mode == 1 ? "D2H" : "H2D+D2H",
           gbps(t, mode == 2 ? 2 : 1));
  };
  run(engines[0], engines[0], 0);
  run(engines[0], engines[0], 1);
  run(engines[0], engines[0], 2);
  if (engines.size() > 1) run(engines[0], engines[1], 2);
  return 0;
}
