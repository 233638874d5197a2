// Back-to-back ingress copies: does the copy engine restart at once when the next H2D is
// already queued?  The step timeline (profiles/r6_summary.md) shows the engine idle 33-40 us
// between one step's ingress H2D and the next even when the next copy was queued long
// before.  K copies of n bytes (pinned host -> device, distinct destinations, like the
// ingress slots) queued at once, then waited for:
//   hip   hipMemcpyAsync on one stream
//   hip2  hipMemcpyAsync alternating over two streams
//   hsa   hsa_amd_memory_async_copy_on_engine on one SDMA engine, no dependencies
// Per copy: (total time) / K against one copy alone; the difference is the restart cost.
// Build: hipcc --offload-arch=gfx950 -O3 bench/micro/h2d_chain_probe.hip -o bench/micro/h2d_chain_probe -lhsa-runtime64
#include <hip/hip_runtime.h>
#include <hsa/amd_hsa_signal.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                  \
  do {                                                                                         \
    hipError_t e = (x);                                                                        \
    if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); }   \
  } while (0)

static double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

struct Agents { std::vector<hsa_agent_t> gpus, cpus; };

__global__ void k_touch(unsigned* p) {
  if (threadIdx.x == 0) p[0] += 1;
}

// waits (bounded) for an HSA completion signal to reach 0, then an acquire at system scope
__global__ void k_wait_sig(const long* v, unsigned* p) {
  if (threadIdx.x == 0) {
    for (unsigned it = 0; it < (1u << 24); ++it) {
      if (__hip_atomic_load(v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0) break;
      __builtin_amdgcn_s_sleep(2);
    }
    __atomic_thread_fence(__ATOMIC_ACQUIRE);
    p[0] += 1;
  }
}

int main(int argc, char** argv) {
  const size_t n = (size_t)(argc > 1 ? atol(argv[1]) : 12700) << 10;   // KB (one step's payload)
  const int K = argc > 2 ? atoi(argv[2]) : 16;
  CK(hipSetDevice(0));
  void* h = nullptr;
  CK(hipHostMalloc(&h, n, hipHostMallocDefault));
  std::vector<void*> d(K);
  for (auto& p : d) CK(hipMalloc(&p, n));
  hipStream_t s[2];
  CK(hipStreamCreateWithFlags(&s[0], hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s[1], hipStreamNonBlocking));
  // warm-up and the single-copy time
  for (int w = 0; w < 3; ++w) CK(hipMemcpyAsync(d[0], h, n, hipMemcpyHostToDevice, s[0]));
  CK(hipStreamSynchronize(s[0]));
  double t0 = now_s();
  for (int r = 0; r < 5; ++r) {
    CK(hipMemcpyAsync(d[0], h, n, hipMemcpyHostToDevice, s[0]));
    CK(hipStreamSynchronize(s[0]));
  }
  const double one = (now_s() - t0) / 5;
  for (int mode = 0; mode < 2; ++mode) {
    CK(hipDeviceSynchronize());
    t0 = now_s();
    for (int k = 0; k < K; ++k) CK(hipMemcpyAsync(d[k], h, n, hipMemcpyHostToDevice, s[mode ? (k & 1) : 0]));
    CK(hipStreamSynchronize(s[0]));
    CK(hipStreamSynchronize(s[1]));
    const double per = (now_s() - t0) / K;
    printf("%-5s %zu KB x %d: %.1f us per copy (one alone %.1f us incl. sync), %.1f GB/s\n", mode ? "hip2" : "hip",
           n >> 10, K, per * 1e6, one * 1e6, n / per / 1e9);
  }
  // as the engine does it: an event recorded behind every copy, a consumer stream waiting on
  // it and running a small kernel (the step)
  {
    std::vector<hipEvent_t> ev(K);
    for (auto& x : ev) CK(hipEventCreateWithFlags(&x, hipEventDisableTiming));
    CK(hipDeviceSynchronize());
    t0 = now_s();
    for (int k = 0; k < K; ++k) {
      CK(hipMemcpyAsync(d[k], h, n, hipMemcpyHostToDevice, s[0]));
      CK(hipEventRecord(ev[k], s[0]));
      CK(hipStreamWaitEvent(s[1], ev[k], 0));
      hipLaunchKernelGGL(k_touch, dim3(1), dim3(64), 0, s[1], (unsigned*)d[k]);
    }
    CK(hipStreamSynchronize(s[0]));
    CK(hipStreamSynchronize(s[1]));
    const double per = (now_s() - t0) / K;
    printf("hipev %zu KB x %d: %.1f us per copy, %.1f GB/s\n", n >> 10, K, per * 1e6, n / per / 1e9);
    // only the events (no consumer)
    CK(hipDeviceSynchronize());
    t0 = now_s();
    for (int k = 0; k < K; ++k) {
      CK(hipMemcpyAsync(d[k], h, n, hipMemcpyHostToDevice, s[0]));
      CK(hipEventRecord(ev[k], s[0]));
    }
    CK(hipStreamSynchronize(s[0]));
    const double per2 = (now_s() - t0) / K;
    printf("hipe  %zu KB x %d: %.1f us per copy, %.1f GB/s\n", n >> 10, K, per2 * 1e6, n / per2 / 1e9);
    for (auto& x : ev) CK(hipEventDestroy(x));
  }
  // the same through HSA on one engine (not engine 0, the runtime's)
  if (hsa_init() != HSA_STATUS_SUCCESS) return 1;
  Agents ag;
  hsa_iterate_agents([](hsa_agent_t a, void* data) {
    hsa_device_type_t t;
    hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
    auto* x = (Agents*)data;
    (t == HSA_DEVICE_TYPE_GPU ? x->gpus : x->cpus).push_back(a);
    return HSA_STATUS_SUCCESS;
  }, &ag);
  uint32_t mask = 0;
  hsa_amd_memory_copy_engine_status(ag.gpus[0], ag.cpus[0], &mask);
  for (int eng : {2, 0}) {
    if (!((mask >> eng) & 1u)) continue;
    std::vector<hsa_signal_t> sg(K);
    for (auto& x : sg) hsa_signal_create(1, 0, nullptr, &x);
    t0 = now_s();
    for (int k = 0; k < K; ++k)
      if (hsa_amd_memory_async_copy_on_engine(d[k], ag.gpus[0], h, ag.cpus[0], n, 0, nullptr, sg[k],
                                              (hsa_amd_sdma_engine_id_t)(1u << eng), true) != HSA_STATUS_SUCCESS) {
        printf("hsa copy on engine %d refused\n", eng);
        return 1;
      }
    for (auto& x : sg)
      hsa_signal_wait_scacquire(x, HSA_SIGNAL_CONDITION_EQ, 0, UINT64_MAX, HSA_WAIT_STATE_ACTIVE);
    const double per = (now_s() - t0) / K;
    printf("hsa   engine %d, %zu KB x %d: %.1f us per copy, %.1f GB/s\n", eng, n >> 10, K, per * 1e6, n / per / 1e9);
    // the same copies, each consumed by a kernel on a HIP stream that waits for its signal
    // on the device (no host round trip, no marker between the copies)
    for (auto& x : sg) hsa_signal_store_screlease(x, 1);
    CK(hipDeviceSynchronize());
    t0 = now_s();
    for (int k = 0; k < K; ++k) {
      if (hsa_amd_memory_async_copy_on_engine(d[k], ag.gpus[0], h, ag.cpus[0], n, 0, nullptr, sg[k],
                                              (hsa_amd_sdma_engine_id_t)(1u << eng), true) != HSA_STATUS_SUCCESS)
        return 1;
      hipLaunchKernelGGL(k_wait_sig, dim3(1), dim3(64), 0, s[1], (const long*)&((amd_signal_t*)sg[k].handle)->value,
                         (unsigned*)d[k]);
    }
    CK(hipStreamSynchronize(s[1]));
    const double per3 = (now_s() - t0) / K;
    printf("hsak  engine %d, %zu KB x %d: %.1f us per copy + device-side wait, %.1f GB/s\n", eng, n >> 10, K,
           per3 * 1e6, n / per3 / 1e9);
    for (auto& x : sg) hsa_signal_destroy(x);
  }
  // one payload split in halves over two engines at once (0 and 2): is the H2D bound by one
  // engine or by the link?
  {
    std::vector<hsa_signal_t> sg(2 * K);
    for (auto& x : sg) hsa_signal_create(1, 0, nullptr, &x);
    const size_t h1 = (n / 2 + 4095) & ~size_t(4095);
    t0 = now_s();
    for (int k = 0; k < K; ++k)
      for (int half = 0; half < 2; ++half) {
        const size_t off = half ? h1 : 0, len = half ? n - h1 : h1;
        if (hsa_amd_memory_async_copy_on_engine((char*)d[k] + off, ag.gpus[0], (char*)h + off, ag.cpus[0], len, 0,
                                                nullptr, sg[2 * k + half],
                                                (hsa_amd_sdma_engine_id_t)(1u << (half ? 2 : 0)), true) !=
            HSA_STATUS_SUCCESS)
          return 1;
      }
    for (auto& x : sg)
      hsa_signal_wait_scacquire(x, HSA_SIGNAL_CONDITION_EQ, 0, UINT64_MAX, HSA_WAIT_STATE_ACTIVE);
    const double per = (now_s() - t0) / K;
    printf("split engines 0+2, %zu KB x %d: %.1f us per payload, %.1f GB/s\n", n >> 10, K, per * 1e6, n / per / 1e9);
    for (auto& x : sg) hsa_signal_destroy(x);
  }
  return 0;
}
