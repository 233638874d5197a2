// Where does k_frame_scan's candidate screen spend its time?  The screen of the headline step
// (256 segments x 48 KB, one 1024-thread block per segment and CU) timed in isolation, one
// ingredient at a time:
//   load      each block reads its segment (16-B words, one per lane, 4 in flight per lane)
//   +shift    the words are re-aligned behind a carry of odd length (two-level barrel shift,
//             the look-ahead word from the neighbour lane)
//   +stage    ... and stored to the LDS stage
//   +copy     ... and to the work buffer in HBM (the fused segment copy)
//   +cand     ... and screened (cand_bits) into the LDS candidate mask -- the full phase
// Build: hipcc --offload-arch=gfx950 -O3 bench/micro/screen_probe.hip -o bench/micro/screen_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e = (x);                                                                    \
    if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } \
  } while (0)

typedef unsigned int u32;
constexpr u32 NT = 1024, SEG = 48u << 10, NSEG = 256, NW = SEG / 16;

__device__ __forceinline__ u32 zero_bytes(u32 v) { return (v - 0x01010101u) & ~v & 0x80808080u; }
__device__ __forceinline__ u32 type_nibble(u32 v) {
  const u32 h = (zero_bytes(v & 0xFCFCFCFCu) & ~zero_bytes(v)) | zero_bytes(v ^ 0x08080808u);
  return (((h >> 7) * 0x00204081u) >> 21) & 0xFu;
}
__device__ __forceinline__ u32 cand_bits(uint4 A, uint4 B, u32 fm) {
  const u32 w[6] = {A.x, A.y, A.z, A.w, B.x, B.y};
  u32 m = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    u32 h = type_nibble(w[i]);
    while (h) {
      const u32 k = __ffs(h) - 1;
      h &= h - 1;
      const u32 v = k == 0 ? __builtin_amdgcn_alignbyte(w[i + 1], w[i], 3)
                           : __builtin_amdgcn_alignbyte(w[i + 2], w[i + 1], k - 1);
      const u32 sz = __builtin_bswap32(v);
      if (fm == 0 || sz <= fm - 8) m |= 1u << (4 * i + k);
    }
  }
  return m;
}
__device__ __forceinline__ uint4 shift_pair(uint4 a, uint4 b, u32 sh) {
  const u32 q = sh >> 2, r = sh & 3;
  const bool q2 = (q & 2) != 0, q1 = (q & 1) != 0;
  const u32 s0 = q2 ? a.z : a.x, s1 = q2 ? a.w : a.y, s2 = q2 ? b.x : a.z;
  const u32 s3 = q2 ? b.y : a.w, s4 = q2 ? b.z : b.x, s5 = q2 ? b.w : b.y;
  const u32 w0 = q1 ? s1 : s0, w1 = q1 ? s2 : s1, w2 = q1 ? s3 : s2, w3 = q1 ? s4 : s3, w4 = q1 ? s5 : s4;
  if (!r) return make_uint4(w0, w1, w2, w3);
  return make_uint4(__builtin_amdgcn_alignbyte(w1, w0, r), __builtin_amdgcn_alignbyte(w2, w1, r),
                    __builtin_amdgcn_alignbyte(w3, w2, r), __builtin_amdgcn_alignbyte(w4, w3, r));
}
__device__ __forceinline__ uint4 shfl_down4(uint4 v) {
  return make_uint4(__shfl_down(v.x, 1), __shfl_down(v.y, 1), __shfl_down(v.z, 1), __shfl_down(v.w, 1));
}

// V: 0 load, 1 +shift, 2 +stage, 3 +copy, 4 +cand
template <int V>
__global__ __launch_bounds__(NT) void k_screen(const uint4* in, uint4* work, u32* sink, u32 sh) {
  __shared__ uint4 stage[NW + 2];
  __shared__ unsigned short am[NW];
  const u32 tid = threadIdx.x, ln = tid & 63, s = blockIdx.x;
  const uint4* N = in + (size_t)s * (NW + 4);
  uint4* WD = work + (size_t)s * (NW + 4);
  u32 acc = 0;
  for (u32 cb = tid - ln; cb < NW; cb += NT * 4) {
    uint4 x[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const u32 c = cb + ln + k * NT;
      x[k] = c <= NW ? N[c] : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const u32 c = cb + ln + k * NT;
      uint4 v = x[k];
      if (V >= 1) {
        uint4 nx = shfl_down4(x[k]);
        if (ln == 63 && c + 1 <= NW) nx = N[c + 1];
        v = shift_pair(x[k], nx, sh);
      }
      if (c < NW) {
        if (V >= 2) stage[c] = v;
        if (V >= 3) WD[c] = v;
        if (V >= 4) {
          uint4 y = shfl_down4(v);
          if (ln == 63) y = shift_pair(N[c + 1], N[c + 2], sh);
          am[c] = (unsigned short)cand_bits(v, y, 131072);
        }
        if (V < 2) acc ^= v.x ^ v.y ^ v.z ^ v.w;
      }
    }
  }
  __syncthreads();
  if (V >= 2) acc ^= stage[tid].x;
  if (V >= 4) acc ^= am[tid];
  if (acc == 0x12345678u) sink[s] = acc;   // keep the work
}

template <int V>
float run(const uint4* in, uint4* work, u32* sink, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(k_screen<V>, dim3(NSEG), dim3(NT), 0, 0, in, work, sink, 5u);
  CK(hipEventRecord(a, 0));
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(k_screen<V>, dim3(NSEG), dim3(NT), 0, 0, in, work, sink, 5u);
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms * 1000.f / reps;
}

int main() {
  const size_t words = (size_t)NSEG * (NW + 4);
  std::vector<uint4> h(words);
  srand(7);
  for (auto& w : h) w = make_uint4(rand(), rand(), rand(), rand());
  uint4 *in, *work;
  u32* sink;
  CK(hipMalloc(&in, words * 16));
  CK(hipMalloc(&work, words * 16));
  CK(hipMalloc(&sink, NSEG * 4));
  CK(hipMemcpy(in, h.data(), words * 16, hipMemcpyHostToDevice));
  const int reps = 200;
  printf("screen of %u segments x %u KB, %u threads per block (us per launch, incl. launch)\n", NSEG, SEG >> 10, NT);
  printf("load          %7.2f\n", run<0>(in, work, sink, reps));
  printf("+shift        %7.2f\n", run<1>(in, work, sink, reps));
  printf("+stage (LDS)  %7.2f\n", run<2>(in, work, sink, reps));
  printf("+copy (HBM)   %7.2f\n", run<3>(in, work, sink, reps));
  printf("+cand         %7.2f\n", run<4>(in, work, sink, reps));
  return 0;
}
