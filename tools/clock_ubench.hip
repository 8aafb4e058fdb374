// clock_ubench.hip -- the shader clock the chip holds under k_rec_main's own point-operation mix,
// measured the way MI355X_MICROARCH.md 'DVFS give-back' item 6 prescribes: back-to-back launches
// for >= 2 s, then one stamped launch; clock = delta s_memtime / delta s_memrealtime x 100 MHz,
// median over workgroups.  The loop body is the u2 R chain's window: 5 doublings + 2 mixed
// additions (gej29_double / gej29_madd<false>, the shipped 29-bit field layer).
//
// Modes (argv[1]):  "rand"  per-lane random points (what the kernel sees)
//                   "same"  every lane of the chip on the SAME point (low toggle activity)
// argv[2] = waves per SIMD (3 = k_rec_main's occupancy), argv[3] = seconds of back-to-back launches.
// Stamps go to a buffer of their own (never an output); the result sink is separate.
//
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -o tools/clock_ubench tools/clock_ubench.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../hashgraph-like-consensus_amd/csrc/hlc_fe29.hpp"
#include "../hashgraph-like-consensus_amd/csrc/hlc_point29.hpp"

using namespace hlc;

#define CHECK(x)                                                                \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

constexpr int TPB = 256;

__device__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16; x *= 0x7FEB352Du; x ^= x >> 15; x *= 0x846CA68Bu; x ^= x >> 16;
  return x;
}
__device__ void seed29r(fe29& a, uint32_t s) {
#pragma unroll
  for (int i = 0; i < 9; ++i) a.v[i] = mix32(s * 9u + (uint32_t)i + 0x1234567u) & M29;
  a.v[8] &= 0xFFFFFFu;
}

// iters windows of (5 doublings + 2 mixed additions) per lane; stamps[2b], stamps[2b+1] =
// (memtime, memrealtime) deltas of workgroup b's lane 0 around the loop.
__global__ void __launch_bounds__(TPB, 2) k_window(uint32_t* sink, unsigned long long* stamps, int iters, int same) {
  const uint32_t t = same ? 1u : blockIdx.x * TPB + threadIdx.x;
  gej29 p;
  ge29 q1, q2;
  seed29r(p.x, t);
  seed29r(p.y, t + 0x100000u);
  seed29r(p.z, t + 0x200000u);
  seed29r(q1.x, t + 0x300000u);
  seed29r(q1.y, t + 0x400000u);
  seed29r(q2.x, t + 0x500000u);
  seed29r(q2.y, t + 0x600000u);
  p.inf = 0;
  const unsigned long long c0 = __builtin_amdgcn_s_memtime(), w0 = __builtin_amdgcn_s_memrealtime();
#pragma unroll 1
  for (int k = 0; k < iters; ++k) {
#pragma unroll 1
    for (int d = 0; d < 5; ++d) gej29_double(p, p);
    gej29_madd<false>(p, p, q1);
    gej29_madd<false>(p, p, q2);
  }
  const unsigned long long c1 = __builtin_amdgcn_s_memtime(), w1 = __builtin_amdgcn_s_memrealtime();
  uint32_t x = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) x ^= p.x.v[i] ^ p.y.v[i] ^ p.z.v[i];
  sink[blockIdx.x * TPB + threadIdx.x] = x;
  if (threadIdx.x == 0) {
    stamps[2 * blockIdx.x] = c1 - c0;
    stamps[2 * blockIdx.x + 1] = w1 - w0;
  }
}

int main(int argc, char** argv) {
  const int same = argc > 1 && std::strcmp(argv[1], "same") == 0;
  const int waves = argc > 2 ? std::atoi(argv[2]) : 3;
  const double seconds = argc > 3 ? std::atof(argv[3]) : 3.0;
  const int iters = argc > 4 ? std::atoi(argv[4]) : 150;
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int blocks = cus * waves;  // 256 threads = one wave on each of the CU's 4 SIMDs
  uint32_t* sink;
  unsigned long long* stamps;
  CHECK(hipMalloc(&sink, (size_t)blocks * TPB * 4));
  CHECK(hipMalloc(&stamps, (size_t)blocks * 16));
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  // back-to-back launches for `seconds`, timing each batch of 10
  auto t0 = std::chrono::steady_clock::now();
  int launches = 0;
  float last_ms = 0;
  for (;;) {
    CHECK(hipEventRecord(a));
    for (int k = 0; k < 10; ++k) hipLaunchKernelGGL(k_window, dim3(blocks), dim3(TPB), 0, 0, sink, stamps, iters, same);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    CHECK(hipEventElapsedTime(&last_ms, a, b));
    launches += 10;
    const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (el >= seconds) break;
  }
  CHECK(hipGetLastError());
  std::vector<unsigned long long> h((size_t)blocks * 2);
  CHECK(hipMemcpy(h.data(), stamps, h.size() * 8, hipMemcpyDeviceToHost));
  std::vector<double> ghz;
  for (int k = 0; k < blocks; ++k)
    if (h[2 * k + 1]) ghz.push_back((double)h[2 * k] / ((double)h[2 * k + 1] / 100e6) / 1e9);
  std::sort(ghz.begin(), ghz.end());
  const double med = ghz.empty() ? 0 : ghz[ghz.size() / 2];
  // issue cost of the loop: instructions per window from the ISA (1087 x 5 + 1750 x 2 = 8935)
  const double win_ns = last_ms / 10.0 * 1e6 / iters;  // one window of all resident waves
  printf("clock_ubench mode=%s waves/SIMD=%d launches=%d (%.1f s back-to-back) ms/launch=%.3f "
         "median clock %.3f GHz (min %.3f, max %.3f) window %.1f ns -> %.2f SIMD-cycles per window-wave at that clock\n",
         same ? "same" : "rand", waves, launches, seconds, last_ms / 10.0, med, ghz.empty() ? 0 : ghz.front(),
         ghz.empty() ? 0 : ghz.back(), win_ns, win_ns * med / waves);
  CHECK(hipFree(sink));
  CHECK(hipFree(stamps));
  return 0;
}
