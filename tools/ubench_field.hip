// ubench_field.hip -- cycle cost of the recovery's field / group operations on gfx950.
//
// Every lane runs ITERS dependent operations on its own data; the grid fills the chip at the
// recovery kernel's occupancy (4 blocks of 256 per CU = 4 waves per SIMD).  Reported per op:
// wall ns per wave-op and SIMD-cycles per wave-op at the given clock, to compare instruction
// counts against issue efficiency.
//
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -o tools/ubench_field tools/ubench_field.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "../hashgraph-like-consensus_amd/csrc/hlc_point.hpp"

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

__device__ void seed_fe(fe& a, uint32_t s) {
#pragma unroll
  for (int i = 0; i < 8; ++i) a.v[i] = ((s + 0x9E3779B9u * (i + 1)) * 0x85EBCA6Bu) ^ (s >> 3);
  a.v[7] &= 0x7FFFFFFFu;
}

__device__ void sink(uint32_t* out, uint32_t x) { out[blockIdx.x * TPB + threadIdx.x] = x; }

__global__ void __launch_bounds__(TPB, 4) k_mul(uint32_t* out, int iters) {
  fe a, b;
  seed_fe(a, threadIdx.x + blockIdx.x * TPB);
  seed_fe(b, 7 * threadIdx.x + 1);
  for (int k = 0; k < iters; ++k) fe_mul(a, a, b);
  uint32_t x = 0;
  for (int i = 0; i < 8; ++i) x ^= a.v[i];
  sink(out, x);
}

__global__ void __launch_bounds__(TPB, 4) k_sqr(uint32_t* out, int iters) {
  fe a;
  seed_fe(a, threadIdx.x + blockIdx.x * TPB);
  for (int k = 0; k < iters; ++k) fe_sqr(a, a);
  uint32_t x = 0;
  for (int i = 0; i < 8; ++i) x ^= a.v[i];
  sink(out, x);
}

__global__ void __launch_bounds__(TPB, 4) k_addsub(uint32_t* out, int iters) {
  fe a, b;
  seed_fe(a, threadIdx.x + blockIdx.x * TPB);
  seed_fe(b, 7 * threadIdx.x + 1);
  for (int k = 0; k < iters; ++k) {
    fe_add(a, a, b);
    fe_sub(b, b, a);
  }
  uint32_t x = 0;
  for (int i = 0; i < 8; ++i) x ^= a.v[i] ^ b.v[i];
  sink(out, x);
}

__global__ void __launch_bounds__(TPB, 4) k_dbl(uint32_t* out, int iters) {
  gej p;
  seed_fe(p.x, threadIdx.x + blockIdx.x * TPB);
  seed_fe(p.y, 3 * threadIdx.x + 5);
  seed_fe(p.z, 11 * threadIdx.x + 2);
  p.inf = 0;
  for (int k = 0; k < iters; ++k) gej_double(p, p);
  uint32_t x = 0;
  for (int i = 0; i < 8; ++i) x ^= p.x.v[i] ^ p.y.v[i] ^ p.z.v[i];
  sink(out, x);
}

__global__ void __launch_bounds__(TPB, 4) k_madd(uint32_t* out, int iters) {
  gej p;
  ge q;
  seed_fe(p.x, threadIdx.x + blockIdx.x * TPB);
  seed_fe(p.y, 3 * threadIdx.x + 5);
  seed_fe(p.z, 11 * threadIdx.x + 2);
  seed_fe(q.x, 13 * threadIdx.x + 7);
  seed_fe(q.y, 17 * threadIdx.x + 9);
  p.inf = 0;
  for (int k = 0; k < iters; ++k) gej_add_ge(p, p, q);
  uint32_t x = 0;
  for (int i = 0; i < 8; ++i) x ^= p.x.v[i] ^ p.y.v[i] ^ p.z.v[i];
  sink(out, x);
}

__global__ void __launch_bounds__(TPB, 4) k_inv(uint32_t* out, int iters) {
  fe a;
  seed_fe(a, threadIdx.x + blockIdx.x * TPB);
  for (int k = 0; k < iters; ++k) fe_inv(a, a);
  uint32_t x = 0;
  for (int i = 0; i < 8; ++i) x ^= a.v[i];
  sink(out, x);
}

// the same field ops at 8 waves per SIMD (latency vs throughput)
__global__ void __launch_bounds__(TPB, 8) k_mul8(uint32_t* out, int iters) {
  fe a, b;
  seed_fe(a, threadIdx.x + blockIdx.x * TPB);
  seed_fe(b, 7 * threadIdx.x + 1);
  for (int k = 0; k < iters; ++k) fe_mul(a, a, b);
  uint32_t x = 0;
  for (int i = 0; i < 8; ++i) x ^= a.v[i];
  sink(out, x);
}
__global__ void __launch_bounds__(TPB, 8) k_sqr8(uint32_t* out, int iters) {
  fe a;
  seed_fe(a, threadIdx.x + blockIdx.x * TPB);
  for (int k = 0; k < iters; ++k) fe_sqr(a, a);
  uint32_t x = 0;
  for (int i = 0; i < 8; ++i) x ^= a.v[i];
  sink(out, x);
}
// two independent chains per lane (ILP 2 at 4 waves per SIMD)
__global__ void __launch_bounds__(TPB, 4) k_mul_x2(uint32_t* out, int iters) {
  fe a, b, c;
  seed_fe(a, threadIdx.x + blockIdx.x * TPB);
  seed_fe(c, threadIdx.x + 3);
  seed_fe(b, 7 * threadIdx.x + 1);
  for (int k = 0; k < iters; ++k) {
    fe_mul(a, a, b);
    fe_mul(c, c, b);
  }
  uint32_t x = 0;
  for (int i = 0; i < 8; ++i) x ^= a.v[i] ^ c.v[i];
  sink(out, x);
}

template <typename K>
float run(K kern, uint32_t* d, int blocks, int iters) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(TPB), 0, 0, d, 4);
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(a));
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(TPB), 0, 0, d, iters);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, a, b));
  return ms;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 2000;
  const double ghz = argc > 2 ? atof(argv[2]) : 2.1;
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int blocks = cus * 4;
  uint32_t* d;
  CHECK(hipMalloc(&d, (size_t)blocks * 2 * TPB * 4));
  struct R {
    const char* name;
    float ms;
    int div;
  } r[] = {{"fe_mul", run(k_mul, d, blocks, iters), 1},
           {"fe_sqr", run(k_sqr, d, blocks, iters), 1},
           {"fe_add+fe_sub", run(k_addsub, d, blocks, iters), 1},
           {"gej_double", run(k_dbl, d, blocks, iters), 1},
           {"gej_add_ge", run(k_madd, d, blocks, iters), 1},
           {"fe_inv", run(k_inv, d, blocks, iters / 20), 20},
           {"fe_mul x2 ILP", run(k_mul_x2, d, blocks, iters), 1}};
  for (auto& x : r) {
    const double ns = x.ms * 1e6 / (iters / x.div);  // per op, 4 waves per SIMD in parallel
    printf("%-14s %8.3f ms  %8.1f ns/op  %8.1f SIMD-cycles/wave-op @%.2f GHz\n", x.name, x.ms, ns,
           ns * ghz / 4.0, ghz);
  }
  // 8 waves per SIMD: twice the blocks, twice the work per SIMD
  const float m8 = run(k_mul8, d, 2 * blocks, iters), s8 = run(k_sqr8, d, 2 * blocks, iters);
  printf("fe_mul @8w     %8.3f ms  %8.1f SIMD-cycles/wave-op\n", m8, m8 * 1e6 / iters * ghz / 8.0);
  printf("fe_sqr @8w     %8.3f ms  %8.1f SIMD-cycles/wave-op\n", s8, s8 * 1e6 / iters * ghz / 8.0);
  CHECK(hipFree(d));
  return 0;
}
