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

__device__ void seed_fe(fe& a, uint32_t s) {
#pragma unroll
  for (int i = 0; i < 8; ++i) a.v[i] = ((s + 0x9E3779B9u * (i + 1)) * 0x85EBCA6Bu) ^ (s >> 3);
  a.v[7] &= 0x7FFFFFFFu;
}

__device__ void sink(uint32_t* out, uint32_t x) { out[blockIdx.x * TPB + threadIdx.x] = x; }
// shader clock during a kernel: block 0, lane 0 brackets its loop with clock64 (shader clock) and
// wall_clock64 (100 MHz)
__device__ unsigned long long g_clk[4];
__device__ void clk_mark(int k) {
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    g_clk[2 * k] = clock64();
    g_clk[2 * k + 1] = wall_clock64();
  }
}

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

// ---- batch inversion in SIMT: three ways to invert 64 x B values per wave ----
// (a) k_inv: one inversion per lane (B = 1).
// (b) k_inv_wavescan: Montgomery's trick ACROSS the 64 lanes (B = 1): inclusive prefix and suffix
//     products by __shfl_up / __shfl_down (6 steps each), ONE inversion of the wave's product
//     (every lane runs the same instruction stream), a_i^-1 = P_(i-1) S_(i+1) / prod.
// (c) k_inv_lanebatch: Montgomery's trick WITHIN each lane over B = 8 values (the recovery's
//     k_rec_prep / k_rec_final).
__device__ void shfl_up_fe(fe& r, const fe& a, int d) {
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = __shfl_up(a.v[i], d, 64);
}
__device__ void shfl_down_fe(fe& r, const fe& a, int d) {
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = __shfl_down(a.v[i], d, 64);
}
__device__ void shfl_fe(fe& r, const fe& a, int src) {
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = __shfl(a.v[i], src, 64);
}
__device__ void wave_batch_inv(fe& a) {
  const int lane = threadIdx.x & 63;
  fe P = a, S = a, t;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    shfl_up_fe(t, P, d);
    if (lane >= d) fe_mul(P, P, t);
  }
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    shfl_down_fe(t, S, d);
    if (lane + d < 64) fe_mul(S, S, t);
  }
  fe tot, ti, pe, se;
  shfl_fe(tot, P, 63);
  fe_inv(ti, tot);
  shfl_up_fe(pe, P, 1);
  shfl_down_fe(se, S, 1);
  if (lane == 0) fe_set(pe, 1);
  if (lane == 63) fe_set(se, 1);
  fe_mul(a, pe, se);
  fe_mul(a, a, ti);
}
__device__ void lane_batch_inv8(fe* a) {
  fe pre[8], acc;
  fe_set(acc, 1);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    pre[j] = acc;
    fe_mul(acc, acc, a[j]);
  }
  fe inv;
  fe_inv(inv, acc);
#pragma unroll
  for (int j = 7; j >= 0; --j) {
    fe t;
    fe_mul(t, pre[j], inv);
    fe_mul(inv, inv, a[j]);
    a[j] = t;
  }
}
__global__ void __launch_bounds__(TPB, 4) k_inv_wavescan(uint32_t* out, int iters) {
  fe a;
  seed_fe(a, threadIdx.x + blockIdx.x * TPB);
  a.v[0] |= 1u;
  for (int k = 0; k < iters; ++k) wave_batch_inv(a);
  uint32_t x = 0;
  for (int i = 0; i < 8; ++i) x ^= a.v[i];
  sink(out, x);
}
__global__ void __launch_bounds__(TPB, 4) k_inv_lanebatch(uint32_t* out, int iters) {
  fe a[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    seed_fe(a[j], threadIdx.x + blockIdx.x * TPB + 977u * j);
    a[j].v[0] |= 1u;
  }
  for (int k = 0; k < iters; ++k) lane_batch_inv8(a);
  uint32_t x = 0;
  for (int j = 0; j < 8; ++j)
    for (int i = 0; i < 8; ++i) x ^= a[j].v[i];
  sink(out, x);
}
// a * a^-1 == 1 for both batch forms (bad lanes counted)
__global__ void k_check_inv(uint32_t* bad) {
  fe a, b, one;
  seed_fe(a, threadIdx.x + blockIdx.x * blockDim.x + 12345u);
  a.v[0] |= 1u;
  b = a;
  wave_batch_inv(b);
  fe_mul(one, a, b);
  fe_normalize(one, one);
  uint32_t d = one.v[0] ^ 1u;
  for (int i = 1; i < 8; ++i) d |= one.v[i];
  fe v[8], w[8];
  for (int j = 0; j < 8; ++j) {
    seed_fe(v[j], threadIdx.x * 8 + j + 777u);
    v[j].v[0] |= 1u;
    w[j] = v[j];
  }
  lane_batch_inv8(w);
  for (int j = 0; j < 8; ++j) {
    fe_mul(one, v[j], w[j]);
    fe_normalize(one, one);
    d |= one.v[0] ^ 1u;
    for (int i = 1; i < 8; ++i) d |= one.v[i];
  }
  if (d) atomicAdd(bad, 1u);
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

// ---- 29-bit unsaturated layer (hlc_fe29.hpp) ----
__device__ void seed29(fe29& a, uint32_t s) {
#pragma unroll
  for (int i = 0; i < 9; ++i) a.v[i] = (((s + 0x9E3779B9u * (i + 1)) * 0x85EBCA6Bu) ^ (s >> 3)) & M29;
}
template <int W>
__global__ void __launch_bounds__(TPB, W) k_mul29(uint32_t* out, int iters) {
  fe29 a, b;
  seed29(a, threadIdx.x + blockIdx.x * TPB);
  seed29(b, 7 * threadIdx.x + 1);
  for (int k = 0; k < iters; ++k) fe29_mul(a, a, b);
  uint32_t x = 0;
  for (int i = 0; i < 9; ++i) x ^= a.v[i];
  sink(out, x);
}
template <int W>
__global__ void __launch_bounds__(TPB, W) k_sqr29(uint32_t* out, int iters) {
  fe29 a;
  seed29(a, threadIdx.x + blockIdx.x * TPB);
  for (int k = 0; k < iters; ++k) fe29_sqr(a, a);
  uint32_t x = 0;
  for (int i = 0; i < 9; ++i) x ^= a.v[i];
  sink(out, x);
}
__global__ void __launch_bounds__(TPB, 4) k_subsub29(uint32_t* out, int iters) {
  fe29 a, b;
  seed29(a, threadIdx.x + blockIdx.x * TPB);
  seed29(b, 7 * threadIdx.x + 1);
  for (int k = 0; k < iters; ++k) {
    fe29_sub(a, a, b);
    fe29_sub(b, b, a);
  }
  uint32_t x = 0;
  for (int i = 0; i < 9; ++i) x ^= a.v[i] ^ b.v[i];
  sink(out, x);
}
__global__ void __launch_bounds__(TPB, 4) k_subsub(uint32_t* out, int iters) {
  fe a, b;
  seed_fe(a, threadIdx.x + blockIdx.x * TPB);
  seed_fe(b, 7 * threadIdx.x + 1);
  for (int k = 0; k < iters; ++k) {
    fe_sub(a, a, b);
    fe_sub(b, b, a);
  }
  uint32_t x = 0;
  for (int i = 0; i < 8; ++i) x ^= a.v[i] ^ b.v[i];
  sink(out, x);
}

template <int W>
__global__ void __launch_bounds__(TPB, W) k_mul29ref(uint32_t* out, int iters) {
  fe29 a, b;
  seed29(a, threadIdx.x + blockIdx.x * TPB);
  seed29(b, 7 * threadIdx.x + 1);
  for (int k = 0; k < iters; ++k) fe29_mul_ref(a, a, b);
  uint32_t x = 0;
  for (int i = 0; i < 9; ++i) x ^= a.v[i];
  sink(out, x);
}

// two independent product chains: separate calls vs one interleaved dual schedule (fe29_mul2)
template <int DUAL>
__global__ void __launch_bounds__(TPB, 4) k_mul29x2(uint32_t* out, int iters) {
  fe29 a, b, c, e;
  seed29(a, threadIdx.x + blockIdx.x * TPB);
  seed29(b, 7 * threadIdx.x + 1);
  seed29(c, 5 * threadIdx.x + 3);
  seed29(e, 9 * threadIdx.x + 4);
  for (int k = 0; k < iters; ++k) {
    if (DUAL) {
      fe29_mul2(a, a, b, c, c, e);
    } else {
      fe29_mul(a, a, b);
      fe29_mul(c, c, e);
    }
  }
  uint32_t x = 0;
  for (int i = 0; i < 9; ++i) x ^= a.v[i] ^ c.v[i];
  sink(out, x);
}
template <int DUAL>
__global__ void __launch_bounds__(TPB, 4) k_sqr29x2(uint32_t* out, int iters) {
  fe29 a, c;
  seed29(a, threadIdx.x + blockIdx.x * TPB);
  seed29(c, 5 * threadIdx.x + 3);
  for (int k = 0; k < iters; ++k) {
    if (DUAL) {
      fe29_sqr2(a, a, c, c);
    } else {
      fe29_sqr(a, a);
      fe29_sqr(c, c);
    }
  }
  uint32_t x = 0;
  for (int i = 0; i < 9; ++i) x ^= a.v[i] ^ c.v[i];
  sink(out, x);
}

__global__ void __launch_bounds__(TPB, 4) k_dbl29(uint32_t* out, int iters) {
  gej29 p;
  seed29(p.x, threadIdx.x + blockIdx.x * TPB);
  seed29(p.y, 3 * threadIdx.x + 5);
  seed29(p.z, 11 * threadIdx.x + 2);
  p.inf = 0;
  clk_mark(0);
  for (int k = 0; k < iters; ++k) gej29_double(p, p);
  clk_mark(1);
  uint32_t x = 0;
  for (int i = 0; i < 9; ++i) x ^= p.x.v[i] ^ p.y.v[i] ^ p.z.v[i];
  sink(out, x);
}
template <bool EXACT>
__global__ void __launch_bounds__(TPB, 4) k_madd29(uint32_t* out, int iters) {
  gej29 p;
  ge29 q;
  seed29(p.x, threadIdx.x + blockIdx.x * TPB);
  seed29(p.y, 3 * threadIdx.x + 5);
  seed29(p.z, 11 * threadIdx.x + 2);
  seed29(q.x, 13 * threadIdx.x + 7);
  seed29(q.y, 17 * threadIdx.x + 9);
  p.inf = 0;
  clk_mark(0);
  for (int k = 0; k < iters; ++k) gej29_madd<EXACT>(p, p, q);
  clk_mark(1);
  uint32_t x = 0;
  for (int i = 0; i < 9; ++i) x ^= p.x.v[i] ^ p.y.v[i] ^ p.z.v[i];
  sink(out, x);
}

// asm schedule == C++ reference on random and extreme inputs (limbs < 2^30.35)
__device__ uint32_t hash32(uint32_t x) {
  x ^= x >> 16; x *= 0x7FEB352Du; x ^= x >> 15; x *= 0x846CA68Bu; x ^= x >> 16;
  return x;
}
__global__ void k_check29(uint32_t* bad, int rounds) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t MAXIN = 1367130551u;  // floor(2^30.35)
  for (int r = 0; r < rounds; ++r) {
    fe29 a, b, x, y;
    const uint32_t mode = hash32(t * 977u + r) & 7u;
    for (int i = 0; i < 9; ++i) {
      uint32_t ha = hash32(t * 131u + r * 7919u + i), hb = hash32(t * 337u + r * 104729u + i + 100);
      a.v[i] = mode == 0 ? MAXIN - (ha & 3u) : ha % MAXIN;
      b.v[i] = mode <= 1 ? MAXIN - (hb & 3u) : hb % MAXIN;
      if (mode == 2) a.v[i] = ha & M29;
    }
    fe29_mul(x, a, b);
    fe29_mul_ref(y, a, b);
    uint32_t d = 0;
    for (int i = 0; i < 9; ++i) d |= x.v[i] ^ y.v[i];
    fe29_sqr(x, a);
    fe29_sqr_ref(y, a);
    for (int i = 0; i < 9; ++i) d |= x.v[i] ^ y.v[i];
    // dual schedules: x = a b, y = b^2 (and a^2, b^2; a b, b a)
    fe29 x2, y2, xr, yr;
    fe29_mulsqr(x2, a, b, y2, b);
    fe29_mul_ref(xr, a, b);
    fe29_sqr_ref(yr, b);
    for (int i = 0; i < 9; ++i) d |= (x2.v[i] ^ xr.v[i]) | (y2.v[i] ^ yr.v[i]);
    fe29_sqr2(x2, a, y2, b);
    fe29_sqr_ref(xr, a);
    for (int i = 0; i < 9; ++i) d |= (x2.v[i] ^ xr.v[i]) | (y2.v[i] ^ yr.v[i]);
    fe29_mul2(x2, a, b, y2, b, a);
    fe29_mul_ref(xr, a, b);
    for (int i = 0; i < 9; ++i) d |= (x2.v[i] ^ xr.v[i]) | (y2.v[i] ^ xr.v[i]);
    // round 3: sum of two products (operands < 2^29: 18 products per column stay < 2^64) and a
    // product / square plus a 32-bit-limb addend
    fe29 c, e;
    uint32_t f[9];
    for (int i = 0; i < 9; ++i) {
      const uint32_t hc = hash32(t * 71u + r * 613u + i + 200), he = hash32(t * 53u + r * 389u + i + 300);
      c.v[i] = mode == 0 ? M29 - (hc & 3u) : hc & M29;
      e.v[i] = mode <= 1 ? M29 - (he & 3u) : he & M29;
      f[i] = mode == 3 ? 0xFFFFFFFFu - (hc & 7u) : hash32(he + i);
    }
    fe29 am, bm;
    for (int i = 0; i < 9; ++i) {
      am.v[i] = a.v[i] & M29;
      bm.v[i] = b.v[i] & M29;
    }
    fe29_muladd(x, am, bm, c, e);
    fe29_muladd_ref(y, am, bm, c, e);
    for (int i = 0; i < 9; ++i) d |= x.v[i] ^ y.v[i];
    fe29_mul_add(x, a, b, f);
    fe29_mul_add_ref(y, a, b, f, false);
    for (int i = 0; i < 9; ++i) d |= x.v[i] ^ y.v[i];
    fe29_sqr_add(x, a, f);
    fe29_mul_add_ref(y, a, a, f, true);
    for (int i = 0; i < 9; ++i) d |= x.v[i] ^ y.v[i];
    if (d) atomicAdd(bad, 1u);
  }
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
    double div;
  } r[] = {{"fe_mul", run(k_mul, d, blocks, iters), 1},
           {"fe_sqr", run(k_sqr, d, blocks, iters), 1},
           {"fe_add+fe_sub", run(k_addsub, d, blocks, iters), 1},
           {"gej_double", run(k_dbl, d, blocks, iters), 1},
           {"gej_add_ge", run(k_madd, d, blocks, iters), 1},
           {"fe_inv", run(k_inv, d, blocks, iters / 20), 0.05},
           {"fe_mul x2 ILP", run(k_mul_x2, d, blocks, iters), 1},
           {"fe_sub x2", run(k_subsub, d, blocks, iters), 1},
           {"fe29_mul", run(k_mul29<4>, d, blocks, iters), 1},
           {"fe29_sqr", run(k_sqr29<4>, d, blocks, iters), 1},
           {"fe29_sub x2", run(k_subsub29, d, blocks, iters), 1},
           {"fe29_mul (C++)", run(k_mul29ref<4>, d, blocks, iters), 1},
           {"fe29_mul x2 sep", run(k_mul29x2<0>, d, blocks, iters), 2},
           {"fe29_mul2 dual", run(k_mul29x2<1>, d, blocks, iters), 2},
           {"fe29_sqr x2 sep", run(k_sqr29x2<0>, d, blocks, iters), 2},
           {"fe29_sqr2 dual", run(k_sqr29x2<1>, d, blocks, iters), 2},
           {"gej29_double", run(k_dbl29, d, blocks, iters), 1},
           {"gej29_madd exact", run(k_madd29<true>, d, blocks, iters), 1},
           {"gej29_madd fast", run(k_madd29<false>, d, blocks, iters), 1}};
  for (auto& x : r) {
    const double ns = x.ms * 1e6 / iters / x.div;  // per op (div ops per iteration), 4 waves per SIMD
    printf("%-14s %8.3f ms  %8.1f ns/op  %8.1f SIMD-cycles/wave-op @%.2f GHz\n", x.name, x.ms, ns,
           ns * ghz / 4.0, ghz);
  }
  // 8 waves per SIMD: twice the blocks, twice the work per SIMD
  const float m8 = run(k_mul8, d, 2 * blocks, iters), s8 = run(k_sqr8, d, 2 * blocks, iters);
  printf("fe_mul @8w     %8.3f ms  %8.1f SIMD-cycles/wave-op\n", m8, m8 * 1e6 / iters * ghz / 8.0);
  printf("fe_sqr @8w     %8.3f ms  %8.1f SIMD-cycles/wave-op\n", s8, s8 * 1e6 / iters * ghz / 8.0);
  const float m29 = run(k_mul29<8>, d, 2 * blocks, iters), s29 = run(k_sqr29<8>, d, 2 * blocks, iters);
  printf("fe29_mul @8w   %8.3f ms  %8.1f SIMD-cycles/wave-op\n", m29, m29 * 1e6 / iters * ghz / 8.0);
  printf("fe29_sqr @8w   %8.3f ms  %8.1f SIMD-cycles/wave-op\n", s29, s29 * 1e6 / iters * ghz / 8.0);
  // batch inversion forms: ns per wave per 64 inverted values
  {
    const int it = iters / 20;
    const float ta = run(k_inv, d, blocks, it), tb = run(k_inv_wavescan, d, blocks, it),
                tc = run(k_inv_lanebatch, d, blocks, it);
    // 4 waves per SIMD in parallel: SIMD-time per wave-iteration = ms / it / 4
    printf("batch inversion, SIMD-ns per 64 values: per-lane fe_inv %.1f | wave scan (Montgomery across "
           "64 lanes, shfl) %.1f | per-lane batch of 8 %.1f\n",
           ta * 1e6 / it / 4.0, tb * 1e6 / it / 4.0, tc * 1e6 / it / 4.0 / 8.0);
    CHECK(hipMemset(d, 0, 4));
    hipLaunchKernelGGL(k_check_inv, dim3(blocks), dim3(TPB), 0, 0, d);
    uint32_t badi = 0;
    CHECK(hipMemcpy(&badi, d, 4, hipMemcpyDeviceToHost));
    printf("batch inversion check: %u bad lanes\n", badi);
    if (badi) return 1;
  }
  // shader clock under the full-chip point-operation loops (the sustained, power-limited clock)
  for (int which = 0; which < 2; ++which) {
    if (which == 0) {
      (void)run(k_dbl29, d, blocks, iters);
    } else {
      (void)run(k_madd29<false>, d, blocks, iters);
    }
    unsigned long long h[4];
    CHECK(hipMemcpyFromSymbol(h, HIP_SYMBOL(g_clk), sizeof h));
    printf("%s: sustained shader clock %.3f GHz\n", which ? "gej29_madd fast" : "gej29_double",
           (double)(h[2] - h[0]) / ((double)(h[3] - h[1]) / 100e6) / 1e9);
  }
  // one wave per SIMD (one 256-thread block per CU): how much a lone wave loses to latency
  const float d1 = run(k_dbl29, d, cus, iters), d4 = run(k_dbl29, d, blocks, iters);
  printf("gej29_double: 1 wave/SIMD %.3f ms, 4 waves/SIMD %.3f ms (lone-wave speed = %.2f of the 4-wave share)\n",
         d1, d4, d4 / 4.0 / d1);
  CHECK(hipMemset(d, 0, 4));
  hipLaunchKernelGGL(k_check29, dim3(blocks), dim3(TPB), 0, 0, d, 64);
  uint32_t bad = 0;
  CHECK(hipMemcpy(&bad, d, 4, hipMemcpyDeviceToHost));
  printf("fe29 asm vs C++ reference: %u mismatching lanes of %d (x64 rounds, mul + sqr + dual schedules + muladd + mul_add + sqr_add)\n", bad, blocks * TPB);
  CHECK(hipFree(d));
  return bad ? 1 : 0;
}
