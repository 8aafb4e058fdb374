// Integer VALU throughput microbenchmark for gfx950 (MI355X).
// Measures wave64 issue throughput of the instructions the secp256k1 field
// arithmetic is built from, so the "VALU integer peak" used by bench.py's
// roofline is a measured number, not a guess.
//
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/ubench_int tools/ubench_int.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); return 1; } } while (0)

constexpr int ITERS = 4096;

// 8 independent chains per lane, 8 instructions of the measured kind per iteration.
__global__ void k_add(uint32_t* out, uint32_t seed) {
  uint32_t a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t b = seed | 1;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile(
        "v_add_u32 %0, %0, %8\n v_add_u32 %1, %1, %8\n v_add_u32 %2, %2, %8\n v_add_u32 %3, %3, %8\n"
        "v_add_u32 %4, %4, %8\n v_add_u32 %5, %5, %8\n v_add_u32 %6, %6, %8\n v_add_u32 %7, %7, %8\n"
        : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void k_addc(uint32_t* out, uint32_t seed) {
  // add-with-carry pairs (v_add_co_u32 / v_addc_co_u32): 4 pairs per iteration = 8 instrs
  uint32_t a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t b = seed | 1;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile(
        "v_add_co_u32 %0, vcc, %0, %8\n v_addc_co_u32 %1, vcc, %1, %8, vcc\n"
        "v_add_co_u32 %2, vcc, %2, %8\n v_addc_co_u32 %3, vcc, %3, %8, vcc\n"
        "v_add_co_u32 %4, vcc, %4, %8\n v_addc_co_u32 %5, vcc, %5, %8, vcc\n"
        "v_add_co_u32 %6, vcc, %6, %8\n v_addc_co_u32 %7, vcc, %7, %8, vcc\n"
        : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b) : "vcc");
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void k_mullo(uint32_t* out, uint32_t seed) {
  uint32_t a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t b = seed | 1;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile(
        "v_mul_lo_u32 %0, %0, %8\n v_mul_lo_u32 %1, %1, %8\n v_mul_lo_u32 %2, %2, %8\n v_mul_lo_u32 %3, %3, %8\n"
        "v_mul_lo_u32 %4, %4, %8\n v_mul_lo_u32 %5, %5, %8\n v_mul_lo_u32 %6, %6, %8\n v_mul_lo_u32 %7, %7, %8\n"
        : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void k_mulhi(uint32_t* out, uint32_t seed) {
  uint32_t a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t b = seed | 1;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile(
        "v_mul_hi_u32 %0, %0, %8\n v_mul_hi_u32 %1, %1, %8\n v_mul_hi_u32 %2, %2, %8\n v_mul_hi_u32 %3, %3, %8\n"
        "v_mul_hi_u32 %4, %4, %8\n v_mul_hi_u32 %5, %5, %8\n v_mul_hi_u32 %6, %6, %8\n v_mul_hi_u32 %7, %7, %8\n"
        : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void k_mad64(uint32_t* out, uint32_t seed) {
  // v_mad_u64_u32 D64 = S0*S1 + S2_64, 8 independent 64-bit accumulators
  uint64_t a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t b = seed | 1, c = seed * 3u + 7u;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile(
        "v_mad_u64_u32 %0, s[0:1], %8, %9, %0\n v_mad_u64_u32 %1, s[0:1], %8, %9, %1\n"
        "v_mad_u64_u32 %2, s[0:1], %8, %9, %2\n v_mad_u64_u32 %3, s[0:1], %8, %9, %3\n"
        "v_mad_u64_u32 %4, s[0:1], %8, %9, %4\n v_mad_u64_u32 %5, s[0:1], %8, %9, %5\n"
        "v_mad_u64_u32 %6, s[0:1], %8, %9, %6\n v_mad_u64_u32 %7, s[0:1], %8, %9, %7\n"
        : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b), "v"(c) : "s0", "s1");
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}

__global__ void k_cndmask(uint32_t* out, uint32_t seed) {
  uint32_t a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t b = seed | 1;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile(
        "v_cmp_gt_u32 vcc, %0, %8\n"
        "v_cndmask_b32 %1, %1, %8, vcc\n v_cndmask_b32 %2, %2, %8, vcc\n v_cndmask_b32 %3, %3, %8, vcc\n"
        "v_cndmask_b32 %4, %4, %8, vcc\n v_cndmask_b32 %5, %5, %8, vcc\n v_cndmask_b32 %6, %6, %8, vcc\n v_cndmask_b32 %7, %7, %8, vcc\n"
        "v_xor_b32 %0, %0, %7\n"
        : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b) : "vcc");
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

typedef void (*kfn)(uint32_t*, uint32_t);

static int run(const char* name, kfn k, int blocks, int threads, uint32_t* d) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, d, 12345u);  // warm
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(e0));
  const int reps = 5;
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, d, 777u + r);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  double instr_lane = (double)blocks * threads * ITERS * 8.0 * reps;  // lane-instructions
  double rate = instr_lane / (ms * 1e-3);                           // lane-instr/s
  // per-SIMD wave-instruction cycles at 2.4 GHz: 256 CU * 4 SIMD
  double wave_instr_per_s = rate / 64.0;
  double cyc_per_wave_instr = (256.0 * 4.0 * 2.4e9) / wave_instr_per_s;
  printf("%-10s blocks=%5d thr=%4d  %8.3f ms  %8.2f T lane-instr/s  ~%.2f cyc/wave-instr/SIMD @2.4GHz\n",
         name, blocks, threads, ms / reps, rate / 1e12, cyc_per_wave_instr);
  return 0;
}

int main() {
  uint32_t* d;
  int blocks = 256 * 8, threads = 256;
  CHECK(hipMalloc(&d, sizeof(uint32_t) * blocks * threads));
  int rc = 0;
  rc |= run("add_u32", k_add, blocks, threads, d);
  rc |= run("addc_pair", k_addc, blocks, threads, d);
  rc |= run("mul_lo", k_mullo, blocks, threads, d);
  rc |= run("mul_hi", k_mulhi, blocks, threads, d);
  rc |= run("mad_u64", k_mad64, blocks, threads, d);
  rc |= run("cndmask", k_cndmask, blocks, threads, d);
  // occupancy sweep for mad_u64 (waves per SIMD = threads*blocks/(256*4*64) approx)
  rc |= run("mad_u64", k_mad64, 256, 256, d);
  rc |= run("mad_u64", k_mad64, 512, 256, d);
  rc |= run("add_u32", k_add, 256, 256, d);
  rc |= run("add_u32", k_add, 512, 256, d);
  CHECK(hipFree(d));
  return rc;
}
