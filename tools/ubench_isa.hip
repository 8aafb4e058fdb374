// Issue cost of single gfx950 VALU instructions in wave64 (MI355X), the inputs of the field-layer
// design: 8 independent chains per lane, 8 instructions of one kind per loop
// iteration, 2048 blocks x 256 threads (8 waves/SIMD).  Reports cycles per wave-instruction per
// SIMD at the measured shader clock (from clock64 / wall time of one kernel).
//
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/ubench_isa tools/ubench_isa.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CHECK(x)                                                                                  \
  do {                                                                                            \
    hipError_t e = (x);                                                                           \
    if (e != hipSuccess) {                                                                        \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__);       \
      return 1;                                                                                   \
    }                                                                                             \
  } while (0)

constexpr int ITERS = 2048;

// 32-bit ops on 8 accumulators a0..a7 with operands b (v), c (v)
#define K32(NAME, INS)                                                                              \
  __global__ void NAME(uint32_t* out, uint32_t seed) {                                              \
    uint32_t a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, \
             a6 = a0 + 6, a7 = a0 + 7;                                                              \
    uint32_t b = seed | 1, c = seed * 3u + 7u;                                                      \
    for (int i = 0; i < ITERS; ++i) {                                                               \
      asm volatile(INS(0) INS(1) INS(2) INS(3) INS(4) INS(5) INS(6) INS(7)                          \
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) \
                   : "v"(b), "v"(c)                                                                 \
                   : "vcc", "s0", "s1");                                                            \
    }                                                                                               \
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;             \
  }

#define S(x) #x
#define I_ADD(k) "v_add_u32 %" S(k) ", %" S(k) ", %8\n"
#define I_ADD3(k) "v_add3_u32 %" S(k) ", %" S(k) ", %8, %9\n"
#define I_AND(k) "v_and_b32 %" S(k) ", %" S(k) ", %8\n"
#define I_LSHR(k) "v_lshrrev_b32 %" S(k) ", 29, %" S(k) "\n"
#define I_ALIGN(k) "v_alignbit_b32 %" S(k) ", %" S(k) ", %8, 29\n"
#define I_BFE(k) "v_bfe_u32 %" S(k) ", %" S(k) ", 3, 29\n"
#define I_LSHLADD(k) "v_lshl_add_u32 %" S(k) ", %" S(k) ", 3, %8\n"
#define I_MUL24(k) "v_mul_u32_u24 %" S(k) ", %" S(k) ", %8\n"
#define I_MULHI24(k) "v_mul_hi_u32_u24 %" S(k) ", %" S(k) ", %8\n"
#define I_MAD24(k) "v_mad_u32_u24 %" S(k) ", %" S(k) ", %8, %9\n"
#define I_MULLO(k) "v_mul_lo_u32 %" S(k) ", %" S(k) ", %8\n"
#define I_ADDCO(k) "v_add_co_u32 %" S(k) ", s[0:1], %" S(k) ", %8\n"
#define I_ADDCO_VCC(k) "v_add_co_u32 %" S(k) ", vcc, %" S(k) ", %8\n"
#define I_ADDC(k) "v_addc_co_u32 %" S(k) ", vcc, %" S(k) ", %8, vcc\n"
#define I_CND(k) "v_cndmask_b32 %" S(k) ", %" S(k) ", %8, vcc\n"
#define I_MOV(k) "v_mov_b32 %" S(k) ", %8\n"
#define I_XOR(k) "v_xor_b32 %" S(k) ", %" S(k) ", %8\n"
#define I_PERM(k) "v_perm_b32 %" S(k) ", %" S(k) ", %8, %9\n"
#define I_ANDLIT(k) "v_and_b32 %" S(k) ", 0x1fffffff, %" S(k) "\n"
#define I_ADDE64(k) "v_add_u32_e64 %" S(k) ", %" S(k) ", %8\n"
#define I_ANDSG(k) "v_and_b32 %" S(k) ", s2, %" S(k) "\n"
#define I_SUB(k) "v_sub_u32 %" S(k) ", %" S(k) ", %8\n"

K32(k_add, I_ADD)
K32(k_add3, I_ADD3)
K32(k_and, I_AND)
K32(k_lshr, I_LSHR)
K32(k_align, I_ALIGN)
K32(k_bfe, I_BFE)
K32(k_lshladd, I_LSHLADD)
K32(k_mul24, I_MUL24)
K32(k_mulhi24, I_MULHI24)
K32(k_mad24, I_MAD24)
K32(k_mullo, I_MULLO)
K32(k_addco, I_ADDCO)
K32(k_addco_vcc, I_ADDCO_VCC)
K32(k_addc, I_ADDC)
K32(k_cnd, I_CND)
K32(k_mov, I_MOV)
K32(k_xor, I_XOR)
K32(k_perm, I_PERM)
K32(k_sub, I_SUB)
K32(k_andlit, I_ANDLIT)
K32(k_adde64, I_ADDE64)
K32(k_andsg, I_ANDSG)

// 64-bit ops on 8 accumulators
#define K64(NAME, INS)                                                                              \
  __global__ void NAME(uint32_t* out, uint32_t seed) {                                              \
    uint64_t a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, \
             a6 = a0 + 6, a7 = a0 + 7;                                                              \
    uint32_t b = seed | 1, c = seed * 3u + 7u;                                                      \
    uint64_t d = ((uint64_t)c << 32) | b;                                                           \
    for (int i = 0; i < ITERS; ++i) {                                                               \
      asm volatile(INS(0) INS(1) INS(2) INS(3) INS(4) INS(5) INS(6) INS(7)                          \
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) \
                   : "v"(b), "v"(c), "v"(d)                                                         \
                   : "s0", "s1");                                                                   \
    }                                                                                               \
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7); \
  }
#define I_MAD64(k) "v_mad_u64_u32 %" S(k) ", s[0:1], %8, %9, %" S(k) "\n"
#define I_LSHR64(k) "v_lshrrev_b64 %" S(k) ", 29, %" S(k) "\n"
#define I_LSHLADD64(k) "v_lshl_add_u64 %" S(k) ", %" S(k) ", 2, %10\n"
#define I_ADDF64(k) "v_add_f64 %" S(k) ", %" S(k) ", %10\n"
#define I_FMAF64(k) "v_fma_f64 %" S(k) ", %" S(k) ", %10, %10\n"
K64(k_mad64, I_MAD64)
K64(k_lshr64, I_LSHR64)
K64(k_lshladd64, I_LSHLADD64)
K64(k_addf64, I_ADDF64)
K64(k_fmaf64, I_FMAF64)

// a mixed stream: 1 mad_u64 + 1 and + 1 alignbit + 1 add per group (the unsaturated column pattern)
__global__ void k_mix_col(uint32_t* out, uint32_t seed) {
  uint64_t a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
  uint32_t l0 = 0, l1 = 0, l2 = 0, l3 = 0;
  uint32_t b = seed | 1, c = seed * 3u + 7u;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile(
        "v_mad_u64_u32 %0, s[0:1], %8, %9, %0\n v_mad_u64_u32 %1, s[0:1], %8, %9, %1\n"
        "v_mad_u64_u32 %2, s[0:1], %8, %9, %2\n v_mad_u64_u32 %3, s[0:1], %8, %9, %3\n"
        "v_and_b32 %4, 0x1fffffff, %4\n v_and_b32 %5, 0x1fffffff, %5\n"
        "v_add_u32 %6, %6, %8\n v_add_u32 %7, %7, %8\n"
        : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(l0), "+v"(l1), "+v"(l2), "+v"(l3)
        : "v"(b), "v"(c)
        : "s0", "s1");
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(a0 ^ a1 ^ a2 ^ a3) ^ l0 ^ l1 ^ l2 ^ l3;
}

// the same mix with the 29-bit mask in a VGPR (%10) instead of a literal
__global__ void k_mix_col_vmask(uint32_t* out, uint32_t seed) {
  uint64_t a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
  uint32_t l0 = 0, l1 = 0, l2 = 0, l3 = 0;
  uint32_t b = seed | 1, c = seed * 3u + 7u, mask = 0x1fffffffu ^ (seed & 0x40000000u);
  for (int i = 0; i < ITERS; ++i) {
    asm volatile(
        "v_mad_u64_u32 %0, s[0:1], %8, %9, %0\n v_mad_u64_u32 %1, s[0:1], %8, %9, %1\n"
        "v_mad_u64_u32 %2, s[0:1], %8, %9, %2\n v_mad_u64_u32 %3, s[0:1], %8, %9, %3\n"
        "v_and_b32 %4, %10, %4\n v_and_b32 %5, %10, %5\n"
        "v_add_u32 %6, %6, %8\n v_add_u32 %7, %7, %8\n"
        : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(l0), "+v"(l1), "+v"(l2), "+v"(l3)
        : "v"(b), "v"(c), "v"(mask)
        : "s0", "s1");
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(a0 ^ a1 ^ a2 ^ a3) ^ l0 ^ l1 ^ l2 ^ l3;
}

// grouping: 8 mads then 8 cheap ops (ands / adds on other registers) vs mad / cheap alternating
#define MIXK(NAME, BODY)                                                                            \
  __global__ void NAME(uint32_t* out, uint32_t seed) {                                              \
    uint64_t a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, \
             a6 = a0 + 6, a7 = a0 + 7;                                                              \
    uint32_t l0 = 0, l1 = 1, l2 = 2, l3 = 3, l4 = 4, l5 = 5, l6 = 6, l7 = 7;                         \
    uint32_t b = seed | 1, c = seed * 3u + 7u;                                                      \
    for (int i = 0; i < ITERS; ++i) {                                                               \
      asm volatile(BODY                                                                             \
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7), \
                     "+v"(l0), "+v"(l1), "+v"(l2), "+v"(l3), "+v"(l4), "+v"(l5), "+v"(l6), "+v"(l7)  \
                   : "v"(b), "v"(c)                                                                 \
                   : "s0", "s1");                                                                   \
    }                                                                                               \
    out[blockIdx.x * blockDim.x + threadIdx.x] =                                                    \
        (uint32_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7) ^ l0 ^ l1 ^ l2 ^ l3 ^ l4 ^ l5 ^ l6 ^ l7;  \
  }
#define M_(k) "v_mad_u64_u32 %" S(k) ", s[0:1], %16, %17, %" S(k) "\n"
#define A_(k) "v_and_b32 %" S(k) ", 0x1fffffff, %" S(k) "\n"
MIXK(k_grp8, M_(0) M_(1) M_(2) M_(3) M_(4) M_(5) M_(6) M_(7) A_(8) A_(9) A_(10) A_(11) A_(12) A_(13) A_(14) A_(15))
MIXK(k_alt8, M_(0) A_(8) M_(1) A_(9) M_(2) A_(10) M_(3) A_(11) M_(4) A_(12) M_(5) A_(13) M_(6) A_(14) M_(7) A_(15))
MIXK(k_grp2, M_(0) M_(1) A_(8) A_(9) M_(2) M_(3) A_(10) A_(11) M_(4) M_(5) A_(12) A_(13) M_(6) M_(7) A_(14) A_(15))

// v_mad_u64_u32 with one SGPR source (a wave-uniform constant, as in the field layer's folds)
__global__ void k_mad64_sgpr(uint32_t* out, uint32_t seed) {
  uint64_t a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
           a7 = a0 + 7;
  uint32_t b = seed | 1;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile(
        "s_mov_b32 s2, 31264\n"
        "v_mad_u64_u32 %0, s[0:1], %8, s2, %0\n v_mad_u64_u32 %1, s[0:1], %8, s2, %1\n"
        "v_mad_u64_u32 %2, s[0:1], %8, s2, %2\n v_mad_u64_u32 %3, s[0:1], %8, s2, %3\n"
        "v_mad_u64_u32 %4, s[0:1], %8, s2, %4\n v_mad_u64_u32 %5, s[0:1], %8, s2, %5\n"
        "v_mad_u64_u32 %6, s[0:1], %8, s2, %6\n v_mad_u64_u32 %7, s[0:1], %8, s2, %7\n"
        : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
        : "v"(b)
        : "s0", "s1", "s2");
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}

__global__ void k_clock(unsigned long long* out) {
  unsigned long long t0 = clock64();
  unsigned long long w0 = wall_clock64();
  uint32_t x = threadIdx.x;
  for (int i = 0; i < 1 << 20; ++i) x = x * 1664525u + 1013904223u;
  unsigned long long t1 = clock64();
  unsigned long long w1 = wall_clock64();
  if (threadIdx.x == 0) {
    out[0] = t1 - t0;
    out[1] = w1 - w0;
    out[2] = x;
  }
}

typedef void (*kfn)(uint32_t*, uint32_t);

static double g_ghz = 2.4;

static int run(const char* name, kfn k, uint32_t* d, int instr_per_iter = 8) {
  const int blocks = 256 * 8, threads = 256;
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, d, 12345u);
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(e0));
  const int reps = 5;
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, d, 777u + r);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  const double wave_instr = (double)blocks * threads / 64.0 * ITERS * instr_per_iter * reps;
  const double per_simd = wave_instr / (256.0 * 4.0);
  const double cycles = ms * 1e-3 * g_ghz * 1e9;
  printf("%-12s %8.3f ms  %6.2f cyc/wave-instr/SIMD @%.2f GHz\n", name, ms / reps, cycles / per_simd, g_ghz);
  return 0;
}

int main() {
  uint32_t* d;
  unsigned long long* c;
  CHECK(hipMalloc(&d, sizeof(uint32_t) * 256 * 8 * 256));
  CHECK(hipMalloc(&c, 64));
  // shader clock: clock64 ticks vs the 100 MHz wall clock over one long single-wave loop
  hipLaunchKernelGGL(k_clock, dim3(1), dim3(64), 0, 0, c);
  CHECK(hipDeviceSynchronize());
  unsigned long long h[3];
  CHECK(hipMemcpy(h, c, sizeof h, hipMemcpyDeviceToHost));
  g_ghz = (double)h[0] / ((double)h[1] / 100e6) / 1e9;
  printf("shader clock estimate: %.3f GHz (clock64 %llu ticks over %llu wall ticks)\n", g_ghz, h[0], h[1]);
  int rc = 0;
  rc |= run("add_u32", k_add, d);
  rc |= run("sub_u32", k_sub, d);
  rc |= run("add3_u32", k_add3, d);
  rc |= run("and_b32", k_and, d);
  rc |= run("xor_b32", k_xor, d);
  rc |= run("and_b32 literal", k_andlit, d);
  rc |= run("and_b32 sgpr", k_andsg, d);
  rc |= run("add_u32_e64 (VOP3 enc)", k_adde64, d);
  rc |= run("mov_b32", k_mov, d);
  rc |= run("lshrrev_b32", k_lshr, d);
  rc |= run("alignbit", k_align, d);
  rc |= run("bfe_u32", k_bfe, d);
  rc |= run("lshl_add_u32", k_lshladd, d);
  rc |= run("perm_b32", k_perm, d);
  rc |= run("mul_u32_u24", k_mul24, d);
  rc |= run("mulhi_u24", k_mulhi24, d);
  rc |= run("mad_u32_u24", k_mad24, d);
  rc |= run("mul_lo_u32", k_mullo, d);
  rc |= run("add_co_sgpr", k_addco, d);
  rc |= run("add_co_vcc", k_addco_vcc, d);
  rc |= run("addc_chain", k_addc, d);
  rc |= run("cndmask_vcc", k_cnd, d);
  rc |= run("mad_u64_u32", k_mad64, d);
  rc |= run("lshrrev_b64", k_lshr64, d);
  rc |= run("lshl_add_u64", k_lshladd64, d);
  rc |= run("add_f64", k_addf64, d);
  rc |= run("fma_f64", k_fmaf64, d);
  rc |= run("mix4mad+4cheap", k_mix_col, d);
  rc |= run("mix4mad+4cheap vmask", k_mix_col_vmask, d);
  rc |= run("mad_u64_u32 sgpr", k_mad64_sgpr, d);
  rc |= run("8 mad, 8 and", k_grp8, d, 16);
  rc |= run("mad/and alternating", k_alt8, d, 16);
  rc |= run("2 mad, 2 and", k_grp2, d, 16);
  CHECK(hipFree(d));
  return rc;
}
