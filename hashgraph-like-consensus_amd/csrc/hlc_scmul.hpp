// hlc_scmul.hpp -- Montgomery multiplication modulo the secp256k1 group order n over 29-bit limbs, the
// scalar products of the recovery's prep stage (r^-1 by Montgomery's trick, u2 = s r^-1, the GLV split)
// and of u1 = -z r^-1 (k256 0.13.4 Scalar arithmetic behind /root/reference/src/signing/ethereum.rs:89).
// Host-compilable (tests/test_modinv_host.py checks it against Python integers).
//
// sc_mont_mul29(r, a, b) returns exactly what the 8 x 32 CIOS form did (hlc_field.hpp sc_mont_mul through
// round 6): t = (a b + M n) / 2^256 with M = -a b n^-1 mod 2^256, then t - n when t >= n.  The CIOS form
// carried every 32 x 32 product through 64-bit adds with zero-extended operand pairs (732 VALU instructions
// on gfx950, 435 of them v_mov_b32).  Here the product columns of 29-bit limbs (< 2^58 each, at most 18 of
// them per column) accumulate in 64 bits with no carries, one v_mad_u64_u32 per product; the reduction runs
// digit-serially, 9 steps of 29 bits over x = 32 a, so it divides by 2^261 and 32 a b 2^-261 = a b 2^-256.
// Its t' = (32 a b + M' n) / 2^261 (M' = -32 a b n^-1 mod 2^261) lies in [a b / 2^256, a b / 2^256 + n) as
// t does, and both are congruent to a b 2^-256 mod n: the same integer.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#endif
#ifndef HLC_HD
#if defined(__HIPCC__)
#define HLC_HD __host__ __device__ __forceinline__
#else
#define HLC_HD inline
#endif
#endif

namespace hlc {

namespace scmul {
constexpr uint32_t M29 = 0x1FFFFFFFu;
constexpr uint32_t NINV29 = 0x1588B13Fu;  // -n^-1 mod 2^29
HLC_HD uint32_t n29(int k) {               // n in 9 limbs of 29 bits
  return k == 0 ? 0x10364141u : k == 1 ? 0x1E92F466u : k == 2 ? 0x12280EEFu : k == 3 ? 0x1DB9CD5Eu
       : k == 4 ? 0x1FFFEBAAu : k == 8 ? 0x00FFFFFFu : 0x1FFFFFFFu;
}
HLC_HD uint32_t n32(int k) {
  return k == 0 ? 0xD0364141u : k == 1 ? 0xBFD25E8Cu : k == 2 ? 0xAF48A03Bu : k == 3 ? 0xBAAEDCE6u
       : k == 4 ? 0xFFFFFFFEu : 0xFFFFFFFFu;
}
// bits [s, s + 29) of the 256-bit w (zeros below bit 0 and above bit 255); s is a constant after unrolling
HLC_HD uint32_t bits29(const uint32_t w[8], int s) {
  if (s < 0) return (w[0] << (-s)) & M29;
  const int q = s >> 5, off = s & 31;
  const uint64_t lo = q < 8 ? w[q] : 0u, hi = q + 1 < 8 ? w[q + 1] : 0u;
  return (uint32_t)(((hi << 32) | lo) >> off) & M29;
}
}  // namespace scmul

HLC_HD void sc_mont_mul29(uint32_t r[8], const uint32_t a[8], const uint32_t b[8]) {
  using namespace scmul;
  uint32_t x[9], y[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    x[k] = bits29(a, 29 * k - 5);  // 32 a
    y[k] = bits29(b, 29 * k);
  }
  uint64_t c[17];
#pragma unroll
  for (int k = 0; k < 17; ++k) c[k] = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i)
#pragma unroll
    for (int j = 0; j < 9; ++j) c[i + j] += (uint64_t)x[i] * y[j];
  // REDC, 29 bits per step: m makes the column's low 29 bits zero; the rest carries into the next column
  uint64_t carry = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const uint64_t ci = c[i] + carry;
    const uint32_t m = ((uint32_t)ci * NINV29) & M29;
    carry = (ci + (uint64_t)m * n29(0)) >> 29;
#pragma unroll
    for (int j = 1; j < 9; ++j) c[i + j] += (uint64_t)m * n29(j);
  }
  // t' = carry + sum_{k >= 9} c[k] 2^(29 (k - 9)) < 2^257, normalised to 29-bit limbs, then 8 x 32 + the top
  uint32_t t[9];
  uint64_t acc = carry;
#pragma unroll
  for (int k = 9; k < 17; ++k) {
    acc += c[k];
    t[k - 9] = (uint32_t)acc & M29;
    acc >>= 29;
  }
  t[8] = (uint32_t)acc;  // bits 232 .. 256 (t' < 2^257)
  uint32_t w[9];
#pragma unroll
  for (int j = 0; j < 9; ++j) {
    const int s = 32 * j, k = s / 29, off = s % 29;  // word j: limbs k, k + 1 (and k + 2) from bit off
    uint64_t v = (uint64_t)t[k] >> off;
    if (k + 1 < 9) v |= (uint64_t)t[k + 1] << (29 - off);
    if (k + 2 < 9 && 58 - off < 32) v |= (uint64_t)t[k + 2] << (58 - off);
    w[j] = (uint32_t)v;
  }
  // t' - n when t' >= n (t' < 2n for a, b < n; the CIOS form's single conditional subtract otherwise too)
  uint32_t d[8], bw = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const uint64_t df = (uint64_t)w[k] - n32(k) - bw;
    d[k] = (uint32_t)df;
    bw = (uint32_t)(df >> 63);
  }
  const uint32_t use_d = (w[8] != 0u) | (bw == 0u);
  const uint32_t mask = 0u - use_d;
#pragma unroll
  for (int k = 0; k < 8; ++k) r[k] = w[k] ^ ((w[k] ^ d[k]) & mask);
}

}  // namespace hlc
