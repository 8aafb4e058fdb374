// hlc_field.hpp -- secp256k1 base-field (mod p) and scalar-field (mod n) arithmetic for
// gfx950, one 256-bit value per lane in 8 x 32-bit little-endian limbs.
//
// Replaces the arithmetic of k256 0.13.4 (FieldElement / Scalar) that
// `VerifyingKey::recover_from_prehash` runs behind /root/reference/src/signing/ethereum.rs:89.
//
// Design (CDNA4):
//  * products use v_mad_u64_u32 (32x32+64 -> 64, half-rate on gfx950, measured
//    profiles/r01_ubench_int.txt) with its carry-out folded by one full-rate v_addc:
//    product scanning, 64 MACs per 256x256 product, 36 per square;
//  * mod p: pseudo-Mersenne fold 2^256 == 2^32 + 977 (two folds, one conditional subtract);
//    all field values are kept fully reduced (< p) so equality tests are limb compares;
//  * mod n: Montgomery multiplication (R = 2^256) over 29-bit limbs (hlc_scmul.hpp; 8 x 32 CIOS
//    through round 6), used for the few scalar ops per vote (r^-1, u1, u2, GLV split products).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hlc_field_asm.hpp"
#include "hlc_modinv.hpp"
#include "hlc_scmul.hpp"

#define HLC_DEV __device__ __forceinline__

namespace hlc {

struct fe {
  uint32_t v[8];
};

// ------------------------------------------------------------------------------------
// constants
// ------------------------------------------------------------------------------------
HLC_DEV uint32_t n_limb(int i) {
  const uint32_t n0 = 0xD0364141u, n1 = 0xBFD25E8Cu, n2 = 0xAF48A03Bu, n3 = 0xBAAEDCE6u,
                 n4 = 0xFFFFFFFEu;
  return i == 0 ? n0 : i == 1 ? n1 : i == 2 ? n2 : i == 3 ? n3 : i == 4 ? n4 : 0xFFFFFFFFu;
}
// (n-1)/2, the high-s threshold used by alloy's normalized_s
HLC_DEV uint32_t nhalf_limb(int i) {
  const uint32_t h[8] = {0x681B20A0u, 0xDFE92F46u, 0x57A4501Du, 0x5D576E73u,
                         0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0x7FFFFFFFu};
  return h[i];
}

// ------------------------------------------------------------------------------------
// limb primitives
// ------------------------------------------------------------------------------------
HLC_DEV uint32_t add_cc(uint32_t a, uint32_t b, uint32_t& carry) {
  uint64_t s = (uint64_t)a + b + carry;
  carry = (uint32_t)(s >> 32);
  return (uint32_t)s;
}
HLC_DEV uint32_t sub_cc(uint32_t a, uint32_t b, uint32_t& borrow) {
  uint64_t d = (uint64_t)a - b - borrow;
  borrow = (uint32_t)(d >> 63);
  return (uint32_t)d;
}

HLC_DEV bool fe_is_zero(const fe& a) {
  uint32_t x = a.v[0];
#pragma unroll
  for (int i = 1; i < 8; ++i) x |= a.v[i];
  return x == 0;
}
HLC_DEV void fe_set(fe& r, uint32_t x) {
  r.v[0] = x;
#pragma unroll
  for (int i = 1; i < 8; ++i) r.v[i] = 0;
}
HLC_DEV void fe_cmov(fe& r, const fe& a, bool c) {
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = c ? a.v[i] : r.v[i];
}
// a < b as 256-bit integers
HLC_DEV bool u256_lt(const fe& a, const fe& b) {
  uint32_t borrow = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) sub_cc(a.v[i], b.v[i], borrow);
  return borrow != 0;
}

// ------------------------------------------------------------------------------------
// mod p -- LAZY representation: a field value is any 256-bit integer congruent to it mod p
// (i.e. in [0, 2^256), so possibly in [p, 2^256)).  Products, sums and differences are
// reduced only back into [0, 2^256) with the fold 2^256 == K = 2^32 + 977; values are made
// canonical (< p) only where a comparison, a parity or an output needs it (fe_normalize,
// fe_is_zero_modp, fe_eq_modp).  Carry chains use __builtin_addc/subc (v_add_co/v_addc with
// SGPR carries); the rare carry propagations past limb 1-2 sit behind a divergent branch that
// the whole wave skips when no lane needs it.
// ------------------------------------------------------------------------------------
HLC_DEV uint32_t adc(uint32_t a, uint32_t b, uint32_t& c) {
  uint32_t co;
  uint32_t r = __builtin_addc(a, b, c, &co);
  c = co;
  return r;
}
HLC_DEV uint32_t sbb(uint32_t a, uint32_t b, uint32_t& c) {
  uint32_t co;
  uint32_t r = __builtin_subc(a, b, c, &co);
  c = co;
  return r;
}

// s += K (s < K on entry: cannot overflow)
HLC_DEV void fe_add_k(uint32_t s[8]) {
  uint32_t c = 0;
  s[0] = adc(s[0], 0x3D1u, c);
  s[1] = adc(s[1], 1u, c);
#pragma unroll
  for (int i = 2; i < 8; ++i) s[i] = adc(s[i], 0u, c);
}

// s (256 bits) + c*2^256 with c in {0, 1} -> [0, 2^256)
HLC_DEV void fe_fold_carry(uint32_t s[8], uint32_t c) {
  uint32_t c2 = 0;
  s[0] = adc(s[0], c * 0x3D1u, c2);
  s[1] = adc(s[1], c, c2);
  if (c2) {  // rare: the fold carries past limb 1
#pragma unroll
    for (int i = 2; i < 8; ++i) s[i] = adc(s[i], 0u, c2);
    if (c2) fe_add_k(s);  // both operands were >= p: one more fold
  }
}

// s (256 bits) - b*2^256 with b in {0, 1} -> [0, 2^256)
HLC_DEV void fe_fold_borrow(uint32_t d[8], uint32_t b) {
  uint32_t b2 = 0;
  d[0] = sbb(d[0], b * 0x3D1u, b2);
  d[1] = sbb(d[1], b, b2);
  if (b2) {  // rare
#pragma unroll
    for (int i = 2; i < 8; ++i) d[i] = sbb(d[i], 0u, b2);
    if (b2) {  // d was < K: subtract K once more (no further borrow)
      uint32_t b3 = 0;
      d[0] = sbb(d[0], 0x3D1u, b3);
      d[1] = sbb(d[1], 1u, b3);
#pragma unroll
      for (int i = 2; i < 8; ++i) d[i] = sbb(d[i], 0u, b3);
    }
  }
}

HLC_DEV void fe_add(fe& r, const fe& a, const fe& b) {
  uint32_t c = 0, s[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) s[i] = adc(a.v[i], b.v[i], c);
  fe_fold_carry(s, c);
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = s[i];
}

HLC_DEV void fe_sub(fe& r, const fe& a, const fe& b) {
  uint32_t bw = 0, d[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) d[i] = sbb(a.v[i], b.v[i], bw);
  fe_fold_borrow(d, bw);
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = d[i];
}

HLC_DEV void fe_neg(fe& r, const fe& a) {
  fe z;
  fe_set(z, 0);
  fe_sub(r, z, a);
}

// r = 2^sh * a, 1 <= sh <= 3 (shift + fold of the sh top bits: e*2^256 == e*K, e < 8)
template <int SH>
HLC_DEV void fe_shl(fe& r, const fe& a) {
  uint32_t s[8];
  const uint32_t e = a.v[7] >> (32 - SH);
#pragma unroll
  for (int i = 7; i > 0; --i) s[i] = __builtin_amdgcn_alignbit(a.v[i], a.v[i - 1], 32 - SH);
  s[0] = a.v[0] << SH;
  uint32_t c2 = 0;
  s[0] = adc(s[0], e * 0x3D1u, c2);
  s[1] = adc(s[1], e, c2);
  if (c2) {
#pragma unroll
    for (int i = 2; i < 8; ++i) s[i] = adc(s[i], 0u, c2);
    if (c2) fe_add_k(s);
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = s[i];
}

HLC_DEV void fe_dbl(fe& r, const fe& a) { fe_shl<1>(r, a); }

// canonical representative (< p): a >= p  <=>  a + K overflows 2^256
HLC_DEV void fe_normalize(fe& r, const fe& a) {
  uint32_t c = 0, t[8];
  t[0] = adc(a.v[0], 0x3D1u, c);
  t[1] = adc(a.v[1], 1u, c);
#pragma unroll
  for (int i = 2; i < 8; ++i) t[i] = adc(a.v[i], 0u, c);
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = c ? t[i] : a.v[i];
}

// a == 0 (mod p), i.e. a in {0, p}
HLC_DEV bool fe_is_zero_modp(const fe& a) {
  uint32_t z = a.v[0], hi = a.v[2];
#pragma unroll
  for (int i = 1; i < 8; ++i) z |= a.v[i];
#pragma unroll
  for (int i = 3; i < 8; ++i) hi &= a.v[i];
  const bool is_p = (a.v[0] == 0xFFFFFC2Fu) & (a.v[1] == 0xFFFFFFFEu) & (hi == 0xFFFFFFFFu);
  return (z == 0) | is_p;
}

HLC_DEV bool fe_eq_modp(const fe& a, const fe& b) {
  fe d;
  fe_sub(d, a, b);
  return fe_is_zero_modp(d);
}

// c3 (<= 2) is the carry out of limb 2 of the fused reduction in hlc_field_asm.hpp: almost always
// 0, so its propagation sits behind a branch the whole wave skips.
HLC_DEV void fe_fix_top(uint32_t r[8], uint32_t c3) {
  if (c3) {
    uint32_t c = 0;
    r[3] = adc(r[3], c3, c);
#pragma unroll
    for (int i = 4; i < 8; ++i) r[i] = adc(r[i], 0u, c);
    if (c) fe_add_k(r);  // the value was within 2^67 of 2^256: one more fold, no further carry
  }
}

HLC_DEV void mul512(uint32_t t[16], const fe& a, const fe& b) { mul512_asm(t, a.v, b.v); }

// r = a * b, r = a^2: product scan with the pseudo-Mersenne reduction interleaved (asm)
HLC_DEV void fe_mul(fe& r, const fe& a, const fe& b) {
  uint32_t c3;
  fe_mul_asm(r.v, c3, a.v, b.v);
  fe_fix_top(r.v, c3);
}

HLC_DEV void fe_sqr(fe& r, const fe& a) {
  uint32_t c3;
  fe_sqr_asm(r.v, c3, a.v);
  fe_fix_top(r.v, c3);
}

// r = a^(2^n) -- one call site per loop keeps code size bounded
HLC_DEV void fe_sqr_n(fe& r, const fe& a, int n) {
  r = a;
  for (int i = 0; i < n; ++i) fe_sqr(r, r);
}

// Addition-chain prefix of the square root exponent (p+1)/4.
HLC_DEV void fe_chain223(const fe& a, fe& x2, fe& x3, fe& x22, fe& x223) {
  fe t, x6, x9, x11, x44, x88, x176, x220;
  fe_sqr(t, a);
  fe_mul(x2, t, a);
  fe_sqr(t, x2);
  fe_mul(x3, t, a);
  fe_sqr_n(t, x3, 3);
  fe_mul(x6, t, x3);
  fe_sqr_n(t, x6, 3);
  fe_mul(x9, t, x3);
  fe_sqr_n(t, x9, 2);
  fe_mul(x11, t, x2);
  fe_sqr_n(t, x11, 11);
  fe_mul(x22, t, x11);
  fe_sqr_n(t, x22, 22);
  fe_mul(x44, t, x22);
  fe_sqr_n(t, x44, 44);
  fe_mul(x88, t, x44);
  fe_sqr_n(t, x88, 88);
  fe_mul(x176, t, x88);
  fe_sqr_n(t, x176, 44);
  fe_mul(x220, t, x44);
  fe_sqr_n(t, x220, 3);
  fe_mul(x223, t, x3);
}

// r = a^-1 mod p (a != 0 mod p), canonical: safegcd divsteps (hlc_modinv.hpp)
HLC_DEV void fe_inv(fe& r, const fe& a) {
  fe n;
  fe_normalize(n, a);
  modinv_safegcd(r.v, n.v, modinfo_p());
}

// r = a^((p+1)/4), canonical; returns whether r^2 == a (a is a quadratic residue)
HLC_DEV bool fe_sqrt(fe& r, const fe& a) {
  fe x2, x3, x22, x223, t;
  fe_chain223(a, x2, x3, x22, x223);
  fe_sqr_n(t, x223, 23);
  fe_mul(t, t, x22);
  fe_sqr_n(t, t, 6);
  fe_mul(t, t, x2);
  fe_sqr_n(r, t, 2);
  fe_normalize(r, r);
  fe_sqr(t, r);
  return fe_eq_modp(t, a);
}

// ------------------------------------------------------------------------------------
// mod n (Montgomery, R = 2^256)
// ------------------------------------------------------------------------------------
static constexpr uint32_t N0INV = 0x5588B13Fu;  // -n^-1 mod 2^32

// r = a*b*R^-1 mod n   (CIOS; inputs < n, output < n)
#ifndef HLC_SC_CIOS
#define HLC_SC_CIOS 0  // 1: the A/B arm with the 8 x 32 CIOS form below (through round 6)
#endif
#if !HLC_SC_CIOS
// a b 2^-256 mod n by 29-bit limbs (hlc_scmul.hpp): the same result as the CIOS form, ~2.3x fewer instructions
HLC_DEV void sc_mont_mul(fe& r, const fe& a, const fe& b) { sc_mont_mul29(r.v, a.v, b.v); }
#else
HLC_DEV void sc_mont_mul(fe& r, const fe& a, const fe& b) {
  uint32_t t[10];
#pragma unroll
  for (int i = 0; i < 10; ++i) t[i] = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    uint64_t c = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      c += (uint64_t)a.v[j] * b.v[i] + t[j];
      t[j] = (uint32_t)c;
      c >>= 32;
    }
    c += t[8];
    t[8] = (uint32_t)c;
    t[9] = (uint32_t)(c >> 32);
    uint32_t m = t[0] * N0INV;
    c = (uint64_t)m * n_limb(0) + t[0];
    c >>= 32;
#pragma unroll
    for (int j = 1; j < 8; ++j) {
      c += (uint64_t)m * n_limb(j) + t[j];
      t[j - 1] = (uint32_t)c;
      c >>= 32;
    }
    c += t[8];
    t[7] = (uint32_t)c;
    t[8] = t[9] + (uint32_t)(c >> 32);
  }
  // conditional subtract n
  uint32_t bw = 0, d[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) d[i] = sub_cc(t[i], n_limb(i), bw);
  bool use_d = (t[8] != 0) || (bw == 0);
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = use_d ? d[i] : t[i];
}
#endif

// r = x mod n for any 256-bit x (n > 2^255 so one conditional subtract suffices)
HLC_DEV void sc_reduce(fe& r, const fe& x) {
  uint32_t bw = 0, d[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) d[i] = sub_cc(x.v[i], n_limb(i), bw);
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = bw ? x.v[i] : d[i];
}

HLC_DEV bool sc_is_ge_n(const fe& x) {
  uint32_t bw = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) sub_cc(x.v[i], n_limb(i), bw);
  return bw == 0;
}

HLC_DEV void sc_neg(fe& r, const fe& a) {
  uint32_t bw = 0, d[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) d[i] = sub_cc(n_limb(i), a.v[i], bw);
  bool z = fe_is_zero(a);
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = z ? 0u : d[i];
}

HLC_DEV void sc_add(fe& r, const fe& a, const fe& b) {
  uint32_t c = 0, s[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) s[i] = add_cc(a.v[i], b.v[i], c);
  uint32_t bw = 0, d[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) d[i] = sub_cc(s[i], n_limb(i), bw);
  bool use_d = c || !bw;
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = use_d ? d[i] : s[i];
}

// R^2 mod n, for conversion into the Montgomery domain
HLC_DEV void sc_r2(fe& r) {
  const uint32_t k[8] = {0x67D7D140u, 0x896CF214u, 0x0E7CF878u, 0x741496C2u,
                         0x5BCD07C6u, 0xE697F5E4u, 0x81C69BC5u, 0x9D671CD5u};
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = k[i];
}

// r = a^-1 mod n (a in [1, n)): safegcd divsteps
HLC_DEV void sc_inv(fe& r, const fe& a) { modinv_safegcd(r.v, a.v, modinfo_n()); }

}  // namespace hlc
