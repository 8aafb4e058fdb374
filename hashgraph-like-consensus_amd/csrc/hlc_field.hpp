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
//  * mod n: Montgomery multiplication (CIOS, R = 2^256), used for the few scalar ops
//    per vote (r^-1, u1, u2, GLV split products).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hlc_modinv.hpp"

#define HLC_DEV __device__ __forceinline__

namespace hlc {

struct fe {
  uint32_t v[8];
};

// ------------------------------------------------------------------------------------
// constants
// ------------------------------------------------------------------------------------
__constant__ static const uint32_t P_LIMBS[8] = {0xFFFFFC2Fu, 0xFFFFFFFEu, 0xFFFFFFFFu, 0xFFFFFFFFu,
                                                  0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
__constant__ static const uint32_t N_LIMBS[8] = {0xD0364141u, 0xBFD25E8Cu, 0xAF48A03Bu, 0xBAAEDCE6u,
                                                  0xFFFFFFFEu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};

HLC_DEV uint32_t p_limb(int i) {
  return i == 0 ? 0xFFFFFC2Fu : (i == 1 ? 0xFFFFFFFEu : 0xFFFFFFFFu);
}
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
// acc(64) += a*b with the 65th bit carried into hi (v_mad_u64_u32 carry-out + v_addc).
HLC_DEV void mac(uint64_t& acc, uint32_t& hi, uint32_t a, uint32_t b) {
  uint64_t c;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc), "=s"(c) : "v"(a), "v"(b));
  asm("v_addc_co_u32_e64 %0, %1, 0, %0, %1" : "+v"(hi), "+s"(c));
}

// acc(64) += 2*a*b (for squaring off-diagonals): two MACs
HLC_DEV void mac2(uint64_t& acc, uint32_t& hi, uint32_t a, uint32_t b) {
  mac(acc, hi, a, b);
  mac(acc, hi, a, b);
}

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
HLC_DEV bool fe_eq(const fe& a, const fe& b) {
  uint32_t x = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) x |= a.v[i] ^ b.v[i];
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
// mod p
// ------------------------------------------------------------------------------------
// r = x - p if x >= p (x < 2^256): x >= p  <=>  x + (2^32+977) overflows 2^256
HLC_DEV void fe_final_sub(fe& r, const uint32_t x[8], uint32_t extra_carry) {
  uint32_t c = 0, t[8];
  t[0] = add_cc(x[0], 0x3D1u, c);
  t[1] = add_cc(x[1], 0x1u, c);
#pragma unroll
  for (int i = 2; i < 8; ++i) t[i] = add_cc(x[i], 0u, c);
  bool ge = (c | extra_carry) != 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = ge ? t[i] : x[i];
}

HLC_DEV void fe_add(fe& r, const fe& a, const fe& b) {
  uint32_t c = 0, s[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) s[i] = add_cc(a.v[i], b.v[i], c);
  fe_final_sub(r, s, c);
}

HLC_DEV void fe_sub(fe& r, const fe& a, const fe& b) {
  uint32_t bw = 0, d[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) d[i] = sub_cc(a.v[i], b.v[i], bw);
  // if borrow: d += p  (== d - (2^32+977) mod 2^256)
  uint32_t bw2 = 0, t[8];
  t[0] = sub_cc(d[0], 0x3D1u, bw2);
  t[1] = sub_cc(d[1], 0x1u, bw2);
#pragma unroll
  for (int i = 2; i < 8; ++i) t[i] = sub_cc(d[i], 0u, bw2);
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = bw ? t[i] : d[i];
}

HLC_DEV void fe_neg(fe& r, const fe& a) {
  fe z;
  fe_set(z, 0);
  fe_sub(r, z, a);
}

HLC_DEV void fe_dbl(fe& r, const fe& a) { fe_add(r, a, a); }

// reduce a 512-bit product t[16] mod p
HLC_DEV void fe_reduce512(fe& r, const uint32_t t[16]) {
  // x = lo + hi*977 + hi*2^32
  uint32_t x[8];
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    c += (uint64_t)t[8 + i] * 977u + t[i];
    if (i > 0) c += t[7 + i];
    x[i] = (uint32_t)c;
    c >>= 32;
  }
  c += t[15];  // T < 2^33: the part at 2^256
  // fold T*(2^32 + 977) into x
  uint64_t e = (c & 0xFFFFFFFFull) * 977u + x[0];
  x[0] = (uint32_t)e;
  e >>= 32;
  e += (uint64_t)(uint32_t)(c >> 32) * 977u + (uint32_t)c + x[1];
  x[1] = (uint32_t)e;
  e >>= 32;
  e += (uint32_t)(c >> 32) + (uint64_t)x[2];
  x[2] = (uint32_t)e;
  uint32_t cc = (uint32_t)(e >> 32);
#pragma unroll
  for (int i = 3; i < 8; ++i) x[i] = add_cc(x[i], 0u, cc);
  // overflow out of 2^256 (only possible when x was near 2^256): add 2^32+977 once more;
  // the result is then tiny and cannot overflow again.
  uint32_t c2 = 0, y[8];
  y[0] = add_cc(x[0], cc ? 0x3D1u : 0u, c2);
  y[1] = add_cc(x[1], cc ? 0x1u : 0u, c2);
#pragma unroll
  for (int i = 2; i < 8; ++i) y[i] = add_cc(x[i], 0u, c2);
  fe_final_sub(r, y, 0);
}

HLC_DEV void mul512(uint32_t t[16], const fe& a, const fe& b) {
  uint64_t acc = 0;
  uint32_t hi = 0;
#pragma unroll
  for (int k = 0; k < 15; ++k) {
#pragma unroll
    for (int i = (k < 8 ? 0 : k - 7); i <= (k < 8 ? k : 7); ++i) mac(acc, hi, a.v[i], b.v[k - i]);
    t[k] = (uint32_t)acc;
    acc = (acc >> 32) | ((uint64_t)hi << 32);
    hi = 0;
  }
  t[15] = (uint32_t)acc;
}

// Squaring: 28 off-diagonal MACs (product scanning over the strict upper triangle),
// one 512-bit doubling (v_alignbit), then the 8 diagonal squares: 36 MACs instead of 64.
HLC_DEV void sqr512(uint32_t t[16], const fe& a) {
  uint32_t x[16];
  uint64_t acc = 0;
  uint32_t hi = 0;
  x[0] = 0;
#pragma unroll
  for (int k = 1; k < 14; ++k) {
#pragma unroll
    for (int i = (k < 8 ? 0 : k - 7); i < k - i; ++i) mac(acc, hi, a.v[i], a.v[k - i]);
    x[k] = (uint32_t)acc;
    acc = (acc >> 32) | ((uint64_t)hi << 32);
    hi = 0;
  }
  x[14] = (uint32_t)acc;
  x[15] = (uint32_t)(acc >> 32);
  // double
#pragma unroll
  for (int k = 15; k > 0; --k) x[k] = __builtin_amdgcn_alignbit(x[k], x[k - 1], 31);
  x[0] = 0;
  // add the diagonal squares a_i^2 at limb 2i with a carry chain
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    uint64_t d = (uint64_t)x[2 * i] | ((uint64_t)x[2 * i + 1] << 32);
    uint64_t sq = (uint64_t)a.v[i] * a.v[i];
    uint64_t s = d + sq;
    uint32_t c1 = s < sq;
    uint64_t s2 = s + c;
    uint32_t c2 = s2 < s;
    t[2 * i] = (uint32_t)s2;
    t[2 * i + 1] = (uint32_t)(s2 >> 32);
    c = c1 + c2;
  }
}

HLC_DEV void fe_mul(fe& r, const fe& a, const fe& b) {
  uint32_t t[16];
  mul512(t, a, b);
  fe_reduce512(r, t);
}

HLC_DEV void fe_sqr(fe& r, const fe& a) {
  uint32_t t[16];
  sqr512(t, a);
  fe_reduce512(r, t);
}

// r = a^(2^n) -- one call site per loop keeps code size bounded
HLC_DEV void fe_sqr_n(fe& r, const fe& a, int n) {
  r = a;
  for (int i = 0; i < n; ++i) fe_sqr(r, r);
}

// Addition-chain prefix shared by inversion (p-2) and square root ((p+1)/4).
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

// r = a^-1 mod p (a != 0): safegcd divsteps (hlc_modinv.hpp), ~5x cheaper than a^(p-2)
HLC_DEV void fe_inv(fe& r, const fe& a) { modinv_safegcd(r.v, a.v, modinfo_p()); }

// r = a^((p+1)/4); returns whether r^2 == a (a is a quadratic residue)
HLC_DEV bool fe_sqrt(fe& r, const fe& a) {
  fe x2, x3, x22, x223, t;
  fe_chain223(a, x2, x3, x22, x223);
  fe_sqr_n(t, x223, 23);
  fe_mul(t, t, x22);
  fe_sqr_n(t, t, 6);
  fe_mul(t, t, x2);
  fe_sqr_n(r, t, 2);
  fe_sqr(t, r);
  return fe_eq(t, a);
}

// ------------------------------------------------------------------------------------
// mod n (Montgomery, R = 2^256)
// ------------------------------------------------------------------------------------
static constexpr uint32_t N0INV = 0x5588B13Fu;  // -n^-1 mod 2^32

// r = a*b*R^-1 mod n   (CIOS; inputs < n, output < n)
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

HLC_DEV void sc_load_const(fe& r, const uint32_t* c) {
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = c[i];
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

// r = a*b mod n (plain domain) = mont(mont(a, b), R^2)
HLC_DEV void sc_mul(fe& r, const fe& a, const fe& b) {
  fe t, r2;
  sc_mont_mul(t, a, b);
  sc_r2(r2);
  sc_mont_mul(r, t, r2);
}

// big-endian 32 bytes <-> limbs
HLC_DEV void fe_from_be_words(fe& r, const uint32_t w_be[8]) {
  // w_be[0] holds bytes 0..3 (most significant) already as a big-endian-decoded u32
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = w_be[7 - i];
}

}  // namespace hlc
