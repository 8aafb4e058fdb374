// hlc_fe29.hpp -- secp256k1 base-field arithmetic in nine unsaturated 29-bit limbs, tuned for the
// gfx950 VALU issue costs measured in profiles/r02_ubench_isa.txt:
//
//   * VOP2 integer ops (v_add_u32, v_sub_u32, v_and_b32, v_lshrrev_b32, v_mov_b32) issue in ~2.5
//     cycles per wave64 instruction; every VOP3 op -- including v_mad_u64_u32 AND every
//     carry-propagating add (v_add_co / v_addc, which write an SGPR carry mask) -- in ~4.4.
//   * The saturated 8 x 32-bit layout (hlc_field.hpp) pays one v_addc per v_mad_u64_u32: its
//     carry chains cost as much as its multiplications.
//   * Here every limb has 3 spare bits, so a column of nine 58-bit products accumulates in the
//     64-bit addend of v_mad_u64_u32 with NO carry instruction; a column is split with one
//     v_and_b32 + one 64-bit shift (v_alignbit + v_lshrrev); additions and subtractions are plain
//     per-limb VOP2 ops with one carry pass.
//
// Value = sum v[i] 2^(29 i), i < 9 (up to 2^261).  Reduction uses 2^261 == 2^37 + 31264 (mod p)
// (31264 = 32 * 977, 2^37 = 256 * 2^29).
//
// Magnitude contract (bounds are per limb):
//   MUL input       : every limb < 2^30.35 (nine products + carry-in < 2^64 per column).
//   mul/sqr output  : limbs < 2^29, except limb 2 < 2^29 + 2^19.            ("normalised")
//   add(n, n)       : < 2^30 + 2^15, a valid MUL input, NOT a valid add/sub input again.
//   sub(a, b)       : a, b any limbs < 2^30.4; output normalised (carry pass included).
//   dbl / mul_small : output normalised (carry pass included).
// fe29_normalize gives the canonical representative (< p) for comparisons, parity, output.
//
// Compiles for host and device (HLC_HD): tests/test_fe29_host.py checks every operation against
// Python integers at the magnitude bounds above (lib/libhlc_fe29_host.so).
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define HLC_HD __host__ __device__ __forceinline__
#else
#define HLC_HD inline
#endif

// Host test build (-DHLC_FE29_CHECK, tests/test_fe29_host.py): every lazy operation and every
// 64-bit column accumulation checks its magnitude contract in wider arithmetic and counts a
// violation instead of silently wrapping.  Compiles to nothing elsewhere.
#if defined(HLC_FE29_CHECK) && !defined(__HIP_DEVICE_COMPILE__)
extern "C" unsigned long long hlc_fe29_violations;
#define FE29_CHECK(c)                 \
  do {                                \
    if (!(c)) ++hlc_fe29_violations;  \
  } while (0)
#else
#define FE29_CHECK(c) \
  do {                \
  } while (0)
#endif

namespace hlc {

struct fe29 {
  uint32_t v[9];
};

constexpr uint32_t M29 = 0x1FFFFFFFu;
constexpr uint32_t FOLD_LO = 31264u;  // 2^261 mod p = 2^37 + 31264: 31264 at limb 0 ...
constexpr uint32_t FOLD_HI = 256u;    // ... and 256 at limb 1 (2^37 = 256 * 2^29)

// p in radix 2^29
HLC_HD uint32_t p29(int i) {
  return i == 0 ? 0x1FFFFC2Fu : i == 1 ? 0x1FFFFFF7u : i == 8 ? 0x00FFFFFFu : 0x1FFFFFFFu;
}
// 128 p with every limb in [2^31 - 5, 2^31.33]: added before a subtraction so that no limb of
// a + K - b goes negative for b limbs < 2^30.4 and none overflows 32 bits for a limbs < 2^30.4.
HLC_HD uint32_t k29(int i) {
  return i == 0 ? 0x9FFE1780u : i == 1 ? 0x9FFFFBFBu : i == 8 ? 0x7FFFFFFBu : 0x9FFFFFFBu;
}

HLC_HD void fe29_set(fe29& r, uint32_t x) {
  r.v[0] = x;
#pragma unroll
  for (int i = 1; i < 9; ++i) r.v[i] = 0;
}

// r = a + b (limbwise; see the contract)
HLC_HD void fe29_add(fe29& r, const fe29& a, const fe29& b) {
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    FE29_CHECK((uint64_t)a.v[i] + b.v[i] <= 0xFFFFFFFFull);
    r.v[i] = a.v[i] + b.v[i];
  }
}

// r = a << s limbwise, NO carry (lazy 2a / 4a / 8a: a valid MUL operand beside a normalised one
// while every limb stays < 2^31.8)
HLC_HD void fe29_shl(fe29& r, const fe29& a, int s) {
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    FE29_CHECK(((uint64_t)a.v[i] << s) <= 0xFFFFFFFFull);
    r.v[i] = a.v[i] << s;
  }
}

// one parallel carry step over limbs < 2^32 (no serial chain: every limb at once) with the 2^261
// fold of limb 8's carry: output limbs < 2^29 + 8, limb 0 < 2^29 + 2^18, limb 1 < 2^29 + 2^12
HLC_HD void fe29_carry(uint32_t d[9]) {
  uint32_t c[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    c[i] = d[i] >> 29;
    d[i] &= M29;
  }
#pragma unroll
  for (int i = 1; i < 9; ++i) d[i] += c[i - 1];
  d[0] += c[8] * FOLD_LO;
  d[1] += c[8] * FOLD_HI;
}

// 64 p with every limb in [2^30 - 62528, 2^30): the lazy subtraction's offset (b normalised).
HLC_HD uint32_t k64(int i) {
  return i == 0 ? 0x3FFF0BC0u : i == 1 ? 0x3FFFFDFEu : 0x3FFFFFFEu;
}

// r = a - b + 64 p, NO carry ("lazy"): b normalised (limbs < 2^29 + 2^19 + 8 < 64p's limbs), a limbs
// < 2^31.35.  For a normalised, r limbs < 2^30.59: a valid MUL operand when the other operand is
// normalised (2^30.59 * 2^29.01 * 9 < 2^64), a valid `a` of another lazy sub, input of
// fe29_carry (-> normalised) and of mul_small(2) (2 r < 2^31.6).  NOT a valid sqr input or `b`.
HLC_HD void fe29_sub_lazy(fe29& r, const fe29& a, const fe29& b) {
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    FE29_CHECK((uint64_t)a.v[i] + k64(i) >= b.v[i] && (uint64_t)a.v[i] + k64(i) - b.v[i] <= 0xFFFFFFFFull);
    r.v[i] = a.v[i] + k64(i) - b.v[i];
  }
}

// in-place carry step of a lazy value (limbs < 2^32) -> normalised
HLC_HD void fe29_norm(fe29& r) { fe29_carry(r.v); }

// r = a - b (mod p), normalised.  a, b limbs < 2^30.4.
HLC_HD void fe29_sub(fe29& r, const fe29& a, const fe29& b) {
  uint32_t d[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    FE29_CHECK((uint64_t)a.v[i] + k29(i) >= b.v[i] && (uint64_t)a.v[i] + k29(i) - b.v[i] <= 0xFFFFFFFFull);
    d[i] = a.v[i] + k29(i) - b.v[i];
  }
  fe29_carry(d);
#pragma unroll
  for (int i = 0; i < 9; ++i) r.v[i] = d[i];
}

// r = a - b - c (mod p), normalised: a + 128 p - b - c, one carry step.  Needs b_i + c_i <= 128p's
// limbs (>= 2^31 - 5: e.g. two normalised values, or three) and a_i < 2^30.58 (a + 128p < 2^32).
HLC_HD void fe29_sub2(fe29& r, const fe29& a, const fe29& b, const fe29& c) {
  uint32_t d[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    FE29_CHECK((uint64_t)a.v[i] + k29(i) <= 0xFFFFFFFFull && (uint64_t)b.v[i] + c.v[i] <= k29(i));
    d[i] = a.v[i] + k29(i) - b.v[i] - c.v[i];
  }
  fe29_carry(d);
#pragma unroll
  for (int i = 0; i < 9; ++i) r.v[i] = d[i];
}

// r = a - b - 2 c (mod p), normalised (same conditions with b_i + 2 c_i <= 128p's limbs)
HLC_HD void fe29_sub_b2c(fe29& r, const fe29& a, const fe29& b, const fe29& c) {
  uint32_t d[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    FE29_CHECK((uint64_t)a.v[i] + k29(i) <= 0xFFFFFFFFull && (uint64_t)b.v[i] + 2ull * c.v[i] <= k29(i));
    d[i] = a.v[i] + k29(i) - b.v[i] - c.v[i] - c.v[i];
  }
  fe29_carry(d);
#pragma unroll
  for (int i = 0; i < 9; ++i) r.v[i] = d[i];
}

HLC_HD void fe29_neg(fe29& r, const fe29& a);
// r = c ? 64p - a : a, branch-free and without a carry step (a limbs <= 64p's, e.g. normalised):
// a lazy value < 2^30 -- the sign of a gathered table entry's y, which only enters products and
// lazy subtractions (hlc_point29.hpp).  64p - a == 64p + ~a + 1 (mod 2^32).
HLC_HD void fe29_cneg_lazy(fe29& r, const fe29& a, bool c) {
  const uint32_t m = 0u - (uint32_t)c;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    FE29_CHECK(a.v[i] <= k64(i));
    r.v[i] = (a.v[i] ^ m) + ((k64(i) + 1u) & m);
  }
}

HLC_HD void fe29_neg(fe29& r, const fe29& a) {
  uint32_t d[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    FE29_CHECK(a.v[i] <= k29(i));
    d[i] = k29(i) - a.v[i];
  }
  fe29_carry(d);
#pragma unroll
  for (int i = 0; i < 9; ++i) r.v[i] = d[i];
}

// r = m * a (mod p), m <= 4, a limbs < 2^29.5 (normalised or sub/mul output), or m = 2 with a a
// lazy-sub output (limbs < 2^31.6 after doubling): normalised
HLC_HD void fe29_mul_small(fe29& r, const fe29& a, uint32_t m) {
  uint32_t d[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    FE29_CHECK((uint64_t)a.v[i] * m <= 0xFFFFFFFFull);
    d[i] = a.v[i] * m;
  }
  fe29_carry(d);
#pragma unroll
  for (int i = 0; i < 9; ++i) r.v[i] = d[i];
}

HLC_HD void fe29_dbl(fe29& r, const fe29& a) { fe29_mul_small(r, a, 2); }

HLC_HD uint64_t mad29(uint32_t a, uint32_t b, uint64_t acc) {
#if defined(HLC_FE29_CHECK) && !defined(__HIP_DEVICE_COMPILE__)
  FE29_CHECK((unsigned __int128)a * b + acc <= (unsigned __int128)0xFFFFFFFFFFFFFFFFull);
#endif
  return (uint64_t)a * b + acc;
}

// Shared tail of mul/sqr: H[0..8] = the high columns 9..17 (29-bit, H[8] the final carry), acc the
// running low column j (already holding the products of column j and the carry of j-1).
// Column j also receives 31264 H_{j+9} and 256 H_{j+8}; 256 H_17 (at 2^261) folds in fe29_top.
// (The asm schedule, hlc_fe29_asm.hpp, performs exactly these steps: bit-identical results.)
#define FE29_LOW_FOLD(j, acc, H)                                    \
  do {                                                              \
    acc = mad29(H[j], FOLD_LO, acc);                                \
    if (j >= 1) acc = mad29(H[(j) - 1], FOLD_HI, acc);              \
  } while (0)

// top: the carry c (< 2^35) out of limb 8 and 256 H_17 sit at 2^261 -> fold into limbs 0, 1 and
// settle limbs 0..2
HLC_HD void fe29_top(uint32_t r[9], uint64_t c, uint32_t h17) {
  uint64_t t = c * FOLD_LO + (uint64_t)h17 * (FOLD_HI * FOLD_LO) + r[0];
  r[0] = (uint32_t)t & M29;
  t = (t >> 29) + c * FOLD_HI + (uint64_t)h17 * (FOLD_HI * FOLD_HI) + r[1];
  r[1] = (uint32_t)t & M29;
  r[2] += (uint32_t)(t >> 29);
}

// r = a * b (mod p).  a, b limbs < 2^30.35; r normalised.  (C++ reference; the device uses the
// generated asm schedule of the same arithmetic, hlc_fe29_asm.hpp)
HLC_HD void fe29_mul_ref(fe29& r, const fe29& a, const fe29& b) {
  uint32_t H[9];
  uint64_t acc = 0;
  // high columns 9..16 first (their 29-bit limbs feed the low columns' fold)
#pragma unroll
  for (int k = 9; k <= 16; ++k) {
#pragma unroll
    for (int i = k - 8; i <= 8; ++i) acc = mad29(a.v[i], b.v[k - i], acc);
    H[k - 9] = (uint32_t)acc & M29;
    acc >>= 29;
  }
  H[8] = (uint32_t)acc;  // column 17 (< 2^31.1)
  uint32_t o[9];
  acc = 0;
#pragma unroll
  for (int j = 0; j <= 8; ++j) {
#pragma unroll
    for (int i = 0; i <= j; ++i) acc = mad29(a.v[i], b.v[j - i], acc);
    FE29_LOW_FOLD(j, acc, H);
    o[j] = (uint32_t)acc & M29;
    acc >>= 29;
  }
  fe29_top(o, acc, H[8]);
#pragma unroll
  for (int i = 0; i < 9; ++i) r.v[i] = o[i];
}

// r = a^2 (mod p).  a limbs < 2^30.35 (2 a_i < 2^31.35: doubled cross products < 2^61.7, at most
// four per column plus one square: < 2^64); r normalised.
HLC_HD void fe29_sqr_ref(fe29& r, const fe29& a) {
  uint32_t d[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    FE29_CHECK(((uint64_t)a.v[i] << 1) <= 0xFFFFFFFFull);
    d[i] = a.v[i] << 1;
  }
  uint32_t H[9];
  uint64_t acc = 0;
#pragma unroll
  for (int k = 9; k <= 16; ++k) {
#pragma unroll
    for (int i = k - 8; i < k - i; ++i) acc = mad29(d[i], a.v[k - i], acc);
    if ((k & 1) == 0) acc = mad29(a.v[k / 2], a.v[k / 2], acc);
    H[k - 9] = (uint32_t)acc & M29;
    acc >>= 29;
  }
  H[8] = (uint32_t)acc;
  uint32_t o[9];
  acc = 0;
#pragma unroll
  for (int j = 0; j <= 8; ++j) {
#pragma unroll
    for (int i = 0; i < j - i; ++i) acc = mad29(d[i], a.v[j - i], acc);
    if ((j & 1) == 0) acc = mad29(a.v[j / 2], a.v[j / 2], acc);
    FE29_LOW_FOLD(j, acc, H);
    o[j] = (uint32_t)acc & M29;
    acc >>= 29;
  }
  fe29_top(o, acc, H[8]);
#pragma unroll
  for (int i = 0; i < 9; ++i) r.v[i] = o[i];
}

// r = a b + c e (mod p) with ONE split / fold / carry pass for the sum: both products accumulate
// into the same 64-bit columns, so every column must hold eighteen products:
// sum_i a_i b_(k-i) + c_i e_(k-i) + carry-in + folds < 2^64 (e.g. a normalised, b < 2^30.6, c < 2^30.01,
// e normalised: 9 (2^59.6 + 2^59.02) < 2^63.5).  r normalised.  (C++ reference of fe29_muladd_asm.)
HLC_HD void fe29_muladd_ref(fe29& r, const fe29& a, const fe29& b, const fe29& c, const fe29& e) {
  uint32_t H[9];
  uint64_t acc = 0;
#pragma unroll
  for (int k = 9; k <= 16; ++k) {
#pragma unroll
    for (int i = k - 8; i <= 8; ++i) {
      acc = mad29(a.v[i], b.v[k - i], acc);
      acc = mad29(c.v[i], e.v[k - i], acc);
    }
    H[k - 9] = (uint32_t)acc & M29;
    acc >>= 29;
  }
  H[8] = (uint32_t)acc;
  uint32_t o[9];
  acc = 0;
#pragma unroll
  for (int j = 0; j <= 8; ++j) {
#pragma unroll
    for (int i = 0; i <= j; ++i) {
      acc = mad29(a.v[i], b.v[j - i], acc);
      acc = mad29(c.v[i], e.v[j - i], acc);
    }
    FE29_LOW_FOLD(j, acc, H);
    o[j] = (uint32_t)acc & M29;
    acc >>= 29;
  }
  fe29_top(o, acc, H[8]);
#pragma unroll
  for (int i = 0; i < 9; ++i) r.v[i] = o[i];
}

// r = a b + f or a^2 + f (mod p) for a nine-limb addend f (limbs < 2^32; in practice 128p minus
// normalised values, i.e. a subtraction that follows the product): f_j joins low column j before
// its split, so the product and the subtraction share one reduction.  Operand contract of mul / sqr;
// r normalised.  (C++ references of fe29_mul_add_asm / fe29_sqr_add_asm.)
HLC_HD void fe29_mul_add_ref(fe29& r, const fe29& a, const fe29& b, const uint32_t f[9], bool square) {
  uint32_t H[9];
  uint64_t acc = 0;
#pragma unroll
  for (int k = 9; k <= 16; ++k) {
#pragma unroll
    for (int i = k - 8; i <= 8; ++i) acc = mad29(a.v[i], square ? a.v[k - i] : b.v[k - i], acc);
    H[k - 9] = (uint32_t)acc & M29;
    acc >>= 29;
  }
  H[8] = (uint32_t)acc;
  uint32_t o[9];
  acc = 0;
#pragma unroll
  for (int j = 0; j <= 8; ++j) {
#pragma unroll
    for (int i = 0; i <= j; ++i) acc = mad29(a.v[i], square ? a.v[j - i] : b.v[j - i], acc);
    acc = mad29(f[j], 1u, acc);
    FE29_LOW_FOLD(j, acc, H);
    o[j] = (uint32_t)acc & M29;
    acc >>= 29;
  }
  fe29_top(o, acc, H[8]);
#pragma unroll
  for (int i = 0; i < 9; ++i) r.v[i] = o[i];
}

// the addend of "... - b - c" after a product: f = 128p - b - c limbwise, NO carry (b_i + c_i <= 128p's
// limbs, as for fe29_sub2; c may be zero)
HLC_HD void fe29_neg_addend(uint32_t f[9], const fe29& b, const fe29& c) {
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    FE29_CHECK((uint64_t)b.v[i] + c.v[i] <= k29(i));
    f[i] = k29(i) - b.v[i] - c.v[i];
  }
}

#if defined(__HIPCC__)
}  // namespace hlc
#include "hlc_fe29_asm.hpp"
namespace hlc {
#endif
// the device runs the generated asm schedule, the host the C++ reference (CPU tests)
HLC_HD void fe29_mul(fe29& r, const fe29& a, const fe29& b) {
#if defined(__HIP_DEVICE_COMPILE__)
  fe29_mul_asm(r.v, a.v, b.v);
#else
  fe29_mul_ref(r, a, b);
#endif
}
// b wave-uniform (e.g. a constant): on the device b lives in SGPRs
HLC_HD void fe29_mul_uniform(fe29& r, const fe29& a, const fe29& b) {
#if defined(__HIP_DEVICE_COMPILE__)
  fe29_mul_sb_asm(r.v, a.v, b.v);
#else
  fe29_mul_ref(r, a, b);
#endif
}
HLC_HD void fe29_sqr(fe29& r, const fe29& a) {
#if defined(__HIP_DEVICE_COMPILE__)
  fe29_sqr_asm(r.v, a.v);
#else
  fe29_sqr_ref(r, a);
#endif
}
HLC_HD void fe29_muladd(fe29& r, const fe29& a, const fe29& b, const fe29& c, const fe29& e) {
#if defined(__HIP_DEVICE_COMPILE__)
  fe29_muladd_asm(r.v, a.v, b.v, c.v, e.v);
#else
  fe29_muladd_ref(r, a, b, c, e);
#endif
}
HLC_HD void fe29_mul_add(fe29& r, const fe29& a, const fe29& b, const uint32_t f[9]) {
#if defined(__HIP_DEVICE_COMPILE__)
  fe29_mul_add_asm(r.v, a.v, b.v, f);
#else
  fe29_mul_add_ref(r, a, b, f, false);
#endif
}
HLC_HD void fe29_sqr_add(fe29& r, const fe29& a, const uint32_t f[9]) {
#if defined(__HIP_DEVICE_COMPILE__)
  fe29_sqr_add_asm(r.v, a.v, f);
#else
  fe29_mul_add_ref(r, a, a, f, true);
#endif
}
// two independent products in one interleaved schedule (two dependency chains in flight per wave)
HLC_HD void fe29_mul2(fe29& x, const fe29& a, const fe29& b, fe29& y, const fe29& c, const fe29& d) {
#if defined(__HIP_DEVICE_COMPILE__)
  fe29_mul2_asm(x.v, a.v, b.v, y.v, c.v, d.v);
#else
  fe29_mul_ref(x, a, b);
  fe29_mul_ref(y, c, d);
#endif
}
HLC_HD void fe29_sqr2(fe29& x, const fe29& a, fe29& y, const fe29& c) {
#if defined(__HIP_DEVICE_COMPILE__)
  fe29_sqr2_asm(x.v, a.v, y.v, c.v);
#else
  fe29_sqr_ref(x, a);
  fe29_sqr_ref(y, c);
#endif
}
HLC_HD void fe29_mulsqr(fe29& x, const fe29& a, const fe29& b, fe29& y, const fe29& c) {
#if defined(__HIP_DEVICE_COMPILE__)
  fe29_mulsqr_asm(x.v, a.v, b.v, y.v, c.v);
#else
  fe29_mul_ref(x, a, b);
  fe29_sqr_ref(y, c);
#endif
}

// Below 2^256 + 2^38 with limbs < 2^29 (input: limbs < 2^30.4): two carry passes, then the bits
// at and above 2^256 (limb 8 bits 24+) fold as t (2^32 + 977) = t 977 at limb 0 + 8 t at limb 1.
HLC_HD void fe29_weak(uint32_t d[9]) {
  fe29_carry(d);
  fe29_carry(d);
  const uint32_t t = d[8] >> 24;
  d[8] &= 0x00FFFFFFu;
  d[0] += t * 977u;
  d[1] += t * 8u;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const uint32_t s = d[i] + c;
    c = s >> 29;
    d[i] = s & M29;
  }
  // c == 0 here: the value is < 2^256 + 2^38 < 2^261
}

// canonical representative (< p), limbs < 2^29
HLC_HD void fe29_normalize(fe29& r, const fe29& a) {
  uint32_t d[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) d[i] = a.v[i];
  fe29_weak(d);
  // value < 2^256 + 2^38 < 2p: subtract p once if value >= p, i.e. if value + (2^256 - p) >= 2^256
  uint32_t e[9];
  uint32_t c = 977u;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const uint32_t s = d[i] + c + (i == 1 ? 8u : 0u);
    c = s >> 29;
    e[i] = s & M29;
  }
  const bool ge = (e[8] >> 24) != 0;  // bit 256 set
  e[8] &= 0x00FFFFFFu;
#pragma unroll
  for (int i = 0; i < 9; ++i) r.v[i] = ge ? e[i] : d[i];
}

HLC_HD bool fe29_is_zero_modp(const fe29& a) {
  uint32_t d[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) d[i] = a.v[i];
  fe29_weak(d);  // < 2p: zero mod p iff 0 or p
  uint32_t z = 0, q = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    z |= d[i];
    q |= d[i] ^ p29(i);
  }
  return z == 0 || q == 0;
}

// 8 x 32-bit little-endian limbs (any value < 2^256) -> 9 x 29
HLC_HD void fe29_from32(fe29& r, const uint32_t w[8]) {
  r.v[0] = w[0] & M29;
  r.v[1] = ((w[0] >> 29) | (w[1] << 3)) & M29;
  r.v[2] = ((w[1] >> 26) | (w[2] << 6)) & M29;
  r.v[3] = ((w[2] >> 23) | (w[3] << 9)) & M29;
  r.v[4] = ((w[3] >> 20) | (w[4] << 12)) & M29;
  r.v[5] = ((w[4] >> 17) | (w[5] << 15)) & M29;
  r.v[6] = ((w[5] >> 14) | (w[6] << 18)) & M29;
  r.v[7] = ((w[6] >> 11) | (w[7] << 21)) & M29;
  r.v[8] = w[7] >> 8;
}

// canonical 8 x 32 (normalises first)
HLC_HD void fe29_to32(uint32_t w[8], const fe29& a) {
  fe29 n;
  fe29_normalize(n, a);
  const uint32_t* v = n.v;
  w[0] = v[0] | (v[1] << 29);
  w[1] = (v[1] >> 3) | (v[2] << 26);
  w[2] = (v[2] >> 6) | (v[3] << 23);
  w[3] = (v[3] >> 9) | (v[4] << 20);
  w[4] = (v[4] >> 12) | (v[5] << 17);
  w[5] = (v[5] >> 15) | (v[6] << 14);
  w[6] = (v[6] >> 18) | (v[7] << 11);
  w[7] = (v[7] >> 21) | (v[8] << 8);
}

}  // namespace hlc
