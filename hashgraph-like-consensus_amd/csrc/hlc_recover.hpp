// hlc_recover.hpp -- per-lane secp256k1 public-key recovery (ecrecover).
//
// Restates, bit-exactly, `Signature::from_raw_array(sig)?.recover_address_from_msg(payload)`
// of alloy-primitives 1.6.0 on top of k256 0.13.4 `VerifyingKey::recover_from_prehash`
// (called at /root/reference/src/signing/ethereum.rs:86-89):
//   normalize_v -> normalized_s (high s flipped) -> r, s in [1, n) -> z = prehash mod n
//   -> R = decompress(r, parity) -> Q = u1 G + u2 R with u1 = -z/r, u2 = s/r
//   -> Q != identity -> address = keccak256(Qx || Qy)[12..32].
// k256's post-recovery verify_prehash always succeeds on a recovered key (it re-derives R)
// and is therefore not repeated.
//
// Scalar multiplication: GLV endomorphism (lambda, beta) splits u1 and u2 into 128-bit
// halves; one shared doubling chain of 129 steps adds
//   u1: width-8 wNAF over odd multiples of G and lambda*G (affine, LDS-resident, 8 KB/block)
//   u2: width-5 wNAF over odd multiples of R and lambda*R (Jacobian, per-lane table kept in a
//       lane-interleaved HBM/L2 workspace, 192 words per lane).
#pragma once
#include "hlc_hash.hpp"
#include "hlc_point.hpp"

namespace hlc {

constexpr int WNAF_G = 8;                       // window for G / lambda G
constexpr int WNAF_R = 5;                       // window for R / lambda R
constexpr int GTAB_N = 1 << (WNAF_G - 2);       // 64 odd multiples
constexpr int RTAB_N = 1 << (WNAF_R - 2);       // 8 odd multiples
constexpr int WNAF_WORDS = 33;                  // 132 digit slots (4 int8 per word) per half
constexpr int RTAB_WORDS = RTAB_N * 24;         // per lane
constexpr int SCRATCH_WORDS = RTAB_WORDS + 4 * WNAF_WORDS;  // per lane workspace

enum { SCHEME_NONE = 0, SCHEME_SIG_LEN = 1, SCHEME_ID_LEN = 2, SCHEME_BAD_PARITY = 3,
       SCHEME_SCALAR_RANGE = 4, SCHEME_NO_POINT = 5, SCHEME_INFINITY = 6 };

// Montgomery-form GLV constants (R = 2^256 mod n)
HLC_DEV void glv_consts(fe& mb1R, fe& mb2R, fe& lamR) {
  const uint32_t a[8] = {0x0AD9263Cu, 0xC50468D0u, 0xFAA6ED42u, 0x1B1C8205u,
                         0x8AC47F71u, 0x1571B4AEu, 0x9DF506C6u, 0x221208ACu};
  const uint32_t b[8] = {0x6A144696u, 0x0CAC5E50u, 0xF3BA5939u, 0x1E8A8DC5u,
                         0xBA244FCEu, 0x176CDF65u, 0x8E173580u, 0xC25575EBu};
  const uint32_t l[8] = {0xC9926C9Eu, 0xF07DEB3Du, 0x83C6944Cu, 0x2C93E7ADu,
                         0x52697D91u, 0x73A96606u, 0x8558D639u, 0x53284017u};
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    mb1R.v[i] = a[i];
    mb2R.v[i] = b[i];
    lamR.v[i] = l[i];
  }
}

// c = round(k * g / 2^384) for 256-bit k and constant g (result < 2^129)
HLC_DEV void mul_shift_384(fe& c, const fe& k, const fe& g) {
  uint32_t t[16];
  mul512(t, k, g);
  uint32_t round_bit = t[11] >> 31;
  uint32_t carry = round_bit;
#pragma unroll
  for (int i = 0; i < 4; ++i) c.v[i] = add_cc(t[12 + i], 0u, carry);
  c.v[4] = carry;
  c.v[5] = c.v[6] = c.v[7] = 0;
}

// k = k1 + k2*lambda (mod n); |k1|, |k2| < 2^128 returned as magnitudes + sign flags
HLC_DEV void glv_split(const fe& k, fe& k1, bool& neg1, fe& k2, bool& neg2) {
  fe g1, g2;
  {
    const uint32_t a[8] = {0x45DBB031u, 0xE893209Au, 0x71E8CA7Fu, 0x3DAA8A14u,
                           0x9284EB15u, 0xE86C90E4u, 0xA7D46BCDu, 0x3086D221u};
    const uint32_t b[8] = {0x8AC47F71u, 0x1571B4AEu, 0x9DF506C6u, 0x221208ACu,
                           0x0ABFE4C4u, 0x6F547FA9u, 0x010E8828u, 0xE4437ED6u};
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      g1.v[i] = a[i];
      g2.v[i] = b[i];
    }
  }
  fe c1, c2, mb1R, mb2R, lamR;
  mul_shift_384(c1, k, g1);
  mul_shift_384(c2, k, g2);
  glv_consts(mb1R, mb2R, lamR);
  fe t1, t2, r2, r1;
  sc_mont_mul(t1, c1, mb1R);  // c1 * (-b1) mod n
  sc_mont_mul(t2, c2, mb2R);  // c2 * (-b2) mod n
  sc_add(r2, t1, t2);
  sc_mont_mul(t1, r2, lamR);  // r2 * lambda
  sc_neg(t1, t1);
  sc_add(r1, k, t1);
  // magnitudes: if r > n/2 use n - r
  fe h;
#pragma unroll
  for (int i = 0; i < 8; ++i) h.v[i] = nhalf_limb(i);
  neg1 = u256_lt(h, r1);
  neg2 = u256_lt(h, r2);
  fe m1, m2;
  sc_neg(m1, r1);
  sc_neg(m2, r2);
  k1 = r1;
  k2 = r2;
  fe_cmov(k1, m1, neg1);
  fe_cmov(k2, m2, neg2);
}

// Width-W wNAF of a (< 2^129) value, LSB first, 4 signed int8 digits per word; written to a
// lane-interleaved workspace column (word q of this lane at ws[q * stride]).
template <int W>
HLC_DEV void wnaf_store(const fe& k, uint32_t* ws, size_t stride) {
  uint32_t x0 = k.v[0], x1 = k.v[1], x2 = k.v[2], x3 = k.v[3], x4 = k.v[4];
  for (int q = 0; q < WNAF_WORDS; ++q) {
    uint32_t packed = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      int d = 0;
      if (x0 & 1u) {
        d = (int)(x0 & ((1u << W) - 1u));
        if (d >= (1 << (W - 1))) d -= (1 << W);
        // x -= d (two's complement add of -d over 160 bits)
        uint32_t nd = (uint32_t)(-d);
        uint32_t ext = (d > 0) ? 0xFFFFFFFFu : 0u;
        uint32_t c = 0;
        x0 = add_cc(x0, nd, c);
        x1 = add_cc(x1, ext, c);
        x2 = add_cc(x2, ext, c);
        x3 = add_cc(x3, ext, c);
        x4 = add_cc(x4, ext, c);
      }
      packed |= ((uint32_t)(d & 0xFF)) << (8 * b);
      x0 = __builtin_amdgcn_alignbit(x1, x0, 1);
      x1 = __builtin_amdgcn_alignbit(x2, x1, 1);
      x2 = __builtin_amdgcn_alignbit(x3, x2, 1);
      x3 = __builtin_amdgcn_alignbit(x4, x3, 1);
      x4 = x4 >> 1;
    }
    ws[(size_t)q * stride] = packed;
  }
}

HLC_DEV int digit_at(uint32_t word, int b) { return (int)(int8_t)(word >> (8 * b)); }

HLC_DEV void load_ge_lds(ge& g, const uint32_t* lds_tab, int idx) {
  const uint4* p = reinterpret_cast<const uint4*>(lds_tab + idx * 16);
  uint4 a = p[0], b = p[1], c = p[2], d = p[3];
  g.x.v[0] = a.x; g.x.v[1] = a.y; g.x.v[2] = a.z; g.x.v[3] = a.w;
  g.x.v[4] = b.x; g.x.v[5] = b.y; g.x.v[6] = b.z; g.x.v[7] = b.w;
  g.y.v[0] = c.x; g.y.v[1] = c.y; g.y.v[2] = c.z; g.y.v[3] = c.w;
  g.y.v[4] = d.x; g.y.v[5] = d.y; g.y.v[6] = d.z; g.y.v[7] = d.w;
}

HLC_DEV void store_gej_ws(const gej& p, uint32_t* ws, size_t stride) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    ws[(size_t)i * stride] = p.x.v[i];
    ws[(size_t)(8 + i) * stride] = p.y.v[i];
    ws[(size_t)(16 + i) * stride] = p.z.v[i];
  }
}

HLC_DEV void load_gej_ws(gej& p, const uint32_t* ws, size_t stride) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    p.x.v[i] = ws[(size_t)i * stride];
    p.y.v[i] = ws[(size_t)(8 + i) * stride];
    p.z.v[i] = ws[(size_t)(16 + i) * stride];
  }
  p.inf = 0;
}

// Recovered address as 5 big-endian u32 words (bytes 12..31 of the keccak of X||Y).
HLC_DEV void pubkey_address(const fe& x, const fe& y, uint32_t addr[5]) {
  uint64_t st[25];
#pragma unroll
  for (int i = 0; i < 25; ++i) st[i] = 0;
  // message bytes: X big-endian (32) || Y big-endian (32); lane i = bytes 8i..8i+7 little-endian
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    uint32_t hiw = x.v[7 - 2 * i], low = x.v[6 - 2 * i];
    st[i] = (uint64_t)bswap32(hiw) | ((uint64_t)bswap32(low) << 32);
    uint32_t hiy = y.v[7 - 2 * i], loy = y.v[6 - 2 * i];
    st[4 + i] = (uint64_t)bswap32(hiy) | ((uint64_t)bswap32(loy) << 32);
  }
  st[8] ^= 0x01ull;                 // pad at byte 64
  st[16] ^= 0x8000000000000000ull;  // final bit at byte 135
  keccak_f1600(st);
  // digest bytes 12..31 = lanes 1 (upper half), 2, 3.  Output words are in memory order
  // (word k holds address bytes 4k..4k+3 as a little-endian u32).
  addr[0] = (uint32_t)(st[1] >> 32);
  addr[1] = (uint32_t)st[2];
  addr[2] = (uint32_t)(st[2] >> 32);
  addr[3] = (uint32_t)st[3];
  addr[4] = (uint32_t)(st[3] >> 32);
}

// Full recovery for one lane.  gtab: LDS, 2*GTAB_N affine entries (G multiples then lambda-G
// multiples).  ws: this lane's workspace column base, stride = total lanes.
// Returns SCHEME_* (0 on success and addr filled).
HLC_DEV int ecrecover_lane(const fe& zraw, fe r, fe s, uint32_t v, uint32_t addr[5],
                           const uint32_t* gtab, uint32_t* ws, size_t stride) {
  // alloy normalize_v
  int parity;
  if (v == 0u || v == 27u) parity = 0;
  else if (v == 1u || v == 28u) parity = 1;
  else if (v >= 35u) parity = (int)((v - 35u) & 1u);
  else return SCHEME_BAD_PARITY;
  // alloy normalized_s: s > n/2 -> n - s (wrapping U256 subtraction), parity flipped
  {
    fe h;
#pragma unroll
    for (int i = 0; i < 8; ++i) h.v[i] = nhalf_limb(i);
    if (u256_lt(h, s)) {
      uint32_t bw = 0;
#pragma unroll
      for (int i = 0; i < 8; ++i) s.v[i] = sub_cc(n_limb(i), s.v[i], bw);
      parity ^= 1;
    }
  }
  // k256 Signature::from_scalars: r, s in [1, n)
  if (fe_is_zero(r) || sc_is_ge_n(r) || fe_is_zero(s) || sc_is_ge_n(s)) return SCHEME_SCALAR_RANGE;
  fe z;
  sc_reduce(z, zraw);
  // R = decompress(r, parity): y^2 = x^3 + 7 (x = r < n < p)
  ge R;
  R.x = r;
  {
    fe x3, alpha, seven;
    fe_sqr(x3, r);
    fe_mul(x3, x3, r);
    fe_set(seven, 7);
    fe_add(alpha, x3, seven);
    if (!fe_sqrt(R.y, alpha)) return SCHEME_NO_POINT;
    if ((int)(R.y.v[0] & 1u) != parity) fe_neg(R.y, R.y);
  }
  // u1 = -z/r, u2 = s/r (mod n), Montgomery domain for the inversion
  fe u1, u2;
  {
    fe r2c, rm, rinv;
    sc_r2(r2c);
    sc_mont_mul(rm, r, r2c);     // r*R
    sc_mont_inv(rinv, rm);       // r^-1 * R
    sc_mont_mul(u2, s, rinv);    // s * r^-1
    sc_mont_mul(u1, z, rinv);    // z * r^-1
    sc_neg(u1, u1);
  }
  // GLV halves + wNAF digits into the workspace
  {
    fe a1, a2, b1, b2;
    bool na1, na2, nb1, nb2;
    glv_split(u1, a1, na1, a2, na2);
    glv_split(u2, b1, nb1, b2, nb2);
    uint32_t* dws = ws + (size_t)RTAB_WORDS * stride;
    // fold sign flags into the digits: negate the magnitude's digits by storing -d
    wnaf_store<WNAF_G>(a1, dws + 0 * WNAF_WORDS * stride, stride);
    wnaf_store<WNAF_G>(a2, dws + 1 * WNAF_WORDS * stride, stride);
    wnaf_store<WNAF_R>(b1, dws + 2 * WNAF_WORDS * stride, stride);
    wnaf_store<WNAF_R>(b2, dws + 3 * WNAF_WORDS * stride, stride);
    // sign flags packed into one word kept in a register below
    parity = (na1 ? 1 : 0) | (na2 ? 2 : 0) | (nb1 ? 4 : 0) | (nb2 ? 8 : 0);
  }
  const int negs = parity;
  // R table: odd multiples 1R, 3R, ..., 15R (Jacobian) in the workspace
  {
    gej cur, d2;
    gej_set_ge(cur, R);
    store_gej_ws(cur, ws, stride);
    gej_double(d2, cur);
    for (int i = 1; i < RTAB_N; ++i) {
      gej_add(cur, cur, d2);
      store_gej_ws(cur, ws + (size_t)(24 * i) * stride, stride);
    }
  }
  fe beta;
  fe_beta(beta);
  const uint32_t* dws = ws + (size_t)RTAB_WORDS * stride;
  gej acc;
  gej_set_inf(acc);
  uint32_t wa1 = 0, wa2 = 0, wb1 = 0, wb2 = 0;
  for (int i = 128; i >= 0; --i) {
    const int q = i >> 2, b = i & 3;
    if (b == 3 || i == 128) {
      wa1 = dws[(size_t)(0 * WNAF_WORDS + q) * stride];
      wa2 = dws[(size_t)(1 * WNAF_WORDS + q) * stride];
      wb1 = dws[(size_t)(2 * WNAF_WORDS + q) * stride];
      wb2 = dws[(size_t)(3 * WNAF_WORDS + q) * stride];
    }
    gej_double(acc, acc);
    int d;
    d = digit_at(wa1, b);
    if (d != 0) {
      ge g;
      int idx = ((d < 0 ? -d : d) - 1) >> 1;
      load_ge_lds(g, gtab, idx);
      if ((d < 0) != ((negs & 1) != 0)) fe_neg(g.y, g.y);
      gej_add_ge(acc, acc, g);
    }
    d = digit_at(wa2, b);
    if (d != 0) {
      ge g;
      int idx = ((d < 0 ? -d : d) - 1) >> 1;
      load_ge_lds(g, gtab, GTAB_N + idx);
      if ((d < 0) != ((negs & 2) != 0)) fe_neg(g.y, g.y);
      gej_add_ge(acc, acc, g);
    }
    d = digit_at(wb1, b);
    if (d != 0) {
      gej p;
      int idx = ((d < 0 ? -d : d) - 1) >> 1;
      load_gej_ws(p, ws + (size_t)(24 * idx) * stride, stride);
      if ((d < 0) != ((negs & 4) != 0)) fe_neg(p.y, p.y);
      gej_add(acc, acc, p);
    }
    d = digit_at(wb2, b);
    if (d != 0) {
      gej p;
      int idx = ((d < 0 ? -d : d) - 1) >> 1;
      load_gej_ws(p, ws + (size_t)(24 * idx) * stride, stride);
      fe_mul(p.x, p.x, beta);
      if ((d < 0) != ((negs & 8) != 0)) fe_neg(p.y, p.y);
      gej_add(acc, acc, p);
    }
  }
  if (acc.inf) return SCHEME_INFINITY;
  fe qx, qy;
  gej_to_affine(qx, qy, acc);
  pubkey_address(qx, qy, addr);
  return SCHEME_NONE;
}

}  // namespace hlc
