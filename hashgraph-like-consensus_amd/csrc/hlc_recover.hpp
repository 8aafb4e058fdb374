// hlc_recover.hpp -- secp256k1 public-key recovery (ecrecover) for a batch of votes, in five
// kernels (hlc_recover.hip: k_rec_prep, k_rec_main, k_rec_comb, k_rec_final, k_rec_addr).
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
// Stages (one lane per vote in main / comb / addr; REC_BATCH votes per lane in prep / final):
//   prep : v / s / range checks, then r^-1 mod n for REC_BATCH votes with ONE inversion
//          (Montgomery's trick: prefix products forward, one safegcd, a backward sweep), u2 = s/r,
//          the GLV split of u2 and its regular signed digits -> a per-vote record in HBM;
//   main : R = decompress(r) (square root), the R table, the u2 R chain -> Jacobian u2 R in HBM
//          (the VALU-bound bulk, ~90% of the work; needs no prehash, so it runs beside it);
//   comb : u1 = -z/r, the u1 G comb and the final addition Q = u2 R + u1 G;
//   final: Z^-1 mod p for REC_BATCH votes with one inversion (the same trick), affine Q;
//   addr : keccak address, owner compare.
// In SIMT a per-lane inversion already costs the wave ONE instruction stream for 64 values, so
// a cross-lane (DPP / ds_swizzle) prefix-product scan only adds multiplications and saves no issue
// slots; the inversion count per wave only drops when each lane folds several of its own values
// into one inversion -- which is what the batch does (measured in DESIGN.md §4.1).
//
// Scalar multiplication Q = u1 G + u2 R, in two independent parts:
//   u2 R: GLV endomorphism (lambda, beta) splits u2 into 128-bit halves b1 + b2 lambda; one
//       doubling chain of 125 steps adds, every 5 bits, one odd multiple of R and one of
//       lambda R ("regular" signed digits: every lane adds at the same positions).  The 16
//       odd multiples 1..31 R live per lane in a lane-contiguous HBM/L2 workspace.  The R
//       table is built on the isomorphic curve y^2 = x^3 + 7 C^6 (C = Z(2R)) by co-Z additions
//       and brought to one common Z ("effective affine", as libsecp256k1's
//       ge_table_set_globalz), so every chain addition is one mixed Jacobian+affine add.
//   u1 G: a fixed-base comb with NO doublings over a table resident in HBM: GC_WINDOWS windows of
//       GC_W bits (11 x 24), T[w][j] = (2j+1) 2^(W w) G (affine), regular signed digits of the odd
//       representative of u1 (u1 or n - u1, the sign folded into the digits); the recoding's
//       top digit is provably 1, so the last window is the constant start point 2^(W windows) G.
//       GC_WINDOWS mixed additions, each table entry prefetched one window ahead.
//   Q = (u2 R) + (u1 G) with one Jacobian addition (exceptional cases exact).
#pragma once
#include "hlc_hash.hpp"
#include "hlc_point.hpp"
#include "hlc_point29.hpp"

namespace hlc {

// Fixed-window "regular" signed-digit recoding (every digit odd, never zero): every lane adds at
// the same bit positions, so a wave executes exactly one addition per window and half-scalar.
// (A sparse wNAF is useless in SIMT: a wave runs an addition whenever ANY of its 64 lanes has a
// non-zero digit, i.e. at nearly every position -- measured 3.0M VALU instructions per vote.)
#ifndef HLC_W_R
#define HLC_W_R 5  // A/B knob (make variant DEFS=-DHLC_W_R=6): the table doubles per extra bit
#endif
constexpr int W_R = HLC_W_R;                    // window for R / lambda R (u2 halves)
constexpr int M_R = (129 + W_R - 1) / W_R;      // windows: 26 * 5 = 130 >= 129 bits
constexpr int TOP_BIT = W_R * (M_R - 1);        // first (most significant) chain position: 125
constexpr int RTAB_N = 1 << (W_R - 1);          // 16 odd multiples 1..31 (per lane)
#ifndef HLC_REG_ENTRIES
#define HLC_REG_ENTRIES 6  // the R table's last entries kept in registers through the build (A/B: profiles/r05/ab_reg_entries_window.txt)
#endif
constexpr int REG_E = HLC_REG_ENTRIES;
static_assert(REG_E >= 0 && REG_E < RTAB_N, "HLC_REG_ENTRIES out of range");
constexpr int DIG_R_WORDS = (M_R + 1) / 2;      // int16 digits, 2 per word
#ifndef HLC_DIGIT_PREFETCH
#define HLC_DIGIT_PREFETCH 1  // the u2 R chain's digit words read after the doublings (+0.5%, profiles/r06/ab_dpf.txt)
#endif
// Per-lane workspace of the main stage (persistent grid):
//  * lane-interleaved (word w of lane t at w * lanes + t: every lane touches the same word, so
//    each access is one coalesced 256-B row per wave): the z-ratios of the table build;
//  * per-lane contiguous R table (RTAB_WORDS words, 64-B entries read by four 16-B vector loads):
//    entries are gathered at lane-dependent indices, so each lane's entry must be one block.
// (128-B entries with beta x beside x and y measured -8.6%: DESIGN.md §8.1, profiles/r06/ab_tab128.txt)
constexpr int RTAB_ENTRY = 16;                  // words per entry: x, y below 2^256 in 8 x 32 bits (64 B)
constexpr int RTAB_WORDS = RTAB_N * RTAB_ENTRY; // per lane (affine, common-Z frame)
constexpr int ZR_OFF = 0;                       // z-ratios of the table build (9 limbs each)
constexpr int IL_WORDS = ZR_OFF + 9 * (RTAB_N - 1);       // interleaved words per lane
constexpr int SCRATCH_WORDS = IL_WORDS + RTAB_WORDS;      // per lane workspace words

// Per-vote records between the stages, word-major (word w of vote i at w * n + i: a wave's 64
// consecutive votes read one coalesced 256-B row per word).
constexpr int REC_RINV = 0;                     // 8 words: r^-1 R mod n (Montgomery form; u1 = -z/r in main)
constexpr int REC_DIG = 8;                      // 2 x DIG_R_WORDS: int16 digit pairs of b1, b2
constexpr int REC_FLAGS = REC_DIG + 2 * DIG_R_WORDS;  // bit 0-1 negs, 2-3 skews, 5 parity, 8-15 prep code
constexpr int REC_WORDS = REC_FLAGS + 1;
constexpr int Q_WORDS = 24;                     // main -> final: Jacobian X, Y, Z
#ifndef HLC_REC_BATCH
#define HLC_REC_BATCH 8
#endif
constexpr int REC_BATCH = HLC_REC_BATCH;        // votes per lane (one inversion) in prep / final
constexpr uint8_t REC_PENDING = 0xFF;           // verify_out state between the stages

// fixed-base comb for u1 G (global memory, built by k_build_gcomb once per device and process and
// shared by its contexts, hlc_api.cpp gen_tables).  Wider windows mean fewer additions per vote and a
// larger table: W = 24 -> 11 additions over 11 x 2^23 affine points (5.9 GB of the 288 GB HBM, out of
// the Infinity Cache; every entry is prefetched one window ahead, so the gather latency hides behind
// an addition).  W = 22 (12 additions, 1.5 GiB) shipped through round 6; with the comb in its own
// kernel after the u2 R stage, 24 measured +0.6% and 26 (10 additions, 21.5 GB) +0.6% on one box,
// three rounds each (profiles/r06g/ab_gc.txt).  W = 24 keeps 2^(W windows) = 2^264, so the comb's
// exceptional additions stay unreachable (tests/crypto_items.py comb_collisions_possible).
#ifndef HLC_GC_W
#define HLC_GC_W 24
#endif
constexpr int GC_W = HLC_GC_W;                  // bits per window
constexpr int GC_WINDOWS = (255 + GC_W - 1) / GC_W;  // W * windows >= 255: the recoding's top is 1
constexpr int GC_ENTRIES = 1 << (GC_W - 1);     // odd multiples 1 .. 2^W - 1
constexpr size_t GC_TOP_OFF = (size_t)GC_WINDOWS * GC_ENTRIES * 16;  // 2^(W windows) G
constexpr size_t GCOMB_WORDS = GC_TOP_OFF + 16;

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

// Regular signed-digit recoding of k (< 2^129): k' = k | 1 (skew = 1 if k was even) written as
// sum d_i 2^(W i), i < M, every d_i odd with |d_i| < 2^W.  Digits go to the lane's workspace
// column as int16 pairs.  Returns the skew.
template <int W, int M>
HLC_DEV uint32_t recode_regular(const fe& k, uint32_t* ws, size_t stride) {
  uint32_t x0 = k.v[0], x1 = k.v[1], x2 = k.v[2], x3 = k.v[3], x4 = k.v[4];
  const uint32_t skew = (x0 & 1u) ^ 1u;
  x0 |= 1u;
#pragma unroll
  for (int q = 0; q < (M + 1) / 2; ++q) {
    uint32_t packed = 0;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int i = 2 * q + h;
      int d = 0;
      if (i < M - 1) {
        d = (int)(x0 & ((1u << (W + 1)) - 1u)) - (1 << W);
        // x -= d, then x >>= W (x - d == 2^W mod 2^(W+1), so the quotient stays odd)
        const uint32_t nd = (uint32_t)(-d);
        const uint32_t ext = d > 0 ? 0xFFFFFFFFu : 0u;
        uint32_t c = 0;
        x0 = add_cc(x0, nd, c);
        x1 = add_cc(x1, ext, c);
        x2 = add_cc(x2, ext, c);
        x3 = add_cc(x3, ext, c);
        x4 = add_cc(x4, ext, c);
        x0 = __builtin_amdgcn_alignbit(x1, x0, W);
        x1 = __builtin_amdgcn_alignbit(x2, x1, W);
        x2 = __builtin_amdgcn_alignbit(x3, x2, W);
        x3 = __builtin_amdgcn_alignbit(x4, x3, W);
        x4 = x4 >> W;
      } else if (i == M - 1) {
        d = (int)x0;  // remaining value: small and odd
      }
      packed |= ((uint32_t)d & 0xFFFFu) << (16 * h);
    }
    ws[(size_t)q * stride] = packed;
  }
  return skew;
}

HLC_DEV int digit16(uint32_t word, int h) { return (int)(int16_t)(word >> (16 * h)); }

HLC_DEV void load_ge_global(ge& g, const uint32_t* t) {
  const uint4* p = reinterpret_cast<const uint4*>(t);
  uint4 a = p[0], b = p[1], c = p[2], d = p[3];
  g.x.v[0] = a.x; g.x.v[1] = a.y; g.x.v[2] = a.z; g.x.v[3] = a.w;
  g.x.v[4] = b.x; g.x.v[5] = b.y; g.x.v[6] = b.z; g.x.v[7] = b.w;
  g.y.v[0] = c.x; g.y.v[1] = c.y; g.y.v[2] = c.z; g.y.v[3] = c.w;
  g.y.v[4] = d.x; g.y.v[5] = d.y; g.y.v[6] = d.z; g.y.v[7] = d.w;
}

// One step of the regular recoding of an odd 256-bit x with W = GC_W, least significant digit
// first: d = (x mod 2^(W+1)) - 2^W (odd, |d| < 2^W), x = (x - d) / 2^W (stays odd).  For
// x < 2^256 the value left after GC_WINDOWS steps is 1 (W * GC_WINDOWS >= 255).
HLC_DEV int comb_digit(fe& x) {
  const int d = (int)(x.v[0] & ((2u << GC_W) - 1u)) - (1 << GC_W);
  const uint32_t nd = (uint32_t)(-d);
  const uint32_t ext = d > 0 ? 0xFFFFFFFFu : 0u;
  uint32_t c = 0;
  x.v[0] = adc(x.v[0], nd, c);
#pragma unroll
  for (int i = 1; i < 8; ++i) x.v[i] = adc(x.v[i], ext, c);
#pragma unroll
  for (int i = 0; i < 7; ++i) x.v[i] = __builtin_amdgcn_alignbit(x.v[i + 1], x.v[i], GC_W);
  x.v[7] = x.v[7] >> GC_W;
  return d;
}

HLC_DEV const uint32_t* comb_entry(const uint32_t* gcomb, int w, int d) {
  const int idx = ((d < 0 ? -d : d) - 1) >> 1;
  return gcomb + ((size_t)w * GC_ENTRIES + (size_t)idx) * 16;
}

HLC_DEV void store_fe_ws(const fe& x, uint32_t* ws, size_t stride) {
#pragma unroll
  for (int i = 0; i < 8; ++i) ws[(size_t)i * stride] = x.v[i];
}

HLC_DEV void load_fe_ws(fe& x, const uint32_t* ws, size_t stride) {
#pragma unroll
  for (int i = 0; i < 8; ++i) x.v[i] = ws[(size_t)i * stride];
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

// alloy normalize_v + normalized_s + k256 from_scalars (range): SCHEME_NONE with the recovery
// parity and the normalised s, or the scheme error.
HLC_DEV int rec_parse(fe& s, const fe& r, uint32_t v, int& parity) {
  if (v == 0u || v == 27u) parity = 0;
  else if (v == 1u || v == 28u) parity = 1;
  else if (v >= 35u) parity = (int)((v - 35u) & 1u);
  else return SCHEME_BAD_PARITY;
  {
    fe h;
#pragma unroll
    for (int i = 0; i < 8; ++i) h.v[i] = nhalf_limb(i);
    if (u256_lt(h, s)) {  // s > n/2 -> n - s (wrapping U256 subtraction), parity flipped
      uint32_t bw = 0;
#pragma unroll
      for (int i = 0; i < 8; ++i) s.v[i] = sub_cc(n_limb(i), s.v[i], bw);
      parity ^= 1;
    }
  }
  if (fe_is_zero(r) || sc_is_ge_n(r) || fe_is_zero(s) || sc_is_ge_n(s)) return SCHEME_SCALAR_RANGE;
  return SCHEME_NONE;
}

// Prep stage, after r^-1 is known: u2 = s/r split by GLV and recoded, r^-1 kept (Montgomery form)
// for u1 = -z/r, which the main stage forms once the prehash z exists: the prep stage needs only
// the signature, so it runs concurrently with the prehash kernels.  Writes the vote's record
// (stride = n, vote-major words).
HLC_DEV void rec_prep_scalars(const fe& s, const fe& rinv, int parity, uint32_t* rec, size_t stride) {
  fe u2, rinvR;
  {
    fe r2c;
    sc_r2(r2c);
    sc_mont_mul(rinvR, rinv, r2c);  // r^-1 * R (Montgomery form)
    sc_mont_mul(u2, s, rinvR);      // s * r^-1
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) rec[(size_t)(REC_RINV + i) * stride] = rinvR.v[i];
  fe b1, b2;
  bool nb1, nb2;
  glv_split(u2, b1, nb1, b2, nb2);
  const uint32_t s2 = recode_regular<W_R, M_R>(b1, rec + (size_t)REC_DIG * stride, stride);
  const uint32_t s3 = recode_regular<W_R, M_R>(b2, rec + (size_t)(REC_DIG + DIG_R_WORDS) * stride, stride);
  rec[(size_t)REC_FLAGS * stride] = (nb1 ? 1u : 0u) | (nb2 ? 2u : 0u) | (s2 << 2) | (s3 << 3) | ((uint32_t)parity << 5);
}

// Main stage: u1 = -z r^-1 mod n from the prehash and the record's r^-1, as its odd representative
// (u1 or n - u1, neg_g set for the latter) -- the comb's recoding needs an odd scalar.
HLC_DEV void rec_u1(const fe& zraw, const uint32_t* rec, size_t stride, fe& u1, bool& neg_g) {
  fe z, rinvR;
  sc_reduce(z, zraw);
#pragma unroll
  for (int i = 0; i < 8; ++i) rinvR.v[i] = rec[(size_t)(REC_RINV + i) * stride];
  sc_mont_mul(u1, z, rinvR);  // z * r^-1
  sc_neg(u1, u1);
  neg_g = (u1.v[0] & 1u) == 0u;
  if (neg_g) {
    uint32_t bw = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) u1.v[i] = sub_cc(n_limb(i), u1.v[i], bw);
  }
}

// ---- main stage helpers over the 29-bit field layer ----
// R-table entries of 64 B: one aligned half line per gather.  (Round 3 stored the lazy limbs, 80 B
// per entry straddling 128-B lines for half of the entries; the 64-B form measured +6.1% on the
// step, profiles/r04/ab_table64.txt.  Also measured and not kept, DESIGN.md §4.1: non-temporal table
// stores / loads -9 ... -27%; the first entries in LDS -0.2 ... -11.5%; LDS-DMA staging of the
// gathers one window ahead -0.8%.)  A stored
// coordinate (a normalised product: limbs < 2^29, limb 2 < 2^29 + 2^19, value < 2^261) is brought
// below 2^256 -- its bits at and above 2^256 fold as t (2^32 + 977), one serial carry, a second
// fold only when that carry reaches bit 256 again (the value was within 2^38 of 2^256) -- and packed
// into 8 words; a gather unpacks with one v_alignbit + one v_and per limb.
HLC_DEV void fe29_pack256(uint32_t w[8], const fe29& a) {
  uint32_t d[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) d[i] = a.v[i];
  const uint32_t t = d[8] >> 24;
  d[8] &= 0x00FFFFFFu;
  d[0] += t * 977u;
  d[1] += t * 8u;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const uint32_t x = d[i] + c;
    c = x >> 29;
    d[i] = x & M29;
  }
  if (d[8] >> 24) {  // bit 256 set again: fold once more (then the value is far below 2^256)
    d[8] &= 0x00FFFFFFu;
    d[0] += 977u;
    d[1] += 8u;
    c = 0;
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      const uint32_t x = d[i] + c;
      c = x >> 29;
      d[i] = x & M29;
    }
  }
  w[0] = d[0] | (d[1] << 29);
  w[1] = (d[1] >> 3) | (d[2] << 26);
  w[2] = (d[2] >> 6) | (d[3] << 23);
  w[3] = (d[3] >> 9) | (d[4] << 20);
  w[4] = (d[4] >> 12) | (d[5] << 17);
  w[5] = (d[5] >> 15) | (d[6] << 14);
  w[6] = (d[6] >> 18) | (d[7] << 11);
  w[7] = (d[7] >> 21) | (d[8] << 8);
}
HLC_DEV void fe29_unpack256(fe29& r, uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3, uint32_t w4, uint32_t w5,
                            uint32_t w6, uint32_t w7) {
  r.v[0] = w0 & M29;
  r.v[1] = __builtin_amdgcn_alignbit(w1, w0, 29) & M29;
  r.v[2] = __builtin_amdgcn_alignbit(w2, w1, 26) & M29;
  r.v[3] = __builtin_amdgcn_alignbit(w3, w2, 23) & M29;
  r.v[4] = __builtin_amdgcn_alignbit(w4, w3, 20) & M29;
  r.v[5] = __builtin_amdgcn_alignbit(w5, w4, 17) & M29;
  r.v[6] = __builtin_amdgcn_alignbit(w6, w5, 14) & M29;
  r.v[7] = __builtin_amdgcn_alignbit(w7, w6, 11) & M29;
  r.v[8] = w7 >> 8;
}
HLC_DEV void store_ge29_tab64(const fe29& x, const fe29& y, uint32_t* t) {
  uint32_t a[8], b[8];
  fe29_pack256(a, x);
  fe29_pack256(b, y);
  uint4* p = reinterpret_cast<uint4*>(t);
  p[0] = make_uint4(a[0], a[1], a[2], a[3]);
  p[1] = make_uint4(a[4], a[5], a[6], a[7]);
  p[2] = make_uint4(b[0], b[1], b[2], b[3]);
  p[3] = make_uint4(b[4], b[5], b[6], b[7]);
}
HLC_DEV void load_ge29_tab64(ge29& g, const uint32_t* t) {
  const uint4* p = reinterpret_cast<const uint4*>(t);
  const uint4 a = p[0], b = p[1], c = p[2], d = p[3];
  fe29_unpack256(g.x, a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w);
  fe29_unpack256(g.y, c.x, c.y, c.z, c.w, d.x, d.y, d.z, d.w);
}

// The lane's R table: RTAB_N entries in its workspace words.
struct rtab29 {
  uint32_t* g;  // the lane's RTAB_WORDS workspace words
  // an entry of the build pass (rescaled and rewritten by store_final)
  HLC_DEV void store(int e, const fe29& x, const fe29& y) const { store_ge29_tab64(x, y, g + RTAB_ENTRY * e); }
  // an entry in its final (common-Z) frame
  HLC_DEV void store_final(int e, const fe29& x, const fe29& y) const { store_ge29_tab64(x, y, g + RTAB_ENTRY * e); }
  HLC_DEV void load(ge29& q, int e) const { load_ge29_tab64(q, g + RTAB_ENTRY * e); }
};

HLC_DEV void store_fe29_ws(const fe29& x, uint32_t* ws, size_t stride) {
#pragma unroll
  for (int i = 0; i < 9; ++i) ws[(size_t)i * stride] = x.v[i];
}
HLC_DEV void load_fe29_ws(fe29& x, const uint32_t* ws, size_t stride) {
#pragma unroll
  for (int i = 0; i < 9; ++i) x.v[i] = ws[(size_t)i * stride];
}
// comb entry (8 x 32 affine, global) -> 29-bit limbs
HLC_DEV void load_ge_global29(ge29& g, const uint32_t* t) {
  ge e;
  load_ge_global(e, t);
  fe29_from32(g.x, e.x.v);
  fe29_from32(g.y, e.y.v);
}

// acc = k G for odd k < 2^256 (neg: acc = -k G) by the comb, 2^(W windows) G + sum_w d_w 2^(W w) G,
// in 29-bit limbs.
// EXACT: see gej29_madd (the fast form leaves exceptional steps to the caller's final-Z test).
template <bool EXACT>
HLC_DEV void comb_mul_g29(gej29& acc, fe k, bool neg, const uint32_t* gcomb) {
  ge29 e;
  load_ge_global29(e, gcomb + GC_TOP_OFF);
  fe29_cneg_lazy(e.y, e.y, neg);
  gej29_set_ge(acc, e);
  int d = comb_digit(k);
  load_ge_global29(e, comb_entry(gcomb, 0, d));
#pragma unroll 1
  for (int w = 0; w < GC_WINDOWS; ++w) {
    ge29 cur = e;
    const int dc = d;
    if (w + 1 < GC_WINDOWS) {  // prefetch the next window's entry
      d = comb_digit(k);
      load_ge_global29(e, comb_entry(gcomb, w + 1, d));
    }
    fe29_cneg_lazy(cur.y, cur.y, (dc < 0) != neg);
    gej29_madd<EXACT>(acc, acc, cur);
  }
}

// u2 R over the lane's R table (odd multiples 1..31 of R in one common-Z frame, zg = that Z):
// regular signed digits of the GLV halves b1, b2 (b2 against lambda R = (beta x, y)).
template <bool EXACT>
HLC_DEV void chain_u2r29(gej29& acc, const uint32_t* rec, size_t stride, const rtab29& tab, const fe29& zg) {
  const uint32_t flags = rec[(size_t)REC_FLAGS * stride];
  const int negs = (int)(flags & 3u), skews = (int)((flags >> 2) & 3u);
  fe29 beta;
  fe29_beta(beta);  // wave-uniform: multiplied from SGPRs (fe29_mul_uniform)
  const uint32_t* dws = rec + (size_t)REC_DIG * stride;
  gej29_set_inf(acc);
  // Additions in order (window 25, b1), (25, b2), 5 doublings, (24, b1), ... -- the two halves add
  // at the same positions (uniform across the wave).
  auto word_at = [&](int win, int k) { return dws[((size_t)(k * DIG_R_WORDS) + (size_t)(win >> 1)) * stride]; };
  auto digit_at = [&](int win, int k) { return digit16(word_at(win, k), win & 1); };
  auto index_of = [&](int d) { return ((d < 0 ? -d : d) - 1) >> 1; };
#pragma unroll 1
  for (int win = M_R - 1; win >= 0; --win) {
    ge29 g;
#if HLC_DIGIT_PREFETCH
    // Both digit words are loaded at the window's top and read after its doublings, so their
    // latency (an L2 miss: the digits of 640k votes do not fit the L2) hides behind the doublings.
    // Read at the top, as before, each window waited on the b1 word before its doublings and on the
    // b2 word before the b2 gather.
    const uint32_t w1 = word_at(win, 0), w2 = word_at(win, 1);
    if (win != M_R - 1) {
#pragma unroll 1
      for (int q = 0; q < W_R - 1; ++q) gej29_double(acc, acc);
    }
    int d = digit16(w1, win & 1);
    tab.load(g, index_of(d));
    if (win != M_R - 1) gej29_double(acc, acc);
    const int d2 = digit16(w2, win & 1);
#else
    int d = digit_at(win, 0);
    if (win != M_R - 1) {
#pragma unroll 1
      for (int q = 0; q < W_R - 1; ++q) gej29_double(acc, acc);
      tab.load(g, index_of(d));
      gej29_double(acc, acc);
    } else {
      tab.load(g, index_of(d));
    }
    // the b2 entry is loaded before the b1 addition: its gather latency hides behind that addition
    const int d2 = digit_at(win, 1);
#endif
    ge29 g2;
    tab.load(g2, index_of(d2));
    fe29_cneg_lazy(g.y, g.y, (d < 0) != ((negs & 1) != 0));
    gej29_madd<EXACT>(acc, acc, g);
    g = g2;
    d = d2;
    fe29_mul_uniform(g.x, g.x, beta);
    fe29_cneg_lazy(g.y, g.y, (d < 0) != ((negs & 2) != 0));
    gej29_madd<EXACT>(acc, acc, g);
  }
#pragma unroll 1
  for (int k = 0; k < 2; ++k) {
    if (((skews >> k) & 1) == 0) continue;
    ge29 g;
    tab.load(g, 0);
    if (k == 1) fe29_mul_uniform(g.x, g.x, beta);
    fe29_cneg_lazy(g.y, g.y, ((negs >> k) & 1) == 0);
    gej29_madd<EXACT>(acc, acc, g);
  }
  if (!acc.inf) fe29_mul(acc.z, acc.z, zg);
}

// The same in two stages, so that the long half needs no prehash: rec_u2r29 (k_rec_main, runs
// beside the prehash kernels) = R = decompress(r, parity), the R table and the u2 R chain, Jacobian
// result in 8 x 32 limbs (inf set for the point at infinity); rec_comb29 (k_rec_comb, after the
// prehash) = the u1 G comb and the one full addition.  Each half re-runs only its own chain checked
// when its own Z comes out zero (the unchecked chain is exact whenever its Z is non-zero, so this
// is the combined stage's test split per chain).
HLC_DEV int rec_u2r29(const fe& r32, const uint32_t* rec, size_t stride, fe& qx, fe& qy, fe& qz, bool& inf,
                      uint32_t* ws, size_t ws_stride, const rtab29& tab, bool force_exact) {
  const uint32_t flags = rec[(size_t)REC_FLAGS * stride];
  const int parity = (int)((flags >> 5) & 1u);
  ge29 R;
  fe29_from32(R.x, r32.v);
  {
    fe29 x3, alpha, seven;
    fe29_sqr(x3, R.x);
    fe29_mul(x3, x3, R.x);
    fe29_set(seven, 7);
    fe29_add(alpha, x3, seven);
    if (!fe29_sqrt(R.y, alpha)) return SCHEME_NO_POINT;
    if ((int)(R.y.v[0] & 1u) != parity) fe29_neg(R.y, R.y);
  }
  fe29 zg;
  {
    gej29 d;
    gej29_set_ge(d, R);
    gej29_double(d, d);
    ge29 dp;
    dp.x = d.x;
    dp.y = d.y;
    fe29 c2, c3;
    fe29_sqr(c2, d.z);
    fe29_mul(c3, c2, d.z);
    ge29 a;
    fe29_mul(a.x, R.x, c2);
    fe29_mul(a.y, R.y, c3);
    tab.store(0, a.x, a.y);
    uint32_t* zrws = ws + (size_t)ZR_OFF * ws_stride;
#if HLC_REG_ENTRIES == 0
    for (int i = 1; i < RTAB_N; ++i) {
      fe29 zr;
      gej29_zaddu(a, dp, zr);
      if (i == RTAB_N - 1) tab.store_final(i, a.x, a.y);  // (the last entry's frame is the common one)
      else tab.store(i, a.x, a.y);
      store_fe29_ws(zr, zrws + (size_t)(9 * (i - 1)) * ws_stride, ws_stride);
    }
    fe29 sc;
    fe29_set(sc, 1);
    for (int i = RTAB_N - 2; i >= 0; --i) {
      fe29 zr, s2, s3;
      load_fe29_ws(zr, zrws + (size_t)(9 * i) * ws_stride, ws_stride);
      fe29_mul(sc, sc, zr);
      fe29_sqr(s2, sc);
      fe29_mul(s3, s2, sc);
      ge29 e;
      tab.load(e, i);
      fe29_mul(e.x, e.x, s2);
      fe29_mul(e.y, e.y, s3);
      tab.store_final(i, e.x, e.y);
    }
#else
    // The last REG_E entries and their z-ratios stay in registers through the build: they are written
    // once, already in the common frame, instead of written, read back and rewritten by the rescale.
    // (Entry i's scale is the product of the z-ratios of steps i+1 .. RTAB_N-1.)
    constexpr int FIRST_REG = RTAB_N - REG_E;
#pragma unroll 1
    for (int i = 1; i < FIRST_REG; ++i) {
      fe29 zr;
      gej29_zaddu(a, dp, zr);
      tab.store(i, a.x, a.y);
      store_fe29_ws(zr, zrws + (size_t)(9 * (i - 1)) * ws_stride, ws_stride);
    }
    ge29 E[REG_E];
    fe29 ZR[REG_E];
#pragma unroll
    for (int j = 0; j < REG_E; ++j) {
      gej29_zaddu(a, dp, ZR[j]);
      E[j] = a;
    }
    fe29 sc;
    fe29_set(sc, 1);
#pragma unroll
    for (int j = REG_E - 1; j >= 0; --j) {
      if (j != REG_E - 1) {
        fe29 s2, s3;
        fe29_sqr(s2, sc);
        fe29_mul(s3, s2, sc);
        fe29_mul(E[j].x, E[j].x, s2);
        fe29_mul(E[j].y, E[j].y, s3);
      }
      tab.store_final(FIRST_REG + j, E[j].x, E[j].y);
      fe29_mul(sc, sc, ZR[j]);
    }
#pragma unroll 1
    for (int i = FIRST_REG - 1; i >= 0; --i) {
      fe29 s2, s3;
      fe29_sqr(s2, sc);
      fe29_mul(s3, s2, sc);
      ge29 e;
      tab.load(e, i);
      fe29_mul(e.x, e.x, s2);
      fe29_mul(e.y, e.y, s3);
      tab.store_final(i, e.x, e.y);
      if (i > 0) {
        fe29 zr;
        load_fe29_ws(zr, zrws + (size_t)(9 * (i - 1)) * ws_stride, ws_stride);
        fe29_mul(sc, sc, zr);
      }
    }
#endif
    fe29_mul(zg, sc, d.z);
  }
  gej29 acc;
  chain_u2r29<false>(acc, rec, stride, tab, zg);
  if (force_exact || (!acc.inf && fe29_is_zero_modp(acc.z))) chain_u2r29<true>(acc, rec, stride, tab, zg);
  inf = acc.inf;
  fe29_to32(qx.v, acc.x);
  fe29_to32(qy.v, acc.y);
  fe29_to32(qz.v, acc.z);
  return SCHEME_NONE;
}

// second half: Q = (u2 R, from rec_u2r29) + u1 G; Q in 8 x 32 limbs.  SCHEME_NONE or SCHEME_INFINITY.
// u2 R (word-major at qin, stride words apart) is read only after the comb, so that its 24 words
// are not live across the comb's chain (register pressure: k_rec_main runs this in its tail).
HLC_DEV int rec_comb29(const fe& u1, bool neg_g, bool inf, const uint32_t* qin, size_t stride, fe& qx, fe& qy, fe& qz,
                       const uint32_t* gcomb, bool force_exact) {
  gej29 acc, ag;
  comb_mul_g29<false>(ag, u1, neg_g, gcomb);
  if (force_exact || fe29_is_zero_modp(ag.z)) comb_mul_g29<true>(ag, u1, neg_g, gcomb);
  load_fe_ws(qx, qin, stride);
  load_fe_ws(qy, qin + 8 * stride, stride);
  load_fe_ws(qz, qin + 16 * stride, stride);
  acc.inf = inf;
  fe29_from32(acc.x, qx.v);
  fe29_from32(acc.y, qy.v);
  fe29_from32(acc.z, qz.v);
  gej29_add(acc, acc, ag);
  if (acc.inf) return SCHEME_INFINITY;
  fe29_to32(qx.v, acc.x);
  fe29_to32(qy.v, acc.y);
  fe29_to32(qz.v, acc.z);
  return SCHEME_NONE;
}


// The same second half in two kernels (HLC_OPT_EARLY_COMB): rec_ucomb29 runs the comb as soon as the
// prehash and the prep stage are done (k_rec_ucomb, dispatched into k_rec_main's tail as its waves
// leave), rec_add29 adds u2 R once k_rec_main is done (k_rec_add).  u1 G goes through memory in
// 8 x 32 limbs: the same point, so Q and every outcome are those of rec_comb29.
HLC_DEV uint32_t rec_ucomb29(const fe& u1, bool neg_g, fe& gx, fe& gy, fe& gz, const uint32_t* gcomb, bool force_exact) {
  gej29 ag;
  comb_mul_g29<false>(ag, u1, neg_g, gcomb);
  if (force_exact || fe29_is_zero_modp(ag.z)) comb_mul_g29<true>(ag, u1, neg_g, gcomb);
  fe29_to32(gx.v, ag.x);
  fe29_to32(gy.v, ag.y);
  fe29_to32(gz.v, ag.z);
  return ag.inf;
}
HLC_DEV int rec_add29(bool inf, const uint32_t* qin, const uint32_t* gin, size_t stride, fe& qx, fe& qy, fe& qz) {
  gej29 acc, ag;
  fe gx, gy, gz;
  load_fe_ws(gx, gin, stride);
  load_fe_ws(gy, gin + 8 * stride, stride);
  load_fe_ws(gz, gin + 16 * stride, stride);
  ag.inf = gin[24 * stride];
  fe29_from32(ag.x, gx.v);
  fe29_from32(ag.y, gy.v);
  fe29_from32(ag.z, gz.v);
  load_fe_ws(qx, qin, stride);
  load_fe_ws(qy, qin + 8 * stride, stride);
  load_fe_ws(qz, qin + 16 * stride, stride);
  acc.inf = inf;
  fe29_from32(acc.x, qx.v);
  fe29_from32(acc.y, qy.v);
  fe29_from32(acc.z, qz.v);
  gej29_add(acc, acc, ag);
  if (acc.inf) return SCHEME_INFINITY;
  fe29_to32(qx.v, acc.x);
  fe29_to32(qy.v, acc.y);
  fe29_to32(qz.v, acc.z);
  return SCHEME_NONE;
}

}  // namespace hlc
