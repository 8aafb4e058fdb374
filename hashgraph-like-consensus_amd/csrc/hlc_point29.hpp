// hlc_point29.hpp -- the secp256k1 group law (a = 0, b = 7, Jacobian coordinates) over the 29-bit
// unsaturated field layer (hlc_fe29.hpp), for the VALU-bound main recovery stage.  The formulas are
// those of hlc_point.hpp (dbl-2009-l, madd-2007-bl, add-2007-bl) with every intermediate kept
// inside hlc_fe29.hpp's magnitude contract: multiplication inputs are normalised values or sums of
// two; every subtraction / small multiple carries once.  Exceptional cases (identity operand,
// P == Q, P == -Q) are exact, so adversarial signatures (a crafted Q = infinity) match k256.
#pragma once
#include "hlc_fe29.hpp"

namespace hlc {

struct gej29 {
  fe29 x, y, z;
  uint32_t inf;  // 1 = point at infinity
};

struct ge29 {
  fe29 x, y;
};

// beta (cube root of unity mod p) in radix 2^29
HLC_HD void fe29_beta(fe29& r) {
  const uint32_t b[9] = {0x119501EEu, 0x09CB6143u, 0x1D626570u, 0x0092EA25u, 0x034E99CFu,
                         0x03CF561Au, 0x1C41B991u, 0x056CAF80u, 0x007AE96Au};
#pragma unroll
  for (int i = 0; i < 9; ++i) r.v[i] = b[i];
}

HLC_HD void gej29_set_inf(gej29& r) {
  fe29_set(r.x, 0);
  fe29_set(r.y, 1);
  fe29_set(r.z, 0);
  r.inf = 1;
}

HLC_HD void gej29_set_ge(gej29& r, const ge29& a) {
  r.x = a.x;
  r.y = a.y;
  fe29_set(r.z, 1);
  r.inf = 0;
}

// dbl-2009-l (a = 0) arranged for lazy reduction: 3M + 3S and three carry steps.  D = 4 X B is ONE
// product of the doubled operands (2X)(2B), so X3 = F - 2D is one 128p-offset subtraction of two
// normalised values; Y3 = E (D - X3) - 2 (2B)^2 is one sum of two products with a single reduction
// (fe29_muladd: E (D - X3) + 4B (-2B)), so (2B)^2 is never reduced on its own.  (secp256k1 has
// prime order: no point with y = 0.)  r may alias a.
HLC_HD void gej29_double(gej29& r, const gej29& a) {
  fe29 A, B, X2, B2, D, E, Z2, t;
  fe29_sqr(A, a.x);
  fe29_sqr(B, a.y);
  fe29_add(X2, a.x, a.x);
  fe29_add(B2, B, B);
  fe29_mul(D, X2, B2);          // 4 X B            (2^30.01 x 2^30.01 operands)
  fe29_mul_small(E, A, 3);      // 3 X^2, normalised: it is squared next
  fe29_add(Z2, a.z, a.z);
  fe29_mul(r.z, a.y, Z2);       // Z3 = 2 Y Z
  {
    uint32_t f[9];
    fe29_neg_addend(f, D, D);
    fe29_sqr_add(r.x, E, f);    // X3 = E^2 + (128p - 2D): one reduction
  }
  fe29_sub_lazy(t, D, r.x);     // D - X3, lazy: multiplies the normalised E
  // Y3 = E (D - X3) - 2 (2B)^2 = E t + 4B (-2B): one sum of two products, one reduction
  // (fe29_muladd).  -2B is carried to normalised form; 4B stays lazy (< 2^31.01).  Column bound:
  // 9 (2^29.01 2^30.59 + 2^31.01 2^29.01) ~= 2^63.995 < 2^64; the fold and carry terms (~2^47) fit the
  // ~2^55.8 left (tests/test_fe29_host.py::test_muladd_doubling_bounds drives every limb of 4B, E,
  // t and -2B at its maximum).  (-4B against 2B would need 4B <= 128p's limb 8, 2^31 - 5, which a
  // normalised B at its limb-8 maximum exceeds.)
  fe29 nb, b4;
  fe29_neg(nb, B2);
  fe29_add(b4, B2, B2);
  fe29_muladd(r.y, E, t, b4, nb);
  r.inf = a.inf;
}

// r = a + b, b affine (madd-2007-bl: 8M + 3S, four carry steps).  Z3 = 2 Z1 H as one product;
// I = 4 HH stays lazy (it only multiplies normalised values); 2V folds into a 128p-offset
// subtraction; Y3 = R (V - X3) - 2 Y1 J is one sum of two products (fe29_muladd, with -J carried
// to normalised form) with a single reduction.  r may alias a.  With zr != nullptr, *zr = Z3 / Z1 = 2H (the R-table build).
// EXACT = true handles the exceptional cases (a == b: doubling; a == -b: infinity) here.
// EXACT = false (the hot chains) does NOT test for them: H == 0 gives Z3 == 0, every later Z
// stays 0 (each step multiplies Z), and the caller tests the chain's final Z once per vote and
// recomputes the vote with EXACT = true (rec_u2r29 / rec_comb29) -- bit-identical results either way.
template <bool EXACT>
HLC_HD void gej29_madd(gej29& r, const gej29& a, const ge29& b, fe29* zr = nullptr) {
  if (a.inf) {
    gej29_set_ge(r, b);
    return;
  }
  fe29 z1z1, u2, s2, h, rr, hh, i4, j, v, h2, z3, x3, t, y3, y1j;
  fe29_sqr(z1z1, a.z);
  {
    uint32_t f[9];
    fe29_neg_addend(f, a.x, fe29{});
    fe29_mul_add(h, b.x, z1z1, f);  // H = U2 - X1 = x2 Z1^2 + (128p - X1): one reduction
  }
  fe29_mul(s2, b.y, a.z);
  fe29_mul(s2, s2, z1z1);
  fe29_sub_lazy(rr, s2, a.y);      // S2 - Y1, lazy
  if (EXACT && fe29_is_zero_modp(h)) {
    fe29_norm(rr);
    if (fe29_is_zero_modp(rr)) {
      gej29_double(r, a);
    } else {
      gej29_set_inf(r);
    }
    return;
  }
  fe29_mul_small(rr, rr, 2);       // R = 2 (S2 - Y1), normalised: it is squared next
  // (operations ordered so that Z1, H, I die early: register pressure, not latency, bounds the
  // chains' occupancy)
  fe29_add(h2, h, h);
  fe29_mul(z3, a.z, h2);           // Z3 = 2 Z1 H
  if (zr) *zr = h2;
  fe29_sqr(hh, h);
  fe29_shl(i4, hh, 2);             // I = 4 HH, lazy (< 2^31.01)
  fe29_mul(j, h, i4);              // J = H I
  fe29_mul(v, a.x, i4);            // V = X1 I
  {
    uint32_t f[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      FE29_CHECK((uint64_t)j.v[i] + 2ull * v.v[i] <= k29(i));
      f[i] = k29(i) - j.v[i] - v.v[i] - v.v[i];
    }
    fe29_sqr_add(x3, rr, f);       // X3 = R^2 + (128p - J - 2V): one reduction
  }
  fe29_sub_lazy(t, v, x3);         // V - X3, lazy: multiplies the normalised R
  fe29_neg(y1j, j);                // -J, normalised
  fe29_add(h2, a.y, a.y);          // 2 Y1 (h2 is dead here)
  fe29_muladd(y3, rr, t, h2, y1j); // Y3 = R (V - X3) + 2 Y1 (-J): one reduction for both products
  r.x = x3;
  r.y = y3;
  r.z = z3;
  r.inf = 0;
}

HLC_HD void gej29_add_ge(gej29& r, const gej29& a, const ge29& b) { gej29_madd<true>(r, a, b); }

// a += b (b affine, a finite, a != +-b: the R-table build, where (2i-1)R and 2R are distinct,
// non-opposite multiples of a point of prime order n); zr = Z(a') / Z(a) = 2H.
HLC_HD void gej29_madd_zr(gej29& a, const ge29& b, fe29& zr) { gej29_madd<false>(a, a, b, &zr); }

// Co-Z addition with update (Meloni's ZADDU; 4M + 2S, four carry steps): a and b share one
// Jacobian Z (not stored).  a <- a + b and b <- b rescaled, both again sharing the new
// Z' = Z (a.x - b.x); zr = Z' / Z = a.x - b.x.  Builds the R table's odd multiples
// (2i+1) R = (2i-1) R + 2R with b = 2R; needs a != +-b (distinct, non-opposite multiples of a
// point of prime order).
HLC_HD void gej29_zaddu(ge29& a, ge29& b, fe29& zr) {
  fe29 A, B, C, u, t, E, X3, Y3;
  fe29_sub(zr, a.x, b.x);          // X2 - X1 (normalised: squared next)
  fe29_sqr(A, zr);
  fe29_mul(B, b.x, A);             // b.x in the new frame
  fe29_mul(C, a.x, A);
  fe29_sub(u, a.y, b.y);           // Y2 - Y1
  fe29_sub_lazy(t, C, B);
  fe29_mul(E, b.y, t);             // b.y in the new frame
  {
    uint32_t f[9];
    fe29_neg_addend(f, B, C);
    fe29_sqr_add(X3, u, f);        // X3 = (Y2 - Y1)^2 - B - C, one reduction
  }
  fe29_sub_lazy(t, B, X3);
  {
    uint32_t f[9];
    fe29_neg_addend(f, E, fe29{});
    fe29_mul_add(Y3, u, t, f);     // Y3 = (Y2 - Y1)(B - X3) - E, one reduction
  }
  a.x = X3;
  a.y = Y3;
  b.x = B;
  b.y = E;
}

// r = a + b, both Jacobian (add-2007-bl: 11M + 5S).  r may alias a.
HLC_HD void gej29_add(gej29& r, const gej29& a, const gej29& b) {
  if (b.inf) {
    r = a;
    return;
  }
  if (a.inf) {
    r = b;
    return;
  }
  fe29 z1z1, z2z2, u1, u2, s1, s2, h, i4, j, rr, v, t;
  fe29_sqr(z1z1, a.z);
  fe29_sqr(z2z2, b.z);
  fe29_mul(u1, a.x, z2z2);
  fe29_mul(u2, b.x, z1z1);
  fe29_mul(s1, a.y, b.z);
  fe29_mul(s1, s1, z2z2);
  fe29_mul(s2, b.y, a.z);
  fe29_mul(s2, s2, z1z1);
  fe29_sub(h, u2, u1);
  fe29_sub(rr, s2, s1);
  if (fe29_is_zero_modp(h)) {
    if (fe29_is_zero_modp(rr)) {
      gej29_double(r, a);
    } else {
      gej29_set_inf(r);
    }
    return;
  }
  fe29_dbl(i4, h);
  fe29_sqr(i4, i4);
  fe29_mul(j, h, i4);
  fe29_dbl(rr, rr);
  fe29_mul(v, u1, i4);
  fe29 z3;
  fe29_add(z3, a.z, b.z);
  fe29_sqr(z3, z3);
  fe29_sub(z3, z3, z1z1);
  fe29_sub(z3, z3, z2z2);
  fe29_mul(z3, z3, h);
  fe29 x3;
  fe29_sqr(x3, rr);
  fe29_sub(x3, x3, j);
  fe29_dbl(t, v);
  fe29_sub(x3, x3, t);
  fe29 y3;
  fe29_sub(t, v, x3);
  fe29_mul(y3, rr, t);
  fe29_mul(t, s1, j);
  fe29_dbl(t, t);
  fe29_sub(y3, y3, t);
  r.x = x3;
  r.y = y3;
  r.z = z3;
  r.inf = 0;
}

HLC_HD void fe29_sqr_n(fe29& r, const fe29& a, int n) {
  r = a;
  for (int i = 0; i < n; ++i) fe29_sqr(r, r);
}

// r = a^((p+1)/4) (canonical); returns whether r^2 == a (a quadratic residue).  The addition
// chain of hlc_field.hpp's fe_sqrt (253 S + 13 M).
HLC_HD bool fe29_sqrt(fe29& r, const fe29& a) {
  fe29 x2, x3, x6, x9, x11, x22, x44, x88, x176, x220, x223, t;
  fe29_sqr(t, a);
  fe29_mul(x2, t, a);
  fe29_sqr(t, x2);
  fe29_mul(x3, t, a);
  fe29_sqr_n(t, x3, 3);
  fe29_mul(x6, t, x3);
  fe29_sqr_n(t, x6, 3);
  fe29_mul(x9, t, x3);
  fe29_sqr_n(t, x9, 2);
  fe29_mul(x11, t, x2);
  fe29_sqr_n(t, x11, 11);
  fe29_mul(x22, t, x11);
  fe29_sqr_n(t, x22, 22);
  fe29_mul(x44, t, x22);
  fe29_sqr_n(t, x44, 44);
  fe29_mul(x88, t, x44);
  fe29_sqr_n(t, x88, 88);
  fe29_mul(x176, t, x88);
  fe29_sqr_n(t, x176, 44);
  fe29_mul(x220, t, x44);
  fe29_sqr_n(t, x220, 3);
  fe29_mul(x223, t, x3);
  fe29_sqr_n(t, x223, 23);
  fe29_mul(t, t, x22);
  fe29_sqr_n(t, t, 6);
  fe29_mul(t, t, x2);
  fe29_sqr_n(r, t, 2);
  fe29_normalize(r, r);
  fe29_sqr(t, r);
  fe29_sub(t, t, a);
  return fe29_is_zero_modp(t);
}

}  // namespace hlc
