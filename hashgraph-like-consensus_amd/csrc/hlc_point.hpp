// hlc_point.hpp -- secp256k1 group law (a = 0, b = 7) in Jacobian coordinates, one point
// per lane.  Exceptional cases (identity operand, P == Q, P == -Q) are handled exactly so
// adversarial signatures (e.g. a crafted Q = infinity) give the same
// outcome as k256's complete projective formulas.
#pragma once
#include "hlc_field.hpp"

namespace hlc {

struct gej {
  fe x, y, z;
  uint32_t inf;  // 1 = point at infinity
};

struct ge {
  fe x, y;
};

// beta: cube root of unity mod p (lambda * (x, y) = (beta*x, y))
HLC_DEV void fe_beta(fe& r) {
  const uint32_t b[8] = {0x719501EEu, 0xC1396C28u, 0x12F58995u, 0x9CF04975u,
                         0xAC3434E9u, 0x6E64479Eu, 0x657C0710u, 0x7AE96A2Bu};
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = b[i];
}

HLC_DEV void ge_generator(ge& g) {
  const uint32_t gx[8] = {0x16F81798u, 0x59F2815Bu, 0x2DCE28D9u, 0x029BFCDBu,
                          0xCE870B07u, 0x55A06295u, 0xF9DCBBACu, 0x79BE667Eu};
  const uint32_t gy[8] = {0xFB10D4B8u, 0x9C47D08Fu, 0xA6855419u, 0xFD17B448u,
                          0x0E1108A8u, 0x5DA4FBFCu, 0x26A3C465u, 0x483ADA77u};
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    g.x.v[i] = gx[i];
    g.y.v[i] = gy[i];
  }
}

HLC_DEV void gej_set_ge(gej& r, const ge& a) {
  r.x = a.x;
  r.y = a.y;
  fe_set(r.z, 1);
  r.inf = 0;
}

HLC_DEV void gej_set_inf(gej& r) {
  fe_set(r.x, 0);
  fe_set(r.y, 1);
  fe_set(r.z, 0);
  r.inf = 1;
}

// dbl-2009-l: 2M + 5S.  (secp256k1 has prime order: no point with y = 0.)
HLC_DEV void gej_double(gej& r, const gej& a) {
  fe A, B, C, D, E, F, t;
  fe_sqr(A, a.x);
  fe_sqr(B, a.y);
  fe_sqr(C, B);
  fe_add(t, a.x, B);
  fe_sqr(t, t);
  fe_sub(t, t, A);
  fe_sub(t, t, C);
  fe_dbl(D, t);
  fe_dbl(E, A);
  fe_add(E, E, A);
  fe_sqr(F, E);
  fe z3;
  fe_mul(z3, a.y, a.z);
  fe_dbl(r.z, z3);
  fe_dbl(t, D);
  fe_sub(r.x, F, t);
  fe_sub(t, D, r.x);
  fe_mul(r.y, E, t);
  fe_dbl(C, C);
  fe_dbl(C, C);
  fe_dbl(C, C);
  fe_sub(r.y, r.y, C);
  r.inf = a.inf;
}

// r = a + b, b affine (madd-2007-bl: 7M + 4S).  r may alias a.
HLC_DEV void gej_add_ge(gej& r, const gej& a, const ge& b) {
  if (a.inf) {
    gej_set_ge(r, b);
    return;
  }
  fe z1z1, u2, s2, h, hh, i4, j, rr, v, t;
  fe_sqr(z1z1, a.z);
  fe_mul(u2, b.x, z1z1);
  fe_mul(s2, b.y, a.z);
  fe_mul(s2, s2, z1z1);
  fe_sub(h, u2, a.x);
  fe_sub(rr, s2, a.y);
  if (fe_is_zero_modp(h)) {
    if (fe_is_zero_modp(rr)) {
      gej_double(r, a);
    } else {
      gej_set_inf(r);
    }
    return;
  }
  fe_sqr(hh, h);
  fe_dbl(i4, hh);
  fe_dbl(i4, i4);
  fe_mul(j, h, i4);
  fe_dbl(rr, rr);
  fe_mul(v, a.x, i4);
  // z3 = (z1 + h)^2 - z1z1 - hh
  fe z3;
  fe_add(z3, a.z, h);
  fe_sqr(z3, z3);
  fe_sub(z3, z3, z1z1);
  fe_sub(z3, z3, hh);
  // x3 = r^2 - j - 2v
  fe x3;
  fe_sqr(x3, rr);
  fe_sub(x3, x3, j);
  fe_dbl(t, v);
  fe_sub(x3, x3, t);
  // y3 = r (v - x3) - 2 y1 j
  fe y3;
  fe_sub(t, v, x3);
  fe_mul(y3, rr, t);
  fe_mul(t, a.y, j);
  fe_dbl(t, t);
  fe_sub(y3, y3, t);
  r.x = x3;
  r.y = y3;
  r.z = z3;
  r.inf = 0;
}

// r = a + b, both Jacobian (add-2007-bl: 11M + 5S).  r may alias a.
HLC_DEV void gej_add(gej& r, const gej& a, const gej& b) {
  if (b.inf) {
    r = a;
    return;
  }
  if (a.inf) {
    r = b;
    return;
  }
  fe z1z1, z2z2, u1, u2, s1, s2, h, i4, j, rr, v, t;
  fe_sqr(z1z1, a.z);
  fe_sqr(z2z2, b.z);
  fe_mul(u1, a.x, z2z2);
  fe_mul(u2, b.x, z1z1);
  fe_mul(s1, a.y, b.z);
  fe_mul(s1, s1, z2z2);
  fe_mul(s2, b.y, a.z);
  fe_mul(s2, s2, z1z1);
  fe_sub(h, u2, u1);
  fe_sub(rr, s2, s1);
  if (fe_is_zero_modp(h)) {
    if (fe_is_zero_modp(rr)) {
      gej_double(r, a);
    } else {
      gej_set_inf(r);
    }
    return;
  }
  fe_dbl(i4, h);
  fe_sqr(i4, i4);
  fe_mul(j, h, i4);
  fe_dbl(rr, rr);
  fe_mul(v, u1, i4);
  fe z3;
  fe_add(z3, a.z, b.z);
  fe_sqr(z3, z3);
  fe_sub(z3, z3, z1z1);
  fe_sub(z3, z3, z2z2);
  fe_mul(z3, z3, h);
  fe x3;
  fe_sqr(x3, rr);
  fe_sub(x3, x3, j);
  fe_dbl(t, v);
  fe_sub(x3, x3, t);
  fe y3;
  fe_sub(t, v, x3);
  fe_mul(y3, rr, t);
  fe_mul(t, s1, j);
  fe_dbl(t, t);
  fe_sub(y3, y3, t);
  r.x = x3;
  r.y = y3;
  r.z = z3;
  r.inf = 0;
}

// affine coordinates (canonical, < p) of a (finite) Jacobian point
HLC_DEV void gej_to_affine(fe& x, fe& y, const gej& a) {
  fe zi, zi2, zi3;
  fe_inv(zi, a.z);
  fe_sqr(zi2, zi);
  fe_mul(zi3, zi2, zi);
  fe_mul(x, a.x, zi2);
  fe_mul(y, a.y, zi3);
  fe_normalize(x, x);
  fe_normalize(y, y);
}

}  // namespace hlc
