// Host build of hlc_fe29.hpp / hlc_point29.hpp for the CPU tests (tests/test_fe29_host.py): one C
// entry point per operation over uint32[9] limb arrays, built with HLC_FE29_CHECK so that every
// magnitude-contract violation is counted.  Test infrastructure, not part of libhlc.so.
#include "hlc_fe29.hpp"
#include "hlc_point29.hpp"

using hlc::fe29;
using hlc::ge29;
using hlc::gej29;

extern "C" {
unsigned long long hlc_fe29_violations = 0;
}

static fe29 ld(const uint32_t* p) {
  fe29 r;
  for (int i = 0; i < 9; ++i) r.v[i] = p[i];
  return r;
}
static void st(uint32_t* p, const fe29& r) {
  for (int i = 0; i < 9; ++i) p[i] = r.v[i];
}

extern "C" {
// op: 0 mul, 1 sqr, 2 add, 3 sub, 4 neg, 5 mul_small(m = b[0]), 6 normalize, 7 is_zero (out[0]),
//     8 from32 (a = 8 words), 9 to32 (out = 8 words), 10 sub_lazy, 11 norm (carry step),
//     12 sub2, 13 sub_b2c, 14 cneg_lazy, 15 muladd (b = [b; c; e] rows), 16 mul_add (a b + f, b =
//     [b; f] rows, f raw addend words), 17 sqr_add (a^2 + f, b = f rows), 18 neg_addend (f = 128p - a - b)
void fe29_op(int op, uint64_t n, const uint32_t* a, const uint32_t* b, uint32_t* out) {
  for (uint64_t k = 0; k < n; ++k) {
    const uint32_t* x = a + 9 * k;
    const uint32_t* y = b + 9 * k;
    uint32_t* o = out + 9 * k;
    fe29 r, u = ld(x), v = ld(y);
    switch (op) {
      case 0: hlc::fe29_mul(r, u, v); st(o, r); break;
      case 1: hlc::fe29_sqr(r, u); st(o, r); break;
      case 2: hlc::fe29_add(r, u, v); st(o, r); break;
      case 3: hlc::fe29_sub(r, u, v); st(o, r); break;
      case 4: hlc::fe29_neg(r, u); st(o, r); break;
      case 5: hlc::fe29_mul_small(r, u, y[0]); st(o, r); break;
      case 6: hlc::fe29_normalize(r, u); st(o, r); break;
      case 7: o[0] = hlc::fe29_is_zero_modp(u) ? 1u : 0u; break;
      case 8: hlc::fe29_from32(r, x); st(o, r); break;
      case 9: hlc::fe29_to32(o, u); break;
      case 10: hlc::fe29_sub_lazy(r, u, v); st(o, r); break;
      case 11: r = u; hlc::fe29_norm(r); st(o, r); break;
      case 12: hlc::fe29_sub2(r, u, v, ld(y + 9 * n)); st(o, r); break;         // a - b - c
      case 13: hlc::fe29_sub_b2c(r, u, v, ld(y + 9 * n)); st(o, r); break;      // a - b - 2c
      case 14: hlc::fe29_cneg_lazy(r, u, y[0] != 0); st(o, r); break;            // b[0] ? -a : a
      case 15: hlc::fe29_muladd(r, u, v, ld(y + 9 * n), ld(y + 18 * n)); st(o, r); break;  // a b + c e
      case 16: hlc::fe29_mul_add(r, u, v, y + 9 * n); st(o, r); break;                     // a b + f
      case 17: hlc::fe29_sqr_add(r, u, y); st(o, r); break;                                // a^2 + f
      case 18: hlc::fe29_neg_addend(o, u, v); break;                                       // 128p - a - b
    }
  }
}

unsigned long long fe29_violations(int reset) {
  const unsigned long long v = hlc_fe29_violations;
  if (reset) hlc_fe29_violations = 0;
  return v;
}

// Point operations over n items.  Jacobian points are 28 words (x 9, y 9, z 9, inf), affine 18.
// op 0: r = 2a; 1: r = a + b unchecked (gej29_madd<false>); 2: r = a + b exact; 3: a += b with the
// z-ratio (out: 28 + 9 words); 4: r = a + b, both Jacobian (b: 28 words); 5: co-Z a += b with
// b updated (a, b share an implicit Z; out: a.x, a.y, zr, then b.x, b.y: 46 words).
void gej29_op(int op, uint64_t n, const uint32_t* a, const uint32_t* b, uint32_t* out) {
  for (uint64_t k = 0; k < n; ++k) {
    const uint32_t* x = a + 28 * k;
    const uint32_t* y = b + (op == 4 ? 28 : 18) * k;
    uint32_t* o = out + (op == 3 ? 37 : op == 5 ? 46 : 28) * k;
    gej29 p, q, res;
    p.x = ld(x);
    p.y = ld(x + 9);
    p.z = ld(x + 18);
    p.inf = x[27];
    ge29 g;
    g.x = ld(y);
    g.y = ld(y + 9);
    fe29 zr;
    switch (op) {
      case 0: hlc::gej29_double(res, p); break;
      case 1: hlc::gej29_madd<false>(res, p, g); break;
      case 2: hlc::gej29_madd<true>(res, p, g); break;
      case 3: res = p; hlc::gej29_madd_zr(res, g, zr); st(o + 28, zr); break;
      case 5:  // co-Z addition: a (affine words of p, same implicit Z as b) += b, b rescaled
        res = p;
        {
          ge29 a2;
          a2.x = p.x;
          a2.y = p.y;
          hlc::gej29_zaddu(a2, g, zr);
          res.x = a2.x;
          res.y = a2.y;
          res.z = zr;
          st(o + 28, g.x);
          st(o + 37, g.y);
        }
        break;
      case 4:
        q.x = ld(y);
        q.y = ld(y + 9);
        q.z = ld(y + 18);
        q.inf = y[27];
        hlc::gej29_add(res, p, q);
        break;
    }
    st(o, res.x);
    st(o + 9, res.y);
    st(o + 18, res.z);
    o[27] = res.inf;
  }
}
}
