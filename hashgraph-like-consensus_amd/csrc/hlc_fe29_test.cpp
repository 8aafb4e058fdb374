// Host build of hlc_fe29.hpp for the CPU tests (tests/test_fe29_host.py): one C entry point per
// operation over uint32[9] limb arrays.  Test infrastructure, not part of libhlc.so.
#include "hlc_fe29.hpp"

using hlc::fe29;

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
//     8 from32 (a = 8 words), 9 to32 (out = 8 words), 10 sub_lazy, 11 norm (carry step)
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
    }
  }
}
}
