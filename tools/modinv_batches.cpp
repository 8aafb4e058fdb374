// How many 30-divstep batches hlc_modinv.hpp's safegcd needs before g == 0, per input and per 64-lane group
// (random 255-bit inputs, mod p and mod n): g++ -O2 -o /tmp/mb tools/modinv_batches.cpp && /tmp/mb
#include "../hashgraph-like-consensus_amd/csrc/hlc_modinv.hpp"
#include <cstdio>
#include <random>
using namespace hlc;
static bool gzero(const s30& g) { int32_t c = 0; for (int i = 0; i < 9; ++i) c |= g.v[i]; return c == 0; }
int batches(const uint32_t a[8], const modinfo30& mi) {
  s30 d = {{0}}, e = {{1}}, f = mi.modulus, g; to_s30(g, a); int32_t zeta = -1;
  for (int i = 0; i < 20; ++i) {
    if (gzero(g)) return i;
    trans2x2 t; zeta = divsteps_30(zeta, (uint32_t)f.v[0], (uint32_t)g.v[0], t);
    update_de_30(d, e, t, mi); update_fg_30(f, g, t);
  }
  return 20 + !gzero(g) * 100;
}
int main() {
  std::mt19937_64 rng(1);
  for (int which = 0; which < 2; ++which) {
    const modinfo30 mi = which ? modinfo_n() : modinfo_p();
    int hist[130] = {0}; int wavemax_hist[130] = {0};
    for (int w = 0; w < 2000; ++w) {
      int mx = 0;
      for (int l = 0; l < 64; ++l) {
        uint32_t a[8]; for (int k = 0; k < 8; ++k) a[k] = (uint32_t)rng();
        a[7] &= 0x7FFFFFFF;
        int b = batches(a, mi); hist[b]++; if (b > mx) mx = b;
      }
      wavemax_hist[mx]++;
    }
    printf("modulus %s lane batches:", which ? "n" : "p"); for (int i = 0; i < 130; ++i) if (hist[i]) printf(" %d:%d", i, hist[i]);
    printf("\n  wave max:"); for (int i = 0; i < 130; ++i) if (wavemax_hist[i]) printf(" %d:%d", i, wavemax_hist[i]); printf("\n");
  }
}
