// Host build of the device-shared safegcd inversion, for CPU tests (tests/test_modinv_host.py).
#include "hlc_modinv.hpp"

extern "C" void hlc_modinv_host(const uint32_t* a, int which_n, uint32_t* out, int count) {
  const hlc::modinfo30 mi = which_n ? hlc::modinfo_n() : hlc::modinfo_p();
  for (int i = 0; i < count; ++i) hlc::modinv_safegcd(out + 8 * i, a + 8 * i, mi);
}

// Host build of the 29-bit Montgomery product mod n (hlc_scmul.hpp) for tests/test_modinv_host.py.
#include "hlc_scmul.hpp"

extern "C" void hlc_sc_mont_mul_host(const uint32_t* a, const uint32_t* b, uint32_t* out, int count) {
  for (int i = 0; i < count; ++i) hlc::sc_mont_mul29(out + 8 * i, a + 8 * i, b + 8 * i);
}
