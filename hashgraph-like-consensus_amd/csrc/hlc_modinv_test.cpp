// Host build of the device-shared safegcd inversion, for CPU tests (tests/test_modinv_host.py).
#include "hlc_modinv.hpp"

extern "C" void hlc_modinv_host(const uint32_t* a, int which_n, uint32_t* out, int count) {
  const hlc::modinfo30 mi = which_n ? hlc::modinfo_n() : hlc::modinfo_p();
  for (int i = 0; i < count; ++i) hlc::modinv_safegcd(out + 8 * i, a + 8 * i, mi);
}
