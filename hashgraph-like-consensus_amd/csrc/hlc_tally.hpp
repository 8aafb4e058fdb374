// hlc_tally.hpp -- the tally / threshold rules shared by validate-many (k_finalize), the timeout
// tally (k_timeout) and the streaming vote path (k_apply_votes).
#pragma once
#include <math.h>
#include <stdint.h>

namespace hlc {

// utils.rs:307-313
__device__ inline uint32_t threshold_value(uint32_t n, double t) {
  if (fabs(t - 2.0 / 3.0) < 2.220446049250313e-16) {
    uint32_t two_n = 2u * n;  // u32 wrap as in a release build
    return two_n / 3u + (two_n % 3u != 0);
  }
  double x = ceil((double)n * t);
  if (!(x > 0)) return 0;
  if (x >= 4294967295.0) return 0xFFFFFFFFu;
  return (uint32_t)x;
}

// utils.rs:227-286 -> -1 None / 0 / 1.  At a timeout silent peers count toward the quorum
// (effective total = n, utils.rs:249-256).
__device__ inline int consensus_result(uint32_t total, uint32_t yes, uint32_t n, double t, bool liveness,
                                bool is_timeout = false) {
  uint32_t no = total > yes ? total - yes : 0;
  uint32_t silent = n > total ? n - total : 0;
  if (n <= 2) {
    if (total < n) return -1;
    return yes == n;
  }
  uint32_t req = threshold_value(n, t);
  if ((is_timeout ? n : total) < req) return -1;
  uint32_t yw = yes + (liveness ? silent : 0), nw = no + (liveness ? 0 : silent);
  if (yw >= req && yw > nw) return 1;
  if (nw >= req && nw > yw) return 0;
  if (total == n && yw == nw) return liveness ? 1 : 0;
  return -1;
}

}  // namespace hlc
