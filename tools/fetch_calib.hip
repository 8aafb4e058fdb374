// fetch_calib.hip -- what rocprofv3's FETCH_SIZE / WRITE_SIZE report on gfx950 for the access shapes
// of this repo's kernels (bench.py doubled FETCH_SIZE for every kernel, but the
// guide's halving is stated for 16-B-per-lane coalesced streams only).  Each kernel touches a known
// number of distinct bytes of a 2 GiB buffer exactly once (far past the 4 MB L2s and the 256 MB
// Infinity Cache), so counter bytes / true bytes is the calibration factor of that shape:
//   stream16   grid-stride 16-B loads, consecutive lanes consecutive   (k_wire_touch, LDS window loads)
//   stream4    grid-stride 4-B loads                                   (word-major records: load_fe_ws)
//   stream1    grid-stride 1-B loads                                   (status / pre bytes)
//   gather64   one 64-B entry per lane, 4 x 16-B loads, entries in a permuted order (k_rec_main's R-table
//              gathers, k_rec_comb's comb gathers)
//   gather32   one 32-B piece per lane, 2 x 16-B loads, permuted      (vote hashes, owners)
//   gather16   one 16-B piece per lane, permuted
//   write16 / write4   the same as stores (WRITE_SIZE)
// Run under `rocprofv3 --pmc FETCH_SIZE` and, separately, `--pmc WRITE_SIZE` (tools/fetch_calib.py).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHK(x)                                                                          \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) {                                                             \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                      \
      std::exit(1);                                                                     \
    }                                                                                   \
  } while (0)

constexpr size_t BYTES = 2ull << 30;
constexpr uint32_t PERM = 0x9E3779B1u;  // odd: i -> i * PERM mod 2^k is a permutation of the slots

__global__ void k_stream16(const uint4* __restrict__ a, size_t n, uint32_t* sink) {
  uint32_t acc = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const uint4 v = a[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) *sink = acc;
}
__global__ void k_stream4(const uint32_t* __restrict__ a, size_t n, uint32_t* sink) {
  uint32_t acc = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    acc ^= a[i];
  if (acc == 0x12345678u) *sink = acc;
}
__global__ void k_stream1(const uint8_t* __restrict__ a, size_t n, uint32_t* sink) {
  uint32_t acc = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    acc += a[i];
  if (acc == 0x12345678u) *sink = acc;
}
template <int PIECES>
__global__ void k_gather(const uint4* __restrict__ a, size_t slots, uint32_t* sink) {  // slots: a power of two
  uint32_t acc = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < slots; i += (size_t)gridDim.x * blockDim.x) {
    const size_t s = (i * PERM) & (slots - 1);
#pragma unroll
    for (int k = 0; k < PIECES; ++k) {
      const uint4 v = a[s * PIECES + k];
      acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
  }
  if (acc == 0x12345678u) *sink = acc;
}
__global__ void k_write16(uint4* __restrict__ a, size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    a[i] = make_uint4((uint32_t)i, 1u, 2u, 3u);
}
__global__ void k_write4(uint32_t* __restrict__ a, size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    a[i] = (uint32_t)i;
}

int main() {
  void* buf = nullptr;
  uint32_t* sink = nullptr;
  CHK(hipMalloc(&buf, BYTES));
  CHK(hipMalloc(&sink, 64));
  CHK(hipMemset(buf, 1, BYTES));
  const dim3 g(8192), b(256);
  // every kernel twice: the first launch of each warms the code object; both launches are counted
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(k_stream16, g, b, 0, 0, (const uint4*)buf, BYTES / 16, sink);
    hipLaunchKernelGGL(k_stream4, g, b, 0, 0, (const uint32_t*)buf, BYTES / 4, sink);
    hipLaunchKernelGGL(k_stream1, g, b, 0, 0, (const uint8_t*)buf, BYTES / 4, sink);  // 512 MiB of bytes
    hipLaunchKernelGGL(k_gather<4>, g, b, 0, 0, (const uint4*)buf, BYTES / 64, sink);
    hipLaunchKernelGGL(k_gather<2>, g, b, 0, 0, (const uint4*)buf, BYTES / 32, sink);
    hipLaunchKernelGGL(k_gather<1>, g, b, 0, 0, (const uint4*)buf, BYTES / 16, sink);
    hipLaunchKernelGGL(k_write16, g, b, 0, 0, (uint4*)buf, BYTES / 16);
    hipLaunchKernelGGL(k_write4, g, b, 0, 0, (uint32_t*)buf, BYTES / 4);
  }
  CHK(hipDeviceSynchronize());
  std::printf("{\"bytes\": {\"k_stream16\": %zu, \"k_stream4\": %zu, \"k_stream1\": %zu, \"k_gather<4>\": %zu, "
              "\"k_gather<2>\": %zu, \"k_gather<1>\": %zu, \"k_write16\": %zu, \"k_write4\": %zu}}\n",
              BYTES, BYTES, BYTES / 4, BYTES, BYTES, BYTES, BYTES, BYTES);
  CHK(hipFree(buf));
  CHK(hipFree(sink));
  return 0;
}
