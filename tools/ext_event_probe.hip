// Probe: what an event costs between two kernels on one stream, recorded as a marker
// (hipEventRecord) or bound to the kernels' own dispatches (hipExtLaunchKernelGGL start / stop), and
// whether a stream can wait on a dispatch-bound stop event.
//   hipcc --offload-arch=gfx950 -O2 tools/ext_event_probe.hip -o /tmp/ext_event_probe && /tmp/ext_event_probe
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      std::printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));    \
      return 1;                                                                \
    }                                                                          \
  } while (0)

// ~`cycles` shader cycles of busy work per wave, then one store per thread
__global__ void k_busy(unsigned long long cycles, unsigned* out, unsigned v) {
  const unsigned long long t0 = clock64();
  while (clock64() - t0 < cycles) {
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = v;
}

// reads what k_busy wrote (dependency check across streams)
__global__ void k_check(const unsigned* in, unsigned want, unsigned* bad) {
  const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
  if (in[i] != want) atomicAdd(bad, 1u);
}

int main() {
  const int K = 12, reps = 200, blocks = 1024;
  unsigned *buf, *bad;
  CK(hipMalloc(&buf, blocks * 256 * sizeof(unsigned)));
  CK(hipMalloc(&bad, sizeof(unsigned)));
  CK(hipMemset(bad, 0, sizeof(unsigned)));
  hipStream_t s, s2;
  CK(hipStreamCreate(&s));
  CK(hipStreamCreate(&s2));
  std::vector<hipEvent_t> ev(2 * K);
  for (auto& e : ev) CK(hipEventCreate(&e));
  const unsigned long long cyc = 4000;  // ~2 us at 2.2 GHz
  const char* names[3] = {"no events", "hipEventRecord between kernels", "dispatch-bound (hipExtLaunchKernelGGL)"};
  for (int mode = 0; mode < 3; ++mode) {
    for (int warm = 0; warm < 2; ++warm) {
      CK(hipDeviceSynchronize());
      auto t0 = std::chrono::steady_clock::now();
      float evsum = 0;
      for (int r = 0; r < reps; ++r) {
        for (int k = 0; k < K; ++k) {
          if (mode == 0) {
            hipLaunchKernelGGL(k_busy, dim3(blocks), dim3(256), 0, s, cyc, buf, (unsigned)k);
          } else if (mode == 1) {
            CK(hipEventRecord(ev[2 * k], s));
            hipLaunchKernelGGL(k_busy, dim3(blocks), dim3(256), 0, s, cyc, buf, (unsigned)k);
            CK(hipEventRecord(ev[2 * k + 1], s));
          } else {
            hipExtLaunchKernelGGL(k_busy, dim3(blocks), dim3(256), 0, s, ev[2 * k], ev[2 * k + 1], 0, cyc, buf,
                                  (unsigned)k);
          }
        }
        if (mode) {
          CK(hipEventSynchronize(ev[2 * K - 1]));
          float ms = 0;
          CK(hipEventElapsedTime(&ms, ev[0], ev[2 * K - 1]));
          evsum += ms;
        }
      }
      CK(hipDeviceSynchronize());
      const double wall = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      if (warm)
        std::printf("%-40s wall %.2f us per %d-kernel sequence, event bracket %.2f us\n", names[mode],
                    1e3 * wall / reps, K, 1e3 * evsum / reps);
    }
  }
  // per-kernel elapsed of one dispatch-bound pair vs the bracket of two kernels
  {
    float a = 0, b = 0;
    CK(hipEventElapsedTime(&a, ev[0], ev[1]));
    CK(hipEventElapsedTime(&b, ev[0], ev[3]));
    std::printf("dispatch-bound: kernel 0 start->stop %.2f us, kernel 0 start -> kernel 1 stop %.2f us\n", 1e3 * a,
                1e3 * b);
  }
  // cross-stream wait on a dispatch-bound stop event: s2's check must see what s's long kernel wrote
  for (int r = 0; r < 20; ++r) {
    const unsigned v = 1000 + r;
    hipExtLaunchKernelGGL(k_busy, dim3(blocks), dim3(256), 0, s, nullptr, ev[1], 0, 200000ull, buf, v);
    CK(hipStreamWaitEvent(s2, ev[1], 0));
    hipLaunchKernelGGL(k_check, dim3(blocks), dim3(256), 0, s2, buf, v, bad);
    CK(hipDeviceSynchronize());  // the next k_busy must not overwrite buf before this check read it
  }
  CK(hipDeviceSynchronize());
  unsigned h = 0;
  CK(hipMemcpy(&h, bad, sizeof h, hipMemcpyDeviceToHost));
  std::printf("cross-stream wait on dispatch-bound stop event: %u mismatching reads (0 = the wait held)\n", h);
  // disable-timing event as a dispatch-bound stop, waited on by another stream
  hipEvent_t nt;
  CK(hipEventCreateWithFlags(&nt, hipEventDisableTiming));
  CK(hipMemset(bad, 0, sizeof(unsigned)));
  for (int r = 0; r < 20; ++r) {
    const unsigned v = 2000 + r;
    hipExtLaunchKernelGGL(k_busy, dim3(blocks), dim3(256), 0, s, nullptr, nt, 0, 200000ull, buf, v);
    CK(hipStreamWaitEvent(s2, nt, 0));
    hipLaunchKernelGGL(k_check, dim3(blocks), dim3(256), 0, s2, buf, v, bad);
    CK(hipDeviceSynchronize());  // the next k_busy must not overwrite buf before this check read it
  }
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(&h, bad, sizeof h, hipMemcpyDeviceToHost));
  std::printf("same with a disable-timing stop event: %u mismatching reads\n", h);
  std::printf("ok\n");
  return 0;
}
