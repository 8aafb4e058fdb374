// Teardown control for rocprofv3 (GPU box): a plain HIP program -- no PyTorch, no libhlc -- that copies
// host -> device, runs one kernel, copies back and exits.  A crash in the process's finalizers under a
// profiler mode here is the profiler's (tools/teardown_probe.py runs the same check with PyTorch and with
// the library).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void k_twice(float* x, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) x[i] *= 2.0f;
}

int main() {
  const int n = 1 << 20;
  std::vector<float> h(n, 1.5f);
  float* d = nullptr;
  if (hipMalloc(&d, n * sizeof(float)) != hipSuccess) return 2;
  if (hipMemcpy(d, h.data(), n * sizeof(float), hipMemcpyHostToDevice) != hipSuccess) return 3;
  hipLaunchKernelGGL(k_twice, dim3(n / 256), dim3(256), 0, 0, d, n);
  if (hipMemcpy(h.data(), d, n * sizeof(float), hipMemcpyDeviceToHost) != hipSuccess) return 4;
  (void)hipFree(d);
  std::printf("hip ok %.1f\n", h[n - 1]);
  return h[n - 1] == 3.0f ? 0 : 5;
}
