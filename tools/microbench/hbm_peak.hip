// HBM read / write / copy microbenchmark on gfx950 (SURVEY.md 8(d) reporting rule (i): the measured
// STREAM-like read peak the roofline fractions are quoted against).  A 4 GiB buffer (16x the Infinity
// Cache) streamed with 16-byte loads per lane, grid-stride, 4 loads in flight per lane, 2048 workgroups of
// 256 threads; the read kernel folds its loads into one store per thread (no dead-code elimination).  Best
// and median of 20 launches each, timed with hipEvents.  Prints one JSON line.
// Build: hipcc -O3 --offload-arch=gfx950 tools/microbench/hbm_peak.hip -o tools/microbench/hbm_peak
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));             \
      return 1;                                                                \
    }                                                                          \
  } while (0)

__global__ void __launch_bounds__(256) k_read(const double4* __restrict__ a, size_t n, double* __restrict__ out) {
  double s = 0.0;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  for (; i + 3 * stride < n; i += 4 * stride) {
    const double4 v0 = a[i], v1 = a[i + stride], v2 = a[i + 2 * stride], v3 = a[i + 3 * stride];
    s += (v0.x + v1.y) + (v2.z + v3.w);
  }
  for (; i < n; i += stride) s += a[i].x;
  out[blockIdx.x * (size_t)blockDim.x + threadIdx.x] = s;
}

__global__ void __launch_bounds__(256) k_write(double4* __restrict__ a, size_t n, double v) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += stride) a[i] = make_double4(v, v, v, v);
}

__global__ void __launch_bounds__(256) k_copy(const double4* __restrict__ a, double4* __restrict__ b, size_t n) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += stride) b[i] = a[i];
}

int main() {
  const size_t bytes = (size_t)4 << 30;
  const size_t n = bytes / sizeof(double4);
  double4 *a = nullptr, *b = nullptr;
  double* out = nullptr;
  const int grid = 2048, block = 256;
  CK(hipMalloc(&a, bytes));
  CK(hipMalloc(&b, bytes / 2));
  CK(hipMalloc(&out, sizeof(double) * 16384 * block));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipLaunchKernelGGL(k_write, dim3(grid), dim3(block), 0, 0, a, n, 1.0);
  CK(hipDeviceSynchronize());
  auto timeit = [&](auto&& launch, double nbytes, double* best, double* med) -> int {
    std::vector<double> v;
    for (int r = 0; r < 22; ++r) {
      CK(hipEventRecord(e0, 0));
      launch();
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms = 0.f;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (r >= 2) v.push_back(nbytes / (ms * 1e-3) / 1e9);
    }
    std::sort(v.begin(), v.end());
    *best = v.back();
    *med = v[v.size() / 2];
    return 0;
  };
  double rb = 0, rm = 0, wb, wm, cb, cm;
  int rgrid = 0;
  for (int g : {1024, 2048, 4096, 8192, 16384}) {   // the read kernel at several grid sizes: the best
    double b_, m_;
    if (timeit([&] { hipLaunchKernelGGL(k_read, dim3(g), dim3(block), 0, 0, a, n, out); }, (double)bytes, &b_, &m_)) return 1;
    if (b_ > rb) { rb = b_; rm = m_; rgrid = g; }
  }
  if (timeit([&] { hipLaunchKernelGGL(k_write, dim3(grid), dim3(block), 0, 0, a, n, 2.0); }, (double)bytes, &wb, &wm)) return 1;
  if (timeit([&] { hipLaunchKernelGGL(k_copy, dim3(grid), dim3(block), 0, 0, a, b, n / 2); }, (double)bytes, &cb, &cm)) return 1;
  std::printf("{\"buffer_bytes\": %zu, \"read_grid\": %d, \"read_gbs_best\": %.1f, \"read_gbs_median\": %.1f, \"write_gbs_best\": %.1f, "
              "\"write_gbs_median\": %.1f, \"copy_gbs_best\": %.1f, \"copy_gbs_median\": %.1f, \"spec_gbs\": 8000.0}\n",
              bytes, rgrid, rb, rm, wb, wm, cb, cm);
  return 0;
}
