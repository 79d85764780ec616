// Host cost of one kernel launch on MI355X (no synchronisation inside the timed loop): hipLaunchKernelGGL,
// hipExtLaunchKernelGGL (null events) and hipModuleLaunchKernel with a pre-packed kernarg buffer, for a kernel with
// ~700 bytes of arguments (the size of k_sigma_tw's).   hipcc --offload-arch=gfx950 -O2 launch_cost.hip -o launch_cost
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <chrono>
#include <cstdio>
#include <cstring>

struct Big { double v[80]; };   // 640 bytes by value

__global__ void k_args(Big b, const double* p, double* q, int n, long long m) {
  if (threadIdx.x == 0 && blockIdx.x == 0 && n < 0) q[0] = b.v[0] + p[0] + (double)m;
}

struct Packed {   // the kernel's explicit arguments in order, natural alignment
  Big b;
  const double* p;
  double* q;
  int n;
  long long m;
};

int main() {
  hipStream_t s;
  hipStreamCreate(&s);
  double* d;
  hipMalloc(&d, 64);
  Big b{};
  const int N = 200;   // (below the queue size: the enqueue never waits for a free slot)
  auto run = [&](const char* name, auto&& launch) {
    for (int i = 0; i < 100; ++i) launch();
    hipStreamSynchronize(s);
    double best = 1e30;
    for (int rep = 0; rep < 5; ++rep) {
      auto t0 = std::chrono::steady_clock::now();
      for (int i = 0; i < N; ++i) launch();
      auto t1 = std::chrono::steady_clock::now();
      hipStreamSynchronize(s);
      const double us = std::chrono::duration<double, std::micro>(t1 - t0).count() / N;
      best = us < best ? us : best;
    }
    std::printf("%-44s %.2f us per launch (enqueue, best of 5 x %d)\n", name, best, N);
  };
  run("hipLaunchKernelGGL", [&] { hipLaunchKernelGGL(k_args, dim3(8), dim3(256), 0, s, b, d, d, 1, 2LL); });
  run("hipExtLaunchKernelGGL (null events)", [&] {
    hipExtLaunchKernelGGL(k_args, dim3(8), dim3(256), 0, s, nullptr, nullptr, 0, b, d, d, 1, 2LL);
  });
  hipFunction_t f = nullptr;
  if (hipGetFuncBySymbol(&f, reinterpret_cast<const void*>(&k_args)) != hipSuccess || !f) {
    std::printf("hipGetFuncBySymbol failed\n");
    return 1;
  }
  Packed pk{};
  pk.b = b; pk.p = d; pk.q = d; pk.n = 1; pk.m = 2;
  size_t sz = sizeof(pk);
  void* extra[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &pk, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz, HIP_LAUNCH_PARAM_END};
  run("hipModuleLaunchKernel (packed kernargs)", [&] {
    hipModuleLaunchKernel(f, 8, 1, 1, 256, 1, 1, 0, s, nullptr, extra);
  });
  void* args[] = {&b, &pk.p, &pk.q, &pk.n, &pk.m};
  run("hipModuleLaunchKernel (kernelParams)", [&] {
    hipModuleLaunchKernel(f, 8, 1, 1, 256, 1, 1, 0, s, args, nullptr);
  });
  std::printf("last error: %s\n", hipGetErrorString(hipGetLastError()));
  return 0;
}
