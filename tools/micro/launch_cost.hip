// Host cost of a kernel launch on this box (diagnostic): empty kernel with a small / large argument block,
// back-to-back on one stream, and the same sequence replayed from a captured hipGraph.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

struct Big { char b[448]; };
__global__ void k_small(int* p) { if (threadIdx.x == 0 && p && blockIdx.x == 1 << 30) *p = 1; }
__global__ void k_big(Big b, int* p) { if (threadIdx.x == 0 && p && blockIdx.x == 1 << 30) *p = b.b[3]; }

int main() {
  hipStream_t s;
  hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  Big b{};
  for (int rep = 0; rep < 2; ++rep) {
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < 2000; ++i) hipLaunchKernelGGL(k_small, dim3(64), dim3(256), 0, s, nullptr);
    auto t1 = std::chrono::steady_clock::now();
    hipStreamSynchronize(s);
    auto t2 = std::chrono::steady_clock::now();
    for (int i = 0; i < 2000; ++i) hipLaunchKernelGGL(k_big, dim3(64), dim3(256), 0, s, b, nullptr);
    auto t3 = std::chrono::steady_clock::now();
    hipStreamSynchronize(s);
    auto t4 = std::chrono::steady_clock::now();
    auto us = [](auto a, auto b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
    std::printf("small: issue %.2f us/launch, drain %.2f us/kernel; big: issue %.2f, drain %.2f\n",
                us(t0, t1) / 2000, us(t0, t2) / 2000, us(t2, t3) / 2000, us(t2, t4) / 2000);
  }
  // graph of 60 kernels
  hipGraph_t g;
  hipGraphExec_t ge;
  hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
  for (int i = 0; i < 60; ++i) hipLaunchKernelGGL(k_big, dim3(64), dim3(256), 0, s, b, nullptr);
  hipStreamEndCapture(s, &g);
  hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
  for (int rep = 0; rep < 3; ++rep) {
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < 50; ++i) hipGraphLaunch(ge, s);
    auto t1 = std::chrono::steady_clock::now();
    hipStreamSynchronize(s);
    auto t2 = std::chrono::steady_clock::now();
    auto us = [](auto a, auto b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
    std::printf("graph of 60: issue %.2f us/graph, drain %.2f us/graph (%.2f us/kernel)\n", us(t0, t1) / 50,
                us(t0, t2) / 50, us(t0, t2) / 3000);
  }
  return 0;
}
