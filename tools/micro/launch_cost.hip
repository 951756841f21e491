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
  // per-iteration capture + hipGraphExecUpdate + launch (parameters change every iteration)
  {
    hipGraphExec_t ex = nullptr;
    for (int rep = 0; rep < 3; ++rep) {
      double tc = 0, tu = 0, tl = 0;
      auto T = [] { return std::chrono::steady_clock::now(); };
      auto us = [](auto a, auto b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
      auto t00 = T();
      for (int it = 0; it < 50; ++it) {
        auto a = T();
        hipGraph_t gg;
        hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
        for (int i = 0; i < 60; ++i) {
          b.b[0] = (char)it;
          hipLaunchKernelGGL(k_big, dim3(64 + (it & 1)), dim3(256), 0, s, b, nullptr);
        }
        hipStreamEndCapture(s, &gg);
        auto c = T();
        if (!ex) {
          hipGraphInstantiate(&ex, gg, nullptr, nullptr, 0);
        } else {
          hipGraphExecUpdateResult r;
          hipGraphNode_t en;
          if (hipGraphExecUpdate(ex, gg, &en, &r) != hipSuccess) {
            hipGraphExecDestroy(ex);
            hipGraphInstantiate(&ex, gg, nullptr, nullptr, 0);
            std::printf("re-instantiated\n");
          }
        }
        auto d = T();
        hipGraphLaunch(ex, s);
        auto e = T();
        hipGraphDestroy(gg);
        tc += us(a, c); tu += us(c, d); tl += us(d, e);
      }
      hipStreamSynchronize(s);
      auto t11 = T();
      std::printf("capture %.1f us, update %.1f us, launch %.1f us per graph of 60; total %.1f us/iter\n", tc / 50,
                  tu / 50, tl / 50, us(t00, t11) / 50);
    }
  }
  // timing events recorded inside a captured graph
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipGraph_t g2;
  hipGraphExec_t ge2;
  hipError_t err = hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
  hipLaunchKernelGGL(k_big, dim3(64), dim3(256), 0, s, b, nullptr);
  hipError_t er0 = hipEventRecord(e0, s);
  for (int i = 0; i < 10; ++i) hipLaunchKernelGGL(k_big, dim3(64), dim3(256), 0, s, b, nullptr);
  hipError_t er1 = hipEventRecord(e1, s);
  hipError_t er2 = hipStreamEndCapture(s, &g2);
  hipError_t er3 = hipGraphInstantiate(&ge2, g2, nullptr, nullptr, 0);
  hipError_t er4 = hipGraphLaunch(ge2, s);
  hipError_t er5 = hipStreamSynchronize(s);
  float ms = -1.f;
  hipError_t er6 = hipEventElapsedTime(&ms, e0, e1);
  std::printf("event nodes: begin %d rec %d %d end %d inst %d launch %d sync %d elapsed %d -> %.2f us for 10 kernels\n",
              (int)err, (int)er0, (int)er1, (int)er2, (int)er3, (int)er4, (int)er5, (int)er6, ms * 1e3);
  return 0;
}
