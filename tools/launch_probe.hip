// Probe: host cost of hipLaunchKernel on this box for an empty kernel with
// small vs ~700-byte kernel arguments, and for a kernel that uses scratch,
// plus a 100-launch hipGraph replay. Build: hipcc --offload-arch=gfx950 -O2
// tools/launch_probe.hip -o tools/launch_probe
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

struct Big { double v[88]; };

__global__ void k_small(int *p) { if (p && threadIdx.x == 1000) p[0] = 1; }
__global__ void k_big(Big b, int *p) { if (p && threadIdx.x == 1000) p[0] = (int)b.v[3]; }
__global__ void k_scratch(int *p, int n) {
  volatile int a[64];
  for (int i = 0; i < 64; i++) a[i] = i * n;
  if (p && threadIdx.x == 1000) p[0] = a[n & 63];
}

template <class F>
double per_call_us(F f, int n) {
  for (int i = 0; i < 100; i++) f();
  (void)hipDeviceSynchronize();
  auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < n; i++) f();
  auto t1 = std::chrono::steady_clock::now();
  (void)hipDeviceSynchronize();
  auto t2 = std::chrono::steady_clock::now();
  double host = std::chrono::duration<double, std::micro>(t1 - t0).count() / n;
  double wall = std::chrono::duration<double, std::micro>(t2 - t0).count() / n;
  printf("  host %.2f us/launch, wall %.2f us/launch\n", host, wall);
  return host;
}

int main() {
  hipStream_t st;
  (void)hipStreamCreate(&st);
  Big b{};
  const int n = 20000;
  printf("small args:\n");
  per_call_us([&] { k_small<<<1024, 128, 0, st>>>(nullptr); }, n);
  printf("700-byte args:\n");
  per_call_us([&] { k_big<<<1024, 128, 0, st>>>(b, nullptr); }, n);
  printf("700-byte args + 39 KB dynamic LDS:\n");
  per_call_us([&] { k_big<<<1024, 128, 39 * 1024, st>>>(b, nullptr); }, n);
  (void)hipFuncSetAttribute((const void *)k_big, hipFuncAttributeMaxDynamicSharedMemorySize, 156 * 1024);
  printf("700-byte args, 512 x 256 threads + 78 KB LDS:\n");
  per_call_us([&] { k_big<<<512, 256, 78 * 1024, st>>>(b, nullptr); }, n);
  printf("700-byte args, 256 x 512 threads + 156 KB LDS:\n");
  per_call_us([&] { k_big<<<256, 512, 156 * 1024, st>>>(b, nullptr); }, n);
  printf("scratch kernel:\n");
  per_call_us([&] { k_scratch<<<1024, 128, 0, st>>>(nullptr, 3); }, n);
  // graph of 100 launches
  hipGraph_t g;
  hipGraphExec_t ge;
  (void)hipStreamBeginCapture(st, hipStreamCaptureModeGlobal);
  for (int i = 0; i < 100; i++) k_big<<<1024, 128, 39 * 1024, st>>>(b, nullptr);
  (void)hipStreamEndCapture(st, &g);
  (void)hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
  printf("graph of 100 (per kernel):\n");
  double h = per_call_us([&] { (void)hipGraphLaunch(ge, st); }, 200);
  printf("  -> %.2f us per kernel host\n", h / 100);
  return 0;
}
