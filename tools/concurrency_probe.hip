// Probe: do kernels on two HIP streams overlap on this box? A ~20 us ALU-spin
// kernel (512 workgroups x 128 threads, 39 KB dynamic LDS: half the step
// kernel's grid) launched 200x on one stream vs alternately on two streams,
// with and without per-lane scratch. Build:
//   hipcc --offload-arch=gfx950 -O2 tools/concurrency_probe.hip -o tools/concurrency_probe
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

__global__ void spin(int *out, int iters) {
  extern __shared__ int lds[];
  float x = threadIdx.x * 0.001f;
  for (int i = 0; i < iters; i++) x = x * 1.0000001f + 0.5f;
  lds[threadIdx.x] = (int)x;
  __syncthreads();
  if (x == 12345.0f) out[blockIdx.x] = lds[threadIdx.x ^ 1];
}

__global__ void spin_scratch(int *out, int iters, int k) {
  extern __shared__ int lds[];
  volatile float a[32];
  for (int i = 0; i < 32; i++) a[i] = i * 0.5f;
  float x = threadIdx.x * 0.001f;
  for (int i = 0; i < iters; i++) x = x * 1.0000001f + a[(i + k) & 31];
  lds[threadIdx.x] = (int)x;
  __syncthreads();
  if (x == 12345.0f) out[blockIdx.x] = lds[threadIdx.x ^ 1];
}

int main() {
  hipStream_t s[2];
  (void)hipStreamCreateWithFlags(&s[0], hipStreamNonBlocking);
  (void)hipStreamCreateWithFlags(&s[1], hipStreamNonBlocking);
  int *out;
  (void)hipMalloc(&out, 4096 * sizeof(int));
  const int lds = 39 * 1024, n = 200;
  for (int scratch = 0; scratch < 2; scratch++) {
    const int iters = scratch ? 2000 : 8000;
    auto launch = [&](hipStream_t st) {
      if (scratch) spin_scratch<<<512, 128, lds, st>>>(out, iters, 3);
      else spin<<<512, 128, lds, st>>>(out, iters);
    };
    for (int mode = 0; mode < 2; mode++) {
      for (int i = 0; i < 10; i++) launch(s[i & mode]);
      (void)hipDeviceSynchronize();
      auto t0 = std::chrono::steady_clock::now();
      for (int i = 0; i < n; i++) launch(s[i & mode]);
      (void)hipDeviceSynchronize();
      auto t1 = std::chrono::steady_clock::now();
      printf("scratch=%d streams=%d: %.2f us per kernel\n", scratch, mode + 1,
             std::chrono::duration<double, std::micro>(t1 - t0).count() / n);
    }
  }
  return 0;
}
