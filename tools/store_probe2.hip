// Probe: write rate of 142.6 MB (the 4v4 observation stream at 65 536 envs)
// for different grid shapes and store kinds, to see whether the emission wave
// count or the store pattern limits the step kernel's observation stream.
// Build: hipcc --offload-arch=gfx950 -O3 tools/store_probe2.hip -o tools/store_probe2
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr size_t N4 = (size_t)65536 * 2 * 4 * 17;  // float4s

// each workgroup writes a contiguous block of N4/nwg float4s
template <bool NT>
__global__ void k_block(f32x4 *out, size_t per) {
  f32x4 v = {1.f, 2.f, 3.f, (float)threadIdx.x};
  f32x4 *b = out + (size_t)blockIdx.x * per;
  for (size_t i = threadIdx.x; i < per; i += blockDim.x) {
    if (NT) __builtin_nontemporal_store(v, b + i);
    else b[i] = v;
  }
}

// one wave per workgroup; each workgroup writes its 64 envs' blocks env-major
// (1088 B per env per side), unrolled by 4 stores in flight
__global__ __launch_bounds__(64) void k_env(f32x4 *out) {
  f32x4 v = {1.f, 2.f, 3.f, (float)threadIdx.x};
  for (int side = 0; side < 2; side++) {
    f32x4 *o = out + (size_t)side * 65536 * 68 + (size_t)blockIdx.x * 64 * 68;
#pragma unroll 4
    for (int i = threadIdx.x; i < 64 * 68; i += 64) __builtin_nontemporal_store(v, o + i);
  }
}

int main() {
  f32x4 *buf;
  hipMalloc(&buf, N4 * 16);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  struct Cfg { int nwg, nthr, nt, env; } cfgs[] = {
      {1024, 64, 0, 0}, {1024, 64, 1, 0}, {1024, 128, 1, 0}, {1024, 256, 1, 0},
      {2048, 64, 1, 0}, {4096, 256, 1, 0}, {8192, 256, 0, 0}, {1024, 64, 1, 1}};
  for (auto &c : cfgs) {
    size_t per = N4 / c.nwg;
    for (int rep = 0; rep < 2; rep++) {
      hipEventRecord(a);
      for (int it = 0; it < 50; it++) {
        if (c.env) k_env<<<1024, 64>>>(buf);
        else if (c.nt) k_block<true><<<c.nwg, c.nthr>>>(buf, per);
        else k_block<false><<<c.nwg, c.nthr>>>(buf, per);
      }
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      double us = ms * 1e3 / 50;
      if (rep)
        printf("wg %d x %d thr, nt %d, env-major %d: %.2f us/launch, %.2f TB/s\n", c.nwg, c.nthr,
               c.nt, c.env, us, N4 * 16 / us / 1e6);
    }
  }
  hipFree(buf);
  return 0;
}
