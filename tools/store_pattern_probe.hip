// Probe: device write rate of the observation stream's store patterns at the
// step kernel's grid shape (1024 workgroups x 1 wave, 64 envs x 8 rows x 272 B
// each = 142.6 MB). Modes: 0 contiguous 1 KB per instruction; 1 emission
// pattern (agent-major row pieces {5,4,4,4} float4s, rows 1088 B apart);
// 2 whole rows (272 B runs). Build: hipcc --offload-arch=gfx950 -O3.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int ENVS = 65536, NS = 4, D4 = 17;

__global__ __launch_bounds__(64) void k_contig(f32x4 *out) {
  // each wave writes its 64 envs x 8 rows x 17 float4 = 8704 float4 contiguous
  f32x4 *b = out + (size_t)blockIdx.x * 64 * 2 * NS * D4;
  f32x4 v = {1.f, 2.f, 3.f, (float)threadIdx.x};
  for (int i = threadIdx.x; i < 64 * 2 * NS * D4; i += 64) b[i] = v;
}

__global__ __launch_bounds__(64) void k_emit(f32x4 *out, int whole) {
  const int lane = threadIdx.x;
  f32x4 v = {1.f, 2.f, 3.f, (float)lane};
  const int GB[5] = {0, 5, 9, 13, D4};
  for (int side = 0; side < 2; side++) {
    f32x4 *o = out + (size_t)side * ENVS * NS * D4 + (size_t)blockIdx.x * 64 * NS * D4;
    for (int kl = 0; kl < NS; kl++) {
      if (whole) {
        for (int i = lane; i < 64 * D4; i += 64) {
          int r = i / D4, cc = i - r * D4;
          o[((size_t)r * NS + kl) * D4 + cc] = v;
        }
      } else {
        for (int g = 0; g < 4; g++) {
          int n = GB[g + 1] - GB[g];
          for (int it = 0; it < n; it++) {
            int i = it * 64 + lane, r = i / n, cc = i - r * n;
            o[((size_t)r * NS + kl) * D4 + GB[g] + cc] = v;
          }
        }
      }
    }
  }
}

int main() {
  size_t n4 = (size_t)ENVS * 2 * NS * D4;
  f32x4 *buf;
  hipMalloc(&buf, n4 * 16);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int mode = 0; mode < 3; mode++) {
    for (int rep = 0; rep < 2; rep++) {
      hipEventRecord(a);
      for (int it = 0; it < 50; it++) {
        if (mode == 0) k_contig<<<ENVS / 64, 64>>>(buf);
        else k_emit<<<ENVS / 64, 64>>>(buf, mode == 2);
      }
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      double us = ms * 1e3 / 50;
      if (rep) printf("mode %d: %.2f us/launch, %.2f TB/s\n", mode, us, n4 * 16 / us / 1e6);
    }
  }
  hipFree(buf);
  return 0;
}
