// tan_probe.hip — device tan(x) for EW-fix slopes: ocml's tan against an
// fdlibm-style reduction + __kernel_tan (lnw_device.h: tan_fd), speed on the
// GPU and agreement with the host libm (glibc) on the bearing domain
// x = radians(b), b in [-1, 370) degrees.
// build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/tan_probe.hip -Ilittoral-naval-warfare-marl_amd/csrc -Iinclude -o /tmp/tan_probe
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <cstdio>
#include <vector>

#include "lnw.h"
#include "lnw_device.h"

using namespace lnw;

template <bool FD>
__global__ void tan_kernel(const double *x, double *y, long long n, int reps) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double v = x[i], acc = 0.0;
  for (int r = 0; r < reps; r++) {
    const double t = FD ? tan_fd(v) : tan(v);
    acc += t;
    v = v + 1e-9;
  }
  y[i] = acc;
}

int main() {
  const long long n = 1 << 22;
  std::vector<double> hx(n);
  for (long long i = 0; i < n; i++) hx[i] = (-1.0 + 371.0 * (double)i / (double)n) * (3.141592653589793 / 180.0);
  double *dx, *dy;
  (void)hipMalloc(&dx, n * 8);
  (void)hipMalloc(&dy, n * 8);
  (void)hipMemcpy(dx, hx.data(), n * 8, hipMemcpyHostToDevice);
  std::vector<double> out(n);
  for (int fd = 0; fd < 2; fd++) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int it = 0; it < 2; it++) {
      (void)hipEventRecord(e0);
      if (fd) tan_kernel<true><<<n / 256, 256>>>(dx, dy, n, 16);
      else tan_kernel<false><<<n / 256, 256>>>(dx, dy, n, 16);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
    }
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (fd) tan_kernel<true><<<n / 256, 256>>>(dx, dy, n, 1);
    else tan_kernel<false><<<n / 256, 256>>>(dx, dy, n, 1);
    (void)hipMemcpy(out.data(), dy, n * 8, hipMemcpyDeviceToHost);
    long long diff = 0, maxulp = 0;
    for (long long i = 0; i < n; i++) {
      const double ref = std::tan(hx[i]);
      if (out[i] != ref) {
        diff++;
        long long a, b;
        std::memcpy(&a, &out[i], 8);
        std::memcpy(&b, &ref, 8);
        long long u = a > b ? a - b : b - a;
        if (u > maxulp) maxulp = u;
      }
    }
    printf("%s: %.3f ms for %lld x 16 tans; vs glibc: %lld of %lld differ, max %lld ulp\n",
           fd ? "tan_fd (fdlibm)" : "ocml tan", ms, n, diff, n, maxulp);
  }
  return 0;
}
