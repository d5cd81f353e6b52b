// Probe (round 5, DESIGN.md "The policy kernel's nondeterminism"): can a VALU
// write to the data or address VGPR of a ds_write_b128, issued right after it,
// change what the LDS write stores when the LDS is busy with other waves?
// lnw_policy_act wrote its fc1 tile with eight ds_write_b128 and hipcc let the
// next VALU instructions overwrite the first write's data (v2, v3) and, in the
// round-4 build, the address of all eight; the tile rows of lanes 48-63 came out
// wrong in waves sharing a SIMD with another wave. Here every even wave writes a
// known 16-B row per lane with ds_write_b128 and overwrites the data (mode 1) or
// the address (mode 2) VGPR in the next instruction (mode 0: after s_waitcnt
// lgkmcnt(0), the control), then checks its row; every odd wave keeps the LDS
// busy with b128 reads and writes of its own area (partner 0) or runs
// v_mfma_f32_16x16x32_bf16 chains on registers (partner 1). Mismatches are
// counted per lane. Mode 3: the data VGPRs written by v_mov right before the
// ds_write_b128 (a read-after-write the hardware interlocks).
// usage: ds_hazard_probe [iters] [partner]
//   hipcc --offload-arch=gfx950 -O3 tools/ds_hazard_probe.hip -o tools/ds_hazard_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

template <int MODE>
__global__ __launch_bounds__(512, 1) void probe(int iters, int partner, int *bad, int *sink) {
  extern __shared__ i32x4 lds[];                 // [8 waves][64 lanes][4] int4 rows
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  i32x4 *mine = lds + (w * 64 + lane) * 4;
  int acc = 0;
  for (int it = 0; it < iters; it++) {
    if ((w & 1) && partner == 1) {  // matrix-core chains of the SIMD's other wave
      bf16x8 a;
#pragma unroll
      for (int j = 0; j < 8; j++) a[j] = (__bf16)(0.001f * (float)(lane + j + it));
      f32x4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = c0, c2 = c0, c3 = c0;
      for (int k = 0; k < 16; k++) {
        c0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, a, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, a, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, a, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, a, c3, 0, 0, 0);
      }
      acc += (int)(c0[0] + c1[1] + c2[2] + c3[3]);
    } else if (w & 1) {  // contention: LDS traffic of the SIMD's other wave
      i32x4 v = mine[0];
#pragma unroll
      for (int k = 0; k < 8; k++) {
        mine[k & 3] = v + k;
        v = mine[(k + 1) & 3];
      }
      acc += v.x;
    } else {
      const i32x4 want = {0x1000000 + (int)threadIdx.x, it, (int)blockIdx.x, 0x7777};
      // the LDS byte address of this lane's row (32-bit)
      const unsigned addr = (unsigned)(size_t)(__attribute__((address_space(3))) i32x4 *)mine;
#define PROBE_SETUP "v_mov_b32 v100, %0\n\tv_mov_b32 v101, %1\n\tv_mov_b32 v102, %2\n\tv_mov_b32 v103, %3\n\t" \
                    "v_mov_b32 v104, %4\n\ts_nop 4\n\tds_write_b128 v104, v[100:103]\n\t"
      if (MODE == 0)
        asm volatile(PROBE_SETUP "s_waitcnt lgkmcnt(0)\n\tv_mov_b32 v100, -1\n\tv_mov_b32 v104, 0"
                     :: "v"(want.x), "v"(want.y), "v"(want.z), "v"(want.w), "v"(addr)
                     : "v100", "v101", "v102", "v103", "v104", "memory");
      else if (MODE == 1)
        asm volatile(PROBE_SETUP "v_mov_b32 v100, -1\n\tv_mov_b32 v101, -1\n\ts_waitcnt lgkmcnt(0)"
                     :: "v"(want.x), "v"(want.y), "v"(want.z), "v"(want.w), "v"(addr)
                     : "v100", "v101", "v102", "v103", "v104", "memory");
      else if (MODE == 2)
        asm volatile(PROBE_SETUP "v_mov_b32 v104, 0\n\ts_waitcnt lgkmcnt(0)"
                     :: "v"(want.x), "v"(want.y), "v"(want.z), "v"(want.w), "v"(addr)
                     : "v100", "v101", "v102", "v103", "v104", "memory");
      else  // mode 3: the data written by VALU right before the write (no wait states between)
        asm volatile("v_mov_b32 v104, %4\n\ts_nop 4\n\t"
                     "v_mov_b32 v100, %0\n\tv_mov_b32 v101, %1\n\tv_mov_b32 v102, %2\n\tv_mov_b32 v103, %3\n\t"
                     "ds_write_b128 v104, v[100:103]\n\ts_waitcnt lgkmcnt(0)"
                     :: "v"(want.x), "v"(want.y), "v"(want.z), "v"(want.w), "v"(addr)
                     : "v100", "v101", "v102", "v103", "v104", "memory");
      const i32x4 got = mine[0];
      if (got.x != want.x || got.y != want.y || got.z != want.z || got.w != want.w) atomicAdd(&bad[lane], 1);
    }
  }
  if (acc == 12345) sink[threadIdx.x] = acc;
}

int main(int argc, char **argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 2000;
  const int partner = argc > 2 ? atoi(argv[2]) : 0;
  int *bad, *sink;
  hipMalloc(&bad, 4 * 64 * sizeof(int));
  hipMalloc(&sink, 512 * sizeof(int));
  hipMemset(bad, 0, 4 * 64 * sizeof(int));
  const size_t lds = 8 * 64 * 4 * sizeof(i32x4);  // 32 KB per block
  const int blocks = 1024;                          // 4 per CU
  probe<0><<<blocks, 512, lds>>>(iters, partner, bad, sink);
  probe<1><<<blocks, 512, lds>>>(iters, partner, bad + 64, sink);
  probe<2><<<blocks, 512, lds>>>(iters, partner, bad + 128, sink);
  probe<3><<<blocks, 512, lds>>>(iters, partner, bad + 192, sink);
  if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); return 1; }
  std::vector<int> h(256);
  hipMemcpy(h.data(), bad, 256 * sizeof(int), hipMemcpyDeviceToHost);
  const char *names[4] = {"wait before overwrite (control)", "data overwritten next", "address overwritten next",
                          "data written by VALU just before"};
  for (int m = 0; m < 4; m++) {
    long long tot = 0;
    int lo = 64, hi = -1;
    for (int l = 0; l < 64; l++) {
      tot += h[m * 64 + l];
      if (h[m * 64 + l]) { lo = l < lo ? l : lo; hi = l; }
    }
    printf("partner %s, mode %d (%s): %lld mismatches of %lld writes", partner ? "mfma" : "lds", m, names[m], tot, (long long)iters * blocks * 4 * 64);
    if (tot) printf(", lanes %d..%d", lo, hi);
    printf("\n");
  }
  return 0;
}
