// Probe (round 5, DESIGN.md "The split contact step with rows"): can an LDS
// read that returns into the data registers of a vector-memory store issued
// just before it change what the store writes, when the wave's store queue is
// backed up? write_obs_t's passes read the next pass's stage into the registers
// the previous pass's buffer_store_dwordx4 took its data from, and its rows came
// out with float4s of other rows until each pass waited for its stores.
// Every lane: a burst of `burst` float4 stores (to back the queue up), then the
// test store of a known float4 from v[100:103] followed at once by a
// ds_read_b128 of a poison value into v[100:103] (mode 0: plain store, 1: sc1
// write-through, 2: nt; mode 3: the same with s_waitcnt vmcnt(0) before the
// LDS read, the control); then the store's target is checked.
//   hipcc --offload-arch=gfx950 -O3 tools/store_lds_war_probe.hip -o tools/store_lds_war_probe
//   usage: store_lds_war_probe [iters] [burst]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef int i32x4 __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ __launch_bounds__(512, 1) void probe(int iters, int burst, i32x4 *junk, i32x4 *target, int *bad) {
  extern __shared__ i32x4 lds[];  // one poison row per lane
  const int lane = threadIdx.x & 63;
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  lds[threadIdx.x] = i32x4{-1, -2, -3, -4};
  const unsigned laddr = (unsigned)(size_t)(__attribute__((address_space(3))) i32x4 *)&lds[threadIdx.x];
  i32x4 *mine = target + t;
  for (int it = 0; it < iters; it++) {
    for (int k = 0; k < burst; k++) junk[(t * 16 + (k & 15)) % (1 << 22)] = i32x4{k, it, (int)t, 5};
    const i32x4 want = {0x1000000 + (int)t, it, (int)blockIdx.x, 0x7777};
#define SETUP "v_mov_b32 v100, %0\n\tv_mov_b32 v101, %1\n\tv_mov_b32 v102, %2\n\tv_mov_b32 v103, %3\n\ts_nop 4\n\t"
    if (MODE == 0)
      asm volatile(SETUP "global_store_dwordx4 %4, v[100:103], off\n\tds_read_b128 v[100:103], %5\n\t"
                   "s_waitcnt vmcnt(0) lgkmcnt(0)"
                   :: "v"(want.x), "v"(want.y), "v"(want.z), "v"(want.w), "v"(mine), "v"(laddr)
                   : "v100", "v101", "v102", "v103", "memory");
    else if (MODE == 1)
      asm volatile(SETUP "global_store_dwordx4 %4, v[100:103], off sc1\n\tds_read_b128 v[100:103], %5\n\t"
                   "s_waitcnt vmcnt(0) lgkmcnt(0)"
                   :: "v"(want.x), "v"(want.y), "v"(want.z), "v"(want.w), "v"(mine), "v"(laddr)
                   : "v100", "v101", "v102", "v103", "memory");
    else if (MODE == 2)
      asm volatile(SETUP "global_store_dwordx4 %4, v[100:103], off nt\n\tds_read_b128 v[100:103], %5\n\t"
                   "s_waitcnt vmcnt(0) lgkmcnt(0)"
                   :: "v"(want.x), "v"(want.y), "v"(want.z), "v"(want.w), "v"(mine), "v"(laddr)
                   : "v100", "v101", "v102", "v103", "memory");
    else
      asm volatile(SETUP "global_store_dwordx4 %4, v[100:103], off sc1\n\ts_waitcnt vmcnt(0)\n\t"
                   "ds_read_b128 v[100:103], %5\n\ts_waitcnt vmcnt(0) lgkmcnt(0)"
                   :: "v"(want.x), "v"(want.y), "v"(want.z), "v"(want.w), "v"(mine), "v"(laddr)
                   : "v100", "v101", "v102", "v103", "memory");
    const i32x4 got = __builtin_nontemporal_load(mine);
    if (got.x != want.x || got.y != want.y || got.z != want.z || got.w != want.w) atomicAdd(&bad[lane], 1);
  }
}

int main(int argc, char **argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 200;
  const int burst = argc > 2 ? atoi(argv[2]) : 16;
  const int blocks = 1024, threads = 512;
  i32x4 *junk, *target;
  int *bad;
  if (hipMalloc(&junk, sizeof(i32x4) << 22) != hipSuccess) return 1;
  if (hipMalloc(&target, sizeof(i32x4) * blocks * threads) != hipSuccess) return 1;
  if (hipMalloc(&bad, 4 * 64 * sizeof(int)) != hipSuccess) return 1;
  if (hipMemset(bad, 0, 4 * 64 * sizeof(int)) != hipSuccess) return 1;
  const size_t lds = threads * sizeof(i32x4);
  probe<0><<<blocks, threads, lds>>>(iters, burst, junk, target, bad);
  probe<1><<<blocks, threads, lds>>>(iters, burst, junk, target, bad + 64);
  probe<2><<<blocks, threads, lds>>>(iters, burst, junk, target, bad + 128);
  probe<3><<<blocks, threads, lds>>>(iters, burst, junk, target, bad + 192);
  if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); return 1; }
  std::vector<int> h(256);
  if (hipMemcpy(h.data(), bad, 256 * sizeof(int), hipMemcpyDeviceToHost) != hipSuccess) return 1;
  const char *names[4] = {"plain store, LDS read next", "sc1 store, LDS read next", "nt store, LDS read next",
                          "sc1 store, vmcnt(0) before the LDS read (control)"};
  for (int m = 0; m < 4; m++) {
    long long tot = 0;
    int lo = 64, hi = -1;
    for (int l = 0; l < 64; l++) {
      tot += h[m * 64 + l];
      if (h[m * 64 + l]) { lo = l < lo ? l : lo; hi = l; }
    }
    printf("burst %d, mode %d (%s): %lld mismatches of %lld stores", burst, m, names[m], tot,
           (long long)iters * blocks * threads);
    if (tot) printf(", lanes %d..%d", lo, hi);
    printf("\n");
  }
  return 0;
}
