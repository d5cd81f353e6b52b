// Probe (round 5, DESIGN.md "The policy kernel's nondeterminism"): does a
// VALU write to a VMEM store's data register, issued right after the store,
// change what the store writes? The round-4 policy kernel spilled a register
// with scratch_store_dwordx2 and overwrote it with the next instruction; its
// outputs came out wrong in lanes 48-63 of some waves under memory contention
// with two workgroups per CU. Here every lane stores a known value to scratch
// (and, as a control, to global memory), overwrites the data register with the
// next instruction, waits, reloads and counts mismatches per lane; in front of
// that each lane issues a burst of widely strided loads so the vector memory
// path is backed up, and two 256-thread workgroups share each CU.
//   hipcc --offload-arch=gfx950 -O3 tools/store_hazard_probe.hip -o tools/store_hazard_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef __attribute__((address_space(5))) int pint;

__global__ __launch_bounds__(256, 2) void probe(const float *big, long long stride, int nburst, int *bad_lane,
                                                int *gbuf, int *bad_glane, float *sink) {
  const int lane = threadIdx.x & 63;
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  // back up the memory path: nburst loads, each lane 'stride' floats apart
  float acc = 0.f;
  for (int k = 0; k < nburst; k++) acc += big[(t * 7 + k * 131) % 4096 * stride];
  volatile int frame[8];  // forces a private segment; the probe stores into its slots
  frame[lane & 7] = (int)acc;
  pint *slot = (pint *)((pint *)&frame[0]);
  const int want = 0x5000000 + (int)t;
  int v = want;
  // scratch store, then the data register overwritten by the very next instruction
  asm volatile("scratch_store_dword %1, %0, off\n\tv_mov_b32 %0, -1" : "+v"(v) : "v"(slot) : "memory");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  int back;
  asm volatile("scratch_load_dword %0, %1, off\n\ts_waitcnt vmcnt(0)" : "=v"(back) : "v"(slot) : "memory");
  if (back != want) atomicAdd(&bad_lane[lane], 1);
  // control: the same with a global store
  int g = want;
  int *gp = gbuf + t;
  asm volatile("global_store_dword %1, %0, off\n\tv_mov_b32 %0, -1" : "+v"(g) : "v"(gp) : "memory");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (__builtin_nontemporal_load(gp) != want) atomicAdd(&bad_glane[lane], 1);
  if (acc == 12345.f) sink[t] = acc + (float)frame[1];
}

int main(int argc, char **argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 50;
  const long long stride = 10880;  // floats: a rollout buffer's env stride (T n D)
  const size_t nbig = 4096ull * stride + 64;
  float *big;
  int *bad, *gbad, *gbuf;
  float *sink;
  const int blocks = 512, threads = 256;
  hipMalloc(&big, nbig * sizeof(float));
  hipMemset(big, 0, nbig * sizeof(float));
  hipMalloc(&bad, 64 * sizeof(int));
  hipMalloc(&gbad, 64 * sizeof(int));
  hipMalloc(&gbuf, (size_t)blocks * threads * sizeof(int));
  hipMalloc(&sink, (size_t)blocks * threads * sizeof(float));
  hipMemset(bad, 0, 64 * sizeof(int));
  hipMemset(gbad, 0, 64 * sizeof(int));
  for (int r = 0; r < reps; r++)
    for (int nb : {0, 8, 32})
      probe<<<blocks, threads>>>(big, stride, nb, bad, gbuf, gbad, sink);
  if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); return 1; }
  std::vector<int> h(64), hg(64);
  hipMemcpy(h.data(), bad, 64 * sizeof(int), hipMemcpyDeviceToHost);
  hipMemcpy(hg.data(), gbad, 64 * sizeof(int), hipMemcpyDeviceToHost);
  long long tot = 0, totg = 0;
  printf("lane: scratch mismatches / global mismatches (of %d stores per lane)\n", reps * 3 * blocks * 4);
  for (int l = 0; l < 64; l++) {
    tot += h[l];
    totg += hg[l];
    if (h[l] || hg[l]) printf("  lane %2d: %d / %d\n", l, h[l], hg[l]);
  }
  printf("total: scratch %lld, global %lld\n", tot, totg);
  return 0;
}
