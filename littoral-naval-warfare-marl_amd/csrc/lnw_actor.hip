// Batched policy forward: the convolutional head of
// the reference actor (network.py:70-82, MLP.forward) for B observation rows at
// once — conv 1->5 (3x3, pad 1) over the 7x7 terrain window, BatchNorm, ReLU,
// 2x2 max pool, conv 5->8, BatchNorm, ReLU, 2x2 max pool, linear 8->12, then the
// LayerNorm over [head, rest of the observation] (network.py:83-85). This is
// the part of the network with no batched BLAS form (per-row BatchNorm
// statistics over 7x7 / 3x3 maps); the tanh MLP and Normal heads run as batched
// GEMMs in lnw.rollout.BatchedActor.
//
// One thread per row; the packed parameters (578 + 2 n_in floats, order below,
// written by BatchedActor.packed_features()) are staged once per workgroup in
// LDS and read as broadcasts. Channels are streamed (49 conv outputs live at a
// time).
// bn_running = 0 normalises with each row's own statistics (the reference's
// one-state-at-a-time training-mode calls, ppo.py:504-512), 1 with the running
// ones.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <string>

#include "lnw.h"
#include "lnw_device.h"

namespace {

using namespace lnw;

constexpr int WIN = 49;       // 7x7 terrain window
constexpr float BN_EPS = 1e-5f;

// packed conv-head parameter layout (floats)
constexpr int C1W = 0, C1B = 45, B1W = 50, B1B = 55, B1M = 60, B1V = 65;
constexpr int C2W = 70, C2B = 430, B2W = 438, B2B = 446, B2M = 454, B2V = 462;
constexpr int HW = 470, HB = 566, CONV_PARAMS = 578;  // then LayerNorm w, b [n_in] each
constexpr int MAX_IN = 64;                            // n_in = obs_dim - 49 + 12 bound
constexpr float LN_EPS = 1e-5f;

extern __shared__ float actor_lds[];

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef double f64x4 __attribute__((ext_vector_type(4)));
// read-only parameters through the constant address space: wave-uniform
// indices then become scalar loads (s_load / s_buffer_load) into SGPRs, one
// load per 16 weights for the whole wave, instead of per-lane vector loads
typedef const __attribute__((address_space(4))) float cfloat;

// BatchNorm of one channel's n values: own statistics (biased variance) or
// running ones, then the affine, then ReLU.
template <int N>
__device__ inline void bn_relu(float (&v)[N], const float *w, const float *b, const float *rm,
                               const float *rv, int c, bool running) {
  float mean, var;
  if (running) {
    mean = rm[c];
    var = rv[c];
  } else {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < N; i++) s += v[i];
    mean = s / (float)N;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < N; i++) q += (v[i] - mean) * (v[i] - mean);
    var = q / (float)N;
  }
  const float inv = 1.0f / sqrtf(var + BN_EPS);
#pragma unroll
  for (int i = 0; i < N; i++) v[i] = fmaxf((v[i] - mean) * inv * w[c] + b[c], 0.f);
}

constexpr int CH_THREADS = 256;
// lnw_policy_act's block (probe builds may change it: tools/build_probes.sh)
#ifndef LNW_PA_THREADS
#define LNW_PA_THREADS 512
#endif
constexpr int PA_THREADS = LNW_PA_THREADS;

// The conv head of one row (network.py:70-82): conv 1->5 over the 7x7 window
// win[0..48] (registers) -> BN -> ReLU -> 2x2 pool, conv 5->8 -> BN -> ReLU ->
// pool, folded into the linear 8->12 (h). P: packed parameters in LDS
// (broadcast reads); pc: the thread's column of a [45][stride] LDS parking area
// for the pooled conv1 maps.
__device__ __forceinline__ void conv_head_win(const float *P, const float (&win)[WIN], float *pc, int stride,
                                              bool running, float (&h)[12]) {
  // multiply-adds fused here (the build's -ffp-contract=off is for the step
  // kernels' bit-exactness; the policy is held to the tolerance of fp32 torch,
  // whose conv kernels fuse them too): half the VALU work of the head
#pragma clang fp contract(fast)
  // conv1 (1 -> 5, 3x3, pad 1) -> BN -> ReLU -> 2x2 max pool (7x7 -> 3x3),
  // one channel at a time (rolled: 49 outputs live)
#pragma unroll 1
  for (int c = 0; c < 5; c++) {
    float v[49];
    const float *w = P + C1W + c * 9;
#pragma unroll
    for (int i = 0; i < 7; i++)
#pragma unroll
      for (int j = 0; j < 7; j++) {
        float s = P[C1B + c];
#pragma unroll
        for (int ki = 0; ki < 3; ki++)
#pragma unroll
          for (int kj = 0; kj < 3; kj++) {
            const int ii = i + ki - 1, jj = j + kj - 1;
            if (ii >= 0 && ii < 7 && jj >= 0 && jj < 7) s += w[ki * 3 + kj] * win[ii * 7 + jj];
          }
        v[i * 7 + j] = s;
      }
    bn_relu<49>(v, P + B1W, P + B1B, P + B1M, P + B1V, c, running);
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
      for (int j = 0; j < 3; j++) {
        const int r0 = 2 * i, c0 = 2 * j;
        pc[(c * 9 + i * 3 + j) * stride] =
            fmaxf(fmaxf(v[r0 * 7 + c0], v[r0 * 7 + c0 + 1]),
                  fmaxf(v[(r0 + 1) * 7 + c0], v[(r0 + 1) * 7 + c0 + 1]));
      }
  }
  // conv2 (5 -> 8, 3x3, pad 1) -> BN -> ReLU -> 2x2 max pool (3x3 -> 1x1),
  // folded straight into the linear 8 -> 12 (convhead). Four output maps at a
  // time accumulate while the input channels stream in from LDS one at a time
  // (36 accumulators and 9 inputs live: the head then fits the kernel's
  // registers without spilling; h sums the maps in the same order).
#pragma unroll
  for (int k = 0; k < 12; k++) h[k] = P[HB + k];
#pragma unroll 1
  for (int c0 = 0; c0 < 8; c0 += 4) {
    float v2[4][9];
#pragma unroll
    for (int co = 0; co < 4; co++)
#pragma unroll
      for (int p = 0; p < 9; p++) v2[co][p] = P[C2B + c0 + co];
#pragma unroll 1
    for (int ci = 0; ci < 5; ci++) {
      float pin[9];
#pragma unroll
      for (int k = 0; k < 9; k++) pin[k] = pc[(ci * 9 + k) * stride];
#pragma unroll
      for (int co = 0; co < 4; co++) {
        const float *w = P + C2W + ((c0 + co) * 5 + ci) * 9;
#pragma unroll
        for (int i = 0; i < 3; i++)
#pragma unroll
          for (int j = 0; j < 3; j++)
#pragma unroll
            for (int ki = 0; ki < 3; ki++)
#pragma unroll
              for (int kj = 0; kj < 3; kj++) {
                const int ii = i + ki - 1, jj = j + kj - 1;
                if (ii >= 0 && ii < 3 && jj >= 0 && jj < 3) v2[co][i * 3 + j] += w[ki * 3 + kj] * pin[ii * 3 + jj];
              }
      }
    }
#pragma unroll
    for (int co = 0; co < 4; co++) {
      bn_relu<9>(v2[co], P + B2W, P + B2B, P + B2M, P + B2V, c0 + co, running);
      const float f = fmaxf(fmaxf(v2[co][0], v2[co][1]), fmaxf(v2[co][3], v2[co][4]));
#pragma unroll
      for (int k = 0; k < 12; k++) h[k] += P[HW + k * 8 + c0 + co] * f;
    }
  }
}

// conv_head_win on a row in memory (features_kernel)
__device__ __forceinline__ void conv_head_row(const float *P, const float *x, float *pc, int stride,
                                              bool running, float (&h)[12]) {
  float win[WIN];
#pragma unroll
  for (int i = 0; i < WIN; i++) win[i] = x[i];
  conv_head_win(P, win, pc, stride, running, h);
}

// LayerNorm over [h, tail] (biased variance; tail = x[49:], n_in - 12 values)
// with its affine, into u[0..n_in)
template <int NI>
__device__ __forceinline__ void layer_norm_tail(const float *P, const float (&tl)[NI - 12], int n_in,
                                                const float (&h)[12], float (&u)[NI]) {
#pragma unroll
  for (int k = 0; k < NI; k++) u[k] = k < 12 ? h[k < 12 ? k : 0] : (k < n_in ? tl[k < 12 ? 0 : k - 12] : 0.f);
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < NI; k++) s += k < n_in ? u[k] : 0.f;
  const float mean = s / (float)n_in;
  float q = 0.f;
#pragma unroll
  for (int k = 0; k < NI; k++) q += k < n_in ? (u[k] - mean) * (u[k] - mean) : 0.f;
  const float inv = 1.0f / sqrtf(q / (float)n_in + LN_EPS);
  const float *lw = P + CONV_PARAMS, *lb = P + CONV_PARAMS + n_in;
#pragma unroll
  for (int k = 0; k < NI; k++) u[k] = k < n_in ? (u[k] - mean) * inv * lw[k] + lb[k] : 0.f;
}

// the LayerNorm tail of a row in memory: x[49 .. D - 1], every load issued at
// once (indices clamped into the row, values past n_in - 12 unused)
template <int NT>
__device__ __forceinline__ void load_tail(const float *x, int D, float (&tl)[NT]) {
#pragma unroll
  for (int k = 0; k < NT; k++) tl[k] = x[WIN + k < D ? WIN + k : D - 1];
}

// The same for a 16-B aligned row of D % 4 == 0 floats (lnw_policy_act checks
// both): the float4 quads from x[48] on, one dwordx4 per quad instead of one
// dword load per value (quad indices clamped into the row; the values past
// n_in - 12 they duplicate are unused)
template <int NT>
__device__ __forceinline__ void load_tail_q(const float *x, int D, float (&tl)[NT]) {
  constexpr int NQ = (NT + 1 + 3) / 4;  // x[48] .. x[48 + NT]
  const int D4 = D >> 2;
  const f32x4 *x4 = (const f32x4 *)x;
  f32x4 q[NQ];
#pragma unroll
  for (int j = 0; j < NQ; j++) q[j] = x4[12 + j < D4 ? 12 + j : D4 - 1];
#pragma unroll
  for (int k = 0; k < NT; k++) tl[k] = q[(k + 1) >> 2][(k + 1) & 3];
}

// (the torch implementation's conv head, off the fused path: one wave per
// SIMD, so the compiler has the registers to keep the head out of scratch)
template <int NI>
__global__ __launch_bounds__(CH_THREADS, 1) void features_kernel(const float *params, int obs_dim,
                                                              const float *obs, int B, int bn_running,
                                                              float *out) {
  const int n_in = obs_dim - WIN + 12;
  const int n_par = CONV_PARAMS + 2 * n_in;
  float *P = actor_lds;                           // [n_par] parameters
  // pooled conv1 maps: per wave [45][64], one column per lane (as lnw_policy_act)
  float *pool1 = actor_lds + n_par + (threadIdx.x / WAVE) * 45 * WAVE + (threadIdx.x & (WAVE - 1));
  for (int i = threadIdx.x; i < n_par; i += blockDim.x) P[i] = params[i];
  __syncthreads();
  const bool running = bn_running != 0;
  // (one row per thread, 32-bit row indices checked on the host; the tail is
  // loaded after the head: nothing but the row index lives across it)
  const int row = blockIdx.x * blockDim.x + threadIdx.x;
  if (row < B) {
    float h[12];
    conv_head_row(P, obs + (long long)row * obs_dim, pool1, WAVE, running, h);
    float tl[NI - 12], u[NI];
    load_tail(obs + (long long)row * obs_dim, obs_dim, tl);
    layer_norm_tail<NI>(P, tl, n_in, h, u);
    float *o = out + (long long)row * n_in;
#pragma unroll
    for (int k = 0; k < NI; k++)
      if (k < n_in) o[k] = u[k];
  }
}

// ---------------------------------------------------------------------------
// Fused policy step (lnw_policy_act): for every row of one side's observation
// block, the whole reference actor forward (network.py:70-115 / get_dist
// :117-152) and what the MAPPO rollout does with it (ppo.py:497-577) in one
// launch, one thread per row:
//   conv head + LayerNorm (as features_kernel), then fc1 64 / fc2 64 / fc3 32
//   tanh layers and the normal / log-std heads with weights read as wave-
//   uniform scalar loads (every lane of the wave uses the same weight), fp32
//   FMA;
//   NaN heads -> N(0, 1) for the row (the reference returns None there);
//   sample: N(mean, std) from keyed Philox normals (+ N(0, noise)), clamped to
//   [0, 1], and its log-probability; or, forced, the log-probability of given
//   actions (get_dist);
//   outputs: the f64 action rows of lnw_step (sunk ships 0), the rollout's
//   action / log-probability rows (0 after the episode ended) and the
//   observation copy for the rollout buffer; the lane of ship 0 also writes its
//   env's scripted red rows (red_steps*.csv, ppo.py:560-566) and the action
//   array's row kinds (np.asarray, ppo.py:577).
// Keyed draws (keyed_normal in lnw/rollout.py): uniform k of global row r at
// Philox counter (slot << 40) / 4 + 2 r (+1), slot = (call * T + t) * 4 + which;
// eps = sqrt(-2 log1p(-u_c)) cos(2 pi u_{4+c}); `call` is read from device
// memory so a replayed graph draws fresh values every rollout.
// ---------------------------------------------------------------------------
constexpr int FC1 = 64, FC2 = 64, FC3 = 32, NOUT = 4;

struct PolicyArgs {
  lnw_policy_args a;
  int n_in;
  int off_b1, off_w1;  // packed MLP: biases b1 | b2 | b3, then the MFMA weight fragments (floats)
};

__device__ __forceinline__ void philox_u8(unsigned long long seed, unsigned long long ctr0, float (&u)[8]) {
#pragma unroll
  for (int b = 0; b < 2; b++) {
    const unsigned long long ctr = ctr0 + (unsigned long long)b;
    uint32_t o[4] = {(uint32_t)ctr, (uint32_t)(ctr >> 32), 0x243F6A88u, 0x85A308D3u};
    philox10(o, (uint32_t)seed, (uint32_t)(seed >> 32));
#pragma unroll
    for (int k = 0; k < 4; k++) u[4 * b + k] = (float)(o[k] >> 8) * 5.9604644775390625e-08f;
  }
}

// standard normals of (slot, global row): keyed_normal's construction
__device__ __forceinline__ void keyed_eps(unsigned long long seed, unsigned long long slot, long long grow,
                                          float (&eps)[NOUT]) {
  float u[8];
  philox_u8(seed, (slot << 38) + (unsigned long long)grow * 2ull, u);
#pragma unroll
  for (int c = 0; c < NOUT; c++)  // (v_cos_f32 takes revolutions: cos(2 pi u) without the range reduction)
    eps[c] = sqrtf(-2.0f * log1pf(-u[c])) * __builtin_amdgcn_cosf(u[4 + c]);
}

// ---- the MLP on the matrix cores -------------------------------------------
// Each wave runs its 64 rows through fc1 / fc2 / fc3 and the two heads with
// v_mfma_f32_16x16x4_f32 (exact f32 products, f32 accumulation), transposed:
// Y^T = W X^T, so the weights are the A operand (lane l: W[n = 16 nt + (l & 15)]
// [k]) and the activations the B operand (lane l: X[r = 16 rt + (l & 15)][k]),
// and a layer's output tile (lane l, register v: Y[r = 16 rt + (l & 15)]
// [n = 16 nt + 4 (l >> 4) + v]) is already the next layer's B operand for the
// k-steps "quad q = nt, element v" — no LDS round trip between layers. Every
// layer therefore sums over k in the order k = 16 q + 4 g + v (g = l >> 4), and
// the host packs each weight matrix as fragments in that order
// (BatchedActor.packed_policy): float4 [nt][q][lane] = W[16 nt + (lane & 15)]
// [16 q + 4 (lane >> 4) + 0..3], read with one 16-B load per lane.
// The first layer's input (the LayerNorm output, one row per lane) goes through
// a wave-private LDS tile [64 rows][KS] to reach the same layout.
typedef float f32x4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4v mfma4(float a, float b, f32x4v c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// acc[rt][nt] += W (frags F, NTO output tiles, Q quads) x X (B operand quads
// xq[rt][q] of float4 = 4 k-steps)
template <int NTO, int Q>
__device__ __forceinline__ void mfma_layer(const f32x4v *__restrict__ F, const f32x4v (&xb)[4][Q],
                                           f32x4v (&acc)[4][NTO], int lane) {
#pragma unroll
  for (int q = 0; q < Q; q++) {
    f32x4v w[NTO];
#pragma unroll
    for (int nt = 0; nt < NTO; nt++) w[nt] = F[(nt * Q + q) * WAVE + lane];
#pragma unroll
    for (int v = 0; v < 4; v++)
#pragma unroll
      for (int rt = 0; rt < 4; rt++)
#pragma unroll
        for (int nt = 0; nt < NTO; nt++) acc[rt][nt] = mfma4(w[nt][v], xb[rt][q][v], acc[rt][nt]);
  }
}

// The same layers on the bf16 matrix cores at f32 accuracy (lnw_policy_act):
// v_mfma_f32_16x16x32_bf16, lane l holding A[l & 15][k = 8 (l >> 4) + j] and
// B[k][l & 15], j = 0..7. Element j of a k-pair p is neuron 32 p + 16 (j / 4) +
// 4 (l >> 4) + j % 4, so the B operand of pair p is just the two f32 quads
// (2p, 2p + 1) of mfma_layer's layout: the chaining stays register-only. Each
// f32 value is split exactly into three bfloat16 terms (x = x0 + x1 + x2, each
// rounded to nearest: 8 + 8 + 8 bits), the weights on the host
// (BatchedActor.packed_policy: planes hi, mid, lo), the activations here; of
// the nine partial products the six above 2^-24 relative are summed (small
// ones first), so a product is exact to about 3 ulp of f32 and the sums match
// the f32 MFMA's within a few ulp, at 6 x 16 cycles per 32 k instead of the
// f32 form's 8 x 32.
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ void split3(const f32x4v &a, const f32x4v &b, bf16x8 &x0, bf16x8 &x1, bf16x8 &x2) {
#pragma unroll
  for (int j = 0; j < 8; j++) {
    const float x = j < 4 ? a[j] : b[j - 4];
    const __bf16 h = (__bf16)x;
    const float r = x - (float)h;
    const __bf16 m = (__bf16)r;
    x0[j] = h;
    x1[j] = m;
    x2[j] = (__bf16)(r - (float)m);
  }
}

__device__ __forceinline__ f32x4v mfma32(const bf16x8 &a, const bf16x8 &b, f32x4v c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// acc[rt][nt] += W (planes F: hi | mid | lo, each bf16x8 [nt][p][lane]) x X
template <int NTO, int Q>
__device__ __forceinline__ void mfma_layer3(const bf16x8 *__restrict__ F, const f32x4v (&xb)[4][Q],
                                            f32x4v (&acc)[4][NTO], int lane, bf16x8 *split_save = nullptr) {
  static_assert(Q % 2 == 0, "k in pairs of quads");
  constexpr int QP = Q / 2, PL = NTO * QP * WAVE;  // plane stride (bf16x8)
#pragma unroll
  for (int p = 0; p < QP; p++) {
    bf16x8 b0[4], b1[4], b2[4];
#pragma unroll
    for (int rt = 0; rt < 4; rt++) split3(xb[rt][2 * p], xb[rt][2 * p + 1], b0[rt], b1[rt], b2[rt]);
#ifdef LNW_MLP_SPLIT_FENCE
    // probe: every split term computed (materialised in its registers) before
    // the first MFMA of the pair is issued: no vector instruction of this block
    // co-executing with its MFMAs
#pragma unroll
    for (int rt = 0; rt < 4; rt++) asm volatile("" : "+v"(b0[rt]), "+v"(b1[rt]), "+v"(b2[rt]));
    __builtin_amdgcn_sched_barrier(0);
#endif
    if (split_save && p == 0) {  // (diagnostics probe 16)
#pragma unroll
      for (int rt = 0; rt < 4; rt++) {
        split_save[3 * rt] = b0[rt];
        split_save[3 * rt + 1] = b1[rt];
        split_save[3 * rt + 2] = b2[rt];
      }
    }
#pragma unroll
    for (int nt = 0; nt < NTO; nt++) {
      const int i = (nt * QP + p) * WAVE + lane;
      const bf16x8 w0 = F[i], w1 = F[PL + i], w2 = F[2 * PL + i];
#pragma unroll
      for (int rt = 0; rt < 4; rt++) acc[rt][nt] = mfma32(w2, b0[rt], acc[rt][nt]);
#pragma unroll
      for (int rt = 0; rt < 4; rt++) acc[rt][nt] = mfma32(w1, b1[rt], acc[rt][nt]);
#pragma unroll
      for (int rt = 0; rt < 4; rt++) acc[rt][nt] = mfma32(w0, b2[rt], acc[rt][nt]);
#pragma unroll
      for (int rt = 0; rt < 4; rt++) acc[rt][nt] = mfma32(w1, b0[rt], acc[rt][nt]);
#pragma unroll
      for (int rt = 0; rt < 4; rt++) acc[rt][nt] = mfma32(w0, b1[rt], acc[rt][nt]);
#pragma unroll
      for (int rt = 0; rt < 4; rt++) acc[rt][nt] = mfma32(w0, b0[rt], acc[rt][nt]);
    }
  }
}

template <int NTO>
__device__ __forceinline__ void bias_init(const float *__restrict__ b, f32x4v (&acc)[4][NTO], int g) {
#pragma unroll
  for (int nt = 0; nt < NTO; nt++) {
    const f32x4v bv = *(const f32x4v *)(b + nt * 16 + 4 * g);
#pragma unroll
    for (int rt = 0; rt < 4; rt++) acc[rt][nt] = bv;
  }
}

// tanh(x) = 1 - 2 / (e^(2x) + 1) with the hardware exp2 and reciprocal
// (v_exp_f32, v_rcp_f32: ~1 ulp each): absolute error below 3e-7 over the
// whole range (+-1 exactly at overflow), against ~40 instructions of ocml's
// tanhf. The policy tolerances are 1e-4 (log-probabilities) and 1e-5 (values).
__device__ __forceinline__ float tanh_fast(float x) {
  const float e = __builtin_amdgcn_exp2f(x * 2.8853900817779268f);  // e^(2x) = 2^(2x log2 e)
  return 1.0f - 2.0f * __builtin_amdgcn_rcpf(e + 1.0f);
}

template <int NTO>
__device__ __forceinline__ void tanh_all(f32x4v (&acc)[4][NTO]) {
#pragma unroll
  for (int rt = 0; rt < 4; rt++)
#pragma unroll
    for (int nt = 0; nt < NTO; nt++)
#pragma unroll
      for (int v = 0; v < 4; v++) acc[rt][nt][v] = tanh_fast(acc[rt][nt][v]);
}

// bf16x8 elements of the MLP's packed weights (three planes per layer: fc1
// 4 x Q1/2, fc2 4 x 2, fc3 2 x 2, heads 1 x 1 tiles of WAVE, as mlp_heads reads them)
template <int NI>
__host__ __device__ constexpr int mlp_bf16x8() {
  return 3 * (4 * (NI / 32) + 4 * 2 + 2 * 2 + 1 * 1) * WAVE;
}

// fc1 / fc2 / fc3 and both heads of the wave's 64 rows on the matrix cores
// (xb: fc1's B operand), then each row's head outputs brought to its own lane
// (hh_save, xb_save: diagnostics probe 14 only)
template <int Q1>
__device__ __forceinline__ void mlp_heads(const PolicyArgs &pa, const bf16x8 *Fw, const float *xt, int lane,
                                          int g, int m, float (&mean)[NOUT], float (&lsd)[NOUT],
                                          f32x4v *hh_save = nullptr, f32x4v *xb_save = nullptr,
                                          f32x4v *layers_save = nullptr, bf16x8 *split_save = nullptr,
                                          f32x4v *pre_save = nullptr) {
  constexpr int KS = 16 * Q1 + 4;  // the tile's row stride (policy_act_kernel)
  const lnw_policy_args &a = pa.a;
  f32x4v xb[4][Q1];
#pragma unroll
  for (int rt = 0; rt < 4; rt++)
#pragma unroll
    for (int q = 0; q < Q1; q++) xb[rt][q] = *(const f32x4v *)(xt + (rt * 16 + m) * KS + 16 * q + 4 * g);
  if (xb_save) {
#pragma unroll
    for (int rt = 0; rt < 4; rt++)
#pragma unroll
      for (int q = 0; q < Q1; q++) xb_save[rt * Q1 + q] = xb[rt][q];
  }
  // weights: three bf16 planes per layer (mfma_layer3), layers in order
  // Fw: the three bf16 planes of every layer (global, or the block's LDS copy)
  constexpr int O2 = 3 * 4 * (Q1 / 2) * WAVE, O3 = O2 + 3 * 4 * 2 * WAVE, OH = O3 + 3 * 2 * 2 * WAVE;
  const float *bias = a.params + pa.off_b1;  // b1 [64] | b2 [64] | b3 [32]
  f32x4v h1[4][4];
  bias_init<4>(bias, h1, g);
  mfma_layer3<4, Q1>(Fw, xb, h1, lane, split_save);
  if (pre_save) {  // (diagnostics probe 16: fc1 before the activation)
#pragma unroll
    for (int rt = 0; rt < 4; rt++)
#pragma unroll
      for (int nt = 0; nt < 4; nt++) pre_save[rt * 4 + nt] = h1[rt][nt];
  }
  tanh_all<4>(h1);
  if (layers_save) {  // probe 15: [layer 0..2][rt][nt] (h1, h2: 4 nt; h3: 2)
#pragma unroll
    for (int rt = 0; rt < 4; rt++)
#pragma unroll
      for (int nt = 0; nt < 4; nt++) layers_save[(0 * 4 + rt) * 4 + nt] = h1[rt][nt];
  }
  f32x4v h2[4][4];
  bias_init<4>(bias + 64, h2, g);
  mfma_layer3<4, 4>(Fw + O2, h1, h2, lane);
  tanh_all<4>(h2);
  if (layers_save) {
#pragma unroll
    for (int rt = 0; rt < 4; rt++)
#pragma unroll
      for (int nt = 0; nt < 4; nt++) layers_save[(1 * 4 + rt) * 4 + nt] = h2[rt][nt];
  }
  f32x4v h3[4][2];
  bias_init<2>(bias + 128, h3, g);
  mfma_layer3<2, 4>(Fw + O3, h2, h3, lane);
  tanh_all<2>(h3);
  if (layers_save) {
#pragma unroll
    for (int rt = 0; rt < 4; rt++)
#pragma unroll
      for (int nt = 0; nt < 2; nt++) layers_save[(2 * 4 + rt) * 4 + nt] = h3[rt][nt];
  }
  f32x4v hh[4][1];
#pragma unroll
  for (int rt = 0; rt < 4; rt++) hh[rt][0] = f32x4v{0.f, 0.f, 0.f, 0.f};
  mfma_layer3<1, 2>(Fw + OH, h3, hh, lane);
  if (hh_save) {
#pragma unroll
    for (int rt = 0; rt < 4; rt++) hh_save[rt] = hh[rt][0];
  }
  // head outputs of row 16 rt + m sit in lane m (normal head, n = v) and lane
  // 16 + m (log-std head, n = 4 + v) of tile rt: bring row `lane` to lane
  // `lane` (rt = g) for the per-row sampling below
#pragma unroll
  for (int v = 0; v < NOUT; v++) {
    float mv = 0.f, lv = 0.f;
#pragma unroll
    for (int rt = 0; rt < 4; rt++) {
      const float sm = __shfl(hh[rt][0][v], m);
      const float sl = __shfl(hh[rt][0][v], 16 + m);
      mv = g == rt ? sm : mv;
      lv = g == rt ? sl : lv;
    }
    mean[v] = mv;
    lsd[v] = lv;
  }
}

// A wave's rows up to the fc1 tile: conv head + LayerNorm (one row per lane),
// the observation copy for the rollout buffer, and the LayerNorm outputs into
// the wave's fc1 input tile in LDS (xt) for mlp_heads.
#if defined(LNW_PROBE_DISTURB) && (LNW_PROBE_DISTURB >= 12)
// Diagnostics probe 12: the first head of every wave (all heads at once) saves
// each stage of its rows here; the partner's second head, run while the other
// wave of its SIMD runs its MLP, compares stage by stage (window loads, pooled
// conv1 maps in LDS, conv head outputs, LayerNorm tail loads, LayerNorm
// outputs) and counts rows that differ per stage and lane (lnw_probe_counts).
constexpr int PROBE_ROWS = 131072, PROBE_W = 256;
__device__ float probe_buf[(size_t)PROBE_ROWS * PROBE_W];
constexpr int PROBE_STAGES = 10;
#if LNW_PROBE_DISTURB >= 15
__device__ f32x4v probe_layers[(size_t)131072 * 48];  // probe 15: every lane's h1 / h2 / h3 from its phase run
#endif
#if LNW_PROBE_DISTURB == 16
__device__ bf16x8 probe_split[(size_t)131072 * 12];  // probe 16: fc1's bf16 split terms (k-pair 0), per rt
__device__ f32x4v probe_pre[(size_t)131072 * 16];    // probe 16: fc1 before tanh
#endif
__device__ unsigned probe_cnt[PROBE_STAGES * 64];
template <int N>
__device__ __forceinline__ void probe_stage(int cmp, int stage, long long row, int off, const float (&v)[N],
                                            int lane) {
  if (row >= PROBE_ROWS) return;
  float *b = probe_buf + (size_t)row * PROBE_W + off;
  if (!cmp) {
#pragma unroll
    for (int k = 0; k < N; k++) b[k] = v[k];
    return;
  }
  bool bad = false;
#pragma unroll
  for (int k = 0; k < N; k++) bad = bad || __float_as_uint(b[k]) != __float_as_uint(v[k]);
  if (bad) atomicAdd(&probe_cnt[stage * 64 + lane], 1u);
}
#if LNW_PROBE_DISTURB == 12
#define PROBE_STAGE(st, off, v) probe_stage(probe_cmp, st, r0 + (threadIdx.x & ~(WAVE - 1)) + lane, off, v, lane)
#else
#define PROBE_STAGE(st, off, v) ((void)0)
#endif
#else
#define PROBE_STAGE(st, off, v) ((void)0)
#endif

template <int NI>
__device__ __forceinline__ void head_to_tile(const PolicyArgs &pa, const float *P, float *warea, int lane,
                                             bool valid, long long e, int i, long long istride, long long r0,
                                             long long rows, int probe_cmp = 0) {
  constexpr int KS = NI + 4;
  const lnw_policy_args &a = pa.a;
  const int n = a.n, D = a.D, n_in = pa.n_in;
  (void)probe_cmp;
  // ---- conv head + LayerNorm, one row per lane -------------------------------
  // The row's window and LayerNorm tail are loaded once, every load issued
  // together, into registers (the tail's loads were one dependent round trip
  // each behind the k < n_in guard).
  float u[NI];
  if (valid) {
    float h[12];
    {
      const float *x = a.obs + e * istride + (long long)i * D;
      float win[WIN];
#pragma unroll
      for (int k = 0; k < WIN; k++) win[k] = x[k];
#ifdef LNW_PROBE_NOCONV  // timing probes only (tools/policy_probe.py): no conv head
      for (int k = 0; k < 12; k++) h[k] = win[k];
#else
      PROBE_STAGE(0, 0, win);
      conv_head_win(P, win, warea + lane, WAVE, a.bn_running != 0, h);
#if defined(LNW_PROBE_DISTURB) && LNW_PROBE_DISTURB == 12
      {
        float pm[45];
        for (int k = 0; k < 45; k++) pm[k] = warea[lane + k * WAVE];
        PROBE_STAGE(1, 49, pm);
      }
#endif
      PROBE_STAGE(2, 94, h);
#endif
    }
    // the tail after the head (its registers are the head's), one batch of loads;
    // the row's address again from an opaque copy of the row index, so no 64-bit
    // address lives across the head (where the register file is full: it went
    // to scratch, and the kernel with it)
    float tl[NI - 12];
    int r_t = (int)(r0 + (threadIdx.x & ~(WAVE - 1)) + lane);
    asm volatile("" : "+v"(r_t));
    const int e_t = r_t / n, i_t = r_t - e_t * n;
    const float *xt = a.obs + (long long)e_t * istride + (long long)i_t * D;
#ifdef LNW_POLICY_SCALAR_TAIL  // (probe builds: the per-value loads, A/B)
    load_tail(xt, D, tl);
#else
    load_tail_q(xt, D, tl);
#endif
    PROBE_STAGE(3, 106, tl);
    layer_norm_tail<NI>(P, tl, n_in, h, u);
    PROBE_STAGE(4, 170, u);
  } else {
#pragma unroll
    for (int k = 0; k < NI; k++) u[k] = 0.f;
  }
  // ---- observation copy for the rollout buffer: the wave's 64 rows, float4
  // chunks (coalesced; the rows are L2-warm from the conv head's reads). Here,
  // between the VALU-bound head and the MFMA layers, rather than ahead of the
  // head: every workgroup starts at once, so a copy there left the memory
  // system idle during the compute and the ALUs idle during the copy.
  // (in place: lnw_observe_ex wrote the rows into the rollout buffer itself;
  // only the rows of envs whose episode ended are zeroed)
  const bool in_place = a.obs_out == a.obs && a.obs_env_stride == istride;
#if defined(LNW_PROBE_DISTURB) && LNW_PROBE_DISTURB == 12
  if (probe_cmp) return;
#endif
  if (a.obs_out && (!in_place || a.live)) {
    const int D4 = D >> 2;
    const long long rw = r0 + (threadIdx.x & ~(WAVE - 1));
    const long long nr = rows - rw < WAVE ? rows - rw : WAVE;
    for (int q = lane; q < nr * D4; q += WAVE) {
      const long long rr = rw + q / D4;
      const int c4 = q - (q / D4) * D4;
      const long long ee = rr / n;
      const int ii = (int)(rr - ee * n);
      const bool dead = a.live && !a.live[ee];
      if (in_place && !dead) continue;
      f32x4 v = dead ? f32x4{0.f, 0.f, 0.f, 0.f} : *(const f32x4 *)(a.obs + ee * istride + (long long)ii * D + 4 * c4);
      *(f32x4 *)(a.obs_out + ee * a.obs_env_stride + (long long)ii * D + 4 * c4) = v;
    }
  }
  // ---- fc1 input tile: the wave's rows into the MFMA B layout ---------------
  // (over the wave's own conv1 area: its lanes are done with it, and a wave's
  // LDS operations complete in order)
  float *xt = warea;
#pragma unroll
  for (int k4 = 0; k4 < NI / 4; k4++)
    *(f32x4v *)(xt + lane * KS + 4 * k4) = f32x4v{u[4 * k4], u[4 * k4 + 1], u[4 * k4 + 2], u[4 * k4 + 3]};
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#if defined(LNW_PROBE_DISTURB) && LNW_PROBE_DISTURB >= 13
  // Diagnostics probe 13 (the head/MLP overlap schedule of probe 10): every head
  // saves the row it wrote; the second head (probe_cmp, beside the SIMD
  // partner's MLP) reads its tile row back at once and counts lanes whose
  // bytes differ from what it wrote (stage 0); head_and_mlp checks the tile
  // again just before this wave's own MLP (stage 1)
  {
    const long long grow = r0 + (threadIdx.x & ~(WAVE - 1)) + lane;
    if (grow < PROBE_ROWS) {
      float *b = probe_buf + (size_t)grow * PROBE_W;
#pragma unroll
      for (int k = 0; k < NI; k++) b[k] = u[k];
    }
    if (probe_cmp) {
      bool bad = false;
#pragma unroll
      for (int k4 = 0; k4 < NI / 4; k4++) {
        f32x4v v = *(const f32x4v *)(xt + lane * KS + 4 * k4);
        asm volatile("" : "+v"(v));
#pragma unroll
        for (int j = 0; j < 4; j++) bad = bad || __float_as_uint(v[j]) != __float_as_uint(u[4 * k4 + j]);
      }
      if (bad) atomicAdd(&probe_cnt[0 * 64 + lane], 1u);
    }
  }
#endif
}

#ifdef LNW_PROBE_DISTURB
// Diagnostics probes only: what the other wave of a SIMD does while a wave
// runs its MLP (1 VALU FMA chains, 2 LDS reads of its own tile, 3 global
// loads, 4 s_sleep, 5 MFMA chains on registers, 6 LDS writes past its tile,
// 7 global stores to its rows' log-prob outputs (rewritten after), 8 v_exp /
// v_log / v_rcp / v_sqrt chains, 9 integer hashing; 10, in head_and_mlp: its
// own head again, rewriting the same tile; 11 its tile rows read and written
// back unchanged; 12 its head again, compared stage by stage, probe_stage);
// nothing it computes is kept.
template <int MODE, int KS>
__device__ __forceinline__ void disturb(const PolicyArgs &pa, float *warea, int lane, long long e, int i) {
  float acc0 = (float)lane, acc1 = 1.f, acc2 = 2.f, acc3 = 3.f;
  if (MODE == 1) {
    for (int it = 0; it < 2000; it++) {
      acc0 = fmaf(acc0, 1.0001f, 0.5f); acc1 = fmaf(acc1, 0.9999f, 0.25f);
      acc2 = fmaf(acc2, 1.0002f, 0.125f); acc3 = fmaf(acc3, 0.9998f, 0.0625f);
    }
  } else if (MODE == 2) {
    for (int it = 0; it < 600; it++) {
      const f32x4v v = *(const f32x4v *)(warea + ((lane + it) & 63) * KS + 4 * (it & 3));
      acc0 += v[0]; acc1 += v[1]; acc2 += v[2]; acc3 += v[3];
    }
  } else if (MODE == 3) {
    const float *q = pa.a.params + pa.off_w1;
    for (int it = 0; it < 300; it++) {
      const f32x4v v = *(const f32x4v *)(q + 4 * ((lane + 64 * it) & 4095));
      acc0 += v[0]; acc1 += v[1]; acc2 += v[2]; acc3 += v[3];
    }
  } else if (MODE == 4) {
    for (int it = 0; it < 100; it++) __builtin_amdgcn_s_sleep(8);
  } else if (MODE == 6) {
    for (int it = 0; it < 600; it++) {
      acc0 = fmaf(acc0, 1.0001f, 0.5f);
      warea[64 * KS + lane + 64 * (it % ((45 * 64 - 64 * KS) / 64 > 0 ? (45 * 64 - 64 * KS) / 64 : 1))] = acc0;
    }
  } else if (MODE == 7) {
    float *o = pa.a.logp_out ? pa.a.logp_out + e * pa.a.act_env_stride + 4 * i : nullptr;
    for (int it = 0; it < 300 && o; it++) {
      acc0 = fmaf(acc0, 1.0001f, 0.5f);
      o[it & 3] = acc0;
    }
  } else if (MODE == 8) {
    for (int it = 0; it < 500; it++) {
      acc0 = __builtin_amdgcn_exp2f(acc0 * 1e-3f); acc1 = __builtin_amdgcn_logf(acc1 + 1.f);
      acc2 = __builtin_amdgcn_rcpf(acc2 + 1.f); acc3 = __builtin_amdgcn_sqrtf(acc3 + 1.f);
    }
  } else if (MODE == 11) {  // its own tile row read and written back, unchanged
    float *row = warea + lane * KS;
    for (int it = 0; it < 60; it++) {
      f32x4v v[KS / 4 - 1];
#pragma unroll
      for (int k4 = 0; k4 < KS / 4 - 1; k4++) {
        v[k4] = *(const f32x4v *)(row + 4 * k4);
        asm volatile("" : "+v"(v[k4]));  // (not a load-store pair the compiler may drop)
      }
#pragma unroll
      for (int k4 = 0; k4 < KS / 4 - 1; k4++) *(f32x4v *)(row + 4 * k4) = v[k4];
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
  } else if (MODE == 9) {
    unsigned h0 = (unsigned)lane, h1 = 7u;
    for (int it = 0; it < 1000; it++) {
      h0 = __umulhi(h0 ^ 0x9E3779B9u, 0xD2511F53u) + h1;
      h1 = h1 * 0xCD9E8D57u + h0;
    }
    acc0 = (float)h0; acc1 = (float)h1;
  } else {
    bf16x8 w;
#pragma unroll
    for (int j = 0; j < 8; j++) w[j] = (__bf16)(0.001f * (float)(lane + j));
    f32x4v c0 = {0.f, 0.f, 0.f, 0.f}, c1 = c0, c2 = c0, c3 = c0;
    for (int it = 0; it < 400; it++) {
      c0 = mfma32(w, w, c0); c1 = mfma32(w, w, c1); c2 = mfma32(w, w, c2); c3 = mfma32(w, w, c3);
    }
    acc0 = c0[0] + c1[1] + c2[2] + c3[3];
  }
  asm volatile("" ::"v"(acc0), "v"(acc1), "v"(acc2), "v"(acc3));
}
#endif

// The phases of a block. PA_THREADS = 512 (one block per CU, two waves per
// SIMD): every wave runs its head, a barrier, then every wave its MLP. A wave's
// head (its conv, LayerNorm and fc1 tile) running while the other wave of its
// SIMD ran its MLP (v_mfma_f32_16x16x32_bf16 chains) came out wrong in lanes
// 48-63 of the head's wave ("The policy kernel's nondeterminism");
// heads beside heads and MLPs beside MLPs are exact. (One block per CU: the
// block's LDS is larger than half the CU's, so no other block's head shares a
// SIMD with these MLPs.) The diagnostics probes keep round 5's schedule, the
// waves of each SIMD taking their MLPs one at a time, to run their partner
// workloads beside each MLP.
template <int NI>
__device__ __forceinline__ void head_and_mlp(const PolicyArgs &pa, const float *P, const bf16x8 *Fw, float *warea, int lane, int g,
                                             int m, bool valid, long long e, int i, long long istride, long long r0,
                                             long long rows, float (&mean)[NOUT], float (&lsd)[NOUT]) {
  constexpr int Q1 = NI / 16;
  head_to_tile<NI>(pa, P, warea, lane, valid, e, i, istride, r0, rows);
#ifndef LNW_PROBE_DISTURB
#ifndef LNW_POLICY_OVERLAP  // (probe builds: each wave's MLP right after its own head)
  if constexpr (PA_THREADS > WAVE) __syncthreads();  // every head done before any MLP
#endif
  mlp_heads<Q1>(pa, Fw, warea, lane, g, m, mean, lsd);
#else
  constexpr int NWB = PA_THREADS / WAVE;
  __shared__ int simd_of[NWB];
  const int wv = (int)(threadIdx.x / WAVE);
  const int simd = (int)((__builtin_amdgcn_s_getreg((31 << 11) | 4) >> 4) & 3);  // hwreg(HW_ID).SIMD_ID
  if (lane == 0) simd_of[wv] = simd;
  __syncthreads();
  int rank = 0, nph = 1;  // this wave's turn on its SIMD; turns needed by the busiest SIMD
#pragma unroll
  for (int w2 = 0; w2 < NWB; w2++) {
    int r2 = 0;
#pragma unroll
    for (int w3 = 0; w3 < w2; w3++) r2 += simd_of[w3] == simd_of[w2] ? 1 : 0;
    nph = r2 + 1 > nph ? r2 + 1 : nph;
    rank = w2 == wv ? r2 : rank;
  }
#if LNW_PROBE_DISTURB >= 14
  f32x4v hh1[4];
#endif
  for (int ph = 0; ph < nph; ph++) {
#if LNW_PROBE_DISTURB == 13 || LNW_PROBE_DISTURB == 14  // this wave's tile row against what its head wrote, just before its MLP
    if (ph == rank) {
      constexpr int KS = NI + 4;
      const long long grow = r0 + (threadIdx.x & ~(WAVE - 1)) + lane;
      bool bad = false;
      if (grow < PROBE_ROWS) {
        const float *b = probe_buf + (size_t)grow * PROBE_W;
#pragma unroll
        for (int k4 = 0; k4 < NI / 4; k4++) {
          f32x4v v = *(const f32x4v *)(warea + lane * KS + 4 * k4);
          asm volatile("" : "+v"(v));
#pragma unroll
          for (int j = 0; j < 4; j++) bad = bad || __float_as_uint(v[j]) != __float_as_uint(b[4 * k4 + j]);
        }
      }
      if (bad) atomicAdd(&probe_cnt[1 * 64 + lane], 1u);
    }
#endif
#if LNW_PROBE_DISTURB == 16
    if (ph == rank) {
      const size_t t = (size_t)blockIdx.x * PA_THREADS + threadIdx.x;
      mlp_heads<Q1>(pa, Fw, warea, lane, g, m, mean, lsd, hh1, nullptr, probe_layers + t * 48,
                    probe_split + t * 12, probe_pre + t * 16);
    }
#elif LNW_PROBE_DISTURB == 15
    if (ph == rank) {
      f32x4v *ls = probe_layers + ((size_t)blockIdx.x * PA_THREADS + threadIdx.x) * 48;
      mlp_heads<Q1>(pa, Fw, warea, lane, g, m, mean, lsd, hh1, nullptr, ls);
    }
#elif LNW_PROBE_DISTURB == 14
    if (ph == rank) {
      // the MLP's fc1 operands as it loaded them from the tile, against the saved
      // rows (stage 2); its head outputs (hh) kept for the rerun below
      f32x4v xs[4 * Q1];
      mlp_heads<Q1>(pa, Fw, warea, lane, g, m, mean, lsd, hh1, xs);
      bool bad = false;
#pragma unroll
      for (int rt = 0; rt < 4; rt++) {
        const long long grow = r0 + (threadIdx.x & ~(WAVE - 1)) + rt * 16 + m;
        if (grow >= PROBE_ROWS) continue;
        const float *b = probe_buf + (size_t)grow * PROBE_W;
#pragma unroll
        for (int q = 0; q < Q1; q++)
#pragma unroll
          for (int j = 0; j < 4; j++)
            bad = bad || __float_as_uint(xs[rt * Q1 + q][j]) != __float_as_uint(b[16 * q + 4 * g + j]);
      }
      if (bad) atomicAdd(&probe_cnt[2 * 64 + lane], 1u);
    }
#else
    if (ph == rank) mlp_heads<Q1>(pa, Fw, warea, lane, g, m, mean, lsd);
#endif
#if LNW_PROBE_DISTURB == 10 || LNW_PROBE_DISTURB >= 13  // the partner redoes its head (same tile)
    else head_to_tile<NI>(pa, P, warea, lane, valid, e, i, istride, r0, rows, LNW_PROBE_DISTURB >= 13);
#elif LNW_PROBE_DISTURB == 12  // ... comparing every stage
    else head_to_tile<NI>(pa, P, warea, lane, valid, e, i, istride, r0, rows, 1);
#else  // the partner's work (tools/build_probes.sh)
    else disturb<LNW_PROBE_DISTURB, NI + 4>(pa, warea, lane, e, i);
#endif
    __syncthreads();
  }
#if LNW_PROBE_DISTURB == 16
  {  // stages: 0/1 split terms (rt 0-2 / rt 3), 2/3 fc1 before tanh, 4/5 h1 after tanh
    float m2[NOUT], l2[NOUT];
    f32x4v hh2[4], l2s[48], pre2[16];
    bf16x8 sp2[12];
    mlp_heads<Q1>(pa, Fw, warea, lane, g, m, m2, l2, hh2, nullptr, l2s, sp2, pre2);
    const size_t t = (size_t)blockIdx.x * PA_THREADS + threadIdx.x;
    const bf16x8 *sp = probe_split + t * 12;
    const f32x4v *pr = probe_pre + t * 16, *ls = probe_layers + t * 48;
    bool bad[3][2] = {{false, false}, {false, false}, {false, false}};
#pragma unroll
    for (int rt = 0; rt < 4; rt++) {
#pragma unroll
      for (int k = 0; k < 3; k++)
#pragma unroll
        for (int j = 0; j < 8; j++)
          bad[0][rt == 3] = bad[0][rt == 3] || __builtin_bit_cast(unsigned short, sp[3 * rt + k][j]) !=
                                                   __builtin_bit_cast(unsigned short, sp2[3 * rt + k][j]);
#pragma unroll
      for (int nt = 0; nt < 4; nt++)
#pragma unroll
        for (int j = 0; j < 4; j++) {
          bad[1][rt == 3] = bad[1][rt == 3] || __float_as_uint(pr[rt * 4 + nt][j]) != __float_as_uint(pre2[rt * 4 + nt][j]);
          bad[2][rt == 3] = bad[2][rt == 3] || __float_as_uint(ls[rt * 4 + nt][j]) != __float_as_uint(l2s[rt * 4 + nt][j]);
        }
    }
#pragma unroll
    for (int L = 0; L < 3; L++)
#pragma unroll
      for (int u = 0; u < 2; u++)
        if (bad[L][u]) atomicAdd(&probe_cnt[(2 * L + u) * 64 + lane], 1u);
  }
#elif LNW_PROBE_DISTURB == 15
  {  // per layer (h1, h2, h3, heads) and row tile: stage 2 L + (rt == 3), L = layer
    float m2[NOUT], l2[NOUT];
    f32x4v hh2[4], l2s[48];
    mlp_heads<Q1>(pa, Fw, warea, lane, g, m, m2, l2, hh2, nullptr, l2s);
    const f32x4v *ls = probe_layers + ((size_t)blockIdx.x * PA_THREADS + threadIdx.x) * 48;
    bool bad[4][2] = {{false, false}, {false, false}, {false, false}, {false, false}};
#pragma unroll
    for (int L = 0; L < 3; L++)
#pragma unroll
      for (int rt = 0; rt < 4; rt++)
#pragma unroll
        for (int nt = 0; nt < (L == 2 ? 2 : 4); nt++)
#pragma unroll
          for (int j = 0; j < 4; j++)
            bad[L][rt == 3] = bad[L][rt == 3] ||
                              __float_as_uint(ls[(L * 4 + rt) * 4 + nt][j]) != __float_as_uint(l2s[(L * 4 + rt) * 4 + nt][j]);
#pragma unroll
    for (int rt = 0; rt < 4; rt++)
#pragma unroll
      for (int j = 0; j < 4; j++) bad[3][rt == 3] = bad[3][rt == 3] || __float_as_uint(hh2[rt][j]) != __float_as_uint(hh1[rt][j]);
#pragma unroll
    for (int L = 0; L < 4; L++)
#pragma unroll
      for (int t = 0; t < 2; t++)
        if (bad[L][t]) atomicAdd(&probe_cnt[(2 * L + t) * 64 + lane], 1u);
  }
#elif LNW_PROBE_DISTURB == 14
  {  // stage 3: the final per-row outputs, stage 4: the head outputs before the gather
    float m2[NOUT], l2[NOUT];
    f32x4v hh2[4];
    mlp_heads<Q1>(pa, Fw, warea, lane, g, m, m2, l2, hh2);
    bool bo = false, bh = false;
#pragma unroll
    for (int v = 0; v < NOUT; v++)
      bo = bo || __float_as_uint(m2[v]) != __float_as_uint(mean[v]) || __float_as_uint(l2[v]) != __float_as_uint(lsd[v]);
#pragma unroll
    for (int rt = 0; rt < 4; rt++)
#pragma unroll
      for (int j = 0; j < 4; j++) bh = bh || __float_as_uint(hh2[rt][j]) != __float_as_uint(hh1[rt][j]);
    if (bo) atomicAdd(&probe_cnt[3 * 64 + lane], 1u);
    if (bh) atomicAdd(&probe_cnt[4 * 64 + lane], 1u);
  }
#endif
#endif
}

template <int NI>
__global__ __launch_bounds__(PA_THREADS, 512 / PA_THREADS) void policy_act_kernel(PolicyArgs pa) {
  constexpr int Q1 = NI / 16;        // fc1 k-quads (n_in zero-padded to NI)
  constexpr int KS = NI + 4;         // row stride of the wave's fc1 input tile (16-B aligned)
  const lnw_policy_args &a = pa.a;
  const int n_in = pa.n_in;
  const int n_par = CONV_PARAMS + 2 * n_in;
  float *P = actor_lds;                // [n_par] conv head + LayerNorm parameters
  // per wave: [45][64] pooled conv1 maps (one column per lane), then the
  // wave's fc1 input tile [64][KS] over the same floats
  constexpr int WAREA = (45 > KS ? 45 : KS) * WAVE;
  float *warea = actor_lds + ((n_par + 3) & ~3) + (threadIdx.x / WAVE) * WAREA;
  for (int i = threadIdx.x; i < n_par; i += blockDim.x) P[i] = a.params[i];
  // the MLP's weights (three bf16 planes per layer, mlp_bf16x8<NI> of them):
  // at NI = 32 a copy in LDS after the wave areas, loaded once per block while
  // the heads run, so each wave's MFMA chains read their A operands from LDS
  // instead of 51 KB apiece from L2 (at NI = 64 they do not fit beside the
  // larger tiles and stay in global memory)
  const bf16x8 *Fw = (const bf16x8 *)(a.params + pa.off_w1);
  if constexpr (NI == 32) {
    bf16x8 *wl = (bf16x8 *)(actor_lds + ((n_par + 3) & ~3) + (PA_THREADS / WAVE) * WAREA);
    for (int i = threadIdx.x; i < mlp_bf16x8<NI>(); i += blockDim.x) wl[i] = Fw[i];
    Fw = wl;
  }
  const int n = a.n, D = a.D;
  const long long rows = a.E * n;
  const long long r0 = (long long)blockIdx.x * PA_THREADS;
  const long long istride = a.obs_in_env_stride ? a.obs_in_env_stride : (long long)n * D;
  __syncthreads();
  const int lane = threadIdx.x & (WAVE - 1), g = lane >> 4, m = lane & 15;
  const long long r = r0 + threadIdx.x;
  const bool valid = r < rows;  // (every lane stays for the wave-wide MFMAs)
  // (32-bit: rows < 2^31, checked on the host; fewer registers live across the head)
  const int e32 = valid ? (int)r / n : 0;
  const long long e = e32;
  const int i = valid ? (int)r - e32 * n : 0;
  const long long E = a.E;
  const bool alive = valid && a.alive[(long long)(a.own0 + i) * E + e] != 0;
  const bool live = !a.live || (valid && a.live[e] != 0);
  // ---- env-level side work by the lane of ship 0 ---------------------------
  if (valid && i == 0) {
    if (a.script) {  // scripted rows: profile j for red ship j < script_n, zeros past the table
      for (int j = 0; j < a.script_cnt; j++) {
        const int ag = a.script_own0 + j;
        const bool al = a.alive[(long long)ag * E + e] != 0;
        const bool has = j < a.script_n && a.t < a.script_steps;
        f64x4 v = {0.0, 0.0, 0.0, 0.0};
        if (al && has) v = *(const f64x4 *)(a.script + ((long long)j * a.script_steps + a.t) * 4);
        *(f64x4 *)(a.full + (e * a.A + ag) * 4) = v;
      }
    }
    if (a.kinds) {
      bool all = true;
      for (int ag = 0; ag < a.A; ag++) all = all && a.alive[(long long)ag * E + e] != 0;
      const uint8_t k = (a.kinds_f32_all_alive && all) ? (uint8_t)LNW_KIND_F32 : (uint8_t)LNW_KIND_F64;
      for (int ag = 0; ag < a.A; ag++) a.kinds[e * a.A + ag] = k;
      if (a.f32_out) a.f32_out[e * a.f32_env_stride] = k == LNW_KIND_F32 ? 1 : 0;
    }
  }
  // ---- head, fc1 tile and MLP (phases: head_and_mlp) --------------------------
  float mean[NOUT], lsd[NOUT];
#ifdef LNW_PROBE_NOMLP  // timing / diagnostics probes only: no MLP (the lane's own fc1 tile row)
  head_to_tile<NI>(pa, P, warea, lane, valid, e, i, istride, r0, rows);
  for (int v = 0; v < NOUT; v++) {
    mean[v] = warea[lane * KS + 12 + v];
    lsd[v] = 0.f;
  }
#else
  head_and_mlp<NI>(pa, P, Fw, warea, lane, g, m, valid, e, i, istride, r0, rows, mean, lsd);
#endif
  if (!valid) return;
  // the row's env and ship again, from an opaque copy of the row index: so
  // they are recomputed here instead of living across the head (where the
  // register file is full and they would go to scratch)
  int r_o = (int)(blockIdx.x * PA_THREADS + threadIdx.x);
  asm volatile("" : "+v"(r_o));
  const int e_o = r_o / n, i_o = r_o - e_o * n;
  float std_[NOUT];
  bool ok = true;
#pragma unroll
  for (int o = 0; o < NOUT; o++) {
    // (the hardware exp2 / reciprocal forms: tanh_fast's absolute error < 3e-7,
    // __expf's a few ulp; NaN, +-inf and overflow behave as tanhf / expf)
    mean[o] = tanh_fast(mean[o]);
    std_[o] = __expf(lsd[o]);
    ok = ok && !isnan(mean[o]) && !isnan(std_[o]);
  }
  // ---- sample / forced actions and log-probabilities -----------------------
  float act[NOUT], lp[NOUT];
  if (a.forced) {  // MLP.get_dist (network.py:117-152): no NaN guard
    const float *fa = a.forced_act + (long long)e_o * a.fa_env_stride + 4 * i_o;
#pragma unroll
    for (int o = 0; o < NOUT; o++) act[o] = fa[o];
  } else {
    if (!ok) {
#pragma unroll
      for (int o = 0; o < NOUT; o++) { mean[o] = 0.f; std_[o] = 1.f; }
    }
    const unsigned long long call = a.call_dev ? (unsigned long long)*a.call_dev : 0ull;
    const unsigned long long slot = (call * (unsigned long long)a.T + (unsigned long long)a.t) * 4ull;
    const long long grow = a.row_base + r_o;
    float eps[NOUT];
    keyed_eps(a.seed, slot + (unsigned long long)a.which, grow, eps);
#pragma unroll
    for (int o = 0; o < NOUT; o++) act[o] = mean[o] + std_[o] * eps[o];
    if (a.noise > 0.f) {
      float ne[NOUT];
      keyed_eps(a.seed, slot + (unsigned long long)a.which + 1ull, grow, ne);
#pragma unroll
      for (int o = 0; o < NOUT; o++) act[o] = act[o] + a.noise * ne[o];
    }
#pragma unroll
    for (int o = 0; o < NOUT; o++) act[o] = fminf(fmaxf(act[o], 0.f), 1.f);
  }
  // Normal.log_prob (torch.distributions): -((x - m)^2) / (2 var) - log(std) - log(sqrt(2 pi))
#pragma unroll
  for (int o = 0; o < NOUT; o++) {
    const float d = act[o] - mean[o];
    const float s = std_[o];
    // log(std) is the log-scale itself (the guarded rows carry std 1: log 0), except
    // where an f32 exp overflows to inf or rounds to 0 (below ln 2^-150; the hardware
    // exp may flush the denormals above that, whose log the log-scale stays), as
    // torch's log(exp(.)) does; v_rcp_f32 for 1 / var (1 ulp)
    const float l = (a.forced || ok) ? lsd[o] : 0.f;
    const float ls = (s < INFINITY && l > -103.972f) ? l : logf(s);
    lp[o] = -(d * d) * (0.5f * __builtin_amdgcn_rcpf(s * s)) - ls - 0.91893853320467274178f;
  }
  // ---- outputs --------------------------------------------------------------
  const bool keep = alive && live;
  if (a.full) {
    f64x4 v = {alive ? (double)act[0] : 0.0, alive ? (double)act[1] : 0.0, alive ? (double)act[2] : 0.0,
               alive ? (double)act[3] : 0.0};
    *(f64x4 *)(a.full + ((long long)e_o * a.A + a.own0 + i_o) * 4) = v;
  }
  if (a.act_out)
    *(f32x4 *)(a.act_out + (long long)e_o * a.act_env_stride + 4 * i_o) =
        keep ? f32x4{act[0], act[1], act[2], act[3]} : f32x4{0.f, 0.f, 0.f, 0.f};
  if (a.logp_out)
    *(f32x4 *)(a.logp_out + (long long)e_o * a.act_env_stride + 4 * i_o) =
        keep ? f32x4{lp[0], lp[1], lp[2], lp[3]} : f32x4{0.f, 0.f, 0.f, 0.f};
}

// ---------------------------------------------------------------------------
// After lnw_step (lnw_rollout_post): the rollout's bookkeeping of step t and
// the critic (network.py:154-172, ppo.py:598-605) on the observations the actor
// saw (the rollout buffer at step t), on the matrix cores like the actor's MLP
// (v_mfma_f32_16x16x4_f32, transposed layers Y^T = W X^T, k order 16 q + 4 g +
// v; see mfma_layer). One workgroup = 64 envs (4 row tiles) x n waves:
//   fc1 (n D -> 32): wave w takes ship w's D inputs (zero-padded to DQ
//        quads), partial sums of all 32 outputs for the 64 envs, added up
//        through LDS by every wave (+ bias, tanh);
//   fc2 (32 -> 64) and fc3 (64 -> 64): the 16-output tiles dealt over the
//        waves, fc2's tiles exchanged through LDS in the MFMA operand layout;
//   fc4 (64 -> 1): each wave's fc3 tiles dotted with w4 in registers, summed
//        over lane groups (shuffles) and waves (LDS);
//   wave 0, lane = env: the value (0 after the episode ended), the rewards,
//   the running flag and the env's new live flag (done == 0 ends it, ppo.py:640).
// Packed critic (BatchedCritic.packed()): fc1 fragments per ship [n][2][DQ]
// [lane] float4, b1 [32], fc2 fragments [4][2][lane], b2 [64], fc3 fragments
// [4][4][lane], b3 [64], w4 [64], b4 (+ 3 zeros).
// ---------------------------------------------------------------------------
constexpr int CF1 = 32, CF2 = 64, CF3 = 64;

struct CriticOffsets { int w1, b1, w2, b2, w3, b3, w4, b4; };

__global__ __launch_bounds__(1024) void rollout_post_kernel(lnw_rollout_post_args a, CriticOffsets co, int dq) {
  const int lane = threadIdx.x & (WAVE - 1), g = lane >> 4, m = lane & 15;
  const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / WAVE));
  const int n = a.n, D = a.D;
  const long long e0 = (long long)blockIdx.x * WAVE;
  const long long e = e0 + lane;
  const bool valid = e < a.E;
  const bool crit = a.critic != nullptr;
  // dynamic LDS: fc1 partials [n][2 nt][4 rt][64] f32x4 | fc2 tiles [4][4 rt][64] f32x4 | fc4 dots [n][64]
  f32x4v *part = (f32x4v *)actor_lds;
  f32x4v *h2s = part + n * 8 * WAVE;
  float *dsum = (float *)(h2s + 16 * WAVE);
  if (crit) {
    const float *C = a.critic;
    // ---- fc1: ship w's inputs --------------------------------------------------
    f32x4v acc[4][2];
#pragma unroll
    for (int rt = 0; rt < 4; rt++) acc[rt][0] = acc[rt][1] = f32x4v{0.f, 0.f, 0.f, 0.f};
    const f32x4v *F1 = (const f32x4v *)(C + co.w1) + (size_t)w * 2 * dq * WAVE;
    // (uniform trip count; MFMAs unrolled inside; quad q + 1's rows and weights
    // are loaded before quad q's MFMAs, so one load latency per wave, not dq)
    auto load_q = [&](int q, f32x4v (&xb)[4], f32x4v &w0, f32x4v &w1) {
      const int k = 16 * q + 4 * g;
#pragma unroll
      for (int rt = 0; rt < 4; rt++) {
        const long long er = e0 + rt * 16 + m;
        xb[rt] = (k < D && er < a.E) ? *(const f32x4v *)(a.obs + er * a.obs_env_stride + (long long)w * D + k)
                                      : f32x4v{0.f, 0.f, 0.f, 0.f};
      }
      w0 = F1[(0 * dq + q) * WAVE + lane];
      w1 = F1[(1 * dq + q) * WAVE + lane];
    };
    f32x4v xb[4], w0, w1;
    load_q(0, xb, w0, w1);
    for (int q = 0; q < dq; q++) {
      f32x4v xn[4], n0, n1;
      if (q + 1 < dq) load_q(q + 1, xn, n0, n1);
#pragma unroll
      for (int v = 0; v < 4; v++)
#pragma unroll
        for (int rt = 0; rt < 4; rt++) {
          acc[rt][0] = mfma4(w0[v], xb[rt][v], acc[rt][0]);
          acc[rt][1] = mfma4(w1[v], xb[rt][v], acc[rt][1]);
        }
      if (q + 1 < dq) {
#pragma unroll
        for (int rt = 0; rt < 4; rt++) xb[rt] = xn[rt];
        w0 = n0;
        w1 = n1;
      }
    }
  #pragma unroll
    for (int rt = 0; rt < 4; rt++)
#pragma unroll
      for (int nt = 0; nt < 2; nt++) part[((w * 2 + nt) * 4 + rt) * WAVE + lane] = acc[rt][nt];
    __syncthreads();
    f32x4v h1[4][2];
    bias_init<2>(C + co.b1, h1, g);
    for (int v = 0; v < n; v++)
#pragma unroll
      for (int rt = 0; rt < 4; rt++)
#pragma unroll
        for (int nt = 0; nt < 2; nt++) h1[rt][nt] += part[((v * 2 + nt) * 4 + rt) * WAVE + lane];
    tanh_all<2>(h1);
    // ---- fc2: tiles w, w + n, ... ------------------------------------------
    for (int nt = w; nt < 4; nt += n) {
      f32x4v t2[4][1];
      const f32x4v bv = *(const f32x4v *)(C + co.b2 + nt * 16 + 4 * g);
#pragma unroll
      for (int rt = 0; rt < 4; rt++) t2[rt][0] = bv;
      mfma_layer<1, 2>((const f32x4v *)(C + co.w2) + nt * 2 * WAVE, h1, t2, lane);
    #pragma unroll
      for (int rt = 0; rt < 4; rt++) {
#pragma unroll
        for (int v = 0; v < 4; v++) t2[rt][0][v] = tanh_fast(t2[rt][0][v]);
        h2s[(nt * 4 + rt) * WAVE + lane] = t2[rt][0];
      }
    }
    __syncthreads();
    // ---- fc3 + fc4 partial dots ----------------------------------------------
    f32x4v h2[4][4];
#pragma unroll
    for (int rt = 0; rt < 4; rt++)
#pragma unroll
      for (int q = 0; q < 4; q++) h2[rt][q] = h2s[(q * 4 + rt) * WAVE + lane];
    float dot[4] = {0.f, 0.f, 0.f, 0.f};
    for (int nt = w; nt < 4; nt += n) {
      f32x4v t3[4][1];
      const f32x4v bv = *(const f32x4v *)(C + co.b3 + nt * 16 + 4 * g);
#pragma unroll
      for (int rt = 0; rt < 4; rt++) t3[rt][0] = bv;
      mfma_layer<1, 4>((const f32x4v *)(C + co.w3) + nt * 4 * WAVE, h2, t3, lane);
          const f32x4v w4 = *(const f32x4v *)(C + co.w4 + nt * 16 + 4 * g);
#pragma unroll
      for (int rt = 0; rt < 4; rt++)
#pragma unroll
        for (int v = 0; v < 4; v++) dot[rt] = fmaf(w4[v], tanh_fast(t3[rt][0][v]), dot[rt]);
    }
    // lane groups g hold outputs 4 g .. 4 g + 3 of each tile: sum over g
#pragma unroll
    for (int rt = 0; rt < 4; rt++) {
      dot[rt] += __shfl_xor(dot[rt], 16);
      dot[rt] += __shfl_xor(dot[rt], 32);
    }
    if (g == 0) {
#pragma unroll
      for (int rt = 0; rt < 4; rt++) dsum[w * WAVE + rt * 16 + m] = dot[rt];
    }
    __syncthreads();
  }
  if (w != 0 || !valid) return;
  const bool L = !a.live || a.live[e] != 0;
  const bool masked = a.stop_at_done != 0;
  if (crit) {
    float s = 0.f;
    for (int q = 0; q < n; q++) s += dsum[q * WAVE + lane];
    const float v = a.critic[co.b4] + s;
    a.val[e * a.val_env_stride] = (masked && !L) ? 0.0f : v;
  }
  if (a.rew && a.rew_out) {
    for (int q = 0; q < a.n_rew; q++) {
      const double rv = a.rew_f64 ? ((const double *)a.rew)[e * a.n_rew + q]
                                  : (double)((const float *)a.rew)[e * a.n_rew + q];
      a.rew_out[e * a.rew_env_stride + q] = (masked && !L) ? 0.0 : rv;
    }
  }
  if (a.running) a.running[e * a.running_env_stride] = L ? 1 : 0;
  if (masked && a.live && a.done) a.live[e] = (L && a.done[e] != 0) ? 1 : 0;
}

}  // namespace

extern "C" {

int lnw_actor_features(const float *params_dev, int32_t obs_dim, const float *obs_dev, int64_t B,
                       int32_t bn_running, float *out_dev, void *stream) {
  if (!params_dev || !obs_dev || !out_dev || B < 0) return LNW_EINVAL;
  if (obs_dim < WIN || obs_dim - WIN + 12 > MAX_IN) return LNW_EUNSUPPORTED;
  if (B == 0) return 0;
  const long long blocks = (B + CH_THREADS - 1) / CH_THREADS;  // one row per thread
  if (B >= (1ll << 31) - CH_THREADS) return LNW_EUNSUPPORTED;  // (32-bit rows)
  const int n_par = CONV_PARAMS + 2 * (obs_dim - WIN + 12);
  const size_t lds = (n_par + 45 * CH_THREADS) * sizeof(float);
  if (obs_dim - WIN + 12 <= 32)
    features_kernel<32><<<dim3((unsigned)blocks), dim3(CH_THREADS), lds, (hipStream_t)stream>>>(
        params_dev, obs_dim, obs_dev, (int)B, bn_running, out_dev);
  else
    features_kernel<MAX_IN><<<dim3((unsigned)blocks), dim3(CH_THREADS), lds, (hipStream_t)stream>>>(
        params_dev, obs_dim, obs_dev, (int)B, bn_running, out_dev);
  return hipGetLastError() == hipSuccess ? 0 : LNW_EDEVICE;
}

// Packed MLP part of lnw_policy_act's parameters (BatchedActor.packed_policy()),
// after the conv head block padded to a multiple of 4 floats: b1 [64], b2 [64],
// b3 [32], then the MFMA A-operand fragments of fc1 (n_in zero-padded to K1 =
// 32, or 64 when n_in > 32), fc2, fc3 and the heads (normal rows 0-3, log-std
// rows 4-7, zero rows to 16), each as float4 [n-tile][k-quad][lane] (see
// mfma_layer).
int lnw_policy_act(const lnw_policy_args *args, void *stream) {
  if (!args) return LNW_EINVAL;
  const lnw_policy_args &a = *args;
  if (!a.obs || !a.params || !a.alive || a.n <= 0 || a.E < 0 || a.A <= 0 || a.own0 < 0 || a.own0 + a.n > a.A)
    return LNW_EINVAL;
  if (a.D < WIN || a.D - WIN + 12 > MAX_IN || (a.D & 3)) return LNW_EUNSUPPORTED;
  if (a.forced && !a.forced_act) return LNW_EINVAL;
  if (!a.forced && a.T <= 0) return LNW_EINVAL;
  if (a.script && (!a.full || a.script_own0 < 0 || a.script_own0 + a.script_cnt > a.A)) return LNW_EINVAL;
  if ((a.kinds_f32_all_alive || a.f32_out) && !a.kinds) return LNW_EINVAL;
  if (a.obs_in_env_stride < 0 || (a.obs_in_env_stride && (a.obs_in_env_stride < (int64_t)a.n * a.D ||
                                                          (a.obs_in_env_stride & 3))))
    return LNW_EINVAL;
  // 16-B aligned rows for the vector copies and stores
  if (((uintptr_t)a.obs & 15) || (a.obs_out && (((uintptr_t)a.obs_out & 15) || (a.obs_env_stride & 3))) ||
      ((a.act_out || a.logp_out) && (a.act_env_stride & 3)) || (a.act_out && ((uintptr_t)a.act_out & 15)) ||
      (a.logp_out && ((uintptr_t)a.logp_out & 15)) || (a.full && ((uintptr_t)a.full & 31)) ||
      (a.script && ((uintptr_t)a.script & 31)))
    return LNW_EINVAL;
  if (a.E == 0) return 0;
  PolicyArgs pa;
  pa.a = a;
  pa.n_in = a.D - WIN + 12;
  int o = CONV_PARAMS + 2 * pa.n_in;
  o = (o + 3) & ~3;     // (16-B aligned biases and fragments)
  pa.off_b1 = o; o += FC1 + FC2 + FC3;
  pa.off_w1 = o;
  const long long rows = a.E * a.n;
  if (rows + PA_THREADS >= (1ll << 31)) return LNW_EUNSUPPORTED;  // (32-bit row indices)
  const unsigned blocks = (unsigned)((rows + PA_THREADS - 1) / PA_THREADS);
  const int npar4 = (CONV_PARAMS + 2 * pa.n_in + 3) & ~3;
  size_t lds = (size_t)(npar4 + (PA_THREADS / WAVE) * (pa.n_in <= 32 ? 45 : MAX_IN + 4) * WAVE) * sizeof(float);
  if (pa.n_in <= 32) lds += (size_t)mlp_bf16x8<32>() * 16;  // the MLP weights' LDS copy
#ifdef LNW_PROBE_ONEBLOCK  // probe builds: one block per CU
  if (lds < 84 * 1024) lds = 84 * 1024;
#endif
  // One block per CU: head_and_mlp's schedule (every head, a barrier, every MLP)
  // keeps a head from running beside an MLP only within the block, so no other
  // block may share the CU. The block asks for more than half of the CU's LDS,
  // padded up should a future layout (a smaller tile, the weights out of LDS, a
  // smaller PA_THREADS) need less.
  static int cu_lds = 0;
  if (!cu_lds) {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&v, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, dev) != hipSuccess || v <= 0)
      v = 160 * 1024;
    cu_lds = v;
  }
  if (lds <= (size_t)cu_lds / 2) lds = (size_t)cu_lds / 2 + 16;
  if (pa.n_in <= 32)
    policy_act_kernel<32><<<blocks, PA_THREADS, lds, (hipStream_t)stream>>>(pa);
  else
    policy_act_kernel<MAX_IN><<<blocks, PA_THREADS, lds, (hipStream_t)stream>>>(pa);
  return hipGetLastError() == hipSuccess ? 0 : LNW_EDEVICE;
}

#if defined(LNW_PROBE_DISTURB) && (LNW_PROBE_DISTURB >= 12)
// probe 12's / 13's counters [stage][lane] since the last call (then zeroed)
int lnw_probe_counts(unsigned *host) {
  if (hipMemcpyFromSymbol(host, HIP_SYMBOL(probe_cnt), sizeof(probe_cnt)) != hipSuccess) return LNW_EDEVICE;
  static const unsigned zero[PROBE_STAGES * 64] = {};
  return hipMemcpyToSymbol(HIP_SYMBOL(probe_cnt), zero, sizeof(zero)) == hipSuccess ? 0 : LNW_EDEVICE;
}
#endif

// Packed critic: see rollout_post_kernel (BatchedCritic.packed()).
int lnw_rollout_post(const lnw_rollout_post_args *args, void *stream) {
  if (!args) return LNW_EINVAL;
  const lnw_rollout_post_args &a = *args;
  if (a.n <= 0 || a.n > 16 || a.E < 0) return LNW_EINVAL;
  if (a.critic && (!a.obs || !a.val || (a.D & 3) || ((uintptr_t)a.obs & 15) || (a.obs_env_stride & 3) ||
                   ((uintptr_t)a.critic & 15)))
    return LNW_EINVAL;
  if (a.rew_out && (!a.rew || a.n_rew <= 0)) return LNW_EINVAL;
  if (a.E == 0) return 0;
  const int dq = (a.D + 15) / 16;
  CriticOffsets co;
  int o = 0;
  co.w1 = o; o += a.n * 2 * dq * WAVE * 4;
  co.b1 = o; o += CF1;
  co.w2 = o; o += 4 * 2 * WAVE * 4;
  co.b2 = o; o += CF2;
  co.w3 = o; o += 4 * 4 * WAVE * 4;
  co.b3 = o; o += CF3;
  co.w4 = o; o += CF3;
  co.b4 = o;
  const unsigned blocks = (unsigned)((a.E + WAVE - 1) / WAVE);
  const size_t lds = a.critic ? (size_t)(a.n * 8 * WAVE + 16 * WAVE) * 16 + (size_t)a.n * WAVE * 4 : 0;
  rollout_post_kernel<<<blocks, WAVE * a.n, lds, (hipStream_t)stream>>>(a, co, dq);
  return hipGetLastError() == hipSuccess ? 0 : LNW_EDEVICE;
}

}  // extern "C"
