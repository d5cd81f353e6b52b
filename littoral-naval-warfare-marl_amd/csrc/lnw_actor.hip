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

__global__ __launch_bounds__(CH_THREADS, 2) void features_kernel(const float *params, int obs_dim,
                                                              const float *obs, long long B,
                                                              int bn_running, float *out) {
  const int n_in = obs_dim - WIN + 12;
  const int n_par = CONV_PARAMS + 2 * n_in;
  float *P = actor_lds;                           // [n_par] parameters
  float *pool1 = actor_lds + n_par;               // [45][CH_THREADS] pooled conv1 maps
  for (int i = threadIdx.x; i < n_par; i += blockDim.x) P[i] = params[i];
  __syncthreads();
  const bool running = bn_running != 0;
  const int t = threadIdx.x;
  for (long long row = (long long)blockIdx.x * blockDim.x + threadIdx.x; row < B;
       row += (long long)gridDim.x * blockDim.x) {
    const float *x = obs + row * obs_dim;
    float win[WIN];
#pragma unroll
    for (int i = 0; i < WIN; i++) win[i] = x[i];
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
          pool1[(c * 9 + i * 3 + j) * CH_THREADS + t] =
              fmaxf(fmaxf(v[r0 * 7 + c0], v[r0 * 7 + c0 + 1]),
                    fmaxf(v[(r0 + 1) * 7 + c0], v[(r0 + 1) * 7 + c0 + 1]));
        }
    }
    float p1[45];
#pragma unroll
    for (int k = 0; k < 45; k++) p1[k] = pool1[k * CH_THREADS + t];
    // conv2 (5 -> 8, 3x3, pad 1) -> BN -> ReLU -> 2x2 max pool (3x3 -> 1x1),
    // folded straight into the linear 8 -> 12 (convhead)
    float h[12];
#pragma unroll
    for (int k = 0; k < 12; k++) h[k] = P[HB + k];
#pragma unroll 1
    for (int co = 0; co < 8; co++) {
      float v[9];
#pragma unroll
      for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = 0; j < 3; j++) {
          float s = P[C2B + co];
#pragma unroll
          for (int ci = 0; ci < 5; ci++) {
            const float *w = P + C2W + (co * 5 + ci) * 9;
#pragma unroll
            for (int ki = 0; ki < 3; ki++)
#pragma unroll
              for (int kj = 0; kj < 3; kj++) {
                const int ii = i + ki - 1, jj = j + kj - 1;
                if (ii >= 0 && ii < 3 && jj >= 0 && jj < 3)
                  s += w[ki * 3 + kj] * p1[ci * 9 + ii * 3 + jj];
              }
          }
          v[i * 3 + j] = s;
        }
      bn_relu<9>(v, P + B2W, P + B2B, P + B2M, P + B2V, co, running);
      const float f = fmaxf(fmaxf(v[0], v[1]), fmaxf(v[3], v[4]));
#pragma unroll
      for (int k = 0; k < 12; k++) h[k] += P[HW + k * 8 + co] * f;
    }
    // LayerNorm over [h, x[49:]] (biased variance), affine
    float u[MAX_IN];
#pragma unroll
    for (int k = 0; k < MAX_IN; k++) u[k] = k < 12 ? h[k < 12 ? k : 0] : (k < n_in ? x[WIN + k - 12] : 0.f);
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < MAX_IN; k++) s += k < n_in ? u[k] : 0.f;
    const float mean = s / (float)n_in;
    float q = 0.f;
#pragma unroll
    for (int k = 0; k < MAX_IN; k++) q += k < n_in ? (u[k] - mean) * (u[k] - mean) : 0.f;
    const float inv = 1.0f / sqrtf(q / (float)n_in + LN_EPS);
    float *o = out + row * n_in;
    const float *lw = P + CONV_PARAMS, *lb = P + CONV_PARAMS + n_in;
#pragma unroll
    for (int k = 0; k < MAX_IN; k++)
      if (k < n_in) o[k] = (u[k] - mean) * inv * lw[k] + lb[k];
  }
}

}  // namespace

extern "C" {

int lnw_actor_features(const float *params_dev, int32_t obs_dim, const float *obs_dev, int64_t B,
                       int32_t bn_running, float *out_dev, void *stream) {
  if (!params_dev || !obs_dev || !out_dev || B < 0) return LNW_EINVAL;
  if (obs_dim < WIN || obs_dim - WIN + 12 > MAX_IN) return LNW_EUNSUPPORTED;
  if (B == 0) return 0;
  long long blocks = (B + CH_THREADS - 1) / CH_THREADS;
  if (blocks > 8192) blocks = 8192;
  const int n_par = CONV_PARAMS + 2 * (obs_dim - WIN + 12);
  features_kernel<<<dim3((unsigned)blocks), dim3(CH_THREADS), (n_par + 45 * CH_THREADS) * sizeof(float),
                    (hipStream_t)stream>>>(params_dev, obs_dim, obs_dev, B, bn_running, out_dev);
  return hipGetLastError() == hipSuccess ? 0 : LNW_EDEVICE;
}

}  // extern "C"
