// lnw_device.h — device-side building blocks of the batched littoral env step
// (gfx950 / CDNA4). Every function cites the reference code it re-implements
// (valauri/Littoral-Naval-Warfare-MARL).
//
// Numerics: the library is built with -ffp-contract=off so every double and
// float operation rounds exactly like CPython/NumPy on x86-64 (no FMA
// contraction). Python round()/np.round are half-to-even -> rint/rintf.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace lnw {

constexpr int WAVE = 64;
constexpr int R_MV = 4;           // move-table window: target offsets in [-4, 4]^2
constexpr int MV_W = 2 * R_MV + 1;
constexpr int MV_WORDS = 3;       // 81 bits per (class, start cell)
constexpr int R_LOS = 40;         // LOS-table window: offsets in [-40, 40]^2
constexpr int LOS_W = 2 * R_LOS + 1;
constexpr int LOS_ROW_WORDS = 6;  // 81 cells x 2 bits = 162 bits per row
constexpr int LOS_CELL_WORDS = LOS_W * LOS_ROW_WORDS;  // 486 words per origin
constexpr int OPEN_CAP = 16;      // A* open list bound is 15 (floor(L/2)+8 from L=1)

// value kinds: NumPy-2 NEP 50 promotion lattice
enum { K_PYINT = 0, K_PYFLOAT = 1, K_F32 = 2, K_F64 = 3 };
enum { T_SMALL = 0, T_LARGE = 1, T_LS = 2, T_MEDIUM = 3 };

constexpr double PY_PI = 3.141592653589793;
constexpr double RAD2DEG = 180.0 / PY_PI;  // CPython math.degrees constant
constexpr double DEG2RAD = PY_PI / 180.0;  // CPython math.radians constant

// Kernel-wide constants (passed by value as a kernel argument).
struct KParams {
  int discrete, landing_ops, aggressive, side_blue, trained_red;
  int move_thr, ew_thr, lz_x, lz_y;
  int episode_steps, auto_reset, los_mode, move_mode;
  int E, nb, nr, A, G, T, W16;
  int rng_mode;
  int act_dtype;
  int rew_f64;        // lnw_set_reward_dtype: rew_blue/rew_red are float64 arrays
  long long env_base;
  unsigned long long seed;
  double red_aggression;
  double hit64[2][9];
  float hit32[2][9];
  double d5[2][2];    // sqrt((4/3)*6370*2)*(sqrt(m_i/1000)+sqrt(m_j/1000))/5, mast class 0=15,1=30
  double den[2];      // aggressive-reward denominator per mast class (game.py:269)
  double det_q[2];    // detected_prob: [0] target radar==1 (0.345-0.1), [1] otherwise
  int box_lo[2], box_hi[2];
  int group_march;    // group kernel: pair LOS marched over the LDS terrain mask instead of LOS-table loads (LNW_GROUP_MARCH)
  int xcd_remap;      // env chunks dealt to workgroups XCD-contiguously (xcd_chunk); LNW_NO_XCD_REMAP turns it off (A/B)
  int wc[2];          // observation window cells per side: 49 (7x7), or 25 for a side of medium ships (5x5, game.py:595-610)
  int epw;            // environments per workgroup (<= EPW; fewer when E is small, to fill the CUs)
  int store_wt;       // observation stream stored write-through (sc1): no dirty lines left in L2 at the launch end
  int atan_odd;       // the host's bearing table is odd in dy (degrees(atan2(-dy, dx)) == -degrees(atan2(dy, dx))): the group kernel stages its dy >= 0 half
  int no_obs;         // lnw_step without observation outputs (both pointers NULL)
  long long obs_stride[2];  // lnw_observe_ex: floats between envs' rows per side (0: packed)
  int dbg_skip;       // diagnostics only (LNW_DEBUG_SKIP): bit0 obs, bit1 phase S, bit2 phase M, bit7 get_obs in S, bit8 reward, bit9 no quiet path, bit10 no window reads in quiet emission, bit11 no phase-S LOS prefetch, bit12 device atan2 instead of the bearing table, bit13 4-ship phase-S rows stored row by row instead of line-aligned, bit15 the group kernel's fire loop entry by entry
  int qdirect;        // (last: the tail padding; the fields above keep their kernarg offsets) quiet workgroups stage whole 64-row side blocks (qbig) and wave 1 writes every row itself, in slabs of 64 / nb envs (step_qdirect)
};

// Device state (SoA, agent-major [field][agent][env] so a wave of envs reads
// one agent's field with coalesced accesses).
struct KState {
  uint32_t *pos;       // [A][E] x | y<<16
  int32_t *radar;      // [A][E]
  uint8_t *miss;       // [A][E]
  uint8_t *mkind;      // [A][E]
  uint8_t *alive;      // [A][E]
  uint8_t *type;       // [A][E]
  int32_t *steps;      // [A][E]
  double *dist_lz;     // [A][E]
  uint16_t *tl_cnt;    // [A][E]
  uint16_t *tl;        // [A][T][E]  x | y<<8
  double *duct;        // [E]
  int32_t *envi;       // [8][E]
  unsigned long long *rng;  // [E]
  uint32_t *err;       // [E]
  double *bear_val;    // [nmax*nmax][E] EW bearing scratch
  uint8_t *bear_ship;  // [nmax*nmax][E]
  const double *atan_deg;  // [LOS_W][LOS_W] degrees(atan2(dy, dx)), host libm (EW bearings)
  const uint8_t *grid;     // [G][G]
  const float *gridf;      // [G][G] grid/255 as float32
  const float *winf;       // [3][G*G][52] Combatant 7x7 | LandingShip 5x5 | medium Combatant 5x5 observation windows
  float *dummy;            // [WAVE * 4] sink for masked-out stores (keeps store counts static)
  unsigned long long *prof;  // diagnostics (LNW_PROF): [n_wg][16] phase timestamps, else null
  lnw_analytics ana;         // analytics side channels (null pointers: off)
  unsigned long long *ctr;   // lnw_set_counters work counters (null: off)
  const uint32_t *mask2;   // [G][W16] 2 bits per cell: bit0 > move_thr, bit1 > ew_thr
  const uint32_t *mvtab;   // [3][G*G][3] move tables: Combatant speed 3 | LandingShip | medium Combatant speed 2
  const uint32_t *lostab;  // [G*G][486]
  const double *tape;
  const long long *tape_off;
  // spawn spec (auto-reset)
  const int32_t *sp_types;   // [A]
  const int32_t *sp_pos;     // [A][2]
  const int32_t *sp_randls;  // [A]
  const int32_t *sp_pos_env; // [E][A][2] or null
  int nmax;
};

__host__ __device__ inline uint32_t pack_pos(int x, int y) {
  return (uint32_t)(x & 0xffff) | ((uint32_t)(y & 0xffff) << 16);
}
__device__ inline int pos_x(uint32_t p) { return (int)(p & 0x7fff); }
__device__ inline int pos_y(uint32_t p) { return (int)((p >> 16) & 0x7fff); }

__device__ inline int kind_promote(int a, int b) {
  if (a == K_F64 || b == K_F64) return K_F64;
  if (a == K_F32 || b == K_F32) return K_F32;
  if (a == K_PYFLOAT || b == K_PYFLOAT) return K_PYFLOAT;
  return K_PYINT;
}

// --------------------------------------------------------------------------
// RNG: Philox4x32-10 keyed by (seed, global env id) with a per-env counter, or
// a recorded tape (parity mode). Call sites follow the reference:
//   random.random()  combatant.py:614,637; game.py:377,379
//   random.gauss()   combatant.py:255
//   random.randint() game.py:589
//   np.random.beta(1,3) game.py:531
// --------------------------------------------------------------------------
__device__ inline void philox10(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; r++) {
    uint32_t hi0 = __umulhi(0xD2511F53u, c[0]), lo0 = 0xD2511F53u * c[0];
    uint32_t hi1 = __umulhi(0xCD9E8D57u, c[2]), lo1 = 0xCD9E8D57u * c[2];
    uint32_t n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
    c[0] = n0; c[1] = lo1; c[2] = n2; c[3] = lo0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}

__device__ inline double u53(uint32_t a, uint32_t b) {
  return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6)) / 9007199254740992.0;
}

// Portable ln and cos(2*pi*u): only + - * / and frexp, identical bits on the CPU
// oracle and the GPU (production-mode gauss draws).
// tan(x) for |x| < 2^19 * pi/2 (EW-fix slopes, combatant.py:270-271): the
// fdlibm algorithm — rem_pio2's medium path (x - n*pi/2 with pi/2 in three
// 33-bit pieces) and __kernel_tan's degree-25 odd polynomial with the
// pi/4 - x reflection above 0.6744 — in plain IEEE double arithmetic
// (error < 1 ulp, like the library tan it replaces; tools/tan_probe.hip
// compares it with the host libm over the bearing domain).
__host__ __device__ inline unsigned long long tan_bits(double x) { return __builtin_bit_cast(unsigned long long, x); }
__host__ __device__ inline double tan_from_bits(unsigned long long b) { return __builtin_bit_cast(double, b); }
__host__ __device__ inline double tan_kernel_fd(double x, double y, int iy) {
  const double T0 = 3.33333333333334091986e-01, T1 = 1.33333333333201242699e-01,
               T2 = 5.39682539762260521377e-02, T3 = 2.18694882948595424599e-02,
               T4 = 8.86323982359930005737e-03, T5 = 3.59207910759131235356e-03,
               T6 = 1.45620945432529025516e-03, T7 = 5.88041240820264096874e-04,
               T8 = 2.46463134818469906812e-04, T9 = 7.81794442939557092300e-05,
               T10 = 7.14072491382608190305e-05, T11 = -1.85586374855275456654e-05,
               T12 = 2.59073051863633712884e-05;
  const double pio4 = 7.85398163397448278999e-01, pio4lo = 3.06161699786838301793e-17;
  const int hx = (int)(tan_bits(x) >> 32), ix = hx & 0x7fffffff;
  if (ix < 0x3e300000) {  // |x| < 2^-28
    if (iy == 1) return x;
    return -1.0 / x;      // (x == 0 never reaches here with iy = -1 from a reduction)
  }
  const bool big = ix >= 0x3FE59428;  // |x| >= 0.6744
  if (big) {
    if (hx < 0) { x = -x; y = -y; }
    const double z = pio4 - x, w = pio4lo - y;
    x = z + w;
    y = 0.0;
  }
  double z = x * x, w = z * z;
  double r = T1 + w * (T3 + w * (T5 + w * (T7 + w * (T9 + w * T11))));
  double v = z * (T2 + w * (T4 + w * (T6 + w * (T8 + w * (T10 + w * T12)))));
  double s = z * x;
  r = y + z * (s * (r + v) + y);
  r += T0 * s;
  w = x + r;
  if (big) {
    v = (double)iy;
    return (double)(1 - ((hx >> 30) & 2)) * (v - 2.0 * (x - (w * w / (w + v) - r)));
  }
  if (iy == 1) return w;
  // -1 / (x + r) accurately
  const double zz = tan_from_bits(tan_bits(w) & 0xffffffff00000000ull);
  v = r - (zz - x);
  const double a = -1.0 / w;
  const double t = tan_from_bits(tan_bits(a) & 0xffffffff00000000ull);
  s = 1.0 + t * zz;
  return t + a * (s + t * v);
}
__host__ __device__ inline double tan_fd(double x) {
  const int ix = (int)(tan_bits(x) >> 32) & 0x7fffffff;
  if (ix <= 0x3fe921fb) return tan_kernel_fd(x, 0.0, 1);  // |x| ~<= pi/4
  if (ix >= 0x7ff00000) return x - x;                      // inf / nan
  // rem_pio2, medium path (|x| < 2^19 * pi/2 here: bearings in degrees < 1e5)
  const double invpio2 = 6.36619772367581382433e-01, pio2_1 = 1.57079632673412561417e+00,
               pio2_1t = 6.07710050650619224932e-11, pio2_2 = 6.07710050630396597660e-11,
               pio2_2t = 2.02226624879595063154e-21, pio2_3 = 2.02226624871116645580e-21,
               pio2_3t = 8.47842766036889956997e-32;
  const double t = fabs(x);
  const int n = (int)(t * invpio2 + 0.5);
  const double fn = (double)n;
  double r = t - fn * pio2_1, w = fn * pio2_1t;  // first round: good to 85 bits
  const int j = ix >> 20;
  double y0 = r - w;
  int i = j - (int)((tan_bits(y0) >> 52) & 0x7ff);
  if (i > 16) {  // second round: good to 118 bits
    double tt = r;
    w = fn * pio2_2;
    r = tt - w;
    w = fn * pio2_2t - ((tt - r) - w);
    y0 = r - w;
    i = j - (int)((tan_bits(y0) >> 52) & 0x7ff);
    if (i > 49) {  // third round: 151 bits
      tt = r;
      w = fn * pio2_3;
      r = tt - w;
      w = fn * pio2_3t - ((tt - r) - w);
      y0 = r - w;
    }
  }
  double y1 = (r - y0) - w;
  int nn = n;
  if (x < 0) { y0 = -y0; y1 = -y1; nn = -n; }
  return tan_kernel_fd(y0, y1, 1 - ((nn & 1) << 1));
}

__device__ inline double p_log(double x) {
  int e;
  double m = frexp(x, &e);
  if (m < 0.70710678118654752) { m *= 2.0; e -= 1; }
  double s = (m - 1.0) / (m + 1.0);
  double z = s * s;
  double p = 1.0 / 19.0;
  p = p * z + 1.0 / 17.0;
  p = p * z + 1.0 / 15.0;
  p = p * z + 1.0 / 13.0;
  p = p * z + 1.0 / 11.0;
  p = p * z + 1.0 / 9.0;
  p = p * z + 1.0 / 7.0;
  p = p * z + 1.0 / 5.0;
  p = p * z + 1.0 / 3.0;
  p = p * z + 1.0;
  return 2.0 * s * p + (double)e * 0.6931471805599453;
}

__device__ inline double p_cos2pi(double u) {
  double t = u * 4.0;
  int q = (int)t;
  double r = t - (double)q;
  double th = r * 1.5707963267948966;
  double z = th * th;
  double c = 1.0 / 2432902008176640000.0;
  c = c * -z + 1.0 / 6402373705728000.0;
  c = c * -z + 1.0 / 20922789888000.0;
  c = c * -z + 1.0 / 87178291200.0;
  c = c * -z + 1.0 / 479001600.0;
  c = c * -z + 1.0 / 3628800.0;
  c = c * -z + 1.0 / 40320.0;
  c = c * -z + 1.0 / 720.0;
  c = c * -z + 1.0 / 24.0;
  c = c * -z + 1.0 / 2.0;
  c = c * -z + 1.0;
  double s = 1.0 / 51090942171709440000.0;
  s = s * -z + 1.0 / 121645100408832000.0;
  s = s * -z + 1.0 / 355687428096000.0;
  s = s * -z + 1.0 / 1307674368000.0;
  s = s * -z + 1.0 / 6227020800.0;
  s = s * -z + 1.0 / 39916800.0;
  s = s * -z + 1.0 / 362880.0;
  s = s * -z + 1.0 / 5040.0;
  s = s * -z + 1.0 / 120.0;
  s = s * -z + 1.0 / 6.0;
  s = s * -z + 1.0;
  s = s * th;
  switch (q & 3) {
    case 0: return c;
    case 1: return -s;
    case 2: return -c;
    default: return s;
  }
}

struct Rng {
  int mode;
  uint32_t k0, k1, g0, g1;
  unsigned long long ctr;   // philox counter, or tape cursor relative to tape_lo
  const double *tape;
  long long tape_lo, tape_hi;
  uint32_t err;

  __device__ void block(uint32_t o[4], uint32_t stream = 0) {
    o[0] = (uint32_t)ctr;
    o[1] = (uint32_t)(ctr >> 32);
    o[2] = g0;
    o[3] = g1 ^ stream;
    philox10(o, k0, k1);
    ctr++;
  }
  __device__ double tnext() {
    long long p = tape_lo + (long long)ctr;
    if (p >= tape_hi) { err |= 4u; return 0.0; }
    ctr++;
    return tape[p];
  }
  __device__ __forceinline__ double uniform() {
    if (mode == 1) return tnext();
    uint32_t o[4];
    block(o);
    return u53(o[0], o[1]);
  }
  // two consecutive uniform draws (fire_missile's detection and hit draws);
  // Philox: both counter blocks evaluated side by side
  __device__ __forceinline__ void uniform2(double &u1, double &u2) {
    if (mode == 1) {
      u1 = tnext();
      u2 = tnext();
      return;
    }
    uint32_t o1[4] = {(uint32_t)ctr, (uint32_t)(ctr >> 32), g0, g1};
    const unsigned long long c2 = ctr + 1;
    uint32_t o2[4] = {(uint32_t)c2, (uint32_t)(c2 >> 32), g0, g1};
    philox10(o1, k0, k1);
    philox10(o2, k0, k1);
    ctr += 2;
    u1 = u53(o1[0], o1[1]);
    u2 = u53(o2[0], o2[1]);
  }
  // the uniform draw with draw number c, without touching the cursor or the
  // error bits (the caller accounts for both: fire_group_chunk); a tape
  // position past the end reads 0.0, as tnext
  __device__ __forceinline__ double uniform_at(unsigned long long c) const {
    if (mode == 1) {
      const long long p = tape_lo + (long long)c;
      return p < tape_hi ? tape[p] : 0.0;
    }
    uint32_t o[4] = {(uint32_t)c, (uint32_t)(c >> 32), g0, g1};
    philox10(o, k0, k1);
    return u53(o[0], o[1]);
  }
  __device__ double gauss() {
    if (mode == 1) return tnext();
    uint32_t o[4];
    block(o);
    double a = u53(o[0], o[1]), b = u53(o[2], o[3]);
    return sqrt(-2.0 * p_log(1.0 - a)) * p_cos2pi(b);
  }
  // the gauss draw with draw number c (Philox counter / tape position), without
  // touching the cursor: deferred bearings (finish_obs_t)
  __device__ double gauss_at(unsigned long long c) const {
    if (mode == 1) {
      const long long p = tape_lo + (long long)c;
      return p < tape_hi ? tape[p] : 0.0;
    }
    return gauss_philox(c, g0, g1);
  }
  // the Philox gauss draw c of the stream keyed (k0, k1, h0, h1): another env's
  // draw (h0, h1 = its global env id) in the pooled bearings of finish_obs_t
  __device__ double gauss_philox(unsigned long long c, uint32_t h0, uint32_t h1) const {
    uint32_t o[4] = {(uint32_t)c, (uint32_t)(c >> 32), h0, h1};
    philox10(o, k0, k1);
    double a = u53(o[0], o[1]), b = u53(o[2], o[3]);
    return sqrt(-2.0 * p_log(1.0 - a)) * p_cos2pi(b);
  }
  __device__ int randint(int a, int b) {
    if (mode == 1) return (int)tnext();
    double u = uniform();
    return a + (int)floor(u * (double)(b - a + 1));
  }
  __device__ double beta13() {
    if (mode == 1) return tnext();
    uint32_t o[4];
    block(o);
    const double s = 2.3283064365386963e-10;
    double m = ((double)o[0] + 0.5) * s;
    double v1 = ((double)o[1] + 0.5) * s, v2 = ((double)o[2] + 0.5) * s;
    if (v1 < m) m = v1;
    if (v2 < m) m = v2;
    return m;
  }
};

// --------------------------------------------------------------------------
// ship attributes (combatant.py:60-88, landingship.py:61-92)
// --------------------------------------------------------------------------
__device__ inline int ship_speed(int t) { return (t == T_LS || t == T_MEDIUM) ? 2 : 3; }
// move-table / A* class (check_path flavour and speed): Combatant speed 3,
// LandingShip, medium Combatant (speed 2)
__host__ __device__ inline int mv_cls(int t) { return t == T_LS ? 1 : (t == T_MEDIUM ? 2 : 0); }
// observation-window record class: Combatant 7x7, LandingShip 5x5 (asymmetric),
// medium Combatant 5x5 (combatant.py:165-181 with speed 2)
__device__ inline int win_cls(int t) { return mv_cls(t); }
__device__ inline int win_len(int t) { return t == T_SMALL || t == T_LARGE ? 49 : 25; }
// radar / EW range class of a target: small, large-like (large, medium: mast
// 30, rcs 1), LandingShip (rcs 0.9)
__device__ inline int rng_cls(int t) { return t == T_SMALL ? 0 : (t == T_LS ? 2 : 1); }
// Env chunk of workgroup b of nwg. Workgroups are dealt round-robin over the 8
// XCDs (b, b + 8, ... share one; speed only, never correctness), and each XCD
// has its own L2: with consecutive chunks on different XCDs, every cache line a
// chunk shares with its neighbour (byte and word fields of 16- or 32-env
// chunks, per-env outputs) is fetched into two or more L2s. Dealing each XCD a
// contiguous run of chunks keeps those lines in one L2. A bijection on
// [0, nwg) when nwg is a multiple of 8 (else the identity).
__device__ __forceinline__ int xcd_chunk(const KParams &P, int b, int nwg) {
  if (!P.xcd_remap || (nwg & 7)) return b;
  return (b & 7) * (nwg >> 3) + (b >> 3);
}
// observation row length of a side: 4 n + window + 3 (game.py:609-610)
__host__ __device__ inline int side_D(const KParams &P, int side) {
  return 4 * (side ? P.nr : P.nb) + P.wc[side ? 1 : 0] + 3;
}
__device__ inline int mast_cls(int t) { return t == T_SMALL ? 0 : 1; }
__device__ inline double ship_rcs(int t) { return t == T_SMALL ? 0.7 : (t == T_LS ? 0.9 : 1.0); }
__device__ inline int missiles0(int t) { return t == T_LS ? 0 : (t == T_SMALL ? 4 : 8); }
__device__ inline double miss_norm(int t) { return t == T_SMALL ? 4.0 : 8.0; }

// Small parameter tables indexed by per-lane values: selects between the
// (wave-uniform, scalar-loaded) entries instead of per-lane loads from the
// kernel-argument segment.
__device__ inline double d5_sel(const KParams &P, int mi, int mj) {
  const double r0 = mj ? P.d5[0][1] : P.d5[0][0];
  const double r1 = mj ? P.d5[1][1] : P.d5[1][0];
  return mi ? r1 : r0;
}
template <class TAB>
__device__ inline auto hit_sel(const TAB &tab, int hp, int n) -> decltype(tab[0][0] + 0) {
  auto row = [&](int h) {
    auto v = tab[h][0];
#pragma unroll
    for (int k = 1; k < 9; k++) v = n == k ? tab[h][k] : v;
    return v;
  };
  return hp ? row(1) : row(0);
}

// radar_range / ew_range (combatant.py:235-247) -> squared integer ranges
__device__ inline int radar_r(const KParams &P, double duct, int ti, int tj) {
  double d = d5_sel(P, mast_cls(ti), mast_cls(tj));
  return (int)ceil(d * ship_rcs(tj) * duct);
}
__device__ inline int ew_r(const KParams &P, double duct, int ti, int tj) {
  double d = d5_sel(P, mast_cls(ti), mast_cls(tj)) * duct;
  d = 2.0 * d;
  return (int)ceil(d);
}

// --------------------------------------------------------------------------
// terrain queries
// --------------------------------------------------------------------------
__device__ inline uint32_t cell_bits(const uint32_t *mask2, int W16, int x, int y) {
  return (mask2[x * W16 + (y >> 4)] >> ((y & 15) * 2)) & 3u;
}

// Bresenham LOS (combatant.py:411-456) over the 2-bit mask. Returns
// bit0 = radar clear (no cell > move_thr), bit1 = EW clear (no cell > ew_thr).
// With early_exit, stops at the first radar-blocked cell (EW is only ever
// consulted after radar LOS passed, combatant.py:110,119).
// ncell (optional): incremented by the number of cells visited.
template <bool early_exit>
__device__ inline uint32_t los_march(const uint32_t *mask2, int W16, int x1, int y1, int x2,
                                     int y2, int *ncell = nullptr) {
  int dx = abs(x2 - x1), dy = abs(y2 - y1);
  int sx = x1 > x2 ? -1 : 1, sy = y1 > y2 ? -1 : 1;
  int err = dx - dy;
  uint32_t blk = 0;
  for (;;) {
    blk |= cell_bits(mask2, W16, x1, y1);
    if (ncell) ++*ncell;
    if (early_exit && (blk & 1u)) return 0u;
    if (x1 == x2 && y1 == y2) break;
    int e2 = 2 * err;
    if (e2 > -dy) { err -= dy; x1 += sx; }
    if (e2 < dx) { err += dx; y1 += sy; }
  }
  return (~blk) & 3u;
}

// A* replica (combatant.py:289-379), literal including its quirks: the open
// list is popped while `enumerate` walks it, only the last inner pass's
// children survive, h = |dx| + dy^2, children limited to sqrt(2)*speed from
// the start, timeout returns the path to the last current node.
// Open entries: f<<14 | g<<8 | (dx+4)<<4 | (dy+4) (offsets relative to start).
// Returns len(path) (g+1) or -1 (None); kind: 0 goal, 1 timeout, 2 none.
template <class Blocked>
__device__ inline int astar_dev(const Blocked &blocked, int G, int speed, int sx, int sy,
                                int ex, int ey, int &kind, uint32_t *open, int ost) {
  const int maxd2 = 2 * speed * speed;
  const int max_it = (2 * speed + 1) * (2 * speed + 1);
  int n = 1;
  open[0] = (0u << 14) | (0u << 8) | (4u << 4) | 4u;
  uint32_t cur = open[0];
  int iterations = 0;
  while (n > 0) {
    iterations++;
    if (iterations > max_it) { kind = 1; return (int)((cur >> 8) & 63u) + 1; }
    cur = open[0];
    int ci = 0;
    int it = 0;
    bool found = false;
    while (it < n) {
      int index = it;
      uint32_t item = open[it * ost];
      it++;
      if ((item >> 14) < (cur >> 14)) { cur = item; ci = index; }
      for (int q = ci; q < n - 1; q++) open[q * ost] = open[(q + 1) * ost];
      n--;
      int cx = sx + (int)((cur >> 4) & 15u) - 4, cy = sy + (int)(cur & 15u) - 4;
      if (cx == ex && cy == ey) { found = true; break; }
    }
    if (found) { kind = 0; return (int)((cur >> 8) & 63u) + 1; }
    int cx = sx + (int)((cur >> 4) & 15u) - 4, cy = sy + (int)(cur & 15u) - 4;
    uint32_t g1 = ((cur >> 8) & 63u) + 1u;
    const int adx[8] = {0, 0, -1, 1, -1, -1, 1, 1};
    const int ady[8] = {-1, 1, 0, 0, -1, 1, -1, 1};
#pragma unroll
    for (int a = 0; a < 8; a++) {
      int nx = cx + adx[a], ny = cy + ady[a];
      if (nx > G - 1 || nx < 0 || ny > G - 1 || ny < 0) continue;
      if (blocked(nx, ny)) continue;
      int ddx = nx - sx, ddy = ny - sy;
      if (ddx * ddx + ddy * ddy > maxd2) continue;
      uint32_t h = (uint32_t)(abs(nx - ex) + (ny - ey) * (ny - ey));
      uint32_t f = g1 + h;
      open[n * ost] = (f << 14) | (g1 << 8) | ((uint32_t)(ddx + 4) << 4) | (uint32_t)(ddy + 4);
      n++;
    }
  }
  kind = 2;
  return -1;
}

struct GridBlocked {
  const uint8_t *grid;
  int G, thr;
  __device__ bool operator()(int x, int y) const { return grid[x * G + y] > thr; }
};
struct MaskBlocked {
  const uint32_t *mask2;
  int W16;
  __device__ bool operator()(int x, int y) const { return cell_bits(mask2, W16, x, y) & 1u; }
};

// check_path (combatant.py:382-408; LandingShip limit landingship.py:393,406)
template <class Blocked>
__device__ inline bool check_path_dev(const Blocked &blocked, bool start_blocked, int G, int type,
                                      int ox, int oy, int tx, int ty, uint32_t *open, int ost) {
  if (tx < 0 || tx > 99 || ty < 0 || ty > 99) return false;
  int speed = ship_speed(type);
  int limit = type == T_LS ? abs(ox - tx) + abs(oy - ty) + 1 : speed + 2;
  int kind;
  int len = astar_dev(blocked, G, speed, ox, oy, tx, ty, kind, open, ost);
  if (len < 0 || len > limit) return false;
  // every path cell is water except possibly the start (children are filtered)
  return !start_blocked;
}

// continuous_to_discrete arithmetic (combatant.py:459-471) in the value kind
// of the action row: float32 rows evaluate in float32 (NEP 50), others in f64.
// Returns false for a non-finite target (round(nan) raises ValueError and
// round(inf) OverflowError, combatant.py:470-471); finite targets beyond
// +-10^6 are only out of the grid.
// The float32 rows' target cell when it is certain without the double sin /
// cos: the cell is rintf(px + float(cos deg) * dist) (and the same with sin),
// so cos / sin are only needed to the precision that decides that rounding.
// Reduced by pi/2 in double (Cody-Waite, exact to ~1e-16 for |deg| < 1e5), then
// float polynomials on |r| <= pi/4: each coordinate is within 3e-5 of the exact
// path's float (cos / sin error < 5e-7 times dist <= 4, plus one float ulp of a
// coordinate below 256), so a coordinate farther than 4e-5 from a half-integer
// rounds the same way. Returns false otherwise (the caller then takes the
// double sincos path, about 1 row in 10^4 for uniform rows): the cell is the
// exact path's for every row either way (CPU check of both paths).
__device__ inline bool move_cell_f32_fast(int px, int py, double deg, float dist, int &nx, int &ny) {
  if (!(fabs(deg) < 1.0e5) || !(fabsf(dist) <= 4.0f)) return false;
  const double k = rint(deg * 6.36619772367581382433e-01);  // 2 / pi
  double rd = fma(-k, 1.57079632673412561417e+00, deg);      // pi/2, first 33 bits: exact
  rd = fma(-k, 6.07710050650619224932e-11, rd);              // the rest of pi/2
  const float r = (float)rd, z = r * r;
  const float sr = r + r * z * (-1.6666667e-1f + z * (8.3333333e-3f + z * (-1.9841270e-4f + z * 2.7557319e-6f)));
  const float cr = 1.0f - 0.5f * z + z * z * (4.1666668e-2f + z * (-1.3888889e-3f + z * 2.4801587e-5f));
  const int n = (int)k & 3;
  const float s = n == 0 ? sr : n == 1 ? cr : n == 2 ? -sr : -cr;
  const float c = n == 0 ? cr : n == 1 ? -sr : n == 2 ? -cr : sr;
  const float fx = (float)px + c * dist, fy = (float)py + s * dist;
  if (!(fabsf(fx) < 256.0f && fabsf(fy) < 256.0f)) return false;
  const float rx = rintf(fx), ry = rintf(fy);
  if (fabsf(fabsf(fx - rx) - 0.5f) < 4e-5f || fabsf(fabsf(fy - ry) - 0.5f) < 4e-5f) return false;
  nx = (int)rx;
  ny = (int)ry;
  return true;
}

__device__ inline bool move_target_dev(int px, int py, int speed, double a2, double a3, int kind,
                                       int &nx, int &ny) {
  double fxd, fyd;
  if (kind == K_F32) {
    float course = (float)(2.0 * PY_PI) * (float)a2;
    float dist = (float)speed * (float)a3;
    double deg = (double)course * RAD2DEG;
    if (move_cell_f32_fast(px, py, deg, dist, nx, ny)) return true;
    double s, c;
    sincos(deg, &s, &c);
    float dx = (float)c * dist;
    float dy = (float)s * dist;
    float fx = (float)px + dx;
    float fy = (float)py + dy;
    fxd = (double)rintf(fx);
    fyd = (double)rintf(fy);
  } else {
    double course = 2.0 * PY_PI * a2;
    double dist = (double)speed * a3;
    double deg = course * RAD2DEG;
    double s, c;
    sincos(deg, &s, &c);
    double dx = c * dist;
    double dy = s * dist;
    fxd = rint((double)px + dx);
    fyd = rint((double)py + dy);
  }
  if (!(fabs(fxd) < 1.0e6) || !(fabs(fyd) < 1.0e6)) {
    nx = -1000000;
    ny = -1000000;
    return isfinite(fxd) && isfinite(fyd);  // huge but finite: just out of bounds
  }
  nx = (int)fxd;
  ny = (int)fyd;
  return true;
}

// numpy mean of n float64 values (pairwise sum for n >= 8), values strided
template <class Get>
__device__ inline double np_mean_dev(const Get &v, int n) {
  double res;
  if (n < 8) {
    res = 0.0;
    for (int i = 0; i < n; i++) res += v(i);
  } else {
    double r0 = v(0), r1 = v(1), r2 = v(2), r3 = v(3), r4 = v(4), r5 = v(5), r6 = v(6), r7 = v(7);
    int i;
    for (i = 8; i < n - (n % 8); i += 8) {
      r0 += v(i); r1 += v(i + 1); r2 += v(i + 2); r3 += v(i + 3);
      r4 += v(i + 4); r5 += v(i + 5); r6 += v(i + 6); r7 += v(i + 7);
    }
    res = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
    for (; i < n; i++) res += v(i);
  }
  return res / (double)n;
}

}  // namespace lnw
