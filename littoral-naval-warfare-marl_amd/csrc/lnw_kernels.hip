// lnw_kernels.hip — MI355X (gfx950) kernels and C-ABI of the batched littoral
// environment step. See include/lnw.h for the boundary and DESIGN.md for the
// layout/roofline discussion.
//
// Step structure (one 64-lane wavefront = one workgroup = 64 environments):
//   L  coalesced load of the agent-major SoA state into padded LDS columns
//   M  movement feasibility for every (env, agent): move target in the row's
//      value kind, then the precomputed A* table (or the A* replica)
//   S  the reference's sequential agent loop per env (one lane per env):
//      firing over the previous target list, radar, commit move, get_obs
//      (LOS table / ray march, EW bearings + fixes), reward; then the team tail
//   O  observations written cooperatively: lanes cover consecutive floats of
//      the [E][n][D] output (256-B coalesced stores), values read from LDS
//   W  coalesced store of the state (or of an in-kernel auto-reset)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "lnw.h"
#include "lnw_device.h"

using namespace lnw;

// native 4 x f32 vector: arrays of it stay in VGPRs (HIP's union-based float4
// defeats SROA and lands such arrays in scratch)
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef int i32x4_t __attribute__((ext_vector_type(4)));

// One 16-B observation store at float4 index i4 of a wave-uniform base.
// Write-through (buffer_store sc1) when wt: the line leaves this XCC's L2
// clean, so the launch does not end by writing back megabytes of dirty
// observation lines at the kernel boundary (P.store_wt; the host enables it
// only while every offset fits the 32-bit buffer range). Else a non-temporal
// store. The base is wave-uniform by contract (every caller passes a block or
// unit base): it is taken from the first active lane, so the resource is built
// in SGPRs once and the store never becomes a per-lane waterfall loop.
__device__ __forceinline__ void st_obs4(f32x4 *base, uint32_t i4, f32x4 v, bool wt) {
  if (wt) {
    const uint64_t bp = (uint64_t)(uintptr_t)base;
    const uint64_t ub = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)bp) |
                        (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(bp >> 32)) << 32;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void *)(uintptr_t)ub, 0, 0x7fffffff, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i32x4_t, v), rs, i4 * 16u, 0, 16 /* sc1 */);
  } else {
    __builtin_nontemporal_store(v, base + i4);
  }
}
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

namespace {

#ifndef LNW_EPW
#define LNW_EPW 64
#endif
constexpr int EPW = LNW_EPW;    // environments per wavefront (= per workgroup)
constexpr int UNITS = 4;        // 64-env units per workgroup of the headline kernel (step_kernel UN)
constexpr int UNITS_LDS_MAX = 156 * 1024;  // its dynamic LDS: the CU's 160 KiB less its static LDS
constexpr int PAD = EPW + 1;    // padded LDS column stride (words) -> no bank conflicts
constexpr int PADB = EPW + 4;   // byte-array stride

// ---------------------------------------------------------------------------
// per-wave LDS carve-up for the step/observe kernels
// ---------------------------------------------------------------------------
struct LdsLayout {
  // persistent through phase O
  int pos_cur, pos_old, radar_cur, radar_old, tcnt, miss_cur, miss_old, type, alive0, obsd;
  // phase-S scratch (dead before phase O) ...
  int pos_new, reward, observed, open, mkind, eng, bcnt, border, steps, act0, act1, akind;
  // ... aliased by the phase-O row staging area
  int stage;
  // terrain mask (phase M), aliased in phase S by the row-emission stage
  int mask, estage, total;
  // quiet path (step_kernel, quiet_emit_t): per-wave row stages and the x/G LUT.
  // qstage0 aliases the scratch that is dead once phase Q has run (actions,
  // pos_new, observed lists); qstage1 the scratch dead after phase W (rewards,
  // steps, missile kinds) plus the mask region; qlut sits at the very end.
  int qstage0, qstage1, qlut;
  // small quiet workgroups (epw * nb <= 64, lnw_quiet.inc): one stage per side
  // holding every row of the workgroup, appended after everything else
  int qbig;
};

// Row staging for phase O: up to 64 observation rows. The row stride S (floats)
// is a multiple of 4 with S/4 odd: rows are 16-B aligned so the copy-out reads
// float4s (ds_read_b128, conflict-free), and row starts spread over 8 banks
// (ds_write_b32 from lanes on different rows is at most 2-way).
__host__ __device__ constexpr int stage_stride(int ns) {
  return (((4 * ns + 52) / 4) & 1) ? (4 * ns + 52) : (4 * ns + 56);
}
// Phase-O LDS: staged rows (one pass = the rows of WAVE/A envs) | x/G LUT.
// (half a wave's worth of rows when a workgroup holds half a wave of envs, to
// keep its LDS within an eighth of the CU's)
constexpr int OBS_PASS_DIV = EPW == WAVE ? 1 : 2;
__host__ __device__ constexpr int envs_per_pass(int A) {
  return WAVE / A / OBS_PASS_DIV > 0 ? WAVE / A / OBS_PASS_DIV : 1;
}
__host__ __device__ inline int stage_rows_bytes(int A, int nb, int nr) {
  int epg = envs_per_pass(A);
  return epg * (nb * stage_stride(nb) + nr * stage_stride(nr)) * 4;
}
__host__ __device__ inline int stage_bytes(int A, int nb, int nr, int G) {
  return stage_rows_bytes(A, nb, nr) + ((G + 3) & ~3) * 4;
}

// Phase-S row emission (emit_rows_t): one group of row chunks for the 64 envs
// (row stride EST4 float4s, odd: conflict-free ds_write_b128) | x/G LUT.
constexpr int EST4 = 5;
__host__ __device__ inline int estage_bytes(int G) { return WAVE * EST4 * 16 + ((G + 3) & ~3) * 4; }
// wave 1's region in the phase-S split (step_kernel, psplit): pos and radar
// copies (A padded columns each) and finish_obs_t's pooled-bearing tables
// (rank -> lane bytes, rank -> draw u16s, fix table [nmax][WAVE] u32)
__host__ __device__ constexpr int psplit_bytes(int A, int nmax) { return 2 * A * PAD * 4 + 3 * WAVE + 4 * WAVE * nmax; }

// Quiet-path row stage: QEPG envs x one side's rows (stride stage_stride(ns)).
constexpr int QEPG = 8;
__host__ __device__ constexpr int qstage_bytes(int ns) { return QEPG * ns * stage_stride(ns) * 4; }

__host__ __device__ inline LdsLayout lds_layout(int A, int nb, int nr, int nmax, int mask_words,
                                                int G, int qbig_rows = 0) {
  LdsLayout L;
  int o = 0;
  L.pos_cur = o; o += A * PAD * 4;
  L.pos_old = o; o += A * PAD * 4;
  L.radar_cur = o; o += A * PAD * 4;
  L.radar_old = o; o += A * PAD * 4;
  L.tcnt = o; o += A * PAD * 4;
  L.miss_cur = o; o += A * PADB;
  L.miss_old = o; o += A * PADB;
  L.type = o; o += A * PADB;
  L.alive0 = o; o += A * PADB;
  L.obsd = o; o += A * PADB;
  o = (o + 15) & ~15;
  const int scratch = o;
  L.stage = scratch;
  // dead once phase Q (quiet path) or phase S has run
  L.act0 = o; o += A * PAD * 8;
  L.act1 = o; o += A * PAD * 8;
  L.pos_new = o; o += A * PAD * 4;
  L.observed = o; o += nmax * PAD * 4;
  L.bcnt = o; o += nmax * PADB;
  L.border = o; o += nmax * PADB;
  L.akind = o; o += A * PADB;
  o = (o + 15) & ~15;
  L.qstage0 = scratch;
  const int qneed = qstage_bytes(nb > nr ? nb : nr);
  if (o - scratch < qneed) o = scratch + qneed;
  // dead once phase W has run; the A* open lists (phase M) alias the rewards
  // (first written in phase Q / S)
  L.qstage1 = o;
  L.reward = o;
  L.open = o;
  o += (A * PAD * 8 > OPEN_CAP * EPW * 4) ? A * PAD * 8 : OPEN_CAP * EPW * 4;
  L.steps = o; o += A * PAD * 4;
  L.mkind = o; o += A * PADB;
  L.eng = o; o += A * PADB;
  int st_end = scratch + stage_bytes(A, nb, nr, G);
  if (st_end > o) o = st_end;
  o = (o + 15) & ~15;
  L.mask = o;
  L.estage = o;
  // the emission stage exists only with full-wave workgroups (two-wave kernels)
  int est = EPW == WAVE ? estage_bytes(G) : 0;
  // the 4v4 phase-S split (psplit) keeps wave 1's pos / radar copies and its
  // pooled-bearing tables here: 2 A PAD words + 3 WAVE + 4 WAVE nmax bytes
  // (5 376 B at 4v4), which estage_bytes covers only from G = 64 on
  if (EPW == WAVE && nb == 4 && nr == 4) {
    const int ps = psplit_bytes(A, nmax);
    if (est < ps) est = ps;
  }
  o += mask_words * 4 > est ? mask_words * 4 : est;
  const int lut = ((G + 3) & ~3) * 4;
  if (o - L.qstage1 < qneed + lut) o = L.qstage1 + qneed + lut;
  L.qlut = o - lut;
  L.qbig = o;
  o += 2 * qbig_rows * stage_stride(nb) * 4;
  L.total = o;
  return L;
}

struct Cols {
  uint32_t *pos_cur, *pos_old, *pos_new, *tcnt, *observed, *open;
  int32_t *radar_cur, *radar_old, *steps;
  double *reward, *act0, *act1;
  uint8_t *miss_cur, *miss_old, *mkind, *type, *alive0, *eng, *obsd, *bcnt, *border, *akind;
  uint32_t *mask;
  float *stage, *estage, *qstage0, *qstage1, *qlut, *qbig;
};

__device__ inline Cols carve(char *base, const LdsLayout &L) {
  Cols c;
  c.pos_cur = (uint32_t *)(base + L.pos_cur);
  c.pos_old = (uint32_t *)(base + L.pos_old);
  c.pos_new = (uint32_t *)(base + L.pos_new);
  c.radar_cur = (int32_t *)(base + L.radar_cur);
  c.radar_old = (int32_t *)(base + L.radar_old);
  c.reward = (double *)(base + L.reward);
  c.act0 = (double *)(base + L.act0);
  c.act1 = (double *)(base + L.act1);
  c.steps = (int32_t *)(base + L.steps);
  c.akind = (uint8_t *)(base + L.akind);
  c.tcnt = (uint32_t *)(base + L.tcnt);
  c.observed = (uint32_t *)(base + L.observed);
  c.open = (uint32_t *)(base + L.open);
  c.miss_cur = (uint8_t *)(base + L.miss_cur);
  c.miss_old = (uint8_t *)(base + L.miss_old);
  c.mkind = (uint8_t *)(base + L.mkind);
  c.type = (uint8_t *)(base + L.type);
  c.alive0 = (uint8_t *)(base + L.alive0);
  c.eng = (uint8_t *)(base + L.eng);
  c.obsd = (uint8_t *)(base + L.obsd);
  c.bcnt = (uint8_t *)(base + L.bcnt);
  c.border = (uint8_t *)(base + L.border);
  c.mask = (uint32_t *)(base + L.mask);
  c.stage = (float *)(base + L.stage);
  c.estage = (float *)(base + L.estage);
  c.qstage0 = (float *)(base + L.qstage0);
  c.qstage1 = (float *)(base + L.qstage1);
  c.qlut = (float *)(base + L.qlut);
  c.qbig = (float *)(base + L.qbig);
  return c;
}

#define COLW(arr, a) ((arr)[(a) * PAD + lane])
#define COLB(arr, a) ((arr)[(a) * PADB + lane])

// LNW_PROF diagnostics clock (100 MHz; 0 when profiling is off)
constexpr int PROF_SLOTS = 32;  // per-workgroup record (slot map at prof_put)
__device__ inline unsigned long long prof_now(const KState &S) {
  return S.prof ? __builtin_amdgcn_s_memrealtime() : 0ull;
}
// adds the time since t0 to a workgroup slot from the first active lane (the
// wave-level span of a section entered by only some lanes); returns now
__device__ inline unsigned long long prof_acc(const KState &S, int slot, unsigned long long t0) {
  if (!S.prof) return 0ull;
  const unsigned long long t = __builtin_amdgcn_s_memrealtime();
  const unsigned long long m = __ballot(1);
  if ((int)(threadIdx.x & 63) == __ffsll((long long)m) - 1)
    atomicAdd(&S.prof[(size_t)blockIdx.x * PROF_SLOTS + slot], t - t0);
  return t;
}

// Per-lane (per-env) context for phase S.
struct Ctx {
  const KParams &P;
  const KState &S;
  Cols &c;
  int lane, env;
  const double *duct_col;  // per-env ducting factor in LDS (kept out of the registers)
  Rng rng;
  const uint32_t *mask;  // LDS (march mode) or global
  long long E;
  int r2max;             // max over ship-type pairs of radar^2, EW^2 and 16 (d < 4)
  int step;              // episode step being played (analytics records)
  // LOS bits of every (own ship, opponent) pair get_obs can query during this
  // step (los_prefetch_t), per side: bit ((i*NOPP + j)*2 + v)*2 -> radar, +1 -> EW,
  // v = own ship i at its new cell. Valid when `pre` is set.
  uint64_t lpre[2];
  bool pre;
  // contact variant (pair_tables_t): per side, pair b = i * NOPP + j (own-major)
  // at bit b (own ship i on its start cell) and 16 + b (on its new cell):
  // radar-detect possible / close / EW candidate, LOS included
  uint32_t ptr_[2] = {0u, 0u}, ptc[2] = {0u, 0u}, ptw[2] = {0u, 0u};
  // the lane that makes the env's shared-counter side effects (analytics
  // records and maps): every lane where one lane steps one env; the first lane
  // of the env's group in the group kernel (lnw_group.inc), whose other lanes
  // repeat the env's serial work in step
  bool leader = true;
  // group kernel: this lane's index in its env's group and the group's first
  // lane in the wave (fire_dev<true> tests the opponents across the group)
  int gsub = 0, gsh = 0;
  // group kernel, work counters bound: EW bearings this lane's opponent
  // columns had evaluated pooled over the group (lnw_set_counters [3])
  unsigned pooled = 0;
#ifdef LNW_GROUP_PROF
  unsigned long long gp[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // group-kernel section timers
#endif
  __device__ double duct() const { return duct_col[lane]; }
};

// analytics (lnw_set_analytics): one 4-word record appended to a capped log
__device__ inline void ana_record(uint32_t *log, uint32_t *count, long long cap, uint32_t w0,
                                  uint32_t w1, uint32_t w2, uint32_t w3) {
  const uint32_t i = atomicAdd(count, 1u);
  if ((long long)i < cap) {
    uint4 *r = (uint4 *)log + i;
    *r = make_uint4(w0, w1, w2, w3);
  }
}
__device__ inline void ana_map(uint32_t *map, uint32_t p) {
  const int x = pos_x(p), y = pos_y(p);
  if (map && x < 100 && y < 100) atomicAdd(&map[x * 100 + y], 1u);
}

__device__ inline int max_range2(const KParams &P, double duct) {
  int m = 16;
  for (int ti = 0; ti < 3; ti++)
    for (int tj = 0; tj < 3; tj++) {
      int r = radar_r(P, duct, ti, tj), e = ew_r(P, duct, ti, tj);
      m = max(m, max(r * r, e * e));
    }
  return m;
}

__device__ inline int floordiv7(int v) { int q = v / 7; if ((v % 7 != 0) && (v < 0)) q--; return q; }
__device__ inline int pymod7(int v) { int m = v % 7; if (m < 0) m += 7; return m; }

// ---------------------------------------------------------------------------
// movement feasibility (combatant.py:459-489, 382-408, 689-704)
// ---------------------------------------------------------------------------
__device__ inline bool check_path_h(const KParams &P, const KState &S, int type, int sx, int sy,
                                    int tx, int ty, uint32_t *open, int ost) {
  if (tx < 0 || tx > 99 || ty < 0 || ty > 99) return false;
  int ox = tx - sx, oy = ty - sy;
  if (P.move_mode == 0 && ox >= -R_MV && ox <= R_MV && oy >= -R_MV && oy <= R_MV) {
    int cls = mv_cls(type);
    int bit = (ox + R_MV) * MV_W + (oy + R_MV);
    uint32_t w = S.mvtab[((size_t)cls * P.G * P.G + (size_t)sx * P.G + sy) * MV_WORDS + (bit >> 5)];
    return (w >> (bit & 31)) & 1u;
  }
  MaskBlocked mb{S.mask2, P.W16};
  bool sb = mb(sx, sy);
  if (S.ctr) atomicAdd(&S.ctr[2], 1ull);  // A* searches run (work counter)
  return check_path_dev(mb, sb, P.G, type, sx, sy, tx, ty, open, ost);
}

__device__ inline bool can_move_to_h(const KParams &P, const KState &S, int x, int y) {
  if (0 <= x && x < 100 && 0 <= y && y < 100) return !(cell_bits(S.mask2, P.W16, x, y) & 1u);
  return false;
}

// Bresenham ray march of the step / observe kernels, counted into the work
// counters when they are bound (lnw_set_counters: [0] rays marched, [1] cells
// visited)
__device__ inline uint32_t los_march_c(const KState &S, const uint32_t *mask, int W16, int x1,
                                       int y1, int x2, int y2) {
  if (!S.ctr) return los_march<true>(mask, W16, x1, y1, x2, y2);
  int n = 0;
  const uint32_t r = los_march<true>(mask, W16, x1, y1, x2, y2, &n);
  atomicAdd(&S.ctr[0], 1ull);
  atomicAdd(&S.ctr[1], (unsigned long long)n);
  return r;
}

// LOS query: table lookup inside the +-40 window, otherwise the ray march
__device__ inline uint32_t los_q(const KParams &P, const KState &S, const uint32_t *mask, int x1,
                                 int y1, int x2, int y2) {
  int dx = x2 - x1, dy = y2 - y1;
  if (P.los_mode != 1 && dx >= -R_LOS && dx <= R_LOS && dy >= -R_LOS && dy <= R_LOS) {
    int col = (dy + R_LOS) * 2;
    uint32_t w = S.lostab[((size_t)x1 * P.G + y1) * LOS_CELL_WORDS + (dx + R_LOS) * LOS_ROW_WORDS +
                          (col >> 5)];
    return (w >> (col & 31)) & 3u;
  }
  return los_march_c(S, mask, P.W16, x1, y1, x2, y2);
}

// ---------------------------------------------------------------------------
// get_obs sensor fusion (combatant.py:90-161 / landingship.py:94-165): refreshes
// the target list of agent `me`. Observation floats are written in phase O.
// ---------------------------------------------------------------------------
struct ObsAcc {
  int obs_n, norder;
};

__device__ inline void pair_after_los(Ctx &X, int i, int jj, int xi, int yi, int xj, int yj,
                                      bool rad_ok, bool close, bool ew_cand, uint32_t los,
                                      ObsAcc &acc);

// One own-ship x opponent check of get_obs (combatant.py:106-124) once the
// squared distance is known: radar / close / EW conditions, LOS (table or
// march), the position-deduplicated observed list and EW bearings (gauss).
__device__ inline void pair_detect(Ctx &X, int myradar, int i, int jj, int xi, int yi, int ti,
                                   int xj, int yj, int tj, int radj, int d2, ObsAcc &acc) {
  const KParams &P = X.P;
  const KState &S = X.S;
  Cols &c = X.c;
  const int lane = X.lane;
  int rr = radar_r(P, X.duct(), ti, tj), re = ew_r(P, X.duct(), ti, tj);
  bool rad_ok = myradar == 1 && d2 < rr * rr;
  bool close = d2 < 16;
  bool ew_cand = d2 < re * re && radj == 1;
  if (!(rad_ok || close || ew_cand)) return;  // LOS result would be unused
  pair_after_los(X, i, jj, xi, yi, xj, yj, rad_ok, close, ew_cand,
                 los_q(P, S, X.mask, xi, yi, xj, yj), acc);
}

// The observed-list part of one get_obs pair (combatant.py:106-118): radar or
// close detection through a clear radar LOS, de-duplicated by position.
// Returns true when the pair yields an EW bearing (combatant.py:119-124).
__device__ inline bool pair_observe(Ctx &X, int xj, int yj, bool rad_ok, bool close, bool ew_cand,
                                    uint32_t los, ObsAcc &acc) {
  Cols &c = X.c;
  const int lane = X.lane;
  if (!(los & 1u)) return false;
  uint32_t pk = pack_pos(xj, yj);
  bool seen = false;
  for (int q = 0; q < acc.obs_n; q++) seen |= COLW(c.observed, q) == pk;
  if ((rad_ok || close) && !seen) {
    COLW(c.observed, acc.obs_n) = pk;
    acc.obs_n++;
    seen = true;
  }
  return ew_cand && (los & 2u) && !seen;
}

// math.degrees(math.atan2(dy, dx)) (combatant.py:253): the host-libm table in
// the +-R_LOS window, the device atan2 outside it (or with LNW_DEBUG_SKIP bit 12)
__device__ inline double bearing_deg(const KParams &P, const KState &S, int dx, int dy) {
  const bool tab = !(P.dbg_skip & 4096) && S.atan_deg && dx >= -R_LOS && dx <= R_LOS &&
                   dy >= -R_LOS && dy <= R_LOS;
  return tab ? S.atan_deg[(dy + R_LOS) * LOS_W + (dx + R_LOS)] : atan2((double)dy, (double)dx) * RAD2DEG;
}

// bearing_deg split in two: bearing_pre loads unconditionally (the dummy buffer
// when the table does not apply, so no branch sits between the load and its
// use), bearing_use returns the table value or falls back to the device atan2
struct BearPre {
  double v;
  bool tab;
};
__device__ inline BearPre bearing_pre(const KParams &P, const KState &S, int dx, int dy) {
  const bool tab = !(P.dbg_skip & 4096) && S.atan_deg && dx >= -R_LOS && dx <= R_LOS &&
                   dy >= -R_LOS && dy <= R_LOS;
  const double *p = tab ? S.atan_deg + (dy + R_LOS) * LOS_W + (dx + R_LOS) : (const double *)S.dummy;
  return {*p, tab};
}
__device__ inline double bearing_use(const BearPre &b, int dx, int dy) {
  return b.tab ? b.v : atan2((double)dy, (double)dx) * RAD2DEG;
}

// calculate_bearing (combatant.py:249-263) with the gauss draw given
__device__ inline double ew_bearing(const KParams &P, const KState &S, int xi, int yi, int xj, int yj,
                                    double distortion) {
  double bearing = bearing_deg(P, S, xj - xi, yj - yi);
  if (bearing + distortion < 0)
    bearing = bearing + distortion + 360.0;
  else
    bearing = bearing + distortion;
  return bearing;
}

// The LOS-dependent part of one get_obs pair (combatant.py:106-124).
__device__ inline void pair_after_los(Ctx &X, int i, int jj, int xi, int yi, int xj, int yj,
                                      bool rad_ok, bool close, bool ew_cand, uint32_t los,
                                      ObsAcc &acc) {
  const KState &S = X.S;
  Cols &c = X.c;
  const int lane = X.lane;
  if (pair_observe(X, xj, yj, rad_ok, close, ew_cand, los, acc)) {
    const double bearing = ew_bearing(X.P, S, xi, yi, xj, yj, X.rng.gauss());
    int k = COLB(c.bcnt, jj);
    if (k == 0) { COLB(c.border, acc.norder) = (uint8_t)jj; acc.norder++; }
    size_t slot = (size_t)(jj * S.nmax + k) * X.E + X.env;
    S.bear_val[slot] = bearing;
    S.bear_ship[slot] = (uint8_t)i;
    COLB(c.bcnt, jj) = (uint8_t)(k + 1);
  }
}

// pair_after_los for the runtime-size walk (get_obs_dev): `obsm` bit k is set
// once opponent k's cell is in `observed`, so the de-duplication is one bit test
// instead of a scan of the LDS list per pair. Cells do not change during a
// get_obs call, so bit k <=> pos(k) in observed, as the reference's test.
__device__ inline void pair_after_los_m(Ctx &X, int i, int jj, int opp0, int nopp, int xi, int yi,
                                        int xj, int yj, bool rad_ok, bool close, bool ew_cand,
                                        uint32_t los, ObsAcc &acc, uint64_t &obsm) {
  const KState &S = X.S;
  Cols &c = X.c;
  const int lane = X.lane;
  if (!(los & 1u)) return;
  bool seen = (obsm >> jj) & 1u;
  if ((rad_ok || close) && !seen) {
    const uint32_t pk = pack_pos(xj, yj);
    COLW(c.observed, acc.obs_n) = pk;
    acc.obs_n++;
    for (int k = 0; k < nopp; k++)  // every opponent on this cell is now observed
      if (COLW(c.pos_cur, opp0 + k) == pk) obsm |= 1ull << k;
    seen = true;
  }
  if (ew_cand && (los & 2u) && !seen) {
    const double bearing = ew_bearing(X.P, S, xi, yi, xj, yj, X.rng.gauss());
    int k = COLB(c.bcnt, jj);
    if (k == 0) { COLB(c.border, acc.norder) = (uint8_t)jj; acc.norder++; }
    size_t slot = (size_t)(jj * S.nmax + k) * X.E + X.env;
    S.bear_val[slot] = bearing;
    S.bear_ship[slot] = (uint8_t)i;
    COLB(c.bcnt, jj) = (uint8_t)(k + 1);
  }
}

// Target list (combatant.py:152-161): observed positions first, then every EW
// fix (combatant.py:128-150) landing within 2 cells of a live opponent.
// Mean of the consecutive-pair EW fixes of opponent jj's n bearings
// (combatant.py:128-150, calculate_fixed_position :265-277), summed in
// np.mean's order (pairwise for >= 8 terms). Returns false on a zero slope
// difference (the reference's ZeroDivisionError).
struct FixAcc {
  double sumx = 0, sumy = 0, resx = 0, resy = 0;
  double r0x = 0, r1x = 0, r2x = 0, r3x = 0, r4x = 0, r5x = 0, r6x = 0, r7x = 0;
  double r0y = 0, r1y = 0, r2y = 0, r3y = 0, r4y = 0, r5y = 0, r6y = 0, r7y = 0;
  bool tail_started = false;
  // every partial sum conditionally updated (no indexed array or address select,
  // which would keep the sums in scratch); folds to one update for constant r
  __device__ void put(int r, bool acc, double x3, double y3) {
#define LNW_PUT(i)                                              \
  r##i##x = r == i ? (acc ? r##i##x + x3 : x3) : r##i##x;      \
  r##i##y = r == i ? (acc ? r##i##y + y3 : y3) : r##i##y;
    LNW_PUT(0) LNW_PUT(1) LNW_PUT(2) LNW_PUT(3) LNW_PUT(4) LNW_PUT(5) LNW_PUT(6) LNW_PUT(7)
#undef LNW_PUT
  }
  __device__ void add(int k, int m, double x3, double y3) {
    const int mblk = m - (m % 8);
    if (m < 8) {
      sumx += x3;
      sumy += y3;
    } else if (k < mblk) {
      put(k & 7, k >= 8, x3, y3);
    } else {
      if (!tail_started) { tree(); tail_started = true; }
      resx += x3;
      resy += y3;
    }
  }
  __device__ void tree() {
    resx = ((r0x + r1x) + (r2x + r3x)) + ((r4x + r5x) + (r6x + r7x));
    resy = ((r0y + r1y) + (r2y + r3y)) + ((r4y + r5y) + (r6y + r7y));
  }
  __device__ void mean(int m, double &mx, double &my) {
    if (m < 8) { mx = sumx / (double)m; my = sumy / (double)m; return; }
    if (!tail_started) tree();
    mx = resx / (double)m;
    my = resy / (double)m;
  }
};

__device__ inline void fix_pair(double m1, double m2, double x1, double y1, double x2, double y2,
                                double &x3, double &y3) {
  x3 = (m1 * x1 - m2 * x2 + y2 - y1) / (m1 - m2);
  y3 = m1 * (x3 - x1) + y1;
}

// any n: one bearing pair at a time from the global scratch
__device__ inline bool fix_mean_loop(Ctx &X, int jj, int n, double &mx, double &my) {
  const KState &S = X.S;
  Cols &c = X.c;
  const int lane = X.lane;
  auto slot = [&](int k) { return (size_t)(jj * S.nmax + k) * X.E + X.env; };
  const int m = n - 1;
  FixAcc f;
  for (int k = 0; k < m; k++) {
    uint8_t s1 = S.bear_ship[slot(k)], s2 = S.bear_ship[slot(k + 1)];
    double b1 = S.bear_val[slot(k)], b2 = S.bear_val[slot(k + 1)];
    uint32_t p1 = COLW(c.pos_cur, s1), p2 = COLW(c.pos_cur, s2);
    double m1 = tan_fd(b1 * DEG2RAD);
    double m2 = tan_fd(b2 * DEG2RAD);
    if (m1 - m2 == 0.0) return false;
    double x3, y3;
    fix_pair(m1, m2, pos_x(p1), pos_y(p1), pos_x(p2), pos_y(p2), x3, y3);
    f.add(k, m, x3, y3);
  }
  f.mean(m, mx, my);
  return true;
}

// n <= BMAX: all bearings loaded together, one tan per bearing, the pairs
// unrolled (same arithmetic and summation order as fix_mean_loop)
template <int BMAX>
__device__ inline bool fix_mean_batched(Ctx &X, int jj, int n, double &mx, double &my) {
  const KState &S = X.S;
  Cols &c = X.c;
  const int lane = X.lane;
  auto slot = [&](int k) { return (size_t)(jj * S.nmax + k) * X.E + X.env; };
  double bv[BMAX];
  int bs[BMAX];
#pragma unroll
  for (int k = 0; k < BMAX; k++) {
    bv[k] = 0.0;
    bs[k] = 0;
    if (k < n) { bv[k] = S.bear_val[slot(k)]; bs[k] = S.bear_ship[slot(k)]; }
  }
  double tv[BMAX], px[BMAX], py[BMAX];
#pragma unroll
  for (int k = 0; k < BMAX; k++) {
    tv[k] = 0.0;
    px[k] = py[k] = 0.0;
    if (k < n) {
      tv[k] = tan_fd(bv[k] * DEG2RAD);
      const uint32_t p = COLW(c.pos_cur, bs[k]);
      px[k] = pos_x(p);
      py[k] = pos_y(p);
    }
  }
  const int m = n - 1;
  FixAcc f;
  bool zero = false;
#pragma unroll
  for (int k = 0; k < BMAX - 1; k++) {
    if (k < m && !zero) {
      if (tv[k] - tv[k + 1] == 0.0) {
        zero = true;
      } else {
        double x3, y3;
        fix_pair(tv[k], tv[k + 1], px[k], py[k], px[k + 1], py[k + 1], x3, y3);
        f.add(k, m, x3, y3);
      }
    }
  }
  if (zero) return false;
  f.mean(m, mx, my);
  return true;
}

// BMAX: bearings per opponent handled by the batched fix path; EXACT: no more
// can occur (compile-time own-team size), so the loop fallback is not built.
template <int BMAX, bool EXACT>
__device__ inline void finish_obs(Ctx &X, int me, int opp0, int opp1, const ObsAcc &acc) {
  const KParams &P = X.P;
  const KState &S = X.S;
  Cols &c = X.c;
  const int lane = X.lane;
  const long long E = X.E;
  const int env = X.env;
  const int obs_n = acc.obs_n, norder = acc.norder;
  const int T = P.T;
  uint16_t *tl = S.tl + (size_t)me * T * E + env;
  int tn = 0;
  for (int q = 0; q < obs_n; q++) {
    uint32_t pk = COLW(c.observed, q);
    tl[(size_t)tn * E] = (uint16_t)(pos_x(pk) | (pos_y(pk) << 8));
    tn++;
  }
  // EW fixes (combatant.py:128-150) and fix targets (combatant.py:156-161)
  for (int o = 0; o < norder; o++) {
    int jj = COLB(c.border, o);
    int n = COLB(c.bcnt, jj);
    if (n < 2) continue;
    double mx, my;
    bool ok;
    if constexpr (EXACT) ok = fix_mean_batched<BMAX>(X, jj, n, mx, my);
    else ok = n <= BMAX ? fix_mean_batched<BMAX>(X, jj, n, mx, my) : fix_mean_loop(X, jj, n, mx, my);
    if (!ok) { X.rng.err |= LNW_ERRF_ZERODIV; continue; }
    if (!isfinite(mx) || !isfinite(my)) { X.rng.err |= LNW_ERRF_NAN_ROUND; continue; }
    double rx = rint(mx), ry = rint(my);
    if (S.ana.ew_log) {  // combatant.py:146-150: (observer position, rounded fix)
      const int fx = (int)fmin(fmax(rx, -32768.0), 32767.0), fy = (int)fmin(fmax(ry, -32768.0), 32767.0);
      ana_record(S.ana.ew_log, S.ana.ew_count, S.ana.ew_cap, (uint32_t)(P.env_base + env),
                 (uint32_t)X.step | (uint32_t)(me >= P.nb) << 16, COLW(c.pos_cur, me),
                 (uint32_t)(uint16_t)fx | (uint32_t)(uint16_t)fy << 16);
    }
    if (!(rx >= 0.0 && rx < (double)P.G && ry >= 0.0 && ry < (double)P.G)) continue;
    int fxi = (int)rx, fyi = (int)ry;
    for (int j = opp0; j < opp1; j++) {
      if (!COLB(c.alive0, j)) continue;
      uint32_t pj = COLW(c.pos_cur, j);
      int ddx = pos_x(pj) - fxi, ddy = pos_y(pj) - fyi;
      if (ddx * ddx + ddy * ddy < 4) {
        tl[(size_t)tn * E] = (uint16_t)(fxi | (fyi << 8));
        tn++;
      }
    }
  }
  COLW(c.tcnt, me) = (uint32_t)tn;
}


// Select a[k] of a small register array without indexing (which would move
// the array to scratch).
template <int N, class T>
__device__ __forceinline__ T rsel(const T (&a)[N], int k) {
  T v = a[0];
#pragma unroll
  for (int q = 1; q < N; q++) v = k == q ? a[q] : v;
  return v;
}

// get_obs sensor fusion (combatant.py:90-161 / landingship.py:94-165) for
// runtime ship counts: refreshes agent me's target list (observation floats are
// written in phase O).
// los_mode 2 (reference work, diagnostics): the reference traces the full
// Bresenham line of every own ship x opponent pair at every get_obs before
// testing any range (combatant.py:106-110, 443-454). March those rays in full
// (no early exit, counted by lnw_set_counters) and discard them; the step's
// own LOS answers still come from the table, so results do not change.
__device__ __forceinline__ void march_pairs_ref(Ctx &X, int me) {
  const KParams &P = X.P;
  const Cols &c = X.c;
  const int lane = X.lane;
  const int side = me >= P.nb;
  const int own0 = side ? P.nb : 0, own1 = side ? P.A : P.nb;
  const int opp0 = side ? 0 : P.nb, opp1 = side ? P.nb : P.A;
  uint32_t acc = 0;
  for (int i = own0; i < own1; i++) {
    if (!COLB(c.alive0, i)) continue;
    const uint32_t pi = COLW(c.pos_cur, i);
    for (int j = opp0; j < opp1; j++) {
      if (!COLB(c.alive0, j)) continue;
      const uint32_t pj = COLW(c.pos_cur, j);
      int n = 0;
      acc += los_march<false>(X.mask, P.W16, pos_x(pi), pos_y(pi), pos_x(pj), pos_y(pj), &n);
      if (X.S.ctr) {
        atomicAdd(&X.S.ctr[0], 1ull);
        atomicAdd(&X.S.ctr[1], (unsigned long long)n);
      }
    }
  }
  if (acc == 0xffffffffu) X.S.dummy[lane] = 0.0f;  // keeps the marches (never true)
}

__device__ __forceinline__ void get_obs_dev(Ctx &X, int me) {
  const KParams &P = X.P;
  const KState &S = X.S;
  Cols &c = X.c;
  const int lane = X.lane;
  const int nb = P.nb, A = P.A;
  const int side = me >= nb;
  const int own0 = side ? nb : 0, own1 = side ? A : nb;
  const int opp0 = side ? 0 : nb, opp1 = side ? nb : A;
  const int nopp = opp1 - opp0, npair = (own1 - own0) * nopp;
  const int myradar = COLW(c.radar_cur, me);
  ObsAcc acc{0, 0};
  uint64_t obsm = 0;  // opponents whose cell is already observed
  for (int q = 0; q < nopp; q++) COLB(c.bcnt, q) = 0;
  // radar / EW ranges of this env's duct for every (own mast class, opponent
  // type) once per call, selected per pair instead of recomputed in f64
  const double duct = X.duct();
  int rr_t[2][3], re_t[2][3];
#pragma unroll
  for (int mi = 0; mi < 2; mi++)
#pragma unroll
    for (int tj = 0; tj < 3; tj++) {
      const int ti = mi ? T_LARGE : T_SMALL;
      rr_t[mi][tj] = radar_r(P, duct, ti, tj);
      re_t[mi][tj] = ew_r(P, duct, ti, tj);
    }
  // pairs (i outer, j inner) in chunks of 16: the sensor tests of a chunk, then
  // its LOS table words loaded together, then the chunk walked in order
  const unsigned long long tw = prof_now(S);
#pragma unroll 1
  for (int b0 = 0; b0 < npair; b0 += 16) {
    uint32_t radm = 0, closem = 0, ewm = 0, tabm = 0, marchm = 0;
    uint32_t wi[16];
    // (i, j) of the chunk's pairs stepped incrementally: one division per chunk
    // (wave-uniform); the own ship's alive flag, cell and mast class are loaded
    // when i changes, not per pair
    int ic = own0 + b0 / nopp, jc = opp0 + b0 % nopp;
    bool al_i = COLB(c.alive0, ic);
    uint32_t pi_c = COLW(c.pos_cur, ic);
    int mi_c = mast_cls(COLB(c.type, ic));
#pragma unroll
    for (int u = 0; u < 16; u++) {
      wi[u] = 0;
      const int b = b0 + u;
      const int j = jc;
      const bool ali = al_i;
      const uint32_t pi = pi_c;
      const int mi = mi_c;
      if (++jc == opp1) {
        jc = opp0;
        if (++ic < own1) {
          al_i = COLB(c.alive0, ic);
          pi_c = COLW(c.pos_cur, ic);
          mi_c = mast_cls(COLB(c.type, ic));
        }
      }
      if (b >= npair) continue;
      if (!ali || !COLB(c.alive0, j)) continue;
      const uint32_t pj = COLW(c.pos_cur, j);
      const int dx = pos_x(pj) - pos_x(pi), dy = pos_y(pj) - pos_y(pi);
      const int d2 = dx * dx + dy * dy;
      if (d2 >= X.r2max) continue;  // beyond every radar / EW / close range: LOS unused
      const int tj = rng_cls(COLB(c.type, j));  // (rr_t / re_t columns: small, large-like, LandingShip)
      const int rr0 = tj == 0 ? rr_t[0][0] : (tj == 1 ? rr_t[0][1] : rr_t[0][2]);
      const int rr1 = tj == 0 ? rr_t[1][0] : (tj == 1 ? rr_t[1][1] : rr_t[1][2]);
      const int re0 = tj == 0 ? re_t[0][0] : (tj == 1 ? re_t[0][1] : re_t[0][2]);
      const int re1 = tj == 0 ? re_t[1][0] : (tj == 1 ? re_t[1][1] : re_t[1][2]);
      const int rr = mi ? rr1 : rr0, re = mi ? re1 : re0;
      const bool rad_ok = myradar == 1 && d2 < rr * rr, close = d2 < 16;
      const bool ew_cand = d2 < re * re && COLW(c.radar_cur, j) == 1;
      if (!(rad_ok || close || ew_cand)) continue;  // LOS result would be unused
      radm |= (rad_ok ? 1u : 0u) << u;
      closem |= (close ? 1u : 0u) << u;
      ewm |= (ew_cand ? 1u : 0u) << u;
      if (P.los_mode != 1 && dx >= -R_LOS && dx <= R_LOS && dy >= -R_LOS && dy <= R_LOS) {
        tabm |= 1u << u;
        wi[u] = ((uint32_t)(pos_x(pi) * P.G + pos_y(pi)) * LOS_CELL_WORDS + (dx + R_LOS) * LOS_ROW_WORDS) *
                    32u + (dy + R_LOS) * 2;
      } else {
        marchm |= 1u << u;
      }
    }
    uint32_t losb = 0;
#pragma unroll
    for (int u = 0; u < 16; u++) {
      const uint32_t w = (tabm >> u) & 1u ? S.lostab[wi[u] >> 5] : 0u;
      losb |= ((w >> (wi[u] & 31)) & 3u) << (2 * u);
    }
    uint32_t todo = tabm | marchm;
    while (todo) {
      const int u = __builtin_ctz(todo);
      todo &= todo - 1;
      const int b = b0 + u;
      const int i = own0 + b / nopp, j = opp0 + b % nopp;
      const uint32_t pi = COLW(c.pos_cur, i), pj = COLW(c.pos_cur, j);
      const int xi = pos_x(pi), yi = pos_y(pi), xj = pos_x(pj), yj = pos_y(pj);
      const uint32_t los = (tabm >> u) & 1u ? (losb >> (2 * u)) & 3u
                                            : los_q(P, S, X.mask, xi, yi, xj, yj);
      pair_after_los_m(X, i, j - opp0, opp0, nopp, xi, yi, xj, yj, (radm >> u) & 1u,
                       (closem >> u) & 1u, (ewm >> u) & 1u, los, acc, obsm);
    }
  }
  const unsigned long long tf = prof_acc(S, 20, tw);
  finish_obs<16, false>(X, me, opp0, opp1, acc);
  prof_acc(S, 22, tf);
}


// Target list of a templated get_obs (combatant.py:128-161) from pass 1's
// observed list and bearing requests. Bearing k of the call (pair
// order) takes gauss draw base+k; the draws of opponents with a single bearing
// are consumed but never evaluated (Philox and the tape are indexed by draw
// number). Per opponent j the bearings come from own ships i ascending, i.e. in
// the order the reference appends them, so consecutive-pair fixes stream
// without storage; the mean of m = n-1 <= 3 fixes is a plain left-to-right sum
// (np.mean below 8 terms). Fix targets are appended in the order of each
// opponent's first bearing.
template <int NOWN, int NOPP, bool CW>
__device__ inline void finish_obs_t(Ctx &X, int me, int own0, int opp0, int obs_n,
                                    uint32_t firstbit, uint32_t bearm,
                                    const uint32_t (&pp)[NOPP], uint32_t oal = 0) {
  static_assert(NOWN < 9, "np.mean pairwise summation starts at 8 terms");
  const KParams &P = X.P;
  const KState &S = X.S;
  Cols &c = X.c;
  const int lane = X.lane;
  const long long E = X.E;
  const int env = X.env;
  const unsigned long long base = X.rng.ctr;
  const int nbear = __builtin_popcount(bearm);
  if (X.rng.mode == 1) {  // tape: a draw past the end sets the flag and does not advance
    const long long avail = X.rng.tape_hi - X.rng.tape_lo - (long long)base;
    if (nbear > avail) X.rng.err |= 4u;
    X.rng.ctr += (unsigned long long)(nbear < avail ? nbear : (avail > 0 ? avail : 0));
  } else {
    X.rng.ctr += (unsigned long long)nbear;
  }
  uint16_t *tl = S.tl + (size_t)me * P.T * E + env;
  unsigned long long tq = prof_now(S);
  int tn = 0;
  // observed positions (combatant.py:152-154)
  if constexpr (CW) {  // one per cell class, in the order of each class's first detecting pair
    for (uint32_t fb = firstbit; fb; fb &= fb - 1) {
      const uint32_t pk = COLW(c.pos_cur, opp0 + __builtin_ctz(fb) % NOPP);
      tl[(size_t)tn * E] = (uint16_t)(pos_x(pk) | (pos_y(pk) << 8));
      tn++;
    }
  } else {  // the list the walk built in LDS
    for (int q = 0; q < obs_n; q++) {
      uint32_t pk = COLW(c.observed, q);
      tl[(size_t)tn * E] = (uint16_t)(pos_x(pk) | (pos_y(pk) << 8));
      tn++;
    }
  }
  tq = prof_acc(S, 21, tq);
  // (contact variant: lanes without bearings stay, to evaluate other lanes' bearings)
  if (!CW && bearm == 0) { COLW(c.tcnt, me) = (uint32_t)tn; return; }
  uint32_t colj = 0;  // bits of opponent 0's column
#pragma unroll
  for (int i = 0; i < NOWN; i++) colj |= 1u << (i * NOPP);
  // the bearings to evaluate, opponent-major (bit j*NOWN + i): opponents with at
  // least two, i.e. a fix. One flat loop over them keeps the lanes of a wave
  // busy (a per-opponent loop would run each opponent's worst-lane count).
  uint32_t need = 0;
#pragma unroll
  for (int j = 0; j < NOPP; j++) {
    const uint32_t bj = bearm & (colj << j);
    if (__builtin_popcount(bj) < 2) continue;
#pragma unroll
    for (int i = 0; i < NOWN; i++) need |= ((bj >> (i * NOPP + j)) & 1u) << (j * NOWN + i);
  }
  if (S.prof) {  // bearing load balance: lane sum and wave max of the bearings evaluated
    const int cnt = __builtin_popcount(need);
    int s = 0, mx = 0;  // over the active lanes, by ballots
    for (int b = 4; b >= 0; b--) {
      s += __popcll(__ballot((cnt >> b) & 1)) << b;
      if (__ballot(cnt >= (mx | (1 << b)))) mx |= 1 << b;
    }
    const unsigned long long m = __ballot(1);
    if ((int)(threadIdx.x & 63) == __ffsll((long long)m) - 1) {
      atomicAdd(&S.prof[(size_t)blockIdx.x * PROF_SLOTS + 24], (unsigned long long)s);
      atomicAdd(&S.prof[(size_t)blockIdx.x * PROF_SLOTS + 25], (unsigned long long)mx);
      atomicAdd(&S.prof[(size_t)blockIdx.x * PROF_SLOTS + 26], (unsigned long long)__popcll(m));
    }
  }
  // opponent j's rounded fix, x | y << 8, in bits 16j..16j+15 (a register
  // array indexed by a runtime j would live in scratch)
  static_assert(NOPP <= 4, "fix cells packed 16 bits per opponent");
  uint64_t fixw = 0;
  uint32_t fok = 0;  // opponent j has a rounded fix inside the grid
  int curj = -1, cnt = 0;
  bool zero = false;
  double sumx = 0.0, sumy = 0.0, mprev = 0.0, xprev = 0.0, yprev = 0.0;
  // mean of opponent curj's fixes (np.mean, m = cnt-1 < 8 terms: left-to-right)
  auto flush = [&]() {
    if (curj < 0) return;
    if (zero) { X.rng.err |= LNW_ERRF_ZERODIV; return; }
    const double mx = sumx / (double)(cnt - 1), my = sumy / (double)(cnt - 1);
    if (!isfinite(mx) || !isfinite(my)) { X.rng.err |= LNW_ERRF_NAN_ROUND; return; }
    const double rx = rint(mx), ry = rint(my);
    if (S.ana.ew_log) {  // combatant.py:146-150: (observer position, rounded fix)
      const int fx = (int)fmin(fmax(rx, -32768.0), 32767.0), fy = (int)fmin(fmax(ry, -32768.0), 32767.0);
      ana_record(S.ana.ew_log, S.ana.ew_count, S.ana.ew_cap, (uint32_t)(P.env_base + env),
                 (uint32_t)X.step | (uint32_t)(me >= P.nb) << 16, COLW(c.pos_cur, me),
                 (uint32_t)(uint16_t)fx | (uint32_t)(uint16_t)fy << 16);
    }
    if (!(rx >= 0.0 && rx < (double)P.G && ry >= 0.0 && ry < (double)P.G)) return;
    fixw |= (uint64_t)((uint32_t)(int)rx | (uint32_t)(int)ry << 8) << (16 * curj);
    fok |= 1u << curj;
  };
  if constexpr (CW) {
  // Two bearings per iteration: their gauss draws and tangents are independent
  // f64 chains the compiler interleaves (with one compute wave per SIMD a single
  // chain leaves the latency of every dependent op exposed); the fix sums then
  // take them in order. The table loads of both go first, the rare atan2
  // fallback after them, so the chains share one basic block.
  auto setup = [&](int t, int &dx, int &dy, int &j, double &x1, double &y1, int &k) {
    j = t / NOWN;
    const int i = t - j * NOWN, b = i * NOPP + j;
    const uint32_t pi = COLW(c.pos_cur, own0 + i), pj = COLW(c.pos_cur, opp0 + j);
    dx = pos_x(pj) - pos_x(pi);
    dy = pos_y(pj) - pos_y(pi);
    x1 = pos_x(pi);
    y1 = pos_y(pi);
    k = __builtin_popcount(bearm & ((1u << b) - 1u));
  };
  auto accum = [&](int j, double m, double x1, double y1) {
    if (j != curj) {
      flush();
      curj = j; cnt = 0; zero = false; sumx = sumy = 0.0;
    }
    if (cnt > 0 && !zero) {
      if (mprev - m == 0.0) {
        zero = true;
      } else {
        double x3, y3;
        fix_pair(mprev, m, xprev, yprev, x1, y1, x3, y3);
        sumx += x3;
        sumy += y3;
      }
    }
    cnt++;
    mprev = m; xprev = x1; yprev = y1;
  };
  // wave max of the per-lane bearing counts (ballots over the active lanes)
  const unsigned long long act = __ballot(1);
  const int ncnt = __builtin_popcount(need);
  int wmax = 0;
#pragma unroll
  for (int b = 4; b >= 0; b--)
    if (__ballot(ncnt >= (wmax | (1 << b)))) wmax |= 1 << b;
  if (NOWN * NOPP > 2 && wmax > 2 && !(P.dbg_skip & 131072)) {  // (LNW_DEBUG_SKIP bit 17: per-lane loop)
    // Pooled: the wave's bearings are numbered owner by owner (lane l's k-th
    // bearing, in need-bit order, is g = excl_l + k) and every active lane takes
    // two consecutive ones per round, g = r0 + 2 rank and g + 1, so a round costs
    // the same whichever lanes own them (the per-lane loop runs the busiest lane's
    // count). An opponent's bearings from one owner are consecutive numbers (a
    // segment of at most NOWN); each slot computes its slope, the fix with the
    // previous slot of its segment (fix_pair, the same operands as the per-lane
    // loop), and the running sum of its segment's fixes, left to right like the
    // per-lane loop, by a segmented scan over the slots. The segment's last slot
    // takes the mean, rounds it and stores the fix (or the error) in an LDS table
    // the owner reads afterwards: identical arithmetic and results.
    const int nact = __popcll(act);
    const int rank = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(act >> 32),
                                                    __builtin_amdgcn_mbcnt_lo((uint32_t)act, 0u));
    int excl = 0, total = 0;
#pragma unroll
    for (int b = 0; b < 5; b++) {
      const unsigned long long bb = __ballot((ncnt >> b) & 1);
      excl += (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bb >> 32),
                                             __builtin_amdgcn_mbcnt_lo((uint32_t)bb, 0u)) << b;
      total += __popcll(bb) << b;
    }
    if (S.ctr && rank == 0) atomicAdd(&S.ctr[3], (unsigned long long)total);  // work counter
    // in the observed-list / bearing-order columns (unused by the contact
    // variant's walk; >= 396 B per opponent slot, this needs 192 + 256 per
    // opponent): rank -> lane, rank -> first bearing number, and the fix table
    // [opponent][owner lane]: fx | fy << 8 | inside << 16 | zero-div << 17 | nan << 18
    uint8_t *lor = (uint8_t *)c.observed;
    uint16_t *exr = (uint16_t *)(lor + WAVE);
    uint32_t *fixt = (uint32_t *)(lor + 3 * WAVE);
    lor[rank] = (uint8_t)lane;
    exr[rank] = (uint16_t)excl;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const int prevl = rank > 0 ? (int)lor[rank - 1] : lane;  // the lane of the previous rank
    const int lastl = 63 - __builtin_clzll(act);              // the lane of the last rank
    const bool tape = X.rng.mode == 1;
    constexpr uint32_t SEGM = (1u << NOWN) - 1u;
    // bearing g: owner lane s, own ship i, opponent j, the owner's bearings on j
    // (bit i), its gauss draw number and the two positions. The shuffles run on
    // every active lane (owners are active).
    auto locate = [&](int g, int &s, int &i, int &j, uint32_t &nsj, unsigned long long &drw,
                      uint32_t &pi, uint32_t &pj) {
      int lo = 0;
#pragma unroll
      for (int st = 32; st; st >>= 1)
        if (lo + st < nact && (int)exr[lo + st] <= g) lo += st;
      s = lor[lo];
      const int kk = g - (int)exr[lo];
      uint32_t ns = (uint32_t)__shfl((int)need, s);
      const uint32_t bs = (uint32_t)__shfl((int)bearm, s);
      drw = __shfl(base, s);
      uint32_t w = ns;
      for (int q = 0; q < kk; q++) w &= w - 1;
      const int t = __builtin_ctz(w);
      j = t / NOWN;
      i = t - j * NOWN;
      const int b = i * NOPP + j;
      drw += (unsigned long long)__builtin_popcount(bs & ((1u << b) - 1u));
      nsj = (ns >> (j * NOWN)) & SEGM;
      pi = c.pos_cur[(own0 + i) * PAD + s];
      pj = c.pos_cur[(opp0 + j) * PAD + s];
    };
    auto draw = [&](int s, unsigned long long d) -> double {
      const int es = env - lane + s;
      if (tape) {
        if (!S.tape_off) return 0.0;
        const long long p = S.tape_off[es] + (long long)d;
        return p < S.tape_off[es + 1] ? S.tape[p] : 0.0;
      }
      const unsigned long long gid = (unsigned long long)(P.env_base + es);
      return X.rng.gauss_philox(d, (uint32_t)gid, (uint32_t)(gid >> 32));
    };
    // mean, rounding and grid test of a finished segment (the per-lane flush)
    auto finish = [&](int s, int j, int n, double sx, double sy, bool z, int stp) {
      uint32_t w = 0;
      if (z) {
        w = 1u << 17;
      } else {
        const double mx = sx / (double)(n - 1), my = sy / (double)(n - 1);
        if (!isfinite(mx) || !isfinite(my)) {
          w = 1u << 18;
        } else {
          const double rx = rint(mx), ry = rint(my);
          if (S.ana.ew_log) {  // combatant.py:146-150: (observer position, rounded fix)
            const int fx = (int)fmin(fmax(rx, -32768.0), 32767.0), fy = (int)fmin(fmax(ry, -32768.0), 32767.0);
            ana_record(S.ana.ew_log, S.ana.ew_count, S.ana.ew_cap, (uint32_t)(P.env_base + env - lane + s),
                       (uint32_t)stp | (uint32_t)(me >= P.nb) << 16, c.pos_cur[me * PAD + s],
                       (uint32_t)(uint16_t)fx | (uint32_t)(uint16_t)fy << 16);
          }
          if (rx >= 0.0 && rx < (double)P.G && ry >= 0.0 && ry < (double)P.G)
            w = (uint32_t)(int)rx | (uint32_t)(int)ry << 8 | 1u << 16;
        }
      }
      fixt[j * WAVE + s] = w;
    };
    // the previous round's last slot (rank nact-1, second slot)
    double cm = 0.0, csx = 0.0, csy = 0.0;
    uint32_t cp = 0;
    int cz = 0;
    for (int r0 = 0; r0 < total; r0 += 2 * nact) {
      const int gA = r0 + 2 * rank, gB = gA + 1;
      int sA, iA, jA, sB, iB, jB;
      uint32_t nA, nB, piA, pjA, piB, pjB;
      unsigned long long dA, dB;
      locate(min(gA, total - 1), sA, iA, jA, nA, dA, piA, pjA);
      locate(min(gB, total - 1), sB, iB, jB, nB, dB, piB, pjB);
      const int dx1 = pos_x(pjA) - pos_x(piA), dy1 = pos_y(pjA) - pos_y(piA);
      const int dx2 = pos_x(pjB) - pos_x(piB), dy2 = pos_y(pjB) - pos_y(piB);
      const BearPre b1 = bearing_pre(P, S, dx1, dy1), b2 = bearing_pre(P, S, dx2, dy2);
      double a1 = b1.v, a2 = b2.v;
      if (!(b1.tab && b2.tab)) {
        a1 = bearing_use(b1, dx1, dy1);
        a2 = bearing_use(b2, dx2, dy2);
      }
      const double gg1 = draw(sA, dA), gg2 = draw(sB, dB);
      // calculate_bearing (combatant.py:249-263)
      const double br1 = a1 + gg1 < 0 ? a1 + gg1 + 360.0 : a1 + gg1;
      const double br2 = a2 + gg2 < 0 ? a2 + gg2 + 360.0 : a2 + gg2;
      const double mA = tan_fd(br1 * DEG2RAD), mB = tan_fd(br2 * DEG2RAD);
      // first / last bearing of its segment
      const bool fA = !(nA & ((1u << iA) - 1u)), fB = !(nB & ((1u << iB) - 1u));
      const bool lA = !(nA >> (iA + 1)), lB = !(nB >> (iB + 1));
      // slot A's predecessor: the previous rank's slot B, or the carry
      const double tm = __shfl(mB, prevl);
      const uint32_t tp = (uint32_t)__shfl((int)piB, prevl);
      const double pm = rank > 0 ? tm : cm;
      const uint32_t pp = rank > 0 ? tp : cp;
      double xA = 0.0, yA = 0.0, xB = 0.0, yB = 0.0;
      const bool zA = !fA && pm - mA == 0.0, zB = !fB && mA - mB == 0.0;
      if (!fA && !zA)
        fix_pair(pm, mA, pos_x(pp), pos_y(pp), pos_x(piA), pos_y(piA), xA, yA);
      if (!fB && !zB)
        fix_pair(mA, mB, pos_x(piA), pos_y(piA), pos_x(piB), pos_y(piB), xB, yB);
      // running sums (0.0 at a segment's first slot, then + each fix, left to
      // right). Each pass carries the sums one lane hop further (a slot reads its
      // predecessor's sum from the previous pass); a segment of at most NOWN slots
      // is final after (NOWN - 1) / 2 + 1 passes
      double sxA = 0.0, syA = 0.0, sxB = 0.0, syB = 0.0;
      bool ZA = false, ZB = false;
#pragma unroll
      for (int pass = 0; pass < (NOWN - 1) / 2 + 1; pass++) {
        const double qx = __shfl(sxB, prevl), qy = __shfl(syB, prevl);
        const int qz = __shfl((int)ZB, prevl);
        const double inx = rank > 0 ? qx : csx, iny = rank > 0 ? qy : csy;
        const bool inz = (rank > 0 ? qz : cz) != 0;
        sxA = fA ? 0.0 : inx + xA;
        syA = fA ? 0.0 : iny + yA;
        ZA = !fA && (inz || zA);
        sxB = fB ? 0.0 : sxA + xB;
        syB = fB ? 0.0 : syA + yB;
        ZB = !fB && (ZA || zB);
      }
      int stA = 0, stB = 0;
      if (S.ana.ew_log) {
        stA = __shfl(X.step, sA);
        stB = __shfl(X.step, sB);
      }
      if (gA < total && lA) finish(sA, jA, __builtin_popcount(nA), sxA, syA, ZA, stA);
      if (gB < total && lB) finish(sB, jB, __builtin_popcount(nB), sxB, syB, ZB, stB);
      // carry the last slot of the round
      cm = __shfl(mB, lastl);
      cp = (uint32_t)__shfl((int)piB, lastl);
      csx = __shfl(sxB, lastl);
      csy = __shfl(syB, lastl);
      cz = __shfl((int)ZB, lastl);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int j = 0; j < NOPP; j++) {
      if (__builtin_popcount((need >> (j * NOWN)) & SEGM) < 2) continue;
      const uint32_t w = fixt[j * WAVE + lane];
      if (w & (1u << 17)) X.rng.err |= LNW_ERRF_ZERODIV;
      else if (w & (1u << 18)) X.rng.err |= LNW_ERRF_NAN_ROUND;
      else if (w & (1u << 16)) {
        fixw |= (uint64_t)(w & 0xffffu) << (16 * j);
        fok |= 1u << j;
      }
    }
  } else
  while (need) {
    const int t1 = __builtin_ctz(need);
    need &= need - 1;
    const bool two = need != 0;
    const int t2 = two ? __builtin_ctz(need) : t1;
    if (two) need &= need - 1;
    int dx1, dy1, j1, k1, dx2, dy2, j2, k2;
    double x1, y1, x2, y2;
    setup(t1, dx1, dy1, j1, x1, y1, k1);
    setup(t2, dx2, dy2, j2, x2, y2, k2);
    const BearPre b1 = bearing_pre(P, S, dx1, dy1), b2 = bearing_pre(P, S, dx2, dy2);
    double a1 = b1.v, a2 = b2.v;
    if (!(b1.tab && b2.tab)) {
      a1 = bearing_use(b1, dx1, dy1);
      a2 = bearing_use(b2, dx2, dy2);
    }
    const double g1 = X.rng.gauss_at(base + (unsigned long long)k1);
    const double g2 = X.rng.gauss_at(base + (unsigned long long)k2);
    // calculate_bearing (combatant.py:249-263)
    const double br1 = a1 + g1 < 0 ? a1 + g1 + 360.0 : a1 + g1;
    const double br2 = a2 + g2 < 0 ? a2 + g2 + 360.0 : a2 + g2;
    const double m1 = tan_fd(br1 * DEG2RAD), m2 = tan_fd(br2 * DEG2RAD);
    accum(j1, m1, x1, y1);
    if (two) accum(j2, m2, x2, y2);
  }
  } else {
  while (need) {
    const int t = __builtin_ctz(need);
    need &= need - 1;
    const int j = t / NOWN, i = t - j * NOWN, b = i * NOPP + j;
    const uint32_t pi = COLW(c.pos_cur, own0 + i), pj = COLW(c.pos_cur, opp0 + j);
    const int dx = pos_x(pj) - pos_x(pi), dy = pos_y(pj) - pos_y(pi);
    const double a0 = bearing_deg(P, S, dx, dy);
    if (j != curj) {
      flush();
      curj = j; cnt = 0; zero = false; sumx = sumy = 0.0;
    }
    const int k = __builtin_popcount(bearm & ((1u << b) - 1u));
    const double g = X.rng.gauss_at(base + (unsigned long long)k);
    const double bearing = a0 + g < 0 ? a0 + g + 360.0 : a0 + g;  // calculate_bearing (combatant.py:249-263)
    const double m = tan_fd(bearing * DEG2RAD);
    const double x1 = pos_x(pi), y1 = pos_y(pi);
    if (cnt > 0 && !zero) {
      if (mprev - m == 0.0) {
        zero = true;
      } else {
        double x3, y3;
        fix_pair(mprev, m, xprev, yprev, x1, y1, x3, y3);
        sumx += x3;
        sumy += y3;
      }
    }
    cnt++;
    mprev = m; xprev = x1; yprev = y1;
  }
  }
  flush();
  tq = prof_acc(S, 22, tq);
  // fix targets (combatant.py:156-161), opponents in order of their first bearing
  uint32_t rem = bearm, done = 0;
  while (rem) {
    const int b = __builtin_ctz(rem);
    rem &= rem - 1;
    const int jj = b % NOPP;
    if ((done >> jj) & 1u) continue;
    done |= 1u << jj;
    if (!((fok >> jj) & 1u)) continue;
    const uint32_t fw = (uint32_t)(fixw >> (16 * jj));
    const int fxi = (int)(fw & 0xffu), fyi = (int)((fw >> 8) & 0xffu);
#pragma unroll
    for (int j = 0; j < NOPP; j++) {
      // (contact variant: the opponents' cells and alive bits from the walk's registers)
      if (CW ? !((oal >> j) & 1u) : !COLB(c.alive0, opp0 + j)) continue;
      const uint32_t pj = CW ? pp[j] : COLW(c.pos_cur, opp0 + j);
      const int ddx = pos_x(pj) - fxi, ddy = pos_y(pj) - fyi;
      if (ddx * ddx + ddy * ddy < 4) {
        tl[(size_t)tn * E] = (uint16_t)(fxi | (fyi << 8));
        tn++;
      }
    }
  }
  COLW(c.tcnt, me) = (uint32_t)tn;
  prof_acc(S, 23, tq);
}

// Default pair walk (step_kernel CW = false). Compile-time ship counts: positions and alive flags of both sides are read
// into registers once, the 16 (4v4) distance tests run branch-free, and only
// pairs inside a sensor range are walked. The walk (pass 1) is integer work: the
// observed list and which pairs yield an EW bearing; the floating-point part —
// bearings, gauss draws, tangents and fixes — runs afterwards (finish_obs_t),
// only for opponents with the two bearings a fix needs. (Keeping the walk's
// operands in registers instead of LDS measured slower: the kernel is at 256
// VGPRs and the extra arrays spill to scratch.)
template <int NOWN, int NOPP>
__device__ __forceinline__ void get_obs_walk_t(Ctx &X, int me, int own0, int opp0) {
  Cols &c = X.c;
  const int lane = X.lane;
  const int myradar = COLW(c.radar_cur, me);
  int xo[NOWN], yo[NOWN];
  int xp[NOPP], yp[NOPP];
  uint32_t amask = 0;
#pragma unroll
  for (int i = 0; i < NOWN; i++) {
    uint32_t p = COLW(c.pos_cur, own0 + i);
    xo[i] = pos_x(p); yo[i] = pos_y(p);
    amask |= (COLB(c.alive0, own0 + i) ? 1u : 0u) << i;
  }
#pragma unroll
  for (int j = 0; j < NOPP; j++) {
    uint32_t p = COLW(c.pos_cur, opp0 + j);
    xp[j] = pos_x(p); yp[j] = pos_y(p);
    amask |= (COLB(c.alive0, opp0 + j) ? 1u : 0u) << (NOWN + j);
  }
  uint32_t near = 0;  // bit i*NOPP+j: both alive and within the max sensor range
#pragma unroll
  for (int i = 0; i < NOWN; i++)
#pragma unroll
    for (int j = 0; j < NOPP; j++) {
      int dx = xp[j] - xo[i], dy = yp[j] - yo[i];
      bool in = ((amask >> i) & (amask >> (NOWN + j)) & 1u) && dx * dx + dy * dy < X.r2max;
      near |= (in ? 1u : 0u) << (i * NOPP + j);
    }
  ObsAcc acc{0, 0};
  const unsigned long long tw = prof_now(X.S);
  const uint64_t lbits = X.lpre[own0 != 0];
  uint32_t bearm = 0;  // bit i*NOPP+j: pair (i, j) yields a bearing (one gauss draw)
  while (near) {  // pairs in index order (i outer, j inner), as the reference loops
    int b = __builtin_ctz(near);
    near &= near - 1;
    int i = b / NOPP, j = b - (b / NOPP) * NOPP;
    uint32_t pi = COLW(c.pos_cur, own0 + i), pj = COLW(c.pos_cur, opp0 + j);
    int xi = pos_x(pi), yi = pos_y(pi), xj = pos_x(pj), yj = pos_y(pj);
    int dx = xj - xi, dy = yj - yi;
    const int d2 = dx * dx + dy * dy;
    const int ti = COLB(c.type, own0 + i), tj = COLB(c.type, opp0 + j);
    const int rr = radar_r(X.P, X.duct(), ti, tj), re = ew_r(X.P, X.duct(), ti, tj);
    const bool rad_ok = myradar == 1 && d2 < rr * rr, close = d2 < 16;
    const bool ew_cand = d2 < re * re && COLW(c.radar_cur, opp0 + j) == 1;
    if (!(rad_ok || close || ew_cand)) continue;  // LOS result would be unused
    uint32_t los;
    if (X.pre) {
      // own ship i stands on its new cell once its turn has come and it moved
      const int v = (own0 + i <= me) && (COLW(c.pos_new, own0 + i) & 0x80000000u) ? 1 : 0;
      los = (uint32_t)(lbits >> (((i * NOPP + j) * 2 + v) * 2)) & 3u;
    } else {
      los = los_q(X.P, X.S, X.mask, xi, yi, xj, yj);
    }
    if (pair_observe(X, xj, yj, rad_ok, close, ew_cand, los, acc)) bearm |= 1u << b;
  }
  prof_acc(X.S, 20, tw);
  const uint32_t nopp[NOPP] = {};
  finish_obs_t<NOWN, NOPP, false>(X, me, own0, opp0, acc.obs_n, 0u, bearm, nopp);
}

// Contact variant (step_kernel CW = true, lnw_set_variant): the pair walk of
// get_obs (combatant.py:106-124) as
// bit masks. Positions, types, alive flags and the opponents' radar states are
// read into registers once; every (own i, opponent j) pair's conditions are
// evaluated independently (LOS bits from los_prefetch_t), giving
//   D  = pairs that detect (radar or close, radar LOS clear),
//   EW = pairs that are EW candidates with radar and EW LOS clear.
// The reference walks pairs in index order (i outer, j inner) appending each
// detected opponent's cell to `observed` unless a cell-mate is already there,
// and takes a bearing when an EW pair's opponent cell is not yet observed
// (after the pair's own append). With f = the first D pair over the opponents
// sharing j's cell, the observed list is the set of those f in increasing
// order, and pair b of column j yields a bearing iff b is in EW and b < f.
// Bearings, gauss draws and fixes then run in finish_obs_t.
template <int NOWN, int NOPP>
__device__ __forceinline__ void mask_walk_t(Ctx &X, int me, int own0, int opp0, uint32_t (&pp)[NOPP],
                                            uint32_t &amask, uint32_t &firstbit, uint32_t &bearm,
                                            bool radv_set = false, int radv = 0) {
  static_assert(NOWN * NOPP <= 16, "pair masks are 16 bits");
  Cols &c = X.c;
  const int lane = X.lane;
  // (radv: the observer's radar as take_action sets it, for a walk counted ahead of its turn)
  const int myradar = radv_set ? radv : COLW(c.radar_cur, me);
  uint32_t rowsel = 0;
  amask = 0;
#pragma unroll
  for (int i = 0; i < NOWN; i++) {
    // own ship i stands on its new cell once its turn has come and it moved
    const bool nw = (own0 + i <= me) && (COLW(c.pos_new, own0 + i) & 0x80000000u);
    rowsel |= nw ? ((1u << NOPP) - 1u) << (i * NOPP) : 0u;
  }
#pragma unroll
  for (int j = 0; j < NOPP; j++) {
    pp[j] = COLW(c.pos_cur, opp0 + j);
    amask |= (COLB(c.alive0, opp0 + j) ? 1u : 0u) << (NOWN + j);
  }
  const unsigned long long tw = prof_now(X.S);
  // the pair tables of this side (pair_tables_t), each pair on the cell its own ship stands on now
  const int sd = own0 != 0;
  auto sel = [&](uint32_t b) { return (b & 0xffffu & ~rowsel) | ((b >> 16) & rowsel); };
  const uint32_t detm = sel(sd ? X.ptc[1] : X.ptc[0]) | (myradar == 1 ? sel(sd ? X.ptr_[1] : X.ptr_[0]) : 0u);
  const uint32_t ewm = sel(sd ? X.ptw[1] : X.ptw[0]);
  uint32_t colj = 0;  // bits of opponent 0's column
#pragma unroll
  for (int i = 0; i < NOWN; i++) colj |= 1u << (i * NOPP);
  firstbit = 0;  // bit b: pair b appends to observed / takes a bearing
  bearm = 0;
#pragma unroll
  for (int j = 0; j < NOPP; j++) {
    uint32_t cls = 0;  // columns of the opponents on j's cell (observed is de-duplicated by cell)
#pragma unroll
    for (int k = 0; k < NOPP; k++) cls |= pp[k] == pp[j] ? colj << k : 0u;
    const uint32_t dc = detm & cls;
    const uint32_t f = dc ? 1u << __builtin_ctz(dc) : 0u;
    firstbit |= f;
    bearm |= ewm & (colj << j) & (f ? f - 1u : 0xffffffffu);
  }
  prof_acc(X.S, 20, tw);
}

template <int NOWN, int NOPP>
__device__ __forceinline__ void get_obs_mask_t(Ctx &X, int me, int own0, int opp0) {
  uint32_t pp[NOPP], amask, firstbit, bearm;
  mask_walk_t<NOWN, NOPP>(X, me, own0, opp0, pp, amask, firstbit, bearm);
  finish_obs_t<NOWN, NOPP, true>(X, me, own0, opp0, 0, firstbit, bearm, pp, amask >> NOWN);
}

// get_obs for compile-time ship counts: CW selects the contact variant
template <int NOWN, int NOPP, bool CW>
__device__ __forceinline__ void get_obs_t(Ctx &X, int me, int own0, int opp0) {
  if constexpr (CW) get_obs_mask_t<NOWN, NOPP>(X, me, own0, opp0);
  else get_obs_walk_t<NOWN, NOPP>(X, me, own0, opp0);
}

// Every LOS query get_obs can make during this step's agent loop, loaded in one
// batch before it (the loop otherwise waits on one table load per pair). While
// blue plays, red ships stand on their old cells and blue ship i on its new cell
// once its turn has come (i <= me) and it moved; while red plays, blue ships stand
// on their final cells. So blue->red rays need blue old/new x red
// old, and red->blue rays red old/new x blue final: 2 * NB * NR * 2 rays at most,
// fewer when pairs are out of every sensor range or a ship kept its cell.
template <int NB, int NR>
__device__ inline void los_prefetch_t(Ctx &X) {
  const KParams &P = X.P;
  const KState &S = X.S;
  Cols &c = X.c;
  const int lane = X.lane;
  constexpr int NPAIR = NB * NR;
  static_assert(NPAIR * 4 <= 64, "LOS prefetch bits exceed 64 per side");
  int bo[NB], bn[NB], ro[NR], rn[NR];  // packed x<<8|y cells: old, final
  uint32_t bmv = 0, rmv = 0, al = 0;
#pragma unroll
  for (int i = 0; i < NB; i++) {
    const uint32_t po = COLW(c.pos_cur, i), pn = COLW(c.pos_new, i);
    const bool mv = (pn & 0x80000000u) != 0;
    bo[i] = pos_x(po) << 8 | pos_y(po);
    bn[i] = mv ? (pos_x(pn & 0x7fffffffu) << 8 | pos_y(pn & 0x7fffffffu)) : bo[i];
    bmv |= (mv ? 1u : 0u) << i;
    al |= (COLB(c.alive0, i) ? 1u : 0u) << i;
  }
#pragma unroll
  for (int j = 0; j < NR; j++) {
    const uint32_t po = COLW(c.pos_cur, NB + j), pn = COLW(c.pos_new, NB + j);
    const bool mv = (pn & 0x80000000u) != 0;
    ro[j] = pos_x(po) << 8 | pos_y(po);
    rn[j] = mv ? (pos_x(pn & 0x7fffffffu) << 8 | pos_y(pn & 0x7fffffffu)) : ro[j];
    rmv |= (mv ? 1u : 0u) << j;
    al |= (COLB(c.alive0, NB + j) ? 1u : 0u) << (NB + j);
  }
  // ray r: side s = r / (2*NPAIR); within a side, ((own*NOPP + opp)*2 + v)
  auto ray = [&](int r, int &x1, int &y1, int &x2, int &y2, bool &need) {
    const int s = r / (2 * NPAIR), q = r % (2 * NPAIR), v = q & 1, p = q >> 1;
    int o, d;
    if (s == 0) {
      const int i = p / NR, j = p % NR;
      o = v ? bn[i] : bo[i];
      d = ro[j];
      need = ((al >> i) & (al >> (NB + j)) & 1u) && (v == 0 || ((bmv >> i) & 1u));
    } else {
      const int j = p / NB, i = p % NB;
      o = v ? rn[j] : ro[j];
      d = bn[i];
      need = ((al >> i) & (al >> (NB + j)) & 1u) && (v == 0 || ((rmv >> j) & 1u));
    }
    x1 = o >> 8; y1 = o & 255; x2 = d >> 8; y2 = d & 255;
    const int dx = x2 - x1, dy = y2 - y1;
    need = need && dx * dx + dy * dy < X.r2max;
  };
  uint64_t bits[2] = {0, 0};
  constexpr int NRAY = 4 * NPAIR;
  constexpr int CH = 16;
#pragma unroll
  for (int r0 = 0; r0 < NRAY; r0 += CH) {
    uint32_t wi[CH], tabm = 0, marchm = 0;
#pragma unroll
    for (int u = 0; u < CH; u++) {
      wi[u] = 0;
      if (r0 + u >= NRAY) continue;
      int x1, y1, x2, y2;
      bool need;
      ray(r0 + u, x1, y1, x2, y2, need);
      const int dx = x2 - x1, dy = y2 - y1;
      const bool tab = dx >= -R_LOS && dx <= R_LOS && dy >= -R_LOS && dy <= R_LOS;
      tabm |= (need && tab ? 1u : 0u) << u;
      marchm |= (need && !tab ? 1u : 0u) << u;
      wi[u] = ((uint32_t)(x1 * P.G + y1) * LOS_CELL_WORDS + (dx + R_LOS) * LOS_ROW_WORDS) * 32u +
              (dy + R_LOS) * 2;
    }
#pragma unroll
    for (int u = 0; u < CH; u++) {
      if (r0 + u >= NRAY) continue;
      const uint32_t w = (tabm >> u) & 1u ? S.lostab[wi[u] >> 5] : 0u;
      const int r = r0 + u, s = r / (2 * NPAIR), q = r % (2 * NPAIR);
      bits[s] |= (uint64_t)((w >> (wi[u] & 31)) & 3u) << (2 * q);
    }
    while (marchm) {  // outside the table window (very long sensor ranges)
      const int u = __builtin_ctz(marchm);
      marchm &= marchm - 1;
      // the ray's cells again from the LDS columns: a runtime index into the
      // register arrays above would put them in scratch for the whole function
      const int r = r0 + u, s = r / (2 * NPAIR), q = r % (2 * NPAIR), v = q & 1, p = q >> 1;
      const int o = s == 0 ? p / NR : NB + p / NB, d = s == 0 ? NB + p % NR : p % NB;
      const uint32_t pn = COLW(c.pos_new, o);
      const uint32_t po = v && (pn & 0x80000000u) ? (pn & 0x7fffffffu) : COLW(c.pos_cur, o);
      uint32_t pd = COLW(c.pos_cur, d);
      if (s == 1) {  // red -> blue rays end at the blue ship's final cell
        const uint32_t qn = COLW(c.pos_new, d);
        if (qn & 0x80000000u) pd = qn & 0x7fffffffu;
      }
      bits[s] |= (uint64_t)los_march_c(X.S, X.mask, P.W16, pos_x(po), pos_y(po), pos_x(pd), pos_y(pd))
                 << (2 * q);
    }
  }
  X.lpre[0] = bits[0];
  X.lpre[1] = bits[1];
  X.pre = true;
}

// Contact variant: every pair condition get_obs can ask for during this step's
// agent loop, evaluated once before it (the pair tables, Ctx::ptr_/ptc/ptw).
// Besides the cells (as los_prefetch_t: blue old/new x red old while blue
// plays, red old/new x blue final while red plays), the rest is fixed for the
// step too: types, ducting, alive flags (hits sink ships only in the tail) and
// the opponents' radar states (red's before the step; blue's as take_action
// sets it, rint(a0) or 0). Only the observer's own radar (radar-detect needs
// it on) and the turn order (which own cell) are applied in get_obs_mask_t.
// STEP = false (observe kernel): no ship moves and every radar is current.
template <int NB, int NR, bool STEP>
__device__ inline void pair_tables_t(Ctx &X) {
  const KParams &P = X.P;
  const KState &S = X.S;
  Cols &c = X.c;
  const int lane = X.lane;
  constexpr int NPAIR = NB * NR;
  static_assert(NPAIR <= 16, "pair tables are 16 bits per cell version");
  const double duct = X.duct();
  int bo[NB], bn[NB], ro[NR], rn[NR];  // packed x<<8|y cells: old, final
  uint32_t bmv = 0, rmv = 0, al = 0, tb = 0, tr = 0, radr = 0, radb = 0;
#pragma unroll
  for (int i = 0; i < NB; i++) {
    const uint32_t po = COLW(c.pos_cur, i), pn = COLW(c.pos_new, i);
    const bool mv = STEP && (pn & 0x80000000u) != 0;
    bo[i] = pos_x(po) << 8 | pos_y(po);
    bn[i] = mv ? (pos_x(pn & 0x7fffffffu) << 8 | pos_y(pn & 0x7fffffffu)) : bo[i];
    bmv |= (mv ? 1u : 0u) << i;
    al |= (COLB(c.alive0, i) ? 1u : 0u) << i;
    tb |= (uint32_t)COLB(c.type, i) << (2 * i);
    int rb;
    if constexpr (STEP) {  // blue's radar once it has acted (take_action)
      const double a0 = COLW(c.act0, i);
      rb = isfinite(a0) ? (int)fmin(fmax(rint(a0), -2147483648.0), 2147483647.0) : 0;
    } else {
      rb = COLW(c.radar_cur, i);
    }
    radb |= (rb == 1 ? 1u : 0u) << i;
  }
#pragma unroll
  for (int j = 0; j < NR; j++) {
    const uint32_t po = COLW(c.pos_cur, NB + j), pn = COLW(c.pos_new, NB + j);
    const bool mv = STEP && (pn & 0x80000000u) != 0;
    ro[j] = pos_x(po) << 8 | pos_y(po);
    rn[j] = mv ? (pos_x(pn & 0x7fffffffu) << 8 | pos_y(pn & 0x7fffffffu)) : ro[j];
    rmv |= (mv ? 1u : 0u) << j;
    al |= (COLB(c.alive0, NB + j) ? 1u : 0u) << (NB + j);
    tr |= (uint32_t)COLB(c.type, NB + j) << (2 * j);
    radr |= (COLW(c.radar_cur, NB + j) == 1 ? 1u : 0u) << j;  // red's radar before the step
  }
  // ray r: side s = r / (2*NPAIR); within a side q = (own*NOPP + opp)*2 + v.
  // The pair's ranges (rr2, re2) are computed on its v = 0 ray and reused by its
  // v = 1 ray (the next one: chunks hold whole pairs)
  int rr2 = 0, re2 = 0;
  auto ray = [&](int r, int &x1, int &y1, int &x2, int &y2, uint32_t &f) {
    const int s = r / (2 * NPAIR), q = r % (2 * NPAIR), v = q & 1, p = q >> 1;
    int o, d, ti, tj;
    bool need, radj;
    if (s == 0) {
      const int i = p / NR, j = p % NR;
      o = v ? bn[i] : bo[i];
      d = ro[j];
      need = ((al >> i) & (al >> (NB + j)) & 1u) && (v == 0 || ((bmv >> i) & 1u));
      ti = (tb >> (2 * i)) & 3u;
      tj = (tr >> (2 * j)) & 3u;
      radj = (radr >> j) & 1u;
    } else {
      const int j = p / NB, i = p % NB;
      o = v ? rn[j] : ro[j];
      d = bn[i];
      need = ((al >> i) & (al >> (NB + j)) & 1u) && (v == 0 || ((rmv >> j) & 1u));
      ti = (tr >> (2 * j)) & 3u;
      tj = (tb >> (2 * i)) & 3u;
      radj = (radb >> i) & 1u;
    }
    x1 = o >> 8; y1 = o & 255; x2 = d >> 8; y2 = d & 255;
    const int dx = x2 - x1, dy = y2 - y1, d2 = dx * dx + dy * dy;
    if (v == 0) {
      const int rr = radar_r(P, duct, ti, tj), re = ew_r(P, duct, ti, tj);
      rr2 = rr * rr;
      re2 = re * re;
    }
    f = 0;
    if (need && d2 < X.r2max)
      f = (d2 < rr2 ? 1u : 0u) | (d2 < 16 ? 2u : 0u) | (d2 < re2 && radj ? 4u : 0u);
  };
  uint32_t tR[2] = {0u, 0u}, tC[2] = {0u, 0u}, tW[2] = {0u, 0u};
  constexpr int NRAY = 4 * NPAIR;
  constexpr int CH = 16;
#pragma unroll
  for (int r0 = 0; r0 < NRAY; r0 += CH) {
    uint32_t wi[CH], tabm = 0, marchm = 0;
    uint64_t fl = 0;  // 3 range bits per ray of the chunk
#pragma unroll
    for (int u = 0; u < CH; u++) {
      wi[u] = 0;
      if (r0 + u >= NRAY) continue;
      int x1, y1, x2, y2;
      uint32_t f;
      ray(r0 + u, x1, y1, x2, y2, f);
      fl |= (uint64_t)f << (3 * u);
      const int dx = x2 - x1, dy = y2 - y1;
      const bool tab = P.los_mode != 1 && dx >= -R_LOS && dx <= R_LOS && dy >= -R_LOS && dy <= R_LOS;
      tabm |= (f && tab ? 1u : 0u) << u;
      marchm |= (f && !tab ? 1u : 0u) << u;
      wi[u] = ((uint32_t)(x1 * P.G + y1) * LOS_CELL_WORDS + (dx + R_LOS) * LOS_ROW_WORDS) * 32u +
              (dy + R_LOS) * 2;
    }
    uint64_t lb = 0;  // 2 LOS bits per ray of the chunk
#pragma unroll
    for (int u = 0; u < CH; u++) {
      if (r0 + u >= NRAY) continue;
      const uint32_t w = (tabm >> u) & 1u ? S.lostab[wi[u] >> 5] : 0u;
      lb |= (uint64_t)((w >> (wi[u] & 31)) & 3u) << (2 * u);
    }
    while (marchm) {  // outside the table window (very long sensor ranges), or march mode
      const int u = __builtin_ctz(marchm);
      marchm &= marchm - 1;
      // the ray's cells again from the LDS columns: a runtime index into the
      // register arrays above would put them in scratch for the whole function
      const int r = r0 + u, s = r / (2 * NPAIR), q = r % (2 * NPAIR), v = q & 1, p = q >> 1;
      const int o = s == 0 ? p / NR : NB + p / NB, d = s == 0 ? NB + p % NR : p % NB;
      const uint32_t pn = COLW(c.pos_new, o);
      const uint32_t po = STEP && v && (pn & 0x80000000u) ? (pn & 0x7fffffffu) : COLW(c.pos_cur, o);
      uint32_t pd = COLW(c.pos_cur, d);
      if (STEP && s == 1) {  // red -> blue rays end at the blue ship's final cell
        const uint32_t qn = COLW(c.pos_new, d);
        if (qn & 0x80000000u) pd = qn & 0x7fffffffu;
      }
      lb |= (uint64_t)los_march_c(X.S, X.mask, P.W16, pos_x(po), pos_y(po), pos_x(pd), pos_y(pd)) << (2 * u);
    }
#pragma unroll
    for (int u = 0; u < CH; u++) {
      if (r0 + u >= NRAY) continue;
      const int r = r0 + u, s = r / (2 * NPAIR), q = r % (2 * NPAIR);
      const uint32_t f = (uint32_t)(fl >> (3 * u)) & 7u, l = (uint32_t)(lb >> (2 * u)) & 3u;
      const int bit = (q & 1) * 16 + (q >> 1);
      tR[s] |= ((f & 1u) && (l & 1u) ? 1u : 0u) << bit;
      tC[s] |= ((f & 2u) && (l & 1u) ? 1u : 0u) << bit;
      tW[s] |= ((f & 4u) && l == 3u ? 1u : 0u) << bit;
    }
  }
  X.ptr_[0] = tR[0]; X.ptr_[1] = tR[1];
  X.ptc[0] = tC[0]; X.ptc[1] = tC[1];
  X.ptw[0] = tW[0]; X.ptw[1] = tW[1];
  X.pre = true;
}

// check_target (combatant.py:570-584): first live opponent within 3.5 cells
template <bool GRP = false>
__device__ inline int check_target_dev(Ctx &X, int side, int tx, int ty) {
  const KParams &P = X.P;
  Cols &c = X.c;
  const int lane = X.lane;
  int opp0 = side ? 0 : P.nb, opp1 = side ? P.nb : P.A;
  if constexpr (GRP) {  // lane gsub of the env's group tests opponent opp0 + gsub; the first one found
    const int j = opp0 + X.gsub;
    bool hit = false;
    if (j < opp1 && COLB(c.alive0, j)) {
      const uint32_t pj = COLW(c.pos_cur, j);
      const int dx = pos_x(pj) - tx, dy = pos_y(pj) - ty;
      hit = dx * dx + dy * dy <= 12;
    }
    const uint32_t m = (uint32_t)(__ballot(hit) >> X.gsh) & 0xffffu;
    return m ? opp0 + __builtin_ctz(m) : -1;
  }
  for (int j = opp0; j < opp1; j++) {
    if (!COLB(c.alive0, j)) continue;
    uint32_t pj = COLW(c.pos_cur, j);
    int dx = pos_x(pj) - tx, dy = pos_y(pj) - ty;
    if (dx * dx + dy * dy <= 12) return j;
  }
  return -1;
}

struct Neut {
  int cnt[2];
  uint32_t mask[2];
};

// fire_missile (combatant.py:587-668) — returns hit
template <bool GRP = false>
__device__ inline bool fire_dev(Ctx &X, int a, int tx, int ty, double salvo, int ksalvo, Neut &N) {
  const KParams &P = X.P;
  Cols &c = X.c;
  const int lane = X.lane;
  const int side = a >= P.nb;
  int t = check_target_dev<GRP>(X, side, tx, ty);
  if (t < 0) return false;
  uint32_t pt = COLW(c.pos_cur, t), pa = COLW(c.pos_cur, a);
  int dx = pos_x(pt) - pos_x(pa), dy = pos_y(pt) - pos_y(pa);
  bool hit = false, missile = false;
  int n = 0;  // missiles fired (0: main gun)
  if (dx * dx + dy * dy < 4) {
    hit = true;  // main gun, no draw
  } else {
    int miss = COLB(c.miss_cur, a);
    if (miss == 0) return false;
    int mk = COLB(c.mkind, a);
    double u1, u2;  // the detection draw, then the hit draw (combatant.py:612, 630)
    X.rng.uniform2(u1, u2);
    bool detected = !(u1 < (COLW(c.radar_cur, t) == 1 ? P.det_q[0] : P.det_q[1]));
    int hp = detected ? 0 : 1;
    double num;
    int kn;
    if (!P.discrete) {
      int kp = kind_promote(mk, ksalvo);
      if (kp == K_F32) {
        num = (double)rintf((float)miss * (float)salvo);
        kn = K_F32;
      } else {
        num = rint((double)miss * salvo);
        kn = K_F64;  // np.round -> np.float64
      }
    } else {
      num = COLB(c.type, a) == T_SMALL ? salvo : salvo * 2.0;
      kn = K_PYINT;
    }
    if (num > (double)miss) { num = (double)miss; kn = mk; }
    n = (int)num;
    COLB(c.miss_cur, a) = (uint8_t)(miss - n);
    COLB(c.mkind, a) = (uint8_t)kind_promote(mk, kn);
    if (n < 0 || n > 8) { X.rng.err |= LNW_ERRF_MISSILES; n = n < 0 ? 0 : 8; }
    if (kn == K_F32)
      hit = (float)u2 < hit_sel(P.hit32, hp, n);
    else
      hit = u2 < hit_sel(P.hit64, hp, n);
    missile = true;
  }
  if (hit && X.leader) {
    const KState &S = X.S;
    if (missile) {  // combatant.py:642-652: maps of the trained side, launch sites of both
      if (side == (P.side_blue ? 0 : 1)) {
        ana_map(S.ana.heatmap, pa);
        ana_map(S.ana.coldmap, pt);
      }
      if (S.ana.launch) ana_map(S.ana.launch + side * 10000, pa);
    }
    if (S.ana.eng_log)  // combatant.py:656-657
      ana_record(S.ana.eng_log, S.ana.eng_count, S.ana.eng_cap, (uint32_t)(P.env_base + X.env),
                 (uint32_t)X.step | (uint32_t)side << 16 | (uint32_t)n << 24, pa, pt);
  }
  if (hit) {
    int ts = t >= P.nb;
    N.cnt[ts]++;
    N.mask[ts] |= 1u << (t - (ts ? P.nb : 0));
  }
  return hit;
}

// The draws take_action's fire loop over ship a's previous target list takes
// (fire_dev without its draws: two per missile shot, combatant.py:612, 630),
// counted ahead of the turn: the targets are found among the opponents' start
// cells and alive flags, and the missile count runs its recurrence.
__device__ inline int fire_draws(Ctx &X, int a, double salvo, int ksalvo) {
  const KParams &P = X.P;
  Cols &c = X.c;
  const int lane = X.lane;
  const int side = a >= P.nb;
  const int tn = (int)COLW(c.tcnt, a);
  int miss = COLB(c.miss_cur, a), mk = COLB(c.mkind, a), nd = 0;
  const uint16_t *tl = X.S.tl + (size_t)a * P.T * X.E + X.env;
  const uint32_t pa = COLW(c.pos_cur, a);
  for (int q = 0; q < tn; q++) {
    const uint16_t tg = tl[(size_t)q * X.E];
    const int t = check_target_dev<false>(X, side, tg & 0xff, tg >> 8);
    if (t < 0) continue;
    const uint32_t pt = COLW(c.pos_cur, t);
    const int dx = pos_x(pt) - pos_x(pa), dy = pos_y(pt) - pos_y(pa);
    if (dx * dx + dy * dy < 4 || miss == 0) continue;  // main gun, or no missiles: no draw
    double num;
    int kn;
    if (!P.discrete) {
      if (kind_promote(mk, ksalvo) == K_F32) {
        num = (double)rintf((float)miss * (float)salvo);
        kn = K_F32;
      } else {
        num = rint((double)miss * salvo);
        kn = K_F64;
      }
    } else {
      num = COLB(c.type, a) == T_SMALL ? salvo : salvo * 2.0;
      kn = K_PYINT;
    }
    if (num > (double)miss) { num = (double)miss; kn = mk; }
    miss = (miss - (int)num) & 0xff;
    mk = kind_promote(mk, kn);
    nd += 2;
  }
  return nd;
}

// calculate_reward (game.py:214-295) for agent a of the env in LDS column `lane`
// dlz: the agent-major LDS copy of dist_lz the group kernel stages in phase L
// (entry a * dlz_stride), else null (read from HBM)
__device__ __forceinline__ double reward_core(const KParams &P, const KState &S, Cols &c, int lane,
                                              long long E, int env, int a, bool moved, bool engage,
                                              int n_hit, const double *dlz = nullptr, int dlz_stride = 0) {
  size_t ai = (size_t)a * E + env;
  int steps = COLW(c.steps, a) + 1;
  COLW(c.steps, a) = steps;
  int tl_n = (int)COLW(c.tcnt, a);
  double r = 0.0;
  if (tl_n > 0) r += (double)(tl_n * 3);
  if (moved) r += 1.0;
  else r = fmax(r - 0.5, 0.0);
  if (tl_n > 0 && !engage) r = r / 2.0;
  else if (tl_n > 0 && engage && n_hit == 0) r += 0.5;
  r += (double)(n_hit * 10);
  int t = COLB(c.type, a);
  uint32_t p = COLW(c.pos_cur, a);
  int x = pos_x(p), y = pos_y(p);
  bool red = a >= P.nb;
  if (red && t != T_LS && !P.aggressive) {
    if (steps > 14) {
      if (x < 19 || x > 55 || y < 40 || y > 70) r = fmax(r - 2.0, 0.0);
      else r += 1.0;
    }
  }
  if (red && P.aggressive && t != T_LS) {
    int dx = x - 15, dy = y - 60;
    double nom = fmax(sqrt((double)(dx * dx + dy * dy)), 1.0);
    double d = (1.0 / (nom / (mast_cls(t) ? P.den[1] : P.den[0]))) * 1.0;
    r += d;
  }
  if (t == T_LS) {
    int dx = x - P.lz_x, dy = y - P.lz_y;
    double dl = sqrt((double)(dx * dx + dy * dy));
    if (dl > 0) {
      double cur = (P.dbg_skip & 2097152) ? 1e9 : (dlz ? dlz[a * dlz_stride] : S.dist_lz[ai]);  // (bit 21: diagnostics)
      if (dl < cur) { r += 1.0; S.dist_lz[ai] = dl; }
      else r -= 1.0;
    } else {
      r += 100.0;
    }
    if (dl == 0) r += 100.0;
    else r += log10(100.0 / dl) * 5.0;
  }
  return r;
}

__device__ inline double reward_dev(Ctx &X, int a, bool moved, bool engage, int n_hit) {
  return reward_core(X.P, X.S, X.c, X.lane, X.E, X.env, a, moved, engage, n_hit);
}

// Game.reset for one env (game.py:528-613), in-kernel
__device__ __forceinline__ void reset_env_dev(const KParams &P, const KState &S, int env, Rng &rng) {
  const long long E = P.E;
  double duct = 1.0 + rng.beta13();
  S.duct[env] = duct;
  // optional "box" spawn stream (build-side melee scenario)
  bool box = P.box_hi[0] > P.box_lo[0] && P.box_hi[1] > P.box_lo[1];
  unsigned long long box_ctr = ((unsigned long long)(uint32_t)S.envi[7 * E + env]) << 32;
  for (int a = 0; a < P.A; a++) {
    size_t ai = (size_t)a * E + env;
    int t = S.sp_types[a];
    int x, y;
    if (S.sp_pos_env) {
      x = S.sp_pos_env[((size_t)env * P.A + a) * 2];
      y = S.sp_pos_env[((size_t)env * P.A + a) * 2 + 1];
    } else {
      x = S.sp_pos[2 * a];
      y = S.sp_pos[2 * a + 1];
    }
    if (box) {
      for (int tries = 0; tries < 64; tries++) {
        uint32_t o[4];
        o[0] = (uint32_t)box_ctr;
        o[1] = (uint32_t)(box_ctr >> 32);
        o[2] = rng.g0;
        o[3] = rng.g1 ^ 0x80000000u;
        philox10(o, rng.k0 ^ 0x5bd1e995u, rng.k1);
        box_ctr++;
        int bx = P.box_lo[0] + (int)(o[0] % (uint32_t)(P.box_hi[0] - P.box_lo[0]));
        int by = P.box_lo[1] + (int)(o[1] % (uint32_t)(P.box_hi[1] - P.box_lo[1]));
        if (!(cell_bits(S.mask2, P.W16, bx, by) & 1u)) { x = bx; y = by; break; }
      }
    }
    if (S.sp_randls[a]) {
      x = rng.randint(98, 99);
      y = rng.randint(48, 56);
    }
    S.pos[ai] = pack_pos(x, y);
    S.radar[ai] = 1;
    S.miss[ai] = (uint8_t)missiles0(t);
    S.mkind[ai] = K_PYINT;
    S.alive[ai] = 1;
    S.type[ai] = (uint8_t)t;
    S.steps[ai] = 0;
    S.tl_cnt[ai] = 0;
    double dl = 0.0;
    if (t == T_LS) {
      int dx = x - P.lz_x, dy = y - P.lz_y;
      dl = sqrt((double)(dx * dx + dy * dy));
    }
    S.dist_lz[ai] = dl;
  }
  S.envi[0 * E + env] = P.nb;
  S.envi[1 * E + env] = P.nr;
  S.envi[2 * E + env] = 0;
  S.envi[3 * E + env] = 0;
  S.envi[4 * E + env] = 0;
  S.envi[7 * E + env] = S.envi[7 * E + env] + 1;
}

__device__ inline Rng make_rng(const KParams &P, const KState &S, int env) {
  Rng r;
  r.mode = P.rng_mode;
  r.k0 = (uint32_t)P.seed;
  r.k1 = (uint32_t)(P.seed >> 32);
  unsigned long long gid = (unsigned long long)(P.env_base + env);
  r.g0 = (uint32_t)gid;
  r.g1 = (uint32_t)(gid >> 32);
  r.ctr = S.rng[env];
  r.err = 0;
  r.tape = S.tape;
  if (P.rng_mode == 1 && S.tape_off) {
    r.tape_lo = S.tape_off[env];
    r.tape_hi = S.tape_off[env + 1];
  } else {
    r.tape_lo = r.tape_hi = 0;
  }
  return r;
}

// ---------------------------------------------------------------------------
// phase O: observation vectors (combatant.py:163-233, landingship.py:167-239)
// One lane per (env, agent) row builds its D floats into a padded LDS row; the
// wave then copies each side's block ([envs][n][D], contiguous in the output)
// out with consecutive lanes on consecutive floats (256-B coalesced stores).
// ---------------------------------------------------------------------------
// Builds one observation row of D floats into an LDS row (stride D+1: odd, so
// a ds_write_b32 across lanes is conflict-free). The terrain window comes from
// the per-cell window table (Combatant 49 floats padded to 52, LandingShip 25
// padded to 28): 13 / 7 independent float4 loads issued together.
__device__ __forceinline__ void build_row(const KParams &P, const KState &S, const Cols &c, const double *duct_col,
                          int el, int k, float *row, const float *xg, bool only_observed) {
  const int side = k >= P.nb;
  const int own0 = side ? P.nb : 0;
  const int ns = side ? P.nr : P.nb;
  const int kl = k - own0;
  const int D = side_D(P, side);
  const int G = P.G;
  if (!c.alive0[k * PADB + el] || (only_observed && !c.obsd[k * PADB + el])) {
    for (int d = 0; d < D; d++) row[d] = 0.0f;
    return;
  }
  const int tk = c.type[k * PADB + el];
  const uint32_t p = c.pos_cur[k * PAD + el];
  const int px = pos_x(p), py = pos_y(p);
  int idx;
  if (tk == T_LS || tk == T_MEDIUM) {
    // 5x5 windows: LandingShip rows/cols pos-1..pos+3 (landingship.py:178-188),
    // medium Combatant pos-2..pos+2 (combatant.py:165-181 at speed 2)
    const f32x4 *w = (const f32x4 *)(S.winf + ((size_t)win_cls(tk) * G * G + (size_t)(px * G + py)) * 52);
    f32x4 v[7];
#pragma unroll
    for (int q = 0; q < 7; q++) v[q] = w[q];
    f32x4 *r4 = (f32x4 *)row;
#pragma unroll
    for (int q = 0; q < 6; q++) r4[q] = v[q];
    row[24] = v[6].x;
    idx = 25;
  } else {
    // 7x7 window around the ship (combatant.py:174-181)
    const f32x4 *w = (const f32x4 *)(S.winf + (size_t)(px * G + py) * 52);
    f32x4 v[13];
#pragma unroll
    for (int q = 0; q < 13; q++) v[q] = w[q];
    f32x4 *r4 = (f32x4 *)row;
#pragma unroll
    for (int q = 0; q < 12; q++) r4[q] = v[q];
    row[48] = v[12].x;
    idx = 49;
  }
  // missiles/4 and missiles/8 are exact in float32
  row[idx++] = xg[px];
  row[idx++] = xg[py];
  row[idx++] = (float)c.radar_cur[k * PAD + el];
  row[idx++] = (float)c.miss_cur[k * PADB + el] * (tk == T_SMALL ? 0.25f : 0.125f);
  for (int il = 0; il < ns; il++) {
    if (il == kl) continue;
    const int i = own0 + il;
    if (c.alive0[i * PADB + el]) {
      // own ships that acted before k this step show their new state
      const bool nw = il < kl;
      const uint32_t q = nw ? c.pos_cur[i * PAD + el] : c.pos_old[i * PAD + el];
      row[idx] = xg[pos_x(q)];
      row[idx + 1] = xg[pos_y(q)];
      row[idx + 2] = (float)(nw ? c.radar_cur[i * PAD + el] : c.radar_old[i * PAD + el]);
      const int m = nw ? c.miss_cur[i * PADB + el] : c.miss_old[i * PADB + el];
      row[idx + 3] = (float)m * (c.type[i * PADB + el] == T_SMALL ? 0.25f : 0.125f);
    } else {
      row[idx] = row[idx + 1] = row[idx + 2] = row[idx + 3] = 0.0f;
    }
    idx += 4;
  }
  row[idx++] = (float)c.tcnt[k * PAD + el];
  row[idx++] = tk == T_LS ? 1.0f : 0.0f;
  row[idx++] = (float)(duct_col[el] / 2.0);
  for (; idx < D; idx++) row[idx] = 0.0f;
}

// Copy one side's block [ne envs][ns rows][D] (contiguous in the output, a
// multiple of 4 floats and 16-B aligned since D = 4*ns + 52, or 4*ns + 28 for
// a side of medium ships) with each lane moving 4 consecutive floats:
// ds_read_b128 from the staged row, dwordx4 store (1 KiB per wave store
// instruction).
// stride: floats between envs' rows in out (0: packed, ns * D)
__device__ inline void copy_side(const float *stage, float *out, int ns, int D, int ne, long long genv0,
                                 long long stride = 0) {
  if (!out) return;
  const int lane = threadIdx.x & (WAVE - 1);
  const int S4 = stage_stride(ns) >> 2;
  const int D4 = D >> 2;
  const int n4 = ne * ns * D4;
  const f32x4 *st4 = (const f32x4 *)stage;
  if (stride && stride != (long long)ns * D) {
    const int per = ns * D4;  // float4 chunks per env
    for (int i = lane; i < n4; i += WAVE) {
      const int e = i / per, q = i - e * per, r = e * ns + q / D4;
      ((f32x4 *)(out + (genv0 + e) * stride))[q] = st4[r * S4 + (q - (q / D4) * D4)];
    }
    return;
  }
  f32x4 *base = (f32x4 *)(out + (size_t)genv0 * ns * D);
  int r = lane / D4, c4 = lane - r * D4;
  for (int i = lane; i < n4; i += WAVE) {
    base[i] = st4[r * S4 + c4];
    c4 += WAVE;
    while (c4 >= D4) { c4 -= D4; r++; }
  }
}

// The workgroup is a single wavefront: LDS traffic between its lanes only needs
// the wave's LDS operations to have completed (DS ops of one wave execute in
// order), not a workgroup barrier, which would also drain every outstanding
// global store (s_waitcnt vmcnt(0)) each group.
__device__ inline void wave_lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

__device__ __forceinline__ void write_obs(const KParams &P, const KState &S, Cols &c, const double *duct_col,
                          float *obs_b, float *obs_r, int env0, int nenv, bool only_observed) {
  const int lane = threadIdx.x & (WAVE - 1);
  const int A = P.A, nb = P.nb, nr = P.nr;
  const int epg = envs_per_pass(A);
  const int my_e = lane / A, my_k = lane - (lane / A) * A;
  const int side = my_k >= nb;
  const int kl = side ? my_k - nb : my_k;
  const int ns = side ? nr : nb;
  float *stage_b = c.stage;
  float *stage_r = c.stage + epg * nb * stage_stride(nb);
  float *row = (side ? stage_r : stage_b) + (my_e * ns + kl) * stage_stride(ns);
  float *xg = stage_r + epg * nr * stage_stride(nr);  // x/G (float32 of the f64 quotient)
  for (int x = lane; x < P.G; x += WAVE) xg[x] = (float)((double)x / (double)P.G);
  wave_lds_sync();
  for (int g0 = 0; g0 < nenv; g0 += epg) {
    const int ne = (nenv - g0) < epg ? (nenv - g0) : epg;
    if (my_e < ne && !(P.dbg_skip & 8))
      build_row(P, S, c, duct_col, g0 + my_e, my_k, row, xg, only_observed);
    wave_lds_sync();
    if (!(P.dbg_skip & 16)) {
      copy_side(stage_b, obs_b, nb, side_D(P, 0), ne, env0 + g0, P.obs_stride[0]);
      copy_side(stage_r, obs_r, nr, side_D(P, 1), ne, env0 + g0, P.obs_stride[1]);
    }
    // (as write_obs_t: the pass's stores complete before the next pass or the
    // end of the wave reuses their registers)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    wave_lds_sync();
  }
}

// Compile-time shapes: the copy-out is fully unrolled (the compiler then knows
// how many stores follow the prefetched window loads), and the next pass's
// window loads are issued before this pass's stores, so waiting for them never
// drains the stores (vmcnt counts loads and stores together in issue order).
// One observation row assembled in registers (same content as build_row):
// every LDS read is issued up front without branches, teammate slot s holds
// own ship s < kl ? s : s + 1 (combatant.py:190-212), and the row leaves as
// D/4 ds_write_b128. Combatant rows: window[49] | tail; LandingShip rows:
// window[25] | tail | zeros (the LS window record is zero past 25 floats).
// The row from its inputs (the own ship's cell, type, alive flag, radar,
// missiles, target count, the env's ducting; teammate slot s's cell, radar,
// missiles, type, alive flag) and the ship's window record in v / w48.
template <int NS>
__device__ __forceinline__ void row_build_t(uint32_t p, int tk, int alive, int rad, int mis, uint32_t tcn, double du,
                                   const uint32_t (&tq)[NS - 1], const int (&tr)[NS - 1], const int (&tm)[NS - 1],
                                   const int (&tt)[NS - 1], const int (&ta)[NS - 1], const f32x4 (&v)[12],
                                   float w48, float *row, const float *xg) {
  constexpr int D = 4 * NS + 52, T = 4 * NS + 3;
  float t[T];
  t[0] = xg[pos_x(p)];
  t[1] = xg[pos_y(p)];
  t[2] = (float)rad;
  t[3] = (float)mis * (tk == T_SMALL ? 0.25f : 0.125f);
#pragma unroll
  for (int s = 0; s < NS - 1; s++) {
    const float fx = xg[pos_x(tq[s])], fy = xg[pos_y(tq[s])];
    const float fm = (float)tm[s] * (tt[s] == T_SMALL ? 0.25f : 0.125f);
    t[4 + 4 * s] = ta[s] ? fx : 0.0f;
    t[5 + 4 * s] = ta[s] ? fy : 0.0f;
    t[6 + 4 * s] = ta[s] ? (float)tr[s] : 0.0f;
    t[7 + 4 * s] = ta[s] ? fm : 0.0f;
  }
  t[T - 3] = (float)tcn;
  t[T - 2] = tk == T_LS ? 1.0f : 0.0f;
  t[T - 1] = (float)(du / 2.0);
  const bool ls = tk == T_LS;
  f32x4 *r4 = (f32x4 *)row;
#pragma unroll
  for (int q = 0; q < D / 4; q++) {
    f32x4 o;
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const int j = 4 * q + u;
      const float w = j < 48 ? v[j >> 2][j & 3] : (j == 48 ? w48 : 0.0f);
      const float xc = j < 49 ? w : t[j - 49 < T ? j - 49 : 0];
      const float xl = j < 25 ? w : (j - 25 < T ? t[j - 25 < T ? j - 25 : 0] : 0.0f);
      o[u] = alive ? (ls ? xl : xc) : 0.0f;
    }
    r4[q] = o;
  }
}

template <int NS>
__device__ inline void row_regs_t(const Cols &c, const double *duct_col, int el, int k, int own0,
                                  const f32x4 (&v)[12], float w48, float *row, const float *xg) {
  const int kl = k - own0;
  uint32_t tq[NS - 1];
  int tr[NS - 1], tm[NS - 1], tt[NS - 1], ta[NS - 1];
#pragma unroll
  for (int s = 0; s < NS - 1; s++) {
    const bool nw = s < kl;  // own ships that acted before k show their new state
    const int i = own0 + (nw ? s : s + 1);
    tq[s] = (nw ? c.pos_cur : c.pos_old)[i * PAD + el];
    tr[s] = (nw ? c.radar_cur : c.radar_old)[i * PAD + el];
    tm[s] = (nw ? c.miss_cur : c.miss_old)[i * PADB + el];
    tt[s] = c.type[i * PADB + el];
    ta[s] = c.alive0[i * PADB + el];
  }
  row_build_t<NS>(c.pos_cur[k * PAD + el], c.type[k * PADB + el], c.alive0[k * PADB + el],
                  c.radar_cur[k * PAD + el], c.miss_cur[k * PADB + el], c.tcnt[k * PAD + el], duct_col[el], tq,
                  tr, tm, tt, ta, v, w48, row, xg);
}

template <int NS, int NPASS4, bool NT = true>
__device__ inline void copy_side_t(const float *stage, float *out, float *dummy, int ne,
                                   long long genv0, bool wt = false) {
  constexpr int D = 4 * NS + 52, D4 = D / 4, S4 = stage_stride(NS) / 4;
  constexpr int IT = (NPASS4 + WAVE - 1) / WAVE;
  const int lane = threadIdx.x & (WAVE - 1);
  const int n4 = ne * NS * D4;
  const f32x4 *st4 = (const f32x4 *)stage;
  f32x4 *base = (f32x4 *)(out + (size_t)genv0 * NS * D);
  f32x4 v[IT];
#pragma unroll
  for (int u = 0; u < IT; u++) {  // all LDS reads first (no per-element branch)
    int i = lane + u * WAVE;
    i = i < n4 ? i : n4 - 1;
    const int r = i / D4, c4 = i - (i / D4) * D4;
    v[u] = st4[r * S4 + c4];
  }
  __builtin_amdgcn_sched_barrier(0);
  if (wt) {
    // write-through stores (buffer_store sc1): the lines leave this XCC's L2
    // clean, so the launch does not end by writing back megabytes of dirty
    // observation lines; lanes past the block fall outside the buffer range
    // and are dropped by the hardware
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(base, 0, n4 * 16, 0x00020000);
#pragma unroll
    for (int u = 0; u < IT; u++)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i32x4_t, v[u]), rs, (lane + u * WAVE) * 16, 0,
                                             16 /* sc1 */);
    return;
  }
#pragma unroll
  for (int u = 0; u < IT; u++) {  // unconditional stores: masked-out lanes hit the sink
    const int i = lane + u * WAVE;
    f32x4 *dst = i < n4 ? base + i : (f32x4 *)dummy + lane;
    if constexpr (NT) __builtin_nontemporal_store(v[u], dst);  // streamed out, not re-read
    else *dst = v[u];
  }
}

template <int NB, int NR>
__device__ __forceinline__ void write_obs_t(const KParams &P, const KState &S, Cols &c, const double *duct_col,
                            float *obs_b, float *obs_r, int env0, int nenv) {
  static_assert(NB == NR, "templated obs rows assume equal team sizes");
  constexpr int A = NB + NR, EPG = envs_per_pass(NB + NR);
  const int lane = threadIdx.x & (WAVE - 1);
  const int my_e = lane / A, my_k = lane - (lane / A) * A;
  const int side = my_k >= NB;
  const int own0 = side ? NB : 0;
  const int kl = my_k - own0;
  const int G = P.G;
  float *stage_b = c.stage;
  float *stage_r = c.stage + EPG * NB * stage_stride(NB);
  float *row = side ? stage_r + (my_e * NR + kl) * stage_stride(NR)
                    : stage_b + (my_e * NB + kl) * stage_stride(NB);
  float *xg = stage_r + EPG * NR * stage_stride(NR);
  for (int x = lane; x < G; x += WAVE) xg[x] = (float)((double)x / (double)G);
  const f32x4 *wtab = (const f32x4 *)S.winf;
  f32x4 v[12];
  float w48;
  // 12 unconditional float4 loads + 1 float of the row's window record (a dead
  // or absent row loads cell 0's record and ignores it)
  auto prefetch = [&](int g0) {
    const int el = g0 + my_e;
    int off = 0;
    if (my_e < EPG && el < nenv) {
      const uint32_t p = c.pos_cur[my_k * PAD + el];
      off = ((c.type[my_k * PADB + el] == T_LS ? G * G : 0) + pos_x(p) * G + pos_y(p)) * 13;
    }
#pragma unroll
    for (int q = 0; q < 12; q++) v[q] = wtab[off + q];
    w48 = ((const float *)(wtab + off))[48];
  };
  prefetch(0);
  wave_lds_sync();
  for (int g0 = 0; g0 < nenv; g0 += EPG) {
    const int ne = (nenv - g0) < EPG ? (nenv - g0) : EPG;
    if (my_e < ne && !(P.dbg_skip & 8))
      row_regs_t<NB>(c, duct_col, g0 + my_e, my_k, own0, v, w48, row, xg);
    wave_lds_sync();
    if (g0 + EPG < nenv) prefetch(g0 + EPG);
    if (!(P.dbg_skip & 16)) {
      copy_side_t<NB, EPG * NB * (4 * NB + 52) / 4>(stage_b, obs_b, S.dummy, ne, env0 + g0, P.store_wt);
      copy_side_t<NR, EPG * NR * (4 * NR + 52) / 4>(stage_r, obs_r, S.dummy, ne, env0 + g0, P.store_wt);
    }
    // this pass's stores complete before the next pass reuses their data
    // registers (and before the wave ends after the last pass): without it the
    // split contact step's rows came out with float4s of other rows in about
    // one 45-step 4 096-env run in four ("The split contact step
    // with rows"); 0 in 28 with it, at ~3 us of a 177 us melee step
#if defined(LNW_DIAG)
    if (!(P.dbg_skip & (1 << 25)))  // diagnostics: bit 25 drops the wait (tools/contact_race.py)
#endif
#ifndef LNW_PROBE_NO_OBS_WAIT  // (probe builds: the shipped code without the wait, tools/contact_race.py)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
    wave_lds_sync();
  }
}

// Phase-S row emission (templated equal team sizes, full wave, LOS table
// mode): Game.step stores ship a's observation as take_action returns it
// (game.py:343-344, 380-381), so row a of all 64 envs is final right after
// agent a's turn: own state, teammates before a in their new (*_cur) and
// teammates after a in their old (*_old) state, the same content write_obs_t
// builds after the loop. Each row leaves in four chunk groups ({5,4,4,4}
// float4s) staged through estage.
// Window record of agent a at its position after phase M's move (pos_new when
// flagged, else unchanged): known before phase S reaches a, so wave 1 loads it
// one agent ahead, before the previous agent's stores.
__device__ inline int window_rec(const KParams &P, const Cols &c, int a, int el) {
  if (!c.alive0[a * PADB + el]) return 0;
  const uint32_t pn = c.pos_new[a * PAD + el];
  const uint32_t p = (pn & 0x80000000u) ? (pn & 0x7fffffffu) : c.pos_old[a * PAD + el];
  return ((c.type[a * PADB + el] == T_LS ? P.G * P.G : 0) + pos_x(p) * P.G + pos_y(p)) * 13;
}

__device__ inline void load_window(const KState &S, int off, f32x4 (&v)[12], float &w48) {
  const f32x4 *rec = (const f32x4 *)S.winf + off;
#pragma unroll
  for (int q = 0; q < 12; q++) v[q] = rec[q];
  w48 = ((const float *)rec)[48];
}

template <int NS>
__device__ __forceinline__ void emit_rows_t(const KParams &P, const KState &S, const Cols &c,
                            const double *duct_col, int a, float *obs_side, int env0,
                            f32x4 (&v)[12], float &w48) {
  constexpr int D4 = (4 * NS + 52) / 4, T = 4 * NS + 3;
  const int lane = threadIdx.x & (WAVE - 1);
  const int el = lane;
  const int own0 = a >= NS ? NS : 0, kl = a - own0;
  const int G = P.G;
  const float *xg = c.estage + WAVE * EST4 * 4;
  const uint32_t p = c.pos_cur[a * PAD + el];
  const int tk = c.type[a * PADB + el];
  const int alive = c.alive0[a * PADB + el];
  const int rad = c.radar_cur[a * PAD + el];
  const int mis = c.miss_cur[a * PADB + el];
  const uint32_t tcn = c.tcnt[a * PAD + el];
  const double du = duct_col[el];
  float t[T];
  t[0] = xg[pos_x(p)];
  t[1] = xg[pos_y(p)];
  t[2] = (float)rad;
  t[3] = (float)mis * (tk == T_SMALL ? 0.25f : 0.125f);
#pragma unroll
  for (int s = 0; s < NS - 1; s++) {
    // teammates before a: new state; after a: the old columns (wave 0 may
    // already have moved them by the time this row is emitted)
    const bool nw = s < kl;
    const int i = own0 + (nw ? s : s + 1);
    const uint32_t q = (nw ? c.pos_cur : c.pos_old)[i * PAD + el];
    const int ta = c.alive0[i * PADB + el];
    const int m = (nw ? c.miss_cur : c.miss_old)[i * PADB + el];
    const float fm = (float)m * (c.type[i * PADB + el] == T_SMALL ? 0.25f : 0.125f);
    t[4 + 4 * s] = ta ? xg[pos_x(q)] : 0.0f;
    t[5 + 4 * s] = ta ? xg[pos_y(q)] : 0.0f;
    t[6 + 4 * s] = ta ? (float)(nw ? c.radar_cur : c.radar_old)[i * PAD + el] : 0.0f;
    t[7 + 4 * s] = ta ? fm : 0.0f;
  }
  t[T - 3] = (float)tcn;
  t[T - 2] = tk == T_LS ? 1.0f : 0.0f;
  t[T - 1] = (float)(du / 2.0);
  const bool ls = tk == T_LS;
  f32x4 vc[12];
#pragma unroll
  for (int q = 0; q < 12; q++) vc[q] = v[q];
  const float wc = w48;
  if (a + 1 < 2 * NS) load_window(S, window_rec(P, c, a + 1, el), v, w48);
  f32x4 *st4 = (f32x4 *)c.estage;
  f32x4 *out4 = (f32x4 *)obs_side + ((size_t)env0 * NS + kl) * D4;
  constexpr int GB[5] = {0, 5, 9, 13, D4};
#pragma unroll
  for (int g = 0; g < 4; g++) {
    const int n = GB[g + 1] - GB[g];
#pragma unroll
    for (int u = 0; u < EST4; u++) {
      if (u >= n) break;
      const int q = GB[g] + u;
      f32x4 o;
#pragma unroll
      for (int w = 0; w < 4; w++) {
        const int j = 4 * q + w;
        const float wv = j < 48 ? vc[j >> 2][j & 3] : (j == 48 ? wc : 0.0f);
        const float xc = j < 49 ? wv : t[j - 49 < T ? j - 49 : 0];
        const float xl = j < 25 ? wv : (j - 25 < T ? t[j - 25 < T ? j - 25 : 0] : 0.0f);
        o[w] = alive ? (ls ? xl : xc) : 0.0f;
      }
      st4[lane * EST4 + u] = o;
    }
    wave_lds_sync();
    f32x4 cv[EST4];
#pragma unroll
    for (int it = 0; it < EST4; it++) {
      if (it >= n) break;
      const int i = it * WAVE + lane;
      const int r = i / n, cc = i - (i / n) * n;
      cv[it] = st4[r * EST4 + cc];
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int it = 0; it < EST4; it++) {
      if (it >= n) break;
      const int i = it * WAVE + lane;
      const int r = i / n, cc = i - (i / n) * n;
      const uint32_t i4 = (uint32_t)(r * NS * D4 + GB[g] + cc);
      if (P.dbg_skip & 32) continue;
      if (P.dbg_skip & 64) out4[i4] = cv[it];
      else st_obs4(out4, i4, cv[it], P.store_wt);
    }
  }
}

// 4-ship sides (D = 68 floats = 17 float4 chunks per row, 68 chunks = 17 whole
// 64-B lines per env block): rows of one agent leave line-aligned. Row kl
// spans chunks [17 kl, 17 kl + 17) of the env's block, so rows 0-2 end inside a
// line the next row finishes; stored as is, every such line is written twice,
// in two partial pieces (the melee step's WRITE_SIZE was 1.19x the algorithmic
// bytes). Pass kl instead emits the whole lines [16 kl, 16 kl + 16) (pass 3:
// [48, 68)): the kl chunks row kl-1 left over (carried in registers) and the
// first 16 - kl chunks of row kl; its last kl + 1 chunks wait for the next
// pass. Same values, same addresses, every line written once, whole.
template <int KL>
__device__ __forceinline__ void emit_rows_al4_t(const KParams &P, const KState &S, const Cols &c,
                                                const double *duct_col, int a, float *obs_side, int env0,
                                                f32x4 (&v)[12], float &w48, f32x4 (&carry)[3]) {
  constexpr int NS = 4, D4 = 17, T = 4 * NS + 3;
  constexpr int DC = KL;                          // chunks carried from row KL - 1
  constexpr int W = KL < NS - 1 ? 16 : 20;        // chunks this pass stores (whole lines)
  constexpr int NOWN = W - DC;                    // row KL's chunks stored now: 0 .. NOWN - 1
  constexpr int NDEF = KL < NS - 1 ? D4 - NOWN : 0;  // row KL's chunks left for the next pass
  constexpr int GS = W / 4;                       // chunks per stage group (4 groups)
  static_assert(GS <= EST4 && NDEF <= 3, "stage / carry sizes");
  const int lane = threadIdx.x & (WAVE - 1);
  const int el = lane;
  const int own0 = a >= NS ? NS : 0;
  const float *xg = c.estage + WAVE * EST4 * 4;
  const uint32_t p = c.pos_cur[a * PAD + el];
  const int tk = c.type[a * PADB + el];
  const int alive = c.alive0[a * PADB + el];
  const int rad = c.radar_cur[a * PAD + el];
  const int mis = c.miss_cur[a * PADB + el];
  const uint32_t tcn = c.tcnt[a * PAD + el];
  const double du = duct_col[el];
  float t[T];
  t[0] = xg[pos_x(p)];
  t[1] = xg[pos_y(p)];
  t[2] = (float)rad;
  t[3] = (float)mis * (tk == T_SMALL ? 0.25f : 0.125f);
#pragma unroll
  for (int s = 0; s < NS - 1; s++) {
    const bool nw = s < KL;
    const int i = own0 + (nw ? s : s + 1);
    const uint32_t q = (nw ? c.pos_cur : c.pos_old)[i * PAD + el];
    const int ta = c.alive0[i * PADB + el];
    const int m = (nw ? c.miss_cur : c.miss_old)[i * PADB + el];
    const float fm = (float)m * (c.type[i * PADB + el] == T_SMALL ? 0.25f : 0.125f);
    t[4 + 4 * s] = ta ? xg[pos_x(q)] : 0.0f;
    t[5 + 4 * s] = ta ? xg[pos_y(q)] : 0.0f;
    t[6 + 4 * s] = ta ? (float)(nw ? c.radar_cur : c.radar_old)[i * PAD + el] : 0.0f;
    t[7 + 4 * s] = ta ? fm : 0.0f;
  }
  t[T - 3] = (float)tcn;
  t[T - 2] = tk == T_LS ? 1.0f : 0.0f;
  t[T - 1] = (float)(du / 2.0);
  const bool ls = tk == T_LS;
  f32x4 vc[12];
#pragma unroll
  for (int q = 0; q < 12; q++) vc[q] = v[q];
  const float wc = w48;
  if (a + 1 < 2 * NS) load_window(S, window_rec(P, c, a + 1, el), v, w48);
  auto chunk = [&](int q) {  // row chunk q (compile-time q after unrolling)
    f32x4 o;
#pragma unroll
    for (int w = 0; w < 4; w++) {
      const int j = 4 * q + w;
      const float wv = j < 48 ? vc[j >> 2][j & 3] : (j == 48 ? wc : 0.0f);
      const float xc = j < 49 ? wv : t[j - 49 < T ? j - 49 : 0];
      const float xl = j < 25 ? wv : (j - 25 < T ? t[j - 25 < T ? j - 25 : 0] : 0.0f);
      o[w] = alive ? (ls ? xl : xc) : 0.0f;
    }
    return o;
  };
  f32x4 *st4 = (f32x4 *)c.estage;
  f32x4 *out4 = (f32x4 *)obs_side + (size_t)env0 * NS * D4;  // the first env's block
  constexpr int LS0 = (D4 * KL) & ~3;                         // the pass's first chunk (line start)
#pragma unroll
  for (int g = 0; g < 4; g++) {
#pragma unroll
    for (int u = 0; u < GS; u++) {
      const int j = g * GS + u;
      st4[lane * EST4 + u] = j < DC ? carry[j < DC ? j : 0] : chunk(j - DC);
    }
    wave_lds_sync();
    f32x4 cv[EST4];
#pragma unroll
    for (int it = 0; it < GS; it++) {
      const int i = it * WAVE + lane;
      const int r = i / GS, cc = i - (i / GS) * GS;
      cv[it] = st4[r * EST4 + cc];
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int it = 0; it < GS; it++) {
      const int i = it * WAVE + lane;
      const int r = i / GS, cc = i - (i / GS) * GS;
      const uint32_t i4 = (uint32_t)(r * NS * D4 + LS0 + g * GS + cc);
      if (P.dbg_skip & 32) continue;
      if (P.dbg_skip & 64) out4[i4] = cv[it];
      else st_obs4(out4, i4, cv[it], P.store_wt);
    }
  }
#pragma unroll
  for (int d = 0; d < NDEF; d++) carry[d] = chunk(NOWN + d);
}

// Wave 1 of a templated step workgroup: emits agent a's rows once wave 0 has
// published progress > a (LDS counter, -1 until phase S starts: the emission
// stage aliases the terrain mask phase M reads). Its stores count on its own
// vmcnt, so wave 0's loads in phase S never wait behind observation stores.
//
// The pair's contract (publish_progress / wait_progress): it orders LDS only.
// publish_progress(v) drains the publishing wave's LDS operations
// (s_waitcnt lgkmcnt(0)) and then stores v; a wave that has read a count >= v
// sees every LDS write the publisher made before it (a completed LDS write is
// visible to every wave of the CU, and the reader's later LDS reads are issued
// after its load of the count returned). It gives no ordering for global
// memory (no vmcnt wait, no release/acquire fence), and none the other way:
// the publisher may overwrite any LDS word the reader has not finished with.
// So a reader may use only LDS data the publisher will not change again in
// this step — the emission path reads agent a's columns, which phase S
// finishes with agent a's turn. (Round 4's per-ship handoff broke the second
// rule: wave 1 read columns and HBM target lists that wave 0's later turns
// rewrite; it stays out.)
__device__ inline int wait_progress(const int *prog, int want) {
  int v;
  while ((v = __hip_atomic_load(prog, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) < want)
    __builtin_amdgcn_s_sleep(1);
  asm volatile("" ::: "memory");
  return v;
}

__device__ inline void publish_progress(int *prog, int v) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // row inputs written before the count
  __hip_atomic_store(prog, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}


template <int NS>
__device__ __forceinline__ void emit_wave_t(const KParams &P, const KState &S, const Cols &c, const double *duct_col,
                            const int *prog, float *obs_b, float *obs_r, int env0) {
  const int lane = threadIdx.x & (WAVE - 1);
  wait_progress(prog, 0);
  float *xg = c.estage + WAVE * EST4 * 4;
  for (int x = lane; x < P.G; x += WAVE) xg[x] = (float)((double)x / (double)P.G);
  f32x4 v[12];
  float w48;
  load_window(S, window_rec(P, c, 0, lane), v, w48);
  int done = 0;
  if constexpr (NS == 4) {
    if (!(P.dbg_skip & 8192)) {  // (diagnostics: bit 13 keeps the row-piece emission)
      // line-aligned passes (emit_rows_al4_t): the compile-time pass index keeps
      // the carried chunks in registers
#pragma unroll 1
      for (int sd = 0; sd < 2; sd++) {
        float *out = sd ? obs_r : obs_b;
        f32x4 carry[3];
        const int a0 = sd * NS;
        if (done <= a0) done = wait_progress(prog, a0 + 1);
        emit_rows_al4_t<0>(P, S, c, duct_col, a0, out, env0, v, w48, carry);
        if (done <= a0 + 1) done = wait_progress(prog, a0 + 2);
        emit_rows_al4_t<1>(P, S, c, duct_col, a0 + 1, out, env0, v, w48, carry);
        if (done <= a0 + 2) done = wait_progress(prog, a0 + 3);
        emit_rows_al4_t<2>(P, S, c, duct_col, a0 + 2, out, env0, v, w48, carry);
        if (done <= a0 + 3) done = wait_progress(prog, a0 + 4);
        emit_rows_al4_t<3>(P, S, c, duct_col, a0 + 3, out, env0, v, w48, carry);
      }
      return;
    }
  }
  for (int a = 0; a < 2 * NS; a++) {
    if (done <= a) done = wait_progress(prog, a + 1);
    emit_rows_t<NS>(P, S, c, duct_col, a, a >= NS ? obs_r : obs_b, env0, v, w48);
  }
}

// The 2-bit terrain mask into LDS: 16-B loads, all of a thread's issued before
// any is stored (a plain word loop waits out one L2 round trip per word).
template <int NW>
__device__ __forceinline__ void stage_mask(const KParams &P, const KState &S, uint32_t *dst,
                                           int tid = (int)threadIdx.x) {
  const int nw = P.G * P.W16, n4 = nw >> 2;
  const u32x4 *src4 = (const u32x4 *)S.mask2;
  u32x4 *dst4 = (u32x4 *)dst;
  constexpr int U = 4;
  for (int i0 = tid; i0 < n4; i0 += U * NW * WAVE) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int i = i0 + u * NW * WAVE;
      if (i < n4) v[u] = src4[i];
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int i = i0 + u * NW * WAVE;
      if (i < n4) dst4[i] = v[u];
    }
  }
  for (int w = (n4 << 2) + tid; w < nw; w += NW * WAVE) dst[w] = S.mask2[w];
}

// ---------------------------------------------------------------------------
// phase L: load state columns
// ---------------------------------------------------------------------------
template <int AT, int NW>
__device__ inline void load_state(const KParams &P, const KState &S, Cols &c, int lane, int env,
                                  bool valid, int wid) {
  const long long E = P.E;
  const int A = AT > 0 ? AT : P.A;
#pragma unroll
  for (int a = 0; a < (AT > 0 ? AT : A); a++) {
    if (NW > 1 && a % NW != wid) continue;  // agents split across the waves
    size_t ai = (size_t)a * E + env;
    if (valid) {
      uint32_t p = S.pos[ai];
      COLW(c.pos_cur, a) = p;
      COLW(c.pos_old, a) = p;
      COLW(c.pos_new, a) = p;
      int rd = S.radar[ai];
      COLW(c.radar_cur, a) = rd;
      COLW(c.radar_old, a) = rd;
      uint8_t m = S.miss[ai];
      COLB(c.miss_cur, a) = m;
      COLB(c.miss_old, a) = m;
      COLB(c.type, a) = S.type[ai];
      COLB(c.alive0, a) = S.alive[ai];
      COLW(c.tcnt, a) = S.tl_cnt[ai];
      COLW(c.steps, a) = S.steps[ai];
      COLB(c.eng, a) = 0;
      COLB(c.mkind, a) = S.mkind[ai];
      COLB(c.obsd, a) = 0;
    } else if (lane < EPW) {
      COLB(c.alive0, a) = 0;
      COLB(c.type, a) = 0;
    }
  }
}

// ---------------------------------------------------------------------------
// phase M (combatant.py:459-489): action decode, move target, can_move_to and
// the check_path feasibility, over (env, agent) pairs: pass p lane l handles
// pair q = 64p + l of the workgroup (env q / A, agent q % A), so each pass
// reads 64 consecutive action rows (one coalesced 1 KB load) and all passes'
// loads of one batch are issued before any is used.
// ---------------------------------------------------------------------------
// PRE (float32 rows, one batch): the rows were loaded before phase L's barrier
// (preload_rows_f32) and arrive in vpre.
template <int DT, int MAXP, bool PRE = false>
__device__ __forceinline__ bool move_batch_t(const KParams &P, const KState &S, Cols &c, const void *actions,
                             const uint8_t *row_kind, const uint32_t *mask, int env0, int nenv,
                             int A, int p0, int np, const f32x4 (&vpre)[MAXP] = {}) {
  const int lane = threadIdx.x & (WAVE - 1);
  const int npair = nenv * A;
  f32x4 vf[DT == LNW_ACT_F32 ? MAXP : 1];
  int4 vi[DT == LNW_ACT_I32 ? MAXP : 1];
  double2 v01[DT == LNW_ACT_F64 ? MAXP : 1], v23[DT == LNW_ACT_F64 ? MAXP : 1];
  int kd[DT == LNW_ACT_F64 ? MAXP : 1];
#pragma unroll
  for (int k = 0; k < MAXP; k++) {
    if (k >= np) break;
    int q = (p0 + k) * WAVE + lane;
    q = q < npair ? q : 0;  // absent pairs re-read pair 0 (ignored)
    const size_t row = ((size_t)env0 * A + q) * 4;
    if constexpr (DT == LNW_ACT_F32) vf[k] = PRE ? vpre[k] : *(const f32x4 *)((const float *)actions + row);
    else if constexpr (DT == LNW_ACT_I32) vi[k] = *(const int4 *)((const int32_t *)actions + row);
    else {
      const double2 *da = (const double2 *)((const double *)actions + row);
      v01[k] = da[0];
      v23[k] = da[1];
      kd[k] = row_kind ? row_kind[(size_t)env0 * A + q] : K_F64;
    }
  }
  uint32_t tg[MAXP];
  int mw[MAXP];
#pragma unroll
  for (int k = 0; k < MAXP; k++) {
    tg[k] = 0;
    mw[k] = -1;
    if (k >= np) break;
    const int q = (p0 + k) * WAVE + lane;
    const int e = q / A, a = q - (q / A) * A;
    if (q >= npair || !c.alive0[a * PADB + e]) continue;
    const uint32_t p = c.pos_old[a * PAD + e];
    const int sx = pos_x(p), sy = pos_y(p);
    const int t = c.type[a * PADB + e];
    uint32_t target = p;  // no candidate
    // DISCRETE rows (value_to_coordinates, combatant.py:689-704): an int32
    // buffer is an integer ndarray; a float64 buffer holds the Python ints of a
    // list of lists (ddqn.py:396), whose salvo entry game.py:379 may turn into a
    // float in place
    bool disc = DT == LNW_ACT_I32;
    if constexpr (DT == LNW_ACT_F64) disc = P.discrete != 0;
    if (disc) {
      int mv = 0;
      if constexpr (DT == LNW_ACT_I32) {
        c.act0[a * PAD + e] = (double)vi[k].x;
        c.act1[a * PAD + e] = (double)vi[k].y;
        mv = vi[k].z;
      } else if constexpr (DT == LNW_ACT_F64) {
        c.act0[a * PAD + e] = v01[k].x;
        c.act1[a * PAD + e] = v01[k].y;
        mv = (int)v23[k].x;
      }
      c.akind[a * PADB + e] = K_PYINT;
      const int x = floordiv7(mv), y = pymod7(mv);
      if (0 <= sx - 3 + x && sx - 3 + x < P.G && 0 <= sy - 3 + y && sy - 3 + y < P.G)
        target = pack_pos(sx - 3 + x, sy - 3 + y) | 0x40000000u;
    } else if constexpr (DT != LNW_ACT_I32) {
      double a2, a3;
      int kind;
      if constexpr (DT == LNW_ACT_F32) {
        c.act0[a * PAD + e] = vf[k].x;
        c.act1[a * PAD + e] = vf[k].y;
        a2 = vf[k].z;
        a3 = vf[k].w;
        kind = K_F32;
      } else {
        c.act0[a * PAD + e] = v01[k].x;
        c.act1[a * PAD + e] = v01[k].y;
        a2 = v23[k].x;
        a3 = v23[k].y;
        kind = kd[k];
      }
      c.akind[a * PADB + e] = (uint8_t)kind;
      int nx, ny;
      if (!move_target_dev(sx, sy, ship_speed(t), a2, a3, kind, nx, ny)) {
        atomicOr(&S.err[env0 + e], (uint32_t)LNW_ERRF_NAN_ROUND);
      } else if (0 <= nx && nx < 100 && 0 <= ny && ny < 100 &&
                 !(cell_bits(mask, P.W16, nx, ny) & 1u)) {  // can_move_to (combatant.py:482-489)
        target = pack_pos(nx, ny) | 0x40000000u;
      }
    }
    tg[k] = target;
    // check_path (combatant.py:382-408) from the move table when the target
    // lies in its window (move_mode 0), else the A* below
    if (target & 0x40000000u) {
      const int tx = pos_x(target & 0x3fffffffu), ty = pos_y(target & 0x3fffffffu);
      const int ox = tx - sx, oy = ty - sy;
      if (P.move_mode == 0 && tx <= 99 && ty <= 99 && ox >= -R_MV && ox <= R_MV && oy >= -R_MV &&
          oy <= R_MV) {
        const int bit = (ox + R_MV) * MV_W + (oy + R_MV);
        mw[k] = (int)(((size_t)mv_cls(t) * P.G * P.G + (size_t)sx * P.G + sy) * MV_WORDS +
                      (bit >> 5)) * 32 + (bit & 31);
      }
    }
  }
  uint32_t w[MAXP];
  bool pend = false;
#pragma unroll
  for (int k = 0; k < MAXP; k++) {
    if (k >= np) break;
    w[k] = S.mvtab[mw[k] >= 0 ? mw[k] >> 5 : 0];
  }
#pragma unroll
  for (int k = 0; k < MAXP; k++) {
    if (k >= np) break;
    const int q = (p0 + k) * WAVE + lane;
    const int e = q / A, a = q - (q / A) * A;
    if (q >= npair || !(tg[k] & 0x40000000u)) continue;  // pos_new stays p (load_state)
    if (mw[k] < 0) {  // outside the table: left flagged for the A* pass below
      c.pos_new[a * PAD + e] = tg[k];
      pend = true;
      continue;
    }
    const bool feas = (w[k] >> (mw[k] & 31)) & 1u;
    c.pos_new[a * PAD + e] = feas ? ((tg[k] & 0x3fffffffu) | 0x80000000u) : c.pos_old[a * PAD + e];
  }
  return pend;
}

// check_path by A* for the candidates the table did not cover (still flagged
// 0x40000000 in pos_new): one copy of the search for every action dtype.
__device__ __forceinline__ void move_astar_pass(const KParams &P, const KState &S, Cols &c,
                                                int nenv, int A) {
  const int lane = threadIdx.x & (WAVE - 1);
  const int npair = nenv * A;
  if (lane >= EPW) return;  // open lists exist for EPW lanes
#pragma unroll 1
  for (int q = lane; q < npair; q += EPW) {
    const int e = q / A, a = q - (q / A) * A;
    const uint32_t tgk = c.pos_new[a * PAD + e];
    if (!(tgk & 0x40000000u)) continue;
    const uint32_t p = c.pos_old[a * PAD + e];
    const uint32_t t2 = tgk & 0x3fffffffu;
    const bool feas = check_path_h(P, S, c.type[a * PADB + e], pos_x(p), pos_y(p), pos_x(t2),
                                   pos_y(t2), c.open + lane, EPW);
    c.pos_new[a * PAD + e] = feas ? (t2 | 0x80000000u) : p;
  }
}

// Compile-time team sizes, float32 rows: a wave's share of the pair passes is at
// most 4 (A <= 8, <= 64 envs), one batch. Its rows are loaded at launch, before
// phase L's barrier, so their HBM round trip overlaps the state loads instead of
// following them (move_phase_pre consumes them after the barrier).
template <int NW, int MAXP>
__device__ __forceinline__ void preload_rows_f32(const void *actions, int env0, int nenv, int A, int wid,
                                                 f32x4 (&v)[MAXP]) {
  const int lane = threadIdx.x & (WAVE - 1);
  const int npair = nenv * A;
  const int npass = (npair + WAVE - 1) / WAVE;
  const int share = (npass + NW - 1) / NW;
  const int pbeg = wid * share, np = (pbeg + share < npass ? pbeg + share : npass) - pbeg;
#pragma unroll
  for (int k = 0; k < MAXP; k++) {
    if (k >= np) break;
    int q = (pbeg + k) * WAVE + lane;
    q = q < npair ? q : 0;  // absent pairs re-read pair 0 (ignored)
    v[k] = *(const f32x4 *)((const float *)actions + ((size_t)env0 * A + q) * 4);
  }
}
template <int NW, int MAXP>
__device__ __forceinline__ bool move_phase_pre(const KParams &P, const KState &S, Cols &c, const void *actions,
                                               const uint8_t *row_kind, const uint32_t *mask, int env0,
                                               int nenv, int A, int wid, const f32x4 (&v)[MAXP]) {
  const int npass = (nenv * A + WAVE - 1) / WAVE;
  const int share = (npass + NW - 1) / NW;
  const int pbeg = wid * share, np = (pbeg + share < npass ? pbeg + share : npass) - pbeg;
  if (np <= 0) return false;
  return move_batch_t<LNW_ACT_F32, MAXP, true>(P, S, c, actions, row_kind, mask, env0, nenv, A, pbeg, np, v);
}

// The NW waves of the workgroup take contiguous halves of the passes.
template <int DT, int NW>
__device__ __forceinline__ bool move_phase(const KParams &P, const KState &S, Cols &c, const void *actions,
                                  const uint8_t *row_kind, const uint32_t *mask, int env0,
                                  int nenv, int A, int wid) {
  // f32 (the rollout dtype) batches 8 passes; f64 / i32 go one pass at a time
  constexpr int B = DT == LNW_ACT_F32 ? 8 : 1;
  const int npass = (nenv * A + WAVE - 1) / WAVE;
  const int share = (npass + NW - 1) / NW;
  const int pbeg = wid * share, pend = pbeg + share < npass ? pbeg + share : npass;
  bool pending = false;  // this lane left a candidate for the A* pass
#pragma unroll 1
  for (int p0 = pbeg; p0 < pend; p0 += B)
    pending |= move_batch_t<DT, B>(P, S, c, actions, row_kind, mask, env0, nenv, A, p0,
                                   pend - p0 < B ? pend - p0 : B);
  return pending;
}

// diagnostics: per-workgroup phase timestamps (100 MHz real-time clock)
// slots: 0 start, 4 L end, 1 S start, 3 wave-0 end, 5 wave-1 end, 6..13 agent
// ends (phase S) or 6..9 quiet-path marks, 14 quiet marker, 16..19 lane-0 phase-S
// section totals (take_action to the move, LOS prefetch, get_obs, reward), 20..23 get_obs parts
__device__ inline void prof_put(const KState &S, int slot, unsigned long long v) {
  if (S.prof && (threadIdx.x & (WAVE - 1)) == 0) S.prof[(size_t)blockIdx.x * PROF_SLOTS + slot] = v;
}
__device__ inline void prof_stamp(const KState &S, int slot) {
  if (S.prof && (threadIdx.x & (WAVE - 1)) == 0)
    S.prof[(size_t)blockIdx.x * PROF_SLOTS + slot] = __builtin_amdgcn_s_memrealtime();
}

// Game.step tail (game.py:409-520) for the env in LDS column `lane` once every
// agent has acted: team bonus, defensive loss penalty, victory / defeat,
// landing-ops termination, episode counters, centre-of-gravity distance of the
// pre-move positions, the per-env outputs, then phase W (state stored back, or
// an in-kernel Game.reset when the episode ends).
// The part of the tail every caller shares: team bonus, loss penalty, victory /
// defeat and landing-ops checks on the reward columns, the env counters in ev,
// the cog distance. Returns done (1 running, 0 terminal); *cog_p gets the cog
// distance (NaN = None).
__device__ __forceinline__ int env_tail_core(const KParams &P, Cols &c, int lane, int nb, int A,
                                             const Neut &N, int (&ev)[8], const int (&hits)[2],
                                             int nbp, int nrp, int bsx, int bsy, int rsx, int rsy,
                                             double *cog_p, bool bonus_folded = false) {
  int done = 1;
  double cog = NAN;
  // quiet steps (bonus_folded: the caller added the zero team bonus, +0.0, to
  // every live ship's reward as it computed it): with both sides afloat and no
  // landing ops nothing below changes a reward, so skip the per-agent passes
  if (bonus_folded && !P.landing_ops && ev[0] != 0 && ev[1] != 0) {
    ev[2] = ev[2] + 1;
    if (nbp > 0 && nrp > 0) {
      double bx = (double)bsx / nbp, by = (double)bsy / nbp, rx = (double)rsx / nrp, ry = (double)rsy / nrp;
      cog = sqrt((bx - rx) * (bx - rx) + (by - ry) * (by - ry));
    }
    *cog_p = cog;
    return done;
  }
  // ---- tail (game.py:409-520) -------------------------------------------
  int nbl = ev[0] - N.cnt[0];
  int nrl = ev[1] - N.cnt[1];
  ev[0] = nbl;
  ev[1] = nrl;
  bool no_blue = nbl == 0, no_red = nrl == 0;
  for (int a = 0; a < A; a++) {
    if (!COLB(c.alive0, a)) continue;
    int side = a >= nb;
    if (!COLB(c.eng, a)) COLW(c.reward, a) += (double)(hits[side] * 2);
  }
  if (!P.aggressive) {
    for (int a = 0; a < A; a++) {
      int side = a >= nb;
      if (N.cnt[side] > 0) COLW(c.reward, a) = fmax(COLW(c.reward, a) - (double)(N.cnt[side] * 5), 0.0);
    }
  }
  if (no_blue && !no_red) {
    done = 0;
    for (int a = 0; a < A; a++) {
      if (a < nb) { if (!P.aggressive) COLW(c.reward, a) = COLW(c.reward, a) - COLW(c.reward, a); }
      else COLW(c.reward, a) += 100.0;
    }
    ev[4] += 1;
  }
  if (no_red && !no_blue) {
    done = 0;
    for (int a = 0; a < A; a++) {
      if (a < nb) COLW(c.reward, a) += 100.0;
      else if (!P.aggressive) COLW(c.reward, a) = COLW(c.reward, a) - COLW(c.reward, a);
    }
    ev[3] += 1;
  }
  if (no_blue && no_red) {
    done = 0;
    for (int a = 0; a < A; a++) COLW(c.reward, a) += 10.0;
  }
  if (P.landing_ops) {
    int rem = 0;
    for (int a = nb; a < A; a++) rem += (COLB(c.alive0, a) && COLB(c.type, a) == T_LS) ? 1 : 0;
    if (!rem) {
      done = 0;
      for (int a = 0; a < A; a++) {
        if (a < nb) COLW(c.reward, a) += 100.0;
        else COLW(c.reward, a) = COLW(c.reward, a) - COLW(c.reward, a);
      }
      ev[3] += 1;
    } else {
      for (int l = nb; l < A; l++) {
        if (!(COLB(c.alive0, l) && COLB(c.type, l) == T_LS)) continue;
        uint32_t pl = COLW(c.pos_cur, l);
        if (pos_x(pl) == P.lz_x && pos_y(pl) == P.lz_y) {
          done = 0;
          for (int a = 0; a < A; a++) {
            if (a < nb) COLW(c.reward, a) = COLW(c.reward, a) - COLW(c.reward, a);
            else COLW(c.reward, a) += 100.0;
          }
          ev[3] += 1;
        }
      }
    }
  }
  ev[2] = ev[2] + 1;
  if (nbp > 0 && nrp > 0) {
    double bx = (double)bsx / nbp, by = (double)bsy / nbp, rx = (double)rsx / nrp, ry = (double)rsy / nrp;
    cog = sqrt((bx - rx) * (bx - rx) + (by - ry) * (by - ry));
  }
  *cog_p = cog;
  return done;
}

// episode end: done == 0 or the horizon (the in-kernel auto-reset)
__device__ __forceinline__ bool env_resets(const KParams &P, int done, int steps_env) {
  return P.auto_reset && (done == 0 || (P.episode_steps > 0 && steps_env >= P.episode_steps));
}

__device__ __forceinline__ void env_tail(const KParams &P, const KState &S, Cols &c, int lane, int env,
                                         int nb, int A, const Neut &N, int (&ev)[8],
                                         const int (&hits)[2], int nbp, int nrp, int bsx, int bsy,
                                         int rsx, int rsy, Rng &rng, float *rew_b, float *rew_r,
                                         int32_t *done_out, float *cog_out, bool quiet = false) {
  const long long E = P.E;
  const int nr = A - nb;
  double cog;
  const int done = env_tail_core(P, c, lane, nb, A, N, ev, hits, nbp, nrp, bsx, bsy, rsx, rsy, &cog, quiet);
  const int steps_env = ev[2];
  // outputs
  // float32 values by default; float64 (the reference's Python floats) when
  // lnw_set_reward_dtype asked for it
  if (P.rew_f64) {
    for (int a = 0; a < nb; a++)
      if (rew_b) ((double *)rew_b)[(size_t)env * nb + a] = COLW(c.reward, a);
    for (int a = 0; a < nr; a++)
      if (rew_r) ((double *)rew_r)[(size_t)env * nr + a] = COLW(c.reward, nb + a);
    if (cog_out) ((double *)cog_out)[env] = cog;
  } else {
    for (int a = 0; a < nb; a++)
      if (rew_b) rew_b[(size_t)env * nb + a] = (float)COLW(c.reward, a);
    for (int a = 0; a < nr; a++)
      if (rew_r) rew_r[(size_t)env * nr + a] = (float)COLW(c.reward, nb + a);
    if (cog_out) cog_out[env] = (float)cog;
  }
  if (done_out) done_out[env] = done;
  prof_stamp(S, 2);
  // ---- phase W: store state (alive updated by the neutralized lists) --
  const bool do_reset = env_resets(P, done, steps_env);
  for (int a = 0; a < A; a++) {
    size_t ai = (size_t)a * E + env;
    int side = a >= nb;
    bool killed = (N.mask[side] >> (a - (side ? nb : 0))) & 1u;
    S.pos[ai] = COLW(c.pos_cur, a);
    S.radar[ai] = COLW(c.radar_cur, a);
    S.steps[ai] = COLW(c.steps, a);
    // a quiet step fires nothing, sinks nothing and leaves every target list
    // empty (it was empty: env_quiet_t), so these four fields keep their values
    if (quiet) continue;
    S.miss[ai] = COLB(c.miss_cur, a);
    S.mkind[ai] = COLB(c.mkind, a);
    S.alive[ai] = COLB(c.alive0, a) && !killed;
    S.tl_cnt[ai] = (uint16_t)COLW(c.tcnt, a);
  }
  if (quiet) {  // the step counter, and the victory counters when the episode ends
    S.envi[2 * E + env] = ev[2];
    if (done == 0) {
      S.envi[3 * E + env] = ev[3];
      S.envi[4 * E + env] = ev[4];
    }
  } else {
#pragma unroll
    for (int q = 0; q < 8; q++) S.envi[q * E + env] = ev[q];
  }
  if (do_reset) reset_env_dev(P, S, env, rng);
  // a quiet step with a trained red draws nothing unless the env resets
  if (!quiet || !P.trained_red || do_reset) S.rng[env] = rng.ctr;
  if (rng.err) S.err[env] |= rng.err;
}

#include "lnw_quiet.inc"

extern __shared__ __attribute__((aligned(16))) char lds_dyn[];

// ---------------------------------------------------------------------------
// step kernel (Game.step, game.py:298-525)
// ---------------------------------------------------------------------------
// NB/NR > 0: compile-time ship counts (register pair loop in get_obs, unrolled
// observation copy-out); NB = NR = 0: runtime counts from P.
// NB/NR > 0 run two waves per workgroup: wave 0 steps the envs, wave 1 emits
// the observation rows (emit_wave_t).
// REFW: los_mode 2's reference LOS work (march_pairs_ref), a separate
// instantiation of the runtime-size kernel so the production kernels carry none
// of its code
// UN > 1 (templated team sizes, full 64-env units, LOS table mode): UN units of
// 64 envs and two waves each share one workgroup (one per CU at UN = 4). Every
// unit runs its own phases L, M, Q or S on its own LDS block; the quiet units'
// observation passes go through one workgroup-wide queue that every free wave
// of a quiet unit serves, so the CU's units finish their stream together
// instead of 4-5 us apart (the spread of separate workgroups on one CU).
template <int NB, int NR, bool CW, bool REFW, int UN, bool PS, bool SL>
__device__ __forceinline__ void step_body(
    const KParams &P, KState S, void *actions, const uint8_t *row_kind, float *obs_b, float *obs_r,
    float *rew_b, float *rew_r, int32_t *done_out, float *cog_out) {
  static_assert(UN == 1 || (NB > 0 && EPW == WAVE && !REFW), "units need the two-wave templated kernel");
  const int unit = UN > 1 ? (int)(threadIdx.x / (2 * WAVE)) : 0;
  const int lane = threadIdx.x & (WAVE - 1);
  const int wid = UN > 1 ? (int)((threadIdx.x / WAVE) & 1) : (int)(threadIdx.x / WAVE);
  const int epw = P.epw;
  const int env0 = (UN > 1 ? blockIdx.x * UN + unit : xcd_chunk(P, (int)blockIdx.x, (int)gridDim.x)) * epw;
  // LNW_PROF: one record per unit (prof_stamp writes S.prof[blockIdx.x * PROF_SLOTS + slot])
  if (UN > 1 && S.prof) S.prof += (size_t)(blockIdx.x * (UN - 1) + unit) * PROF_SLOTS;
  const int env = env0 + lane;
  const long long E = P.E;
  const bool valid = lane < epw && env < E;
  const int nenv = (E - env0) < epw ? (int)(E - env0) : epw;
  constexpr bool ST = NB > 0;
  const int nb = ST ? NB : P.nb, nr = ST ? NR : P.nr;
  const int A = nb + nr;
  // small quiet workgroups get whole-side row stages (quiet_step_t's direct mode)
  // (the host's rows, step_launch_lds_bytes: one slab below 64 / NB envs, two in
  // the SL instantiation; the one-slab kernels keep their own test of epw)
  const int qbig_rows = !(ST && NB == NR && EPW == WAVE && P.los_mode == 0) ? 0
                        : SL ? (P.qdirect ? WAVE : 0)
                             : (epw * NB <= WAVE ? epw * NB : 0);
  LdsLayout L = lds_layout(A, nb, nr, S.nmax, P.G * P.W16, P.G, qbig_rows);
  const int lstride = (L.total + 15) & ~15;  // one LDS block per unit
  Cols c = carve(lds_dyn + unit * lstride, L);
  __shared__ double duct_all[UN][WAVE];
  __shared__ int prog_all[UN], qclaim_all[UN];
  __shared__ int r2_all[UN][WAVE];  // per-env max sensor reach^2 (max_range2)
  __shared__ int ushare[2];         // UN > 1: [0] mask of quiet units, [1] shared pass counter
  double *duct_col = duct_all[unit];
  int &prog = prog_all[unit], &qclaim = qclaim_all[unit];
  int *r2col = r2_all[unit];
  if (UN > 1 && threadIdx.x == 0) { ushare[0] = 0; ushare[1] = 0; }  // (before phase L's barrier)
  // rows leave during phase S from wave 1 (emit_wave_t) for full waves in LOS
  // table mode; the terrain mask LDS is then reused as the emission stage, so
  // the rare out-of-table LOS march reads the global copy
  // the contact variant's phase S split by side (step_kernel PS, below): its rows
  // are written after phase S
  const bool psplit = PS && CW && NB == 4 && NR == 4 && UN == 1 && EPW == WAVE && P.los_mode == 0 &&
                      !(P.dbg_skip & 515) && !(P.dbg_skip & 16384);
  const bool emit = ST && P.los_mode != 1 && nenv == WAVE && !(P.dbg_skip & 3) && !P.no_obs && !psplit;
  // two-wave workgroups share phases L and M (agents / pair passes split);
  // after M wave 1 turns to emission and wave 0 runs S
  constexpr int NW = ST && EPW == WAVE ? 2 : 1;
  if (NW == 1 && wid == 1) return;
  // templated team sizes, float32 rows: this wave's action rows in flight across phase L
  // (LNW_DEBUG_SKIP bit 23: loaded in phase M instead)
  constexpr int MAXPRE = 4;  // passes per wave: A <= 8 ships x <= 64 envs over two waves
  const int dt = P.act_dtype;
  const bool pre = ST && NW == 2 && dt == LNW_ACT_F32 && !(P.dbg_skip & 4) && !(P.dbg_skip & 8388608);
  f32x4 vpre[MAXPRE];
  if (pre) preload_rows_f32<NW, MAXPRE>(actions, env0, nenv, A, wid, vpre);
  // small quiet-capable workgroups (quiet_step_t's direct mode, epw * NB <= 64):
  // wave 0's env counters and draw counter loaded at launch, their HBM round
  // trip inside phase L's instead of between phase Q and the tail (nothing
  // before the tail writes them; LNW_DEBUG_SKIP bit 29: loaded in phase Q)
  int evp[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  Rng rngp{};
  // (not in the contact variants: their registers run out in phase S, and these
  // live ranges put 52 B per lane of scratch into them — melee 2.3 us slower)
  const bool evpre = ST && !CW && NW == 2 && UN == 1 && NB == NR && epw * NB <= WAVE && P.los_mode == 0 &&
                     !(P.dbg_skip & (1 << 29));
  if (evpre && wid == 0 && valid) {
#pragma unroll
    for (int q = 0; q < 8; q++) evp[q] = S.envi[q * E + env];
    rngp = make_rng(P, S, env);
  }
  if (wid == 0) {
    prof_stamp(S, 0);
    // XCC id (hwreg 20, bits 3:0) and HW_ID (hwreg 4: CU, SH, SE) of this workgroup
    prof_put(S, 30, (unsigned long long)__builtin_amdgcn_s_getreg((3 << 11) | 20));
    prof_put(S, 31, (unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 4));
  } else if (wid == 1) {
    prof_put(S, 29, (unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 4));
  }

  stage_mask<NW>(P, S, c.mask, (int)threadIdx.x - unit * NW * WAVE);
  const uint32_t *mask = c.mask;
  load_state<NB + NR, NW>(P, S, c, lane, env, valid, wid);
  double duct = valid ? S.duct[env] : 1.0;
  if (wid == 0) {
    duct_col[lane] = duct;
    r2col[lane] = max_range2(P, duct);
    if (lane == 0) prog = -1;
  }
  __syncthreads();
  if (wid == 0) prof_stamp(S, 4);

  // ---- phase M: movement feasibility for every agent of this env --------
  // M1: load each action row once (a0/a1 kept in LDS for phase S) and compute
  //     the move target; M2: feasibility lookups (independent across agents).
  bool pend = false;
  if (!(P.dbg_skip & 4)) {
    if (pre)
      pend = move_phase_pre<NW, MAXPRE>(P, S, c, actions, row_kind, mask, env0, nenv, A, wid, vpre);
    else if (dt == LNW_ACT_F32)
      pend = move_phase<LNW_ACT_F32, NW>(P, S, c, actions, row_kind, mask, env0, nenv, A, wid);
    else if (dt == LNW_ACT_F64)
      pend = move_phase<LNW_ACT_F64, NW>(P, S, c, actions, row_kind, mask, env0, nenv, A, wid);
    else
      pend = move_phase<LNW_ACT_I32, NW>(P, S, c, actions, row_kind, mask, env0, nenv, A, wid);
  }
  // quiet workgroups (lnw_quiet.inc) skip phase S; deciding it needs the final
  // moves, so wave 0 runs the A* fallback before a second barrier
  // (any workgroup size: a partial or small-epw workgroup idles its extra lanes)
  const bool qcap = ST && P.los_mode == 0 && !(P.dbg_skip & 3) && !(P.dbg_skip & 512);
  // workgroup-wide: did any pair leave the move table's window (A* pass needed)?
  // (round 4 measured unit-local barriers here and after phase Q instead,
  // each unit streaming as soon as its own moves were final: 43.3 vs 42.3 us)
  const bool astar = NW > 1 ? __syncthreads_or(pend) != 0 : true;
  if constexpr (ST && NW > 1) {
    if (qcap) {
      if (wid == 0) prof_stamp(S, 6);
      if (astar) {
        if (wid == 0) move_astar_pass(P, S, c, nenv, A);
        __syncthreads();
      }
      if (wid == 0) prof_stamp(S, 7);
      // small workgroups (epw * NB <= 64): the test spread over (ship, env) lanes
      bool wq;
      if (NB == NR && UN == 1 && P.epw * NB <= WAVE && !(P.dbg_skip & 268435456))  // (bit 28: per-env test)
        wq = wg_quiet_spread_t<NB, NB>(P, c, lane, r2col);
      else
        wq = __all(env_quiet_t<NB, NR>(P, c, lane, r2col[lane]));
      if (wid == 0) prof_stamp(S, 8);
#ifdef LNW_DIAG
      if (P.dbg_skip & (1 << 24)) {  // diagnostics: the quiet test again, its code now cached
        wq = __all(env_quiet_t<NB, NR>(P, c, lane, r2col[lane] + (P.dbg_skip >> 30)));
        if (wid == 0) prof_stamp(S, 12);
      }
#endif
      if (__builtin_expect(wq, 1)) {  // (quiet path laid out as the fall-through)
        if constexpr (UN > 1)
          quiet_step_units_t<NB, NR, UN>(P, S, c, lds_dyn, L, lstride, unit, lane, env, wid, duct_all,
                                         ushare, actions, obs_b, obs_r, rew_b, rew_r, done_out, cog_out,
                                         env0, valid);
        else
          quiet_step_t<NB, NR, SL>(P, S, c, lane, env, wid, duct_col, &qclaim, actions, obs_b, obs_r, rew_b,
                               rew_r, done_out, cog_out, env0, nenv, valid, evpre, evp, rngp);
        return;
      }
      if (UN > 1) __syncthreads();  // a loud unit: the barrier the quiet units pass after phase Q
    }
  }
#ifdef LNW_PROBE_QUIET_ONLY
  // timing probe (tools/gpu): the templated kernels without phase S / O code, so
  // the quiet path's registers are allocated without phase S live; loud
  // workgroups then do nothing (wrong results)
  if constexpr (ST && NW > 1) return;
#endif
  // The contact variant's phase S splits by side (templated 4v4, loud
  // workgroups; step_kernel PS): wave 0 plays blue's turns and wave 1 red's, and
  // the rows are written after it (phase O) instead of emitted by wave 1 during
  // it. Red's turns read blue only at its final cells and radars (SURVEY §9 Q1:
  // known after phase M — the moves, and radar = rint(a0)), and blue's read red
  // at its start cells and radars, so each wave works on its own view of the
  // cells and radars (wave 1's copy: blue final, red at the start, in the
  // emission stage's LDS, unused without emission). What ties the sides together
  // is the draw counter: wave 1 counts blue's draws first — the fire loops'
  // missile shots before a barrier (blue's get_obs then rewrites those lists),
  // the get_obs walks' bearings after it — and starts red's turns past them.
  // After a second barrier wave 0 merges red's hits, sums, counter and cells and
  // runs the tail. (The analytics logs' records then interleave the two sides'
  // turns; their order across envs is the atomics' order anyway.)
  // (rows written after phase S by wave 0 alone, behind a barrier: phase O)
  const bool phase_o = !((P.dbg_skip & 1) || emit || P.no_obs);
  if (wid == 1 && !psplit) {
    if constexpr (ST) {
      if (emit) emit_wave_t<NB>(P, S, c, duct_col, &prog, obs_b, obs_r, env0);
    }
    prof_stamp(S, 5);
    return;
  }
  if (!qcap && astar && !(P.dbg_skip & 4)) {
    // the rare A* fallback (open lists sized for one wave; psplit implies qcap)
    move_astar_pass(P, S, c, nenv, A);
    wave_lds_sync();
  }

  // ---- phase S: sequential agent loop ------------------------------------
  prof_stamp(S, 1);
  if (valid && !(P.dbg_skip & 2)) {
    if (emit) publish_progress(&prog, 0);
    Ctx X{P, S, c, lane, env, duct_col, make_rng(P, S, env), (emit || psplit) ? S.mask2 : mask, E,
          r2col[lane], 0};
    unsigned long long tp[4] = {0, 0, 0, 0}, t0 = prof_now(S);  // LNW_PROF part totals
    if constexpr (ST && CW) {
      pair_tables_t<NB, NR, true>(X);
    } else if constexpr (ST) {
      if (P.los_mode != 1 && !(P.dbg_skip & 2048)) los_prefetch_t<NB, NR>(X);
    }
    tp[1] += prof_now(S) - t0;
    Neut N{{0, 0}, {0u, 0u}};
    int ev[8];
#pragma unroll
    for (int q = 0; q < 8; q++) ev[q] = S.envi[q * E + env];
    X.step = ev[2];
    int hits[2] = {0, 0};
    int bsx = 0, bsy = 0, rsx = 0, rsy = 0;  // exact integer sums
    int nbp = 0, nrp = 0;
    if constexpr (PS && ST && CW && NB == 4 && NR == 4) {
      // one ship's turn (take_action, get_obs, calculate_reward: game.py:338-381)
      // on the view X.c: wave 0's is the workgroup's columns, the split's wave 1
      // its own (the parameters shadow the loop state they update)
      // (the hit state is copied in and out: a runtime index into an array behind a
      // reference would keep it in scratch)
      auto turn = [&](Ctx &X, int a, Neut &Nio, int (&evio)[8], int (&hio)[2], int &bsx, int &bsy, int &nbp,
                      int &rsx, int &rsy, int &nrp, unsigned long long (&tp)[4], unsigned long long &t0) {
        Cols &c = X.c;
        Neut N = Nio;
        int ev[8] = {0, 0, 0, 0, 0, 0, 0, 0}, hits[2] = {0, 0};
        const bool al = COLB(c.alive0, a) != 0;  // sunk ships skip their turn (reward 0)
        const int side = a >= nb;
        bool engage = false, moved = false;
        int destroyed = 0;
        t0 = prof_now(S);
        if (al) {
          uint32_t p0 = COLW(c.pos_cur, a);
          if (!side) {
            if (P.side_blue) { bsx += pos_x(p0); bsy += pos_y(p0); nbp++; }
          } else {
            rsx += pos_x(p0); rsy += pos_y(p0); nrp++;
          }
          size_t row = ((size_t)env * A + a) * 4;
          double a0 = COLW(c.act0, a), a1 = COLW(c.act1, a);
          int kind = COLB(c.akind, a);
          // untrained red: random salvo (game.py:375-379), written back in place
          if (side && !P.trained_red) {
            if (X.rng.uniform() < P.red_aggression) {
              double v = X.rng.uniform();
              if (dt == LNW_ACT_F32) { float f = (float)v; ((float *)actions)[row + 1] = f; a1 = f; }
              else if (dt == LNW_ACT_F64) {
                if (kind == K_F32) v = (double)(float)v;
                ((double *)actions)[row + 1] = v; a1 = v;
              } else { ((int32_t *)actions)[row + 1] = 0; a1 = 0.0; }
            }
          }
          // take_action (combatant.py:501-565)
          double engagement = P.discrete ? rint(a1) : a1;
          int keng = P.discrete ? K_PYINT : kind;
          int mk = COLB(c.mkind, a);
          double thr_v;
          if (kind_promote(keng, mk) == K_F32)
            thr_v = (double)rintf((float)engagement * (float)COLB(c.miss_cur, a));
          else
            thr_v = rint(engagement * (double)COLB(c.miss_cur, a));
          // round(nan/inf) of engagement * missiles raises (combatant.py:528): flagged, no engagement
          if (!isfinite(thr_v)) { X.rng.err |= LNW_ERRF_NAN_ROUND; thr_v = 0.0; }
          engage = thr_v > 0.0;
          int tn = (int)COLW(c.tcnt, a);
          if (engage && tn > 0 && !(P.dbg_skip & 65536)) {  // (bit 16: diagnostics, no fire)
            const uint16_t *tl = S.tl + (size_t)a * P.T * E + env;
            if constexpr (CW) {
              // contact variant: the list read 8 entries at a time, the loads of a
              // chunk in flight together (packed in a register pair: a runtime index
              // into a register array would put it in scratch)
              for (int q0 = 0; q0 < tn; q0 += 8) {
                uint64_t pk0 = 0, pk1 = 0;
#pragma unroll
                for (int u = 0; u < 8; u++) {
                  const uint64_t v = q0 + u < tn ? (uint64_t)tl[(size_t)(q0 + u) * E] : 0ull;
                  if (u < 4) pk0 |= v << (16 * u);
                  else pk1 |= v << (16 * (u - 4));
                }
                const int nq = tn - q0 < 8 ? tn - q0 : 8;
                for (int u = 0; u < nq; u++) {
                  const uint16_t tg = (uint16_t)((u < 4 ? pk0 : pk1) >> (16 * (u & 3)));
                  if (fire_dev(X, a, tg & 0xff, tg >> 8, engagement, keng, N)) destroyed++;
                }
              }
            } else {
              uint16_t nx = tl[0];  // the next target's load is in flight while one fires
              for (int q = 0; q < tn; q++) {
                const uint16_t tg = nx;
                if (q + 1 < tn) nx = tl[(size_t)(q + 1) * E];
                if (fire_dev(X, a, tg & 0xff, tg >> 8, engagement, keng, N)) destroyed++;
              }
            }
          }
          if (side) ev[6] += destroyed; else ev[5] += destroyed;
          if (!isfinite(a0)) { X.rng.err |= LNW_ERRF_NAN_ROUND; COLW(c.radar_cur, a) = 0; }
          else {
            double rr = rint(a0);
            COLW(c.radar_cur, a) = (int)fmin(fmax(rr, -2147483648.0), 2147483647.0);
          }
          uint32_t pn = COLW(c.pos_new, a);
          moved = (pn & 0x80000000u) != 0;
          if (moved) COLW(c.pos_cur, a) = pn & 0x7fffffffu;
        }
        tp[0] += prof_now(S) - t0;
        t0 = prof_now(S);
        if (al && !(P.dbg_skip & 128)) {
          if constexpr (REFW) march_pairs_ref(X, a);
          if constexpr (ST) {
            if (!side) get_obs_t<NB, NR, CW>(X, a, 0, NB);
            else get_obs_t<NR, NB, CW>(X, a, NB, 0);
          } else {
            get_obs_dev(X, a);
          }
        }
        tp[2] += prof_now(S) - t0;
        t0 = prof_now(S);
        double r = 0.0;
        if (al && !(P.dbg_skip & 256)) r = reward_dev(X, a, moved, engage, destroyed);
        COLW(c.reward, a) = r;
        if (al) {
          if (!side) {
            if (P.side_blue ? destroyed > 0 : engage) COLB(c.eng, a) = 1;
          } else {
            if (!P.trained_red ? engage : destroyed > 1) COLB(c.eng, a) = 1;
          }
          hits[side] += destroyed;
        }
        tp[3] += prof_now(S) - t0;
        Nio = N;
        evio[5] += ev[5];
        evio[6] += ev[6];
        hio[0] += hits[0];
        hio[1] += hits[1];
      };
      if (psplit) {
        // wave 1's view: pos / radar copies and its pooled-bearing tables in the
        // emission stage (psplit_bytes: 2 x 2 080 + 1 216 B; lds_layout sizes
        // the region to at least that for 4v4 whatever G is)
        Cols cr = c;
        cr.pos_cur = (uint32_t *)(lds_dyn + L.mask);
        cr.radar_cur = (int32_t *)(lds_dyn + L.mask + A * PAD * 4);
        cr.observed = (uint32_t *)(lds_dyn + L.mask + 2 * A * PAD * 4);
        long long nd = 0;  // blue's draws (wave 1)
        if (wid == 1) {
#pragma unroll
          for (int a = 0; a < A; a++) {
            uint32_t p = COLW(c.pos_cur, a);
            int r = COLW(c.radar_cur, a);
            if (a < NB && COLB(c.alive0, a)) {  // blue's final cell and radar
              const uint32_t pn = COLW(c.pos_new, a);
              if (pn & 0x80000000u) p = pn & 0x7fffffffu;
              const double a0 = COLW(c.act0, a);
              r = !isfinite(a0) ? 0 : (int)fmin(fmax(rint(a0), -2147483648.0), 2147483647.0);
            }
            COLW(cr.pos_cur, a) = p;
            COLW(cr.radar_cur, a) = r;
          }
          for (int a = 0; a < NB; a++) {  // fire loops, before blue's get_obs rewrites the lists
            if (!COLB(c.alive0, a)) continue;
            const double a1 = COLW(c.act1, a);
            const int kind = COLB(c.akind, a);
            const double engagement = P.discrete ? rint(a1) : a1;
            const int keng = P.discrete ? K_PYINT : kind;
            const int mk = COLB(c.mkind, a);
            const double thr_v = kind_promote(keng, mk) == K_F32
                                     ? (double)rintf((float)engagement * (float)COLB(c.miss_cur, a))
                                     : rint(engagement * (double)COLB(c.miss_cur, a));
            if (isfinite(thr_v) && thr_v > 0.0 && COLW(c.tcnt, a) > 0 && !(P.dbg_skip & 65536))
              nd += fire_draws(X, a, engagement, keng);
          }
        }
        __syncthreads();
        if (wid == 1) {
#pragma unroll
          for (int a = 0; a < NB; a++) {  // get_obs walks (their bearings), radar as take_action sets it
            if (!COLB(c.alive0, a)) continue;
            uint32_t pp[NR], am, fb, bm;
            mask_walk_t<NB, NR>(X, a, 0, NB, pp, am, fb, bm, true, COLW(cr.radar_cur, a));
            nd += __builtin_popcount(bm);
          }
          Ctx Y{P, S, cr, lane, env, duct_col, X.rng, S.mask2, E, r2col[lane], X.step};
          Y.ptr_[0] = X.ptr_[0]; Y.ptr_[1] = X.ptr_[1];
          Y.ptc[0] = X.ptc[0]; Y.ptc[1] = X.ptc[1];
          Y.ptw[0] = X.ptw[0]; Y.ptw[1] = X.ptw[1];
          Y.pre = X.pre;
          Y.lpre[0] = X.lpre[0]; Y.lpre[1] = X.lpre[1];
          if (Y.rng.mode == 1) {  // a tape stops at its end (blue's turns flag it)
            const long long len = Y.rng.tape_hi - Y.rng.tape_lo, cur = (long long)Y.rng.ctr;
            Y.rng.ctr = (unsigned long long)(cur + nd <= len ? cur + nd : (cur > len ? cur : len));
          } else {
            Y.rng.ctr += (unsigned long long)nd;
          }
          Neut NR_{{0, 0}, {0u, 0u}};
          int evr[8] = {0, 0, 0, 0, 0, 0, 0, 0}, hr[2] = {0, 0}, zb = 0, zby = 0, znb = 0;
          for (int a = NB; a < A; a++) turn(Y, a, NR_, evr, hr, zb, zby, znb, rsx, rsy, nrp, tp, t0);
          // red's results into the copies' blue rows (dead now)
          COLW(cr.pos_cur, 0) = (uint32_t)NR_.cnt[0] | (uint32_t)NR_.cnt[1] << 16;
          COLW(cr.pos_cur, 1) = NR_.mask[0] | NR_.mask[1] << 16;
          COLW(cr.pos_cur, 2) = (uint32_t)rsx | (uint32_t)rsy << 16;
          COLW(cr.pos_cur, 3) = (uint32_t)nrp | (uint32_t)hr[1] << 8;
          COLW(cr.radar_cur, 0) = (int32_t)(uint32_t)Y.rng.ctr;
          COLW(cr.radar_cur, 1) = (int32_t)(uint32_t)(Y.rng.ctr >> 32);
          COLW(cr.radar_cur, 2) = (int32_t)Y.rng.err;
        } else {
          for (int a = 0; a < NB; a++) turn(X, a, N, ev, hits, bsx, bsy, nbp, rsx, rsy, nrp, tp, t0);
        }
        __syncthreads();
        if (wid == 1) return;
        {
          const uint32_t w0 = COLW(cr.pos_cur, 0), w1 = COLW(cr.pos_cur, 1), w2 = COLW(cr.pos_cur, 2),
                         w3 = COLW(cr.pos_cur, 3);
          N.cnt[0] += (int)(w0 & 0xffffu);
          N.cnt[1] += (int)(w0 >> 16);
          N.mask[0] |= w1 & 0xffffu;
          N.mask[1] |= w1 >> 16;
          rsx = (int)(w2 & 0xffffu);
          rsy = (int)(w2 >> 16);
          nrp = (int)(w3 & 0xffu);
          hits[1] += (int)(w3 >> 8);
          ev[6] += (int)(w3 >> 8);
          X.rng.ctr = (unsigned long long)(uint32_t)COLW(cr.radar_cur, 0) |
                      (unsigned long long)(uint32_t)COLW(cr.radar_cur, 1) << 32;
          X.rng.err |= (uint32_t)COLW(cr.radar_cur, 2);
#pragma unroll
          for (int a = NB; a < A; a++) {  // red's final cells and radars
            COLW(c.pos_cur, a) = COLW(cr.pos_cur, a);
            COLW(c.radar_cur, a) = COLW(cr.radar_cur, a);
          }
        }
      } else {
        for (int a = 0; a < A; a++) {
          turn(X, a, N, ev, hits, bsx, bsy, nbp, rsx, rsy, nrp, tp, t0);
          if (emit) publish_progress(&prog, a + 1);
          if (a < 8) prof_stamp(S, 6 + a);
        }
      }
    } else {  // (the loop written out: behind a lambda it keeps state in scratch)
      for (int a = 0; a < A; a++) {
        const bool al = COLB(c.alive0, a) != 0;  // sunk ships skip their turn (reward 0)
        const int side = a >= nb;
        bool engage = false, moved = false;
        int destroyed = 0;
        t0 = prof_now(S);
        if (al) {
          uint32_t p0 = COLW(c.pos_cur, a);
          if (!side) {
            if (P.side_blue) { bsx += pos_x(p0); bsy += pos_y(p0); nbp++; }
          } else {
            rsx += pos_x(p0); rsy += pos_y(p0); nrp++;
          }
          size_t row = ((size_t)env * A + a) * 4;
          double a0 = COLW(c.act0, a), a1 = COLW(c.act1, a);
          int kind = COLB(c.akind, a);
          // untrained red: random salvo (game.py:375-379), written back in place
          if (side && !P.trained_red) {
            if (X.rng.uniform() < P.red_aggression) {
              double v = X.rng.uniform();
              if (dt == LNW_ACT_F32) { float f = (float)v; ((float *)actions)[row + 1] = f; a1 = f; }
              else if (dt == LNW_ACT_F64) {
                if (kind == K_F32) v = (double)(float)v;
                ((double *)actions)[row + 1] = v; a1 = v;
              } else { ((int32_t *)actions)[row + 1] = 0; a1 = 0.0; }
            }
          }
          // take_action (combatant.py:501-565)
          double engagement = P.discrete ? rint(a1) : a1;
          int keng = P.discrete ? K_PYINT : kind;
          int mk = COLB(c.mkind, a);
          double thr_v;
          if (kind_promote(keng, mk) == K_F32)
            thr_v = (double)rintf((float)engagement * (float)COLB(c.miss_cur, a));
          else
            thr_v = rint(engagement * (double)COLB(c.miss_cur, a));
          // round(nan/inf) of engagement * missiles raises (combatant.py:528): flagged, no engagement
          if (!isfinite(thr_v)) { X.rng.err |= LNW_ERRF_NAN_ROUND; thr_v = 0.0; }
          engage = thr_v > 0.0;
          int tn = (int)COLW(c.tcnt, a);
          if (engage && tn > 0 && !(P.dbg_skip & 65536)) {  // (bit 16: diagnostics, no fire)
            const uint16_t *tl = S.tl + (size_t)a * P.T * E + env;
            if constexpr (CW) {
              // contact variant: the list read 8 entries at a time, the loads of a
              // chunk in flight together (packed in a register pair: a runtime index
              // into a register array would put it in scratch)
              for (int q0 = 0; q0 < tn; q0 += 8) {
                uint64_t pk0 = 0, pk1 = 0;
#pragma unroll
                for (int u = 0; u < 8; u++) {
                  const uint64_t v = q0 + u < tn ? (uint64_t)tl[(size_t)(q0 + u) * E] : 0ull;
                  if (u < 4) pk0 |= v << (16 * u);
                  else pk1 |= v << (16 * (u - 4));
                }
                const int nq = tn - q0 < 8 ? tn - q0 : 8;
                for (int u = 0; u < nq; u++) {
                  const uint16_t tg = (uint16_t)((u < 4 ? pk0 : pk1) >> (16 * (u & 3)));
                  if (fire_dev(X, a, tg & 0xff, tg >> 8, engagement, keng, N)) destroyed++;
                }
              }
            } else {
              uint16_t nx = tl[0];  // the next target's load is in flight while one fires
              for (int q = 0; q < tn; q++) {
                const uint16_t tg = nx;
                if (q + 1 < tn) nx = tl[(size_t)(q + 1) * E];
                if (fire_dev(X, a, tg & 0xff, tg >> 8, engagement, keng, N)) destroyed++;
              }
            }
          }
          if (side) ev[6] += destroyed; else ev[5] += destroyed;
          if (!isfinite(a0)) { X.rng.err |= LNW_ERRF_NAN_ROUND; COLW(c.radar_cur, a) = 0; }
          else {
            double rr = rint(a0);
            COLW(c.radar_cur, a) = (int)fmin(fmax(rr, -2147483648.0), 2147483647.0);
          }
          uint32_t pn = COLW(c.pos_new, a);
          moved = (pn & 0x80000000u) != 0;
          if (moved) COLW(c.pos_cur, a) = pn & 0x7fffffffu;
        }
        tp[0] += prof_now(S) - t0;
        t0 = prof_now(S);
        if (al && !(P.dbg_skip & 128)) {
          if constexpr (REFW) march_pairs_ref(X, a);
          if constexpr (ST) {
            if (!side) get_obs_t<NB, NR, CW>(X, a, 0, NB);
            else get_obs_t<NR, NB, CW>(X, a, NB, 0);
          } else {
            get_obs_dev(X, a);
          }
        }
        tp[2] += prof_now(S) - t0;
        t0 = prof_now(S);
        double r = 0.0;
        if (al && !(P.dbg_skip & 256)) r = reward_dev(X, a, moved, engage, destroyed);
        COLW(c.reward, a) = r;
        if (al) {
          if (!side) {
            if (P.side_blue ? destroyed > 0 : engage) COLB(c.eng, a) = 1;
          } else {
            if (!P.trained_red ? engage : destroyed > 1) COLB(c.eng, a) = 1;
          }
          hits[side] += destroyed;
        }
        tp[3] += prof_now(S) - t0;
        if (emit) publish_progress(&prog, a + 1);
        if (a < 8) prof_stamp(S, 6 + a);
      }
    }
    env_tail(P, S, c, lane, env, nb, A, N, ev, hits, nbp, nrp, bsx, bsy, rsx, rsy, X.rng, rew_b,
             rew_r, done_out, cog_out);
    if (S.prof && lane == 0)
      for (int q = 0; q < 4; q++) prof_put(S, 16 + q, tp[q]);
  }
  prof_stamp(S, 3);
  if (!phase_o) return;
  __syncthreads();
  // ---- phase O: observations ---------------------------------------------
  if constexpr (ST) write_obs_t<NB, NR>(P, S, c, duct_col, obs_b, obs_r, env0, nenv);
  else write_obs(P, S, c, duct_col, obs_b, obs_r, env0, nenv, false);
}

// One step of every env (lnw_step; lnw_step_seq makes one launch per step)
// SL: quiet workgroups of up to 128 / NB envs write their rows in two slabs
// (step_qdirect; a separate instantiation, so the one-slab kernels keep their code)
template <int NB, int NR, bool CW = false, bool REFW = false, int UN = 1, bool PS = false, bool SL = false>
__global__ __launch_bounds__(NB > 0 && EPW == WAVE ? 2 * WAVE * UN : WAVE, NB > 0 ? 2 : 1) void step_kernel(
    KParams P, KState S, void *actions, const uint8_t *row_kind, float *obs_b, float *obs_r,
    float *rew_b, float *rew_r, int32_t *done_out, float *cog_out) {
  step_body<NB, NR, CW, REFW, UN, PS, SL>(P, S, actions, row_kind, obs_b, obs_r, rew_b, rew_r, done_out, cog_out);
}

#include "lnw_group.inc"

// ---------------------------------------------------------------------------
// observe kernel (ship.get_obs() for a selection of ships)
// ---------------------------------------------------------------------------
// NB/NR > 0: compile-time team sizes — every LOS word the calls need loaded in
// one batch (los_prefetch_t: no ship moves here, so only the current cells) and
// the templated get_obs (get_obs_t; CW: the contact variant's mask walk), as
// the step kernel's phase S; NB = NR = 0: runtime sizes (get_obs_dev).
// CW with compile-time sizes: two waves, blue's calls on wave 0 and red's on
// wave 1. No ship moves and a call changes only its own ship's target list, so
// the calls are independent but for the draw counter: blue's calls take their
// draws first, and a call takes one draw per bearing of its walk. Wave 1 runs
// blue's walks alone (register bit arithmetic, no draws) to count them, starts
// red's calls past them, and keeps its pooled-bearing tables in the actions'
// LDS columns (unused here); the env's final counter and error bits are merged
// after a barrier. (A single side or ship keeps the calls on wave 0; the EW-fix
// log's records then interleave the sides, their order across envs being the
// atomics' order anyway.)
template <int NB = 0, int NR = 0, bool CW = false>
__global__ __launch_bounds__(NB > 0 && CW ? 2 * WAVE : WAVE) void observe_kernel(KParams P, KState S, int sel,
                                                                                 float *obs_b, float *obs_r) {
  constexpr int NW = NB > 0 && CW ? 2 : 1;
  const int lane = threadIdx.x & (WAVE - 1);
  const int wid = NW > 1 ? (int)(threadIdx.x / WAVE) : 0;
  const int epw = P.epw;
  const int env0 = xcd_chunk(P, (int)blockIdx.x, (int)gridDim.x) * epw;
  const int env = env0 + lane;
  const long long E = P.E;
  const bool valid = lane < epw && env < E;
  const int nenv = (E - env0) < epw ? (int)(E - env0) : epw;
  const int A = P.A, nb = P.nb;
  LdsLayout L = lds_layout(A, P.nb, P.nr, S.nmax, P.G * P.W16, P.G);
  Cols c = carve(lds_dyn, L);
  __shared__ double duct_col[WAVE];
  __shared__ unsigned long long ctr1[NW > 1 ? WAVE : 1];  // wave 1's final draw counter and error bits
  __shared__ uint32_t err1[NW > 1 ? WAVE : 1];
  for (int w = (int)threadIdx.x; w < P.G * P.W16; w += NW * WAVE) c.mask[w] = S.mask2[w];
  const uint32_t *mask = c.mask;
  load_state<NB + NR, NW>(P, S, c, lane, env, valid, wid);
  double duct = valid ? S.duct[env] : 1.0;
  if (wid == 0) duct_col[lane] = duct;
  __syncthreads();
  int a0 = 0, a1 = A;
  if (sel >= 0) { a0 = sel; a1 = sel + 1; }
  else if (sel == LNW_OBS_BLUE) { a1 = nb; }
  else if (sel == LNW_OBS_RED) { a0 = nb; }
  const bool split = NW > 1 && sel == LNW_OBS_ALL;
  int wa0 = a0, wa1 = a1;  // this wave's calls
  if (NW > 1) {
    if (split) { wa0 = wid ? nb : 0; wa1 = wid ? A : nb; }
    else if (wid == 1) { wa1 = wa0; }
  }
  unsigned long long fctr = 0;
  uint32_t ferr = 0;
  if (valid) {
    Cols cw = c;
    if (NW > 1 && wid == 1) cw.observed = (uint32_t *)(lds_dyn + L.act0);
    Ctx X{P, S, cw, lane, env, duct_col, make_rng(P, S, env), mask, E, max_range2(P, duct),
          S.envi[2 * E + env]};
    if constexpr (NB > 0 && CW) {
      pair_tables_t<NB, NR, false>(X);
      if (split && wid == 1) {  // past blue's draws
        long long nd = 0;
        for (int a = 0; a < nb; a++) {
          if (!COLB(c.alive0, a)) continue;
          uint32_t pp[NR], am, fb, bm;
          mask_walk_t<NB, NR>(X, a, 0, NB, pp, am, fb, bm);
          nd += __builtin_popcount(bm);
        }
        if (X.rng.mode == 1) {  // a tape stops at its end (blue's calls flag it)
          const long long len = X.rng.tape_hi - X.rng.tape_lo, cur = (long long)X.rng.ctr;
          X.rng.ctr = (unsigned long long)(cur + nd <= len ? cur + nd : (cur > len ? cur : len));
        } else {
          X.rng.ctr += (unsigned long long)nd;
        }
      }
    } else if constexpr (NB > 0) {
      if (P.los_mode != 1) los_prefetch_t<NB, NR>(X);
    }
    for (int a = wa0; a < wa1; a++) {
      if (!COLB(c.alive0, a)) continue;
      if constexpr (NB > 0) {
        if (a < NB) get_obs_t<NB, NR, CW>(X, a, 0, NB);
        else get_obs_t<NR, NB, CW>(X, a, NB, 0);
      } else {
        if (P.los_mode == 2) march_pairs_ref(X, a);
        get_obs_dev(X, a);
      }
      COLB(c.obsd, a) = 1;
      S.tl_cnt[(size_t)a * E + env] = (uint16_t)COLW(c.tcnt, a);
    }
    fctr = X.rng.ctr;
    ferr = X.rng.err;
    if (NW > 1 && wid == 1) {
      ctr1[lane] = split ? fctr : 0ull;
      err1[lane] = ferr;
    }
  }
  if constexpr (NW > 1) {
    __syncthreads();
    if (wid == 1) return;
    if (valid) {  // (counters only grow: wave 1 started where wave 0 ends)
      fctr = fctr > ctr1[lane] ? fctr : ctr1[lane];
      ferr |= err1[lane];
    }
  }
  if (valid) {
    S.rng[env] = fctr;
    if (ferr) S.err[env] |= ferr;
  }
  if constexpr (NW == 1) __syncthreads();
  // rows of ships not observed in this call are written as zeros
  write_obs(P, S, c, duct_col, obs_b, obs_r, env0, nenv, true);
}

__global__ void reset_kernel(KParams P, KState S, const uint8_t *mask) {
  int env = blockIdx.x * blockDim.x + threadIdx.x;
  if (env >= P.E) return;
  if (mask && !mask[env]) return;
  Rng r = make_rng(P, S, env);
  reset_env_dev(P, S, env, r);
  S.rng[env] = r.ctr;
  if (r.err) S.err[env] |= r.err;
}

// ---------------------------------------------------------------------------
// terrain structures
// ---------------------------------------------------------------------------
__global__ void build_mask_kernel(const uint8_t *grid, int G, int W16, int move_thr, int ew_thr,
                                  uint32_t *mask2) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= G * W16) return;
  int x = i / W16, w = i % W16;
  uint32_t v = 0;
  for (int b = 0; b < 16; b++) {
    int y = w * 16 + b;
    if (y >= G) break;
    uint8_t g = grid[x * G + y];
    v |= ((g > move_thr ? 1u : 0u) | (g > ew_thr ? 2u : 0u)) << (2 * b);
  }
  mask2[i] = v;
}

// move table: check_path(start, start + off) for off in [-4,4]^2, per class
// (mv_cls: Combatant speed 3, LandingShip, medium Combatant speed 2)
constexpr int MV_CLASSES = 3;
__global__ __launch_bounds__(64) void build_move_table_kernel(const uint32_t *mask2, int G, int W16,
                                                              uint32_t *mvtab) {
  __shared__ uint32_t open[OPEN_CAP * WAVE];
  long long i = (long long)blockIdx.x * WAVE + threadIdx.x;
  long long n = (long long)MV_CLASSES * G * G * MV_W * MV_W;
  if (i >= n) return;
  int off = (int)(i % (MV_W * MV_W));
  long long cell = (i / (MV_W * MV_W)) % ((long long)G * G);
  int cls = (int)(i / ((long long)MV_W * MV_W * G * G));
  int sx = (int)(cell / G), sy = (int)(cell % G);
  int tx = sx + off / MV_W - R_MV, ty = sy + off % MV_W - R_MV;
  MaskBlocked mb{mask2, W16};
  const int type = cls == 0 ? T_SMALL : (cls == 1 ? T_LS : T_MEDIUM);  // (mv_cls inverse)
  bool feas = check_path_dev(mb, mb(sx, sy), G, type, sx, sy, tx, ty,
                             open + threadIdx.x, WAVE);
  if (feas) atomicOr(&mvtab[(cls * (long long)G * G + cell) * MV_WORDS + (off >> 5)], 1u << (off & 31));
}

// LOS table: for every origin cell and offset in [-40,40]^2, bit0 radar clear,
// bit1 EW clear (full march, no early exit). The 2-bit terrain mask is staged
// into LDS once per workgroup (mwords words, when it fits the launch's LDS),
// and each workgroup then walks many (cell, row) items in a grid-stride loop,
// so the mask is read once per resident workgroup rather than once per 256
// items (G = 512: 64 KiB per workgroup).
__global__ __launch_bounds__(256) void build_los_table_kernel(const uint32_t *mask2, int G, int W16,
                                                              uint32_t *lostab, int mwords) {
  uint32_t *lm = (uint32_t *)lds_dyn;
  for (int w = threadIdx.x; w < mwords; w += blockDim.x) lm[w] = mask2[w];
  __syncthreads();
  const uint32_t *msk = mwords ? lm : mask2;
  const long long n = (long long)G * G * LOS_W;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const int row = (int)(i % LOS_W);
    const long long cell = i / LOS_W;
    const int x1 = (int)(cell / G), y1 = (int)(cell % G);
    const int x2 = x1 + row - R_LOS;
    uint32_t words[LOS_ROW_WORDS] = {0, 0, 0, 0, 0, 0};
    if (x2 >= 0 && x2 < G) {
      for (int c = 0; c < LOS_W; c++) {
        const int y2 = y1 + c - R_LOS;
        if (y2 < 0 || y2 >= G) continue;
        const uint32_t b = los_march<false>(msk, W16, x1, y1, x2, y2);
        const int col = c * 2;
        words[col >> 5] |= b << (col & 31);
      }
    }
    uint32_t *dst = lostab + cell * LOS_CELL_WORDS + row * LOS_ROW_WORDS;
#pragma unroll
    for (int w = 0; w < LOS_ROW_WORDS; w++) dst[w] = words[w];
  }
}

// ---------------------------------------------------------------------------
// unit kernels
// ---------------------------------------------------------------------------
// lnw_los_batch (combatant.py:436-456 per ray): every workgroup first builds the
// grid's 2-bit terrain mask (bit0 cell > move_thr, bit1 cell > ew_thr) in LDS,
// then its waves march their share of the rays from it. A lane whose ray has
// ended takes the wave's next unclaimed ray (ballot + popcount of the lanes
// asking), so a wave advances at its lanes' mean ray length instead of
// waiting on its longest ray; a ray stops early once both bits are blocked
// (the result cannot change).
constexpr int LB_THREADS = 256, LB_RAYS_PER_WAVE = 1024;
__global__ __launch_bounds__(LB_THREADS) void los_batch_kernel(const uint8_t *grid, int G, const int16_t *pairs,
                                                               long long n, int move_thr, int ew_thr, uint8_t *out) {
  const int W16 = (G + 15) >> 4;
  uint32_t *lm = (uint32_t *)lds_dyn;
  for (int w = threadIdx.x; w < G * W16; w += LB_THREADS) {
    const int x = w / W16, y0 = (w - x * W16) * 16;
    uint32_t v = 0;
    for (int b = 0; b < 16 && y0 + b < G; b++) {
      const uint8_t g = grid[(size_t)x * G + y0 + b];
      v |= ((g > move_thr ? 1u : 0u) | (g > ew_thr ? 2u : 0u)) << (2 * b);
    }
    lm[w] = v;
  }
  __syncthreads();
  const int lane = threadIdx.x & (WAVE - 1);
  const long long w0 = ((long long)blockIdx.x * (LB_THREADS / WAVE) + (threadIdx.x / WAVE)) * LB_RAYS_PER_WAVE;
  const long long wend = w0 + LB_RAYS_PER_WAVE < n ? w0 + LB_RAYS_PER_WAVE : n;
  long long next = w0;  // the wave's next unclaimed ray (uniform)
  long long idx = -1;   // this lane's ray
  int x = 0, y = 0, x2 = 0, y2 = 0, dx = 0, dy = 0, sx = 1, sy = 1, err = 0;
  uint32_t blk = 0;
  const unsigned long long below = (1ull << lane) - 1ull;
  auto claim = [&]() {
    const unsigned long long need = __ballot(idx < 0);
    if (idx < 0) {
      const long long k = next + __popcll(need & below);
      if (k < wend) {
        const uint64_t pr = *(const uint64_t *)(pairs + 4 * k);
        x = (int16_t)(pr & 0xffffu);
        y = (int16_t)((pr >> 16) & 0xffffu);
        x2 = (int16_t)((pr >> 32) & 0xffffu);
        y2 = (int16_t)(pr >> 48);
        dx = abs(x2 - x);
        dy = abs(y2 - y);
        sx = x > x2 ? -1 : 1;
        sy = y > y2 ? -1 : 1;
        err = dx - dy;
        blk = 0;
        idx = k;
      }
    }
    next += __popcll(need);
  };
  claim();
  while (__any(idx >= 0)) {
    if (idx >= 0) {
#pragma unroll 4
      for (int s = 0; s < 8; s++) {
        blk |= cell_bits(lm, W16, x, y);
        if (blk == 3u || (x == x2 && y == y2)) {
          out[idx] = (uint8_t)((~blk) & 3u);
          idx = -1;
          break;
        }
        const int e2 = 2 * err;
        if (e2 > -dy) { err -= dy; x += sx; }
        if (e2 < dx) { err += dx; y += sy; }
      }
    }
    if (next < wend) claim();
  }
}

// grids whose mask does not fit the launch's LDS: one lane per ray from HBM
__global__ void los_batch_global_kernel(const uint8_t *grid, int G, const int16_t *pairs, long long n,
                                        int move_thr, int ew_thr, uint8_t *out) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  int x1 = pairs[4 * i], y1 = pairs[4 * i + 1], x2 = pairs[4 * i + 2], y2 = pairs[4 * i + 3];
  int dx = abs(x2 - x1), dy = abs(y2 - y1);
  int sx = x1 > x2 ? -1 : 1, sy = y1 > y2 ? -1 : 1;
  int err = dx - dy;
  bool rb = false, eb = false;
  for (;;) {
    uint8_t g = grid[x1 * G + y1];
    rb |= g > move_thr;
    eb |= g > ew_thr;
    if (x1 == x2 && y1 == y2) break;
    int e2 = 2 * err;
    if (e2 > -dy) { err -= dy; x1 += sx; }
    if (e2 < dx) { err += dx; y1 += sy; }
  }
  out[i] = (rb ? 0 : 1) | (eb ? 0 : 2);
}

__global__ __launch_bounds__(64) void astar_batch_kernel(const uint8_t *grid, int G, int thr,
                                                         const int8_t *types, const int16_t *st,
                                                         const int16_t *tg, long long n,
                                                         int16_t *plen, int8_t *kind,
                                                         uint8_t *feas) {
  __shared__ uint32_t open[OPEN_CAP * WAVE];
  long long i = (long long)blockIdx.x * WAVE + threadIdx.x;
  if (i >= n) return;
  int t = types[i];
  int sx = st[2 * i], sy = st[2 * i + 1], tx = tg[2 * i], ty = tg[2 * i + 1];
  GridBlocked gb{grid, G, thr};
  if (abs(tx) > 500 || abs(ty) > 500 || sx < 0 || sy < 0 || sx >= G || sy >= G) {
    plen[i] = -2; kind[i] = -1; feas[i] = 0;
    return;
  }
  int k;
  int len = astar_dev(gb, G, ship_speed(t), sx, sy, tx, ty, k, open + threadIdx.x, WAVE);
  plen[i] = (int16_t)len;
  kind[i] = (int8_t)k;
  feas[i] = check_path_dev(gb, gb(sx, sy), G, t, sx, sy, tx, ty, open + threadIdx.x, WAVE) ? 1 : 0;
}

__global__ __launch_bounds__(64) void move_batch_kernel(KParams P, KState S, const int8_t *types,
                                                        const int16_t *pos, const double *act,
                                                        const uint8_t *is_f32, long long n,
                                                        int32_t *rounded, uint8_t *ok) {
  __shared__ uint32_t open[OPEN_CAP * WAVE];
  long long i = (long long)blockIdx.x * WAVE + threadIdx.x;
  if (i >= n) return;
  int t = types[i];
  int sx = pos[2 * i], sy = pos[2 * i + 1];
  int nx, ny;
  bool fin = move_target_dev(sx, sy, ship_speed(t), act[2 * i], act[2 * i + 1],
                             is_f32[i] ? K_F32 : K_F64, nx, ny);
  rounded[2 * i] = nx;
  rounded[2 * i + 1] = ny;
  bool f = fin && can_move_to_h(P, S, nx, ny) &&
           check_path_h(P, S, t, sx, sy, nx, ny, open + threadIdx.x, WAVE);
  ok[i] = f ? 1 : 0;
}

__global__ __launch_bounds__(64) void path_query_kernel(KParams P, KState S, const int8_t *types,
                                                        const int16_t *st, const int16_t *tg,
                                                        long long n, uint8_t *out) {
  __shared__ uint32_t open[OPEN_CAP * WAVE];
  long long i = (long long)blockIdx.x * WAVE + threadIdx.x;
  if (i >= n) return;
  out[i] = check_path_h(P, S, types[i], st[2 * i], st[2 * i + 1], tg[2 * i], tg[2 * i + 1],
                        open + threadIdx.x, WAVE) ? 1 : 0;
}

__global__ void los_query_kernel(KParams P, KState S, const int16_t *pairs, long long n,
                                 uint8_t *out) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  out[i] = (uint8_t)los_q(P, S, S.mask2, pairs[4 * i], pairs[4 * i + 1], pairs[4 * i + 2],
                          pairs[4 * i + 3]);
}

__global__ void fill_uniform_kernel(float *out, long long n, unsigned long long seed,
                                    unsigned long long offset) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  long long base = i * 4;
  if (base >= n) return;
  unsigned long long ctr = (offset >> 2) + (unsigned long long)i;
  uint32_t o[4] = {(uint32_t)ctr, (uint32_t)(ctr >> 32), 0x243F6A88u, 0x85A308D3u};
  philox10(o, (uint32_t)seed, (uint32_t)(seed >> 32));
#pragma unroll
  for (int k = 0; k < 4; k++)
    if (base + k < n) out[base + k] = (float)(o[k] >> 8) * 5.9604644775390625e-08f;
}

// ===========================================================================
// host side
// ===========================================================================
thread_local std::string g_err;

int fail(int code, const std::string &msg) {
  g_err = msg;
  return code;
}

#define HIPCHK(expr)                                                                  \
  do {                                                                                \
    hipError_t _e = (expr);                                                           \
    if (_e != hipSuccess)                                                             \
      return fail(LNW_EDEVICE, std::string(#expr) + ": " + hipGetErrorString(_e));    \
  } while (0)

void host_constants(KParams &k) {
  const double base = std::sqrt((4.0 / 3.0) * 6370.0 * 2.0);
  const int masts[2] = {15, 30};
  for (int i = 0; i < 2; i++)
    for (int j = 0; j < 2; j++) {
      double d = base * (std::sqrt((double)masts[i] / 1000.0) + std::sqrt((double)masts[j] / 1000.0));
      k.d5[i][j] = d / 5.0;
    }
  for (int i = 0; i < 2; i++)
    k.den[i] = (base * (std::sqrt((double)masts[i] / 1000.0) + std::sqrt(15.0 / 1000.0))) / 5.0;
  k.det_q[0] = 0.345 - 0.1;
  k.det_q[1] = 0.345 + 0.1;
  const double ps[2] = {0.45, 0.63};
  for (int h = 0; h < 2; h++)
    for (int n = 0; n < 9; n++) {
      k.hit64[h][n] = 1.0 - std::pow(1.0 - ps[h], (double)n);
      float pn = powf((float)(1.0 - ps[h]), (float)n);
      k.hit32[h][n] = 1.0f - pn;
    }
}

}  // namespace

struct lnw_handle {
  int device = 0;
  lnw_params params{};
  KParams kp{};
  int E = 0, nb = 0, nr = 0, A = 0, T = 0, nmax = 0;
  long long env_base = 0;
  int G = 0, W16 = 0;
  bool terrain = false;
  // device buffers
  uint8_t *d_grid = nullptr;
  float *d_gridf = nullptr, *d_winf = nullptr, *d_dummy = nullptr;
  unsigned long long *d_prof = nullptr;  // LNW_PROF phase timestamps
  size_t prof_cap = 0;                   // d_prof capacity in slots (grown to the launch grid)
  lnw_analytics ana{};                   // bound analytics buffers (lnw_set_analytics)
  unsigned long long *ctr = nullptr;     // bound work counters (lnw_set_counters)
  // diagnostics knobs, read once at lnw_create (LNW_DEBUG_SKIP / LNW_PROF / LNW_FORCE_GENERIC)
  int dbg_skip = 0;
  bool prof = false, force_generic = false, no_group = false, group_fits = false, no_units = false;
  bool no_slab = false;  // LNW_NO_SLAB: no two-slab direct rows (A/B)
  bool force_group = false;  // LNW_FORCE_GROUP (A/B): the group kernel for templated team sizes too
  bool no_split_rows = false;  // LNW_NO_SPLIT_ROWS (A/B): row-writing contact steps keep phase S on one wave
  bool store_wt = false;
  bool units_fit = false;  // UNITS blocks of the step layout fit one workgroup (lnw_load_terrain)
  bool contact = false;  // lnw_set_variant: contact-heavy phase-S code in the templated kernels
  int last_kernel = LNW_KERNEL_NONE;     // lnw_step_kernel: what the last lnw_step launched
  bool has_medium = false;               // the spawn spec has medium ships (runtime-size kernels only)
  unsigned long long terrain_hash = 0;   // FNV-1a of the loaded grid (state snapshots name their terrain)
  uint32_t *d_mask2 = nullptr, *d_mvtab = nullptr, *d_lostab = nullptr;
  uint32_t *pos = nullptr;
  int32_t *radar = nullptr, *steps = nullptr, *envi = nullptr;
  uint8_t *miss = nullptr, *mkind = nullptr, *alive = nullptr, *type = nullptr;
  double *dist_lz = nullptr, *duct = nullptr, *bear_val = nullptr, *d_atan = nullptr;
  uint8_t *bear_ship = nullptr;
  uint16_t *tl_cnt = nullptr, *tl = nullptr;
  unsigned long long *rng = nullptr;
  uint32_t *err = nullptr;
  int32_t *sp_types = nullptr, *sp_pos = nullptr, *sp_randls = nullptr, *sp_pos_env = nullptr;
  bool sp_pos_env_on = false;  // auto-reset respawns on the per-env cells of the last lnw_reset
  const double *tape = nullptr;
  const long long *tape_off = nullptr;
  std::vector<void *> allocs;
};

namespace {

template <class T>
int dalloc(lnw_handle *h, T **p, size_t n) {
  void *q = nullptr;
  hipError_t e = hipMalloc(&q, n * sizeof(T) + 16);
  if (e != hipSuccess) return fail(LNW_ENOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
  (void)hipMemset(q, 0, n * sizeof(T) + 16);
  h->allocs.push_back(q);
  *p = (T *)q;
  return 0;
}

KState make_state(lnw_handle *h) {
  KState s{};
  s.pos = h->pos; s.radar = h->radar; s.miss = h->miss; s.mkind = h->mkind; s.alive = h->alive;
  s.type = h->type; s.steps = h->steps; s.dist_lz = h->dist_lz; s.tl_cnt = h->tl_cnt; s.tl = h->tl;
  s.duct = h->duct; s.envi = h->envi; s.rng = h->rng; s.err = h->err;
  s.bear_val = h->bear_val; s.bear_ship = h->bear_ship; s.atan_deg = h->d_atan;
  s.grid = h->d_grid; s.gridf = h->d_gridf; s.winf = h->d_winf; s.dummy = h->d_dummy; s.prof = nullptr; s.ana = h->ana; s.ctr = h->ctr; s.mask2 = h->d_mask2; s.mvtab = h->d_mvtab; s.lostab = h->d_lostab;
  s.tape = h->tape; s.tape_off = h->tape_off;
  s.sp_types = h->sp_types; s.sp_pos = h->sp_pos; s.sp_randls = h->sp_randls;
  s.sp_pos_env = h->sp_pos_env_on ? h->sp_pos_env : nullptr;
  s.nmax = h->nmax;
  return s;
}

size_t step_lds_bytes(const lnw_handle *h) {
  LdsLayout L = lds_layout(h->A, h->nb, h->nr, h->nmax, h->G * h->W16, h->G);
  return (size_t)L.total;
}

// the step launch's LDS: step_lds_bytes plus the whole-side row stages of
// small quiet workgroups (the same condition step_kernel evaluates)
// compute units of the handle's device (cached per device)
int device_ncu(int dev) {
  static int cache[64] = {0};
  int &c = cache[dev & 63];
  if (c == 0) {
    int n = 0;
    c = hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0 ? n : 256;
  }
  return c;
}

// Quiet workgroups' direct rows (quiet_step_t): a workgroup of up to 64 / nb envs
// stages both sides' rows whole (qbig) and wave 1 builds and stores every row
// from registers; up to 128 / nb envs it does so in two slabs of 64 / nb envs,
// for the non-contact kernels and only when the larger LDS still holds the whole
// grid at once (config 3 at N = 4: 16 384 envs, 32 per workgroup). Larger
// workgroups stream their rows in staged passes (quiet_emit_t).
bool step_qdirect(const lnw_handle *h, int epw) {
  const bool tmpl = !h->force_generic && !h->has_medium && h->params.los_mode == 0 && h->nb == h->nr &&
                    h->nb >= 2 && h->nb <= 4 && EPW == WAVE;
  if (!tmpl) return false;
  if (epw * h->nb <= WAVE) return true;
  // (4v4 only: step_kernel<4, 4, .., SL> is the one two-slab instantiation)
  if (h->nb != 4 || h->contact || h->no_slab || epw * h->nb > 2 * WAVE) return false;
  const LdsLayout L = lds_layout(h->A, h->nb, h->nr, h->nmax, h->G * h->W16, h->G, WAVE);
  int per_cu = (int)((160 * 1024) / ((size_t)L.total + 1024));
  if (per_cu > 4) per_cu = 4;  // 256 VGPRs: two waves per SIMD
  return (h->E + epw - 1) / epw <= (long long)device_ncu(h->device) * per_cu;
}

size_t step_launch_lds_bytes(const lnw_handle *h, int epw) {
  const int rows = step_qdirect(h, epw) ? (epw * h->nb < WAVE ? epw * h->nb : WAVE) : 0;
  LdsLayout L = lds_layout(h->A, h->nb, h->nr, h->nmax, h->G * h->W16, h->G, rows);
  return (size_t)L.total;
}

// Environments per workgroup: EPW (one env per lane) unless that leaves the GPU
// with fewer workgroups than it can hold at once; then halve it (down to 16 for
// the two-wave kernels, 1 otherwise) until the grid fills every resident slot. A step is a per-lane latency chain, so a
// workgroup with fewer live lanes takes about as long as a full one, and more
// workgroups in flight finish the batch in fewer rounds (config 4: 8 192 envs
// -> 512 workgroups of 16 instead of 128 of 64). LNW_EPW_RT overrides.
int choose_epw(const lnw_handle *h) {
  if (const char *e = getenv("LNW_EPW_RT")) {
    int v = atoi(e);
    if (v >= 1 && v <= EPW) return v;
  }
  int ncu = 256;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, h->device) == hipSuccess && prop.multiProcessorCount > 0)
    ncu = prop.multiProcessorCount;
  const bool two_wave = !h->force_generic && h->params.los_mode != 2 && h->nb == h->nr && h->nb >= 2 && h->nb <= 4 && EPW == WAVE;
  const int by_waves = two_wave ? 4 : 8;  // 256 VGPRs: two waves per SIMD
  // resident workgroups at a given epw (the launch's LDS depends on it: small
  // quiet workgroups carry whole-side row stages)
  auto slots = [&](int e) {
    const size_t lds = step_launch_lds_bytes(h, e) + 1024;
    int per_cu = (int)((160 * 1024) / lds);
    if (per_cu > by_waves) per_cu = by_waves;
    if (per_cu < 1) per_cu = 1;
    return (long long)ncu * per_cu;
  };
  // two-wave kernels stop at 16 envs per workgroup: below that each workgroup's
  // fixed head (terrain mask staging, state columns) outweighs the shorter
  // chain (8 192 envs: 20.2 us at 16, 20.5 at 8, 22.3 at 32, 29.0 at 64)
  const int min_epw = two_wave ? 16 : 1;
  int epw = EPW;
  while (epw > min_epw && (h->E + epw - 1) / epw < slots(epw)) epw /= 2;
  if ((h->E + epw - 1) / epw > slots(epw) && epw < EPW) epw *= 2;  // never more rounds than EPW needs
  return epw;
}

}  // namespace

// LNW_PROF diagnostics: mean per-workgroup phase spans and the grid-wide
// start / end spread of one step launch (synchronises the stream).
void prof_report(lnw_handle *h, hipStream_t st, int nwg) {
  std::vector<unsigned long long> t((size_t)nwg * PROF_SLOTS);
  if (hipMemcpyAsync(t.data(), h->d_prof, t.size() * 8, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)
    return;
  double sL = 0, sM = 0, sS = 0, sW = 0, s1 = 0, sa[8] = {0}, sq[4] = {0}, sp[4] = {0}, sg[4] = {0},
         st3[3] = {0, 0, 0};
  int nq = 0;
  unsigned long long t0 = ~0ull, tend0 = 0, tend1 = 0;
  int n1 = 0;
  for (int w = 0; w < nwg; w++) {
    const unsigned long long *r = &t[(size_t)w * PROF_SLOTS];
    sL += (double)(r[4] - r[0]);
    sM += (double)(r[1] - r[4]);
    sS += (double)(r[2] - r[1]);
    sW += (double)(r[3] - r[2]);
    if (r[5]) { s1 += (double)(r[5] - r[0]); n1++; if (r[5] > tend1) tend1 = r[5]; }
    for (int q = 0; q < 4; q++) sp[q] += (double)r[16 + q];
    for (int q = 0; q < 4; q++) sg[q] += (double)r[20 + q];
    if (r[14]) {  // quiet workgroup: M end | A* + barrier | predicate | phase Q + barrier
      nq++;
      sq[0] += (double)(r[6] - r[4]);
      sq[1] += (double)(r[7] - r[6]);
      sq[2] += (double)(r[8] - r[7]);
      sq[3] += (double)(r[9] - r[8]);
      if (r[10] && r[11]) {  // tail: rewards | cog | env_tail + outputs
        st3[0] += (double)(r[10] - r[1]);
        st3[1] += (double)(r[11] - r[10]);
        st3[2] += (double)(r[2] - r[11]);
      }
    } else {
      for (int a = 0; a < 8; a++)
        if (r[6 + a]) sa[a] += (double)(r[6 + a] - (a ? r[5 + a] : r[1]));
    }
    if (r[0] < t0) t0 = r[0];
    if (r[3] > tend0) tend0 = r[3];
  }
  const double us = 0.01;  // 100 MHz ticks
  {  // spread of the per-workgroup phase-S spans (slot 1 -> 2)
    std::vector<double> sv;
    for (int w = 0; w < nwg; w++) {
      const unsigned long long *r = &t[(size_t)w * PROF_SLOTS];
      if (r[2] > r[1]) sv.push_back((double)(r[2] - r[1]) * 0.01);
    }
    {  // the slowest workgroup's parts (slots 16..23)
      int wm = -1;
      double best = -1;
      for (int w = 0; w < nwg; w++) {
        const unsigned long long *r = &t[(size_t)w * PROF_SLOTS];
        if (r[2] > r[1] && (double)(r[2] - r[1]) > best) { best = (double)(r[2] - r[1]); wm = w; }
      }
      if (wm >= 0) {
        const unsigned long long *r = &t[(size_t)wm * PROF_SLOTS];
        fprintf(stderr, "[lnw prof] slowest workgroup %d: S %.1f us = take_action %.1f, LOS prefetch %.1f, get_obs %.1f "
                        "(walk %.1f, observed %.1f, bearings %.1f, fix targets %.1f), reward %.1f\n",
                wm, best * 0.01, r[16] * 0.01, r[17] * 0.01, r[18] * 0.01, r[20] * 0.01, r[21] * 0.01,
                r[22] * 0.01, r[23] * 0.01, r[19] * 0.01);
      }
    }
    std::sort(sv.begin(), sv.end());
    if (!sv.empty())
      fprintf(stderr, "[lnw prof] phase S span per workgroup: p10 %.1f, p50 %.1f, p90 %.1f, max %.1f us\n",
              sv[sv.size() / 10], sv[sv.size() / 2], sv[sv.size() * 9 / 10], sv.back());
  }
  fprintf(stderr, "[lnw prof] wg=%d mean L %.2f us, M %.2f us, S %.2f us, W %.2f us, wave1 end-from-start %.2f us; "
                  "grid: last wave0 end %.2f us, last wave1 end %.2f us after first start\n",
          nwg, sL / nwg * us, sM / nwg * us, sS / nwg * us, sW / nwg * us, n1 ? s1 / n1 * us : 0.0,
          (double)(tend0 - t0) * us, tend1 ? (double)(tend1 - t0) * us : 0.0);
  {
    double bs = 0, bm = 0, bl = 0;
    for (int w = 0; w < nwg; w++) {
      const unsigned long long *r = &t[(size_t)w * PROF_SLOTS];
      bs += (double)r[24]; bm += (double)r[25]; bl += (double)r[26];
    }
    if (bl > 0)
      fprintf(stderr, "[lnw prof] EW bearings (contact variant): %.0f evaluated, wave max summed %.0f, "
                      "active lanes %.0f; balanced/actual %.3f\n",
              bs, bm, bl, bs / 64.0 / bm);
  }
  {  // grid timeline: workgroup start (slot 0), stream / phase S start (slot 1),
     // wave-1 end (slot 5), each as p10 / p50 / p90 / max after the first start
    const int slots[3] = {0, 1, 5};
    const char *names[3] = {"start", "S/stream start", "wave-1 end"};
    for (int k = 0; k < 3; k++) {
      std::vector<double> sv;
      for (int w = 0; w < nwg; w++) {
        const unsigned long long v = t[(size_t)w * PROF_SLOTS + slots[k]];
        if (v >= t0) sv.push_back((double)(v - t0) * us);
      }
      std::sort(sv.begin(), sv.end());
      if (!sv.empty())
        fprintf(stderr, "[lnw prof] timeline %s: p10 %.2f, p50 %.2f, p90 %.2f, max %.2f us\n", names[k],
                sv[sv.size() / 10], sv[sv.size() / 2], sv[sv.size() * 9 / 10], sv.back());
    }
  }
  {  // wave-1 end (slot 5) per XCC: count, mean, max after the first start
    double se[16] = {0}, mx[16] = {0};
    int nx[16] = {0};
    for (int w = 0; w < nwg; w++) {
      const unsigned long long *r = &t[(size_t)w * PROF_SLOTS];
      if (!r[5] || r[5] < t0) continue;
      const int x = (int)(r[30] & 15);
      const double e = (double)(r[5] - t0) * us;
      se[x] += e; nx[x]++;
      if (e > mx[x]) mx[x] = e;
    }
    {  // per CU (XCC, SE, SH, CU from HW_ID bits 15:8): spread of CU means vs within-CU spread
      std::vector<std::pair<int, double>> v;
      for (int w = 0; w < nwg; w++) {
        const unsigned long long *r = &t[(size_t)w * PROF_SLOTS];
        if (!r[5] || r[5] < t0) continue;
        v.push_back({(int)((r[30] & 15) << 8 | ((r[31] >> 8) & 0xff)), (double)(r[5] - t0) * us});
      }
      std::sort(v.begin(), v.end());
      std::vector<double> means, spans;
      for (size_t i = 0; i < v.size();) {
        size_t j = i;
        double sm = 0, lo = 1e30, hi = -1e30;
        while (j < v.size() && v[j].first == v[i].first) { sm += v[j].second; lo = std::min(lo, v[j].second); hi = std::max(hi, v[j].second); j++; }
        means.push_back(sm / (double)(j - i));
        spans.push_back(hi - lo);
        i = j;
      }
      std::sort(means.begin(), means.end());
      std::sort(spans.begin(), spans.end());
      if (!means.empty())
        fprintf(stderr, "[lnw prof] CUs %zu: CU-mean wave-1 end p10 %.1f p50 %.1f p90 %.1f max %.1f; within-CU span p50 %.1f p90 %.1f max %.1f us\n",
                means.size(), means[means.size() / 10], means[means.size() / 2], means[means.size() * 9 / 10], means.back(),
                spans[spans.size() / 2], spans[spans.size() * 9 / 10], spans.back());
    }
    {  // SIMD placement: wave 0 (phase S) sharing its SIMD with another workgroup's wave 0
      std::vector<int> key(nwg);
      for (int w = 0; w < nwg; w++) {
        const unsigned long long *r = &t[(size_t)w * PROF_SLOTS];
        key[w] = (int)((r[30] & 15) << 12 | ((r[31] >> 8) & 0xff) << 4 | ((r[31] >> 4) & 3));
      }
      std::vector<int> sk = key;
      std::sort(sk.begin(), sk.end());
      double e0[2] = {0, 0}, m0[2] = {0, 0};
      int n0[2] = {0, 0}, same = 0;
      for (int w = 0; w < nwg; w++) {
        const unsigned long long *r = &t[(size_t)w * PROF_SLOTS];
        const int cnt = (int)(std::upper_bound(sk.begin(), sk.end(), key[w]) - std::lower_bound(sk.begin(), sk.end(), key[w]));
        const int k = cnt > 1 ? 1 : 0;
        if (r[3] < t0) continue;
        const double e = (double)(r[3] - t0) * us;
        e0[k] += e; n0[k]++;
        if (e > m0[k]) m0[k] = e;
        same += ((r[31] >> 4) & 3) == ((r[29] >> 4) & 3);
      }
      fprintf(stderr, "[lnw prof] wave-0 SIMD: alone %d (end mean %.1f max %.1f us), shared %d (mean %.1f max %.1f us); "
                      "waves 0/1 on one SIMD in %d workgroups\n",
              n0[0], n0[0] ? e0[0] / n0[0] : 0.0, m0[0], n0[1], n0[1] ? e0[1] / n0[1] : 0.0, m0[1], same);
    }
    fprintf(stderr, "[lnw prof] wave-1 end by XCC (n/mean/max us):");
    for (int x = 0; x < 16; x++)
      if (nx[x]) fprintf(stderr, " %d:%d/%.1f/%.1f", x, nx[x], se[x] / nx[x], mx[x]);
    fprintf(stderr, "; block%%8==xcc for %d of %d\n",
            [&] { int k = 0; for (int w = 0; w < nwg; w++) k += (int)(t[(size_t)w * PROF_SLOTS + 30] & 15) == (w & 7); return k; }(), nwg);
  }
  {
    double rq = 0;
    int nr2 = 0;
    for (int w = 0; w < nwg; w++) {
      const unsigned long long *r = &t[(size_t)w * PROF_SLOTS];
      if (r[14] && r[12] > r[8] && r[8]) { rq += (double)(r[12] - r[8]); nr2++; }
    }
    if (nr2) fprintf(stderr, "[lnw prof] repeated quiet test (diagnostics): %.2f us\n", rq / nr2 * us);
  }
  {  // quiet small workgroups (direct mode): each wave's phase-Q work from the
     // test's end (slots 27 / 15), wave 1's rows staged (28) and stored (5)
     // from the barrier (9)
    double q0 = 0, q1 = 0, rb = 0, rc = 0;
    int nd = 0;
    for (int w = 0; w < nwg; w++) {
      const unsigned long long *r = &t[(size_t)w * PROF_SLOTS];
      if (!r[14] || !r[28] || !r[15] || !r[27] || r[28] < r[9]) continue;
      nd++;
      q0 += (double)(r[27] - r[8]);
      q1 += (double)(r[15] - r[8]);
      rb += (double)(r[28] - r[9]);
      rc += (double)(r[5] - r[28]);
    }
    if (nd)
      fprintf(stderr, "[lnw prof] quiet direct %d: phase-Q work wave 0 %.2f, wave 1 %.2f us; after the barrier "
                      "rows staged %.2f, stored %.2f us\n",
              nd, q0 / nd * us, q1 / nd * us, rb / nd * us, rc / nd * us);
  }
  if (nq)
    fprintf(stderr, "[lnw prof] quiet workgroups %d: M %.2f us, A*+barrier %.2f us, quiet test %.2f us, Q+barrier %.2f us; "
                    "tail: rewards %.2f, cog %.2f, env_tail+outputs %.2f us\n",
            nq, sq[0] / nq * us, sq[1] / nq * us, sq[2] / nq * us, sq[3] / nq * us, st3[0] / nq * us,
            st3[1] / nq * us, st3[2] / nq * us);
  const int ns = nwg - nq;
  fprintf(stderr, "[lnw prof] phase S workgroups %d, per agent (us):", ns);
  for (int a = 0; a < 8; a++) fprintf(stderr, " %.2f", ns ? sa[a] / ns * us : 0.0);
  fprintf(stderr, "; section totals take_action %.2f, LOS prefetch %.2f, get_obs %.2f, reward %.2f us\n",
          ns ? sp[0] / ns * us : 0.0, ns ? sp[1] / ns * us : 0.0, ns ? sp[2] / ns * us : 0.0,
          ns ? sp[3] / ns * us : 0.0);
  fprintf(stderr, "[lnw prof] get_obs parts (templated): pair walk %.2f, observed stores %.2f, bearings+fixes %.2f, fix targets %.2f us\n",
          ns ? sg[0] / ns * us : 0.0, ns ? sg[1] / ns * us : 0.0, ns ? sg[2] / ns * us : 0.0,
          ns ? sg[3] / ns * us : 0.0);
}

extern "C" {

int lnw_abi_version(void) { return LNW_ABI_VERSION; }
const char *lnw_last_error(void) { return g_err.c_str(); }

int lnw_set_analytics(lnw_handle *h, const lnw_analytics *a) {
  if (!h) return fail(LNW_EINVAL, "null handle");
  if (!a) { h->ana = lnw_analytics{}; return 0; }
  if ((a->eng_log && (!a->eng_count || a->eng_cap < 0)) || (a->ew_log && (!a->ew_count || a->ew_cap < 0)))
    return fail(LNW_EINVAL, "analytics log without a counter or with a negative capacity");
  h->ana = *a;
  return 0;
}

int lnw_hit_tables(double *tab64, float *tab32) {
  KParams k{};
  host_constants(k);
  for (int h = 0; h < 2; h++)
    for (int n = 0; n < 9; n++) {
      if (tab64) tab64[h * 9 + n] = k.hit64[h][n];
      if (tab32) tab32[h * 9 + n] = k.hit32[h][n];
    }
  return 0;
}

int lnw_create(const lnw_params *params, int32_t n_envs, int32_t nb, int32_t nr, int32_t device,
               int64_t env_id_base, lnw_handle **out) {
  if (!params || !out) return fail(LNW_EINVAL, "null argument");
  if (n_envs <= 0) return fail(LNW_EINVAL, "n_envs must be > 0");
  if (nb < 1 || nr < 1 || nb > 16 || nr > 16)
    return fail(LNW_EUNSUPPORTED, "need 1 <= nb, nr <= 16 ships per side");
  HIPCHK(hipSetDevice(device));
  lnw_handle *h = new lnw_handle();
  h->device = device;
  if (const char *dbg = getenv("LNW_DEBUG_SKIP")) h->dbg_skip = atoi(dbg);
#ifndef LNW_DIAG
  // the shipped library honours only the knobs that change the launch shape or
  // code path, never the results (bit 9: no quiet path, 15: the group kernel's
  // fire loop entry by entry, 17: per-lane bearing loop, 22/23: where the
  // head's loads are issued, 28: the per-env quiet test in small workgroups,
  // 29: their env counters loaded in phase Q); section skips and
  // replaced arithmetic exist only in the diagnostics build (-DLNW_DIAG,
  // lnw.build.build_diag)
  constexpr int kResultPreserving = 512 | 32768 | 131072 | 4194304 | 8388608 | (1 << 28) | (1 << 29);
  if (h->dbg_skip & ~kResultPreserving) {
    const int bad = h->dbg_skip & ~kResultPreserving;
    delete h;
    return fail(LNW_EINVAL, "LNW_DEBUG_SKIP bits " + std::to_string(bad) +
                                " change results; they exist only in the diagnostics build (-DLNW_DIAG)");
  }
#endif
  h->prof = getenv("LNW_PROF") != nullptr;
  h->force_generic = getenv("LNW_FORCE_GENERIC") != nullptr;
  // LNW_NO_GROUP: runtime team sizes on the one-lane-per-env kernel (A/B tests)
  h->no_group = getenv("LNW_NO_GROUP") != nullptr;
  h->force_group = getenv("LNW_FORCE_GROUP") != nullptr;
  h->no_split_rows = getenv("LNW_NO_SPLIT_ROWS") != nullptr;
  // LNW_NO_UNITS: one 64-env unit per workgroup for the headline shape (A/B tests)
  h->no_units = getenv("LNW_NO_UNITS") != nullptr;
  h->no_slab = getenv("LNW_NO_SLAB") != nullptr;
  h->kp.xcd_remap = getenv("LNW_NO_XCD_REMAP") == nullptr ? 1 : 0;
  // LNW_GROUP_MARCH=1: the group kernel marches its pair LOS over the LDS
  // terrain mask instead of loading LOS-table words (A/B)
  h->kp.group_march = getenv("LNW_GROUP_MARCH") != nullptr ? 1 : 0;
  // write-through observation stores (st_obs4) while a side's output fits the
  // 32-bit buffer offsets; LNW_NO_STORE_WT keeps non-temporal stores (A/B)
  {
    const int ns = nb > nr ? nb : nr;
    const double side_bytes = (double)n_envs * ns * (4 * ns + 52) * 4.0;
    h->store_wt = getenv("LNW_NO_STORE_WT") == nullptr && side_bytes < 2147483648.0;
  }
  h->params = *params;
  h->E = n_envs; h->nb = nb; h->nr = nr; h->A = nb + nr;
  h->nmax = nb > nr ? nb : nr;
  h->T = h->nmax + h->nmax * h->nmax;
  h->env_base = env_id_base;
  const size_t E = (size_t)n_envs, A = (size_t)h->A;
  int rc = 0;
  rc |= dalloc(h, &h->pos, A * E);
  rc |= dalloc(h, &h->radar, A * E);
  rc |= dalloc(h, &h->miss, A * E);
  rc |= dalloc(h, &h->mkind, A * E);
  rc |= dalloc(h, &h->alive, A * E);
  rc |= dalloc(h, &h->type, A * E);
  rc |= dalloc(h, &h->steps, A * E);
  rc |= dalloc(h, &h->dist_lz, A * E);
  rc |= dalloc(h, &h->tl_cnt, A * E);
  rc |= dalloc(h, &h->tl, A * (size_t)h->T * E);
  rc |= dalloc(h, &h->duct, E);
  rc |= dalloc(h, &h->envi, 8 * E);
  rc |= dalloc(h, &h->rng, E);
  rc |= dalloc(h, &h->err, E);
  rc |= dalloc(h, &h->bear_val, (size_t)h->nmax * h->nmax * E);
  rc |= dalloc(h, &h->bear_ship, (size_t)h->nmax * h->nmax * E);
  rc |= dalloc(h, &h->sp_types, 64);
  rc |= dalloc(h, &h->sp_pos, 128);
  rc |= dalloc(h, &h->sp_randls, 64);
  rc |= dalloc(h, &h->d_dummy, 4 * 64);
  rc |= dalloc(h, &h->d_atan, (size_t)LOS_W * LOS_W);
  if (rc) {
    std::string m = g_err;
    lnw_destroy(h);
    return fail(LNW_ENOMEM, m);
  }
  {  // EW bearing table: math.degrees(math.atan2(dy, dx)) for integer offsets in
     // [-R_LOS, R_LOS]^2, computed by the host libm as the reference does
     // (combatant.py:253), so the device needs no atan2 of its own in range
    std::vector<double> at((size_t)LOS_W * LOS_W);
    for (int dy = -R_LOS; dy <= R_LOS; dy++)
      for (int dx = -R_LOS; dx <= R_LOS; dx++)
        at[(size_t)(dy + R_LOS) * LOS_W + (dx + R_LOS)] = atan2((double)dy, (double)dx) * (180.0 / PY_PI);
    HIPCHK(hipMemcpy(h->d_atan, at.data(), at.size() * sizeof(double), hipMemcpyHostToDevice));
    // odd in dy (glibc's atan2 is; checked, not assumed): the group kernel then
    // keeps only the dy >= 0 rows in LDS and negates for dy < 0
    bool odd = true;
    for (int dy = 1; dy <= R_LOS; dy++)
      for (int dx = -R_LOS; dx <= R_LOS; dx++)
        odd = odd && at[(size_t)(R_LOS - dy) * LOS_W + (dx + R_LOS)] == -at[(size_t)(R_LOS + dy) * LOS_W + (dx + R_LOS)];
    h->kp.atan_odd = odd ? 1 : 0;
  }
  KParams &k = h->kp;
  k.discrete = params->discrete; k.landing_ops = params->landing_ops;
  k.aggressive = params->aggressive; k.side_blue = params->side_blue;
  k.trained_red = params->trained_red; k.move_thr = params->move_thr; k.ew_thr = params->ew_thr;
  k.lz_x = params->lz_x; k.lz_y = params->lz_y; k.red_aggression = params->red_aggression;
  k.episode_steps = params->episode_steps; k.auto_reset = params->auto_reset;
  k.los_mode = params->los_mode; k.move_mode = params->move_mode;
  k.E = n_envs; k.nb = nb; k.nr = nr; k.A = h->A; k.T = h->T;
  k.env_base = env_id_base;
  k.rng_mode = LNW_RNG_PHILOX;
  k.seed = 0;
  k.epw = EPW;  // refined by lnw_load_terrain (choose_epw) once the LDS size is known
  k.wc[0] = k.wc[1] = 49;  // 7x7 windows until a reset spawns a side of medium ships
  host_constants(k);
  *out = h;
  return 0;
}

int lnw_destroy(lnw_handle *h) {
  if (!h) return 0;
  (void)hipSetDevice(h->device);
  (void)hipDeviceSynchronize();
  for (void *p : h->allocs) (void)hipFree(p);
  if (h->d_prof) (void)hipFree(h->d_prof);
  delete h;
  return 0;
}

int lnw_load_terrain(lnw_handle *h, const uint8_t *grid_host, int32_t G) {
  if (!h || !grid_host) return fail(LNW_EINVAL, "null argument");
  if (G < 8 || G > 1024) return fail(LNW_EINVAL, "grid size out of range");
  HIPCHK(hipSetDevice(h->device));
  h->G = G;
  h->W16 = (G + 15) / 16;
  int rc = 0;
  if (h->d_grid) {  // re-load: release the previous terrain structures
    HIPCHK(hipDeviceSynchronize());
    void *old[6] = {h->d_grid, h->d_gridf, h->d_winf, h->d_mask2, h->d_mvtab, h->d_lostab};
    for (void *p : old) {
      for (size_t i = 0; i < h->allocs.size(); i++)
        if (h->allocs[i] == p) { (void)hipFree(p); h->allocs.erase(h->allocs.begin() + i); break; }
    }
  }
  rc |= dalloc(h, &h->d_grid, (size_t)G * G);
  rc |= dalloc(h, &h->d_gridf, (size_t)G * G);
  rc |= dalloc(h, &h->d_winf, (size_t)3 * G * G * 52);
  rc |= dalloc(h, &h->d_mask2, (size_t)G * h->W16);
  rc |= dalloc(h, &h->d_mvtab, (size_t)MV_CLASSES * G * G * MV_WORDS);
  rc |= dalloc(h, &h->d_lostab, (size_t)G * G * LOS_CELL_WORDS);
  if (rc) return rc;
  HIPCHK(hipMemcpy(h->d_grid, grid_host, (size_t)G * G, hipMemcpyHostToDevice));
  {
    unsigned long long fh = 1469598103934665603ull ^ (unsigned long long)G;
    for (size_t i = 0; i < (size_t)G * G; i++) fh = (fh ^ grid_host[i]) * 1099511628211ull;
    h->terrain_hash = fh;
  }
  {  // observation window values grid/255 (combatant.py:177), float64 quotient -> float32
    std::vector<float> gf((size_t)G * G);
    for (size_t i = 0; i < gf.size(); i++) gf[i] = (float)((double)grid_host[i] / 255.0);
    HIPCHK(hipMemcpy(h->d_gridf, gf.data(), gf.size() * sizeof(float), hipMemcpyHostToDevice));
    // per-cell observation windows, one 52-float (13 x float4) record per cell
    // and class: [0] Combatant 7x7 around the ship (49 floats), [1] LandingShip
    // 5x5 rows/cols pos-1..pos+3 (25 floats), [2] medium Combatant 5x5 around
    // the ship (speed 2: combatant.py:165-181); cells outside the hard-coded
    // 0..99 are 0 (combatant.py:176, landingship.py:183)
    std::vector<float> wf((size_t)3 * G * G * 52, 0.0f);
    auto cellv = [&](int x, int y) {
      return (0 <= x && x < 100 && 0 <= y && y < 100 && x < G && y < G) ? gf[(size_t)x * G + y] : 0.0f;
    };
    for (int x = 0; x < G; x++)
      for (int y = 0; y < G; y++) {
        float *w7 = &wf[((size_t)x * G + y) * 52];
        for (int i = 0; i < 7; i++)
          for (int j = 0; j < 7; j++) w7[i * 7 + j] = cellv(x - 3 + i, y - 3 + j);
        float *w5 = &wf[((size_t)G * G + (size_t)x * G + y) * 52];
        for (int i = 0; i < 5; i++)
          for (int j = 0; j < 5; j++) w5[i * 5 + j] = cellv(x - 1 + i, y - 1 + j);
        float *wm = &wf[((size_t)2 * G * G + (size_t)x * G + y) * 52];
        for (int i = 0; i < 5; i++)
          for (int j = 0; j < 5; j++) wm[i * 5 + j] = cellv(x - 2 + i, y - 2 + j);
      }
    HIPCHK(hipMemcpy(h->d_winf, wf.data(), wf.size() * sizeof(float), hipMemcpyHostToDevice));
  }
  KParams &k = h->kp;
  k.G = G;
  k.W16 = h->W16;
  int n = G * h->W16;
  build_mask_kernel<<<(n + 255) / 256, 256>>>(h->d_grid, G, h->W16, k.move_thr, k.ew_thr, h->d_mask2);
  HIPCHK(hipGetLastError());
  long long nm = (long long)MV_CLASSES * G * G * MV_W * MV_W;
  build_move_table_kernel<<<(unsigned)((nm + WAVE - 1) / WAVE), WAVE>>>(h->d_mask2, G, h->W16, h->d_mvtab);
  HIPCHK(hipGetLastError());
  long long nl = (long long)G * G * LOS_W;
  const int mwords = G * h->W16 * 4 <= 64 * 1024 ? G * h->W16 : 0;  // terrain mask staged in LDS
  {  // a few resident rounds of workgroups, each looping over its items
    int ncu = 256;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, h->device) == hipSuccess && prop.multiProcessorCount > 0)
      ncu = prop.multiProcessorCount;
    const long long need = (nl + 255) / 256, cap = (long long)ncu * 8;
    build_los_table_kernel<<<(unsigned)(need < cap ? need : cap), 256, (size_t)mwords * 4>>>(
        h->d_mask2, G, h->W16, h->d_lostab, mwords);
  }
  HIPCHK(hipGetLastError());
  HIPCHK(hipDeviceSynchronize());
  h->terrain = true;
  // dynamic LDS above the 64 KiB default needs an explicit opt-in
  {
    // the largest step launch (64 / nb envs per workgroup: the biggest row stages)
    const size_t need = step_launch_lds_bytes(h, WAVE / h->nb);
    // the same bound the launch attribute below grants
    if (need > (size_t)GROUP_LDS_MAX) return fail(LNW_EUNSUPPORTED, "agent count needs more LDS than a CU has");
    const LdsLayout GLy = lds_layout(h->A, h->nb, h->nr, h->nmax, h->G * h->W16, h->G);
    const size_t gneed = (size_t)group_lds(GLy, h->G * h->W16, h->A, h->nb * h->nr, h->kp.atan_odd != 0).total + 1024;
    // (else runtime sizes stay on step_kernel<0, 0>)
    h->group_fits = group_lds(GLy, h->G * h->W16, h->A, h->nb * h->nr, h->kp.atan_odd != 0).ms >= 0;
    // the limit is per kernel function and device, shared by every handle of
    // the process on that device: set to GROUP_LDS_MAX once per device, so a
    // smaller handle never lowers it under a larger one's launch (the launch's
    // own size sets the occupancy); hipSetDevice(h->device) above selects it
    static unsigned long long lds_opt_in = 0;  // bit d: device d done
    const unsigned long long dbit = 1ull << (h->device & 63);
    const size_t uneed = (size_t)UNITS * ((step_lds_bytes(h) + 15) & ~(size_t)15);
    h->units_fit = uneed <= (size_t)UNITS_LDS_MAX;
    if (!(lds_opt_in & dbit) && (need > 64 * 1024 || gneed > 64 * 1024 || uneed > 64 * 1024)) {
      HIPCHK(hipFuncSetAttribute((const void *)step_kernel<4, 4, false, false, 1, false, true>,
                                 hipFuncAttributeMaxDynamicSharedMemorySize, GROUP_LDS_MAX));
      const void *ks[17] = {(const void *)step_kernel<4, 4, true, false, 1, true>,
                            (const void *)step_kernel<0, 0>,       (const void *)step_kernel<2, 2>,
                            (const void *)step_kernel<3, 3>,       (const void *)step_kernel<4, 4>,
                            (const void *)step_kernel<2, 2, true>, (const void *)step_kernel<3, 3, true>,
                            (const void *)step_kernel<4, 4, true>, (const void *)step_kernel<0, 0, false, true>,
                            (const void *)observe_kernel<0, 0, false>, (const void *)step_group_kernel,
                            (const void *)observe_kernel<2, 2, false>, (const void *)observe_kernel<3, 3, false>,
                            (const void *)observe_kernel<4, 4, false>, (const void *)observe_kernel<2, 2, true>,
                            (const void *)observe_kernel<3, 3, true>, (const void *)observe_kernel<4, 4, true>};
      for (const void *kk : ks)
        HIPCHK(hipFuncSetAttribute(kk, hipFuncAttributeMaxDynamicSharedMemorySize, GROUP_LDS_MAX));
      HIPCHK(hipFuncSetAttribute((const void *)step_kernel<4, 4, false, false, UNITS>,
                                 hipFuncAttributeMaxDynamicSharedMemorySize, UNITS_LDS_MAX));
      lds_opt_in |= dbit;
    }
  }
  (void)hipGetLastError();
  h->kp.epw = choose_epw(h);
  return 0;
}

int lnw_set_rng(lnw_handle *h, int32_t mode, uint64_t seed, const double *tape_dev,
                const int64_t *tape_off_dev) {
  if (!h) return fail(LNW_EINVAL, "null handle");
  if (mode != LNW_RNG_PHILOX && mode != LNW_RNG_TAPE) return fail(LNW_EINVAL, "bad rng mode");
  if (mode == LNW_RNG_TAPE && (!tape_dev || !tape_off_dev))
    return fail(LNW_EINVAL, "tape mode needs tape and offsets");
  HIPCHK(hipSetDevice(h->device));
  h->kp.rng_mode = mode;
  h->kp.seed = seed;
  h->tape = tape_dev;
  h->tape_off = (const long long *)tape_off_dev;
  HIPCHK(hipMemset(h->rng, 0, sizeof(unsigned long long) * h->E));
  return 0;
}

// Validate a spawn spec's ship types (blue then red) and derive what the
// kernels key on: each side's window cells (wc) and whether the runtime-size
// kernels must run (has_medium). Shared by lnw_reset and lnw_set_state, so a
// snapshot restored into any handle selects the same kernels and row lengths
// as the handle it was taken from. apply = false only validates.
static int apply_side_types(lnw_handle *h, const int32_t *types, bool apply) {
  int nmed[2] = {0, 0};
  for (int a = 0; a < h->A; a++) {
    const int t = types[a];
    if (t != LNW_SMALL && t != LNW_LARGE && t != LNW_LS && t != LNW_MEDIUM)
      return fail(LNW_EUNSUPPORTED, "ship type must be small, large, ls or medium");
    if (t == LNW_MEDIUM) nmed[a >= h->nb]++;
    if (h->params.discrete && t == LNW_LS)
      return fail(LNW_EUNSUPPORTED, "LandingShip has no value_to_coordinates (DISCRETE mode)");
  }
  // a side's row length follows its fastest ship (game.py:595-610), and a
  // medium ship's get_obs row has a 5x5 window (combatant.py:165-181): a side
  // of medium ships only has 4 n + 28-float rows; medium ships beside speed-3
  // ships make the reference's row assignment raise (game.py:344, 381)
  for (int sd = 0; sd < 2; sd++) {
    const int ns = sd ? h->nr : h->nb;
    if (nmed[sd] && nmed[sd] != ns)
      return fail(LNW_EUNSUPPORTED, "medium ships need a side of medium ships only (the reference's "
                                    "rows are sized by the fastest ship, game.py:595-610)");
  }
  if (apply) {
    h->kp.wc[0] = nmed[0] ? 25 : 49;
    h->kp.wc[1] = nmed[1] ? 25 : 49;
    h->has_medium = nmed[0] || nmed[1];
  }
  return 0;
}

int lnw_reset(lnw_handle *h, const uint8_t *env_mask_dev, const lnw_spawn *spawn,
              const int32_t *pos_dev, void *stream) {
  if (!h || !spawn) return fail(LNW_EINVAL, "null argument");
  if (!h->terrain) return fail(LNW_ESTATE, "lnw_load_terrain must be called first");
  HIPCHK(hipSetDevice(h->device));
  if (int rc = apply_side_types(h, spawn->types, false)) return rc;
  for (int a = 0; a < h->A; a++)
    if (!spawn->rand_ls[a] && (spawn->pos[a][0] < 0 || spawn->pos[a][0] >= h->G ||
                               spawn->pos[a][1] < 0 || spawn->pos[a][1] >= h->G))
      return fail(LNW_EINVAL, "spawn position outside the grid");
  apply_side_types(h, spawn->types, true);
  hipStream_t st = (hipStream_t)stream;
  HIPCHK(hipMemcpy(h->sp_types, spawn->types, sizeof(int32_t) * h->A, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(h->sp_pos, spawn->pos, sizeof(int32_t) * 2 * h->A, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(h->sp_randls, spawn->rand_ls, sizeof(int32_t) * h->A, hipMemcpyHostToDevice));
  h->kp.box_lo[0] = spawn->box_lo[0]; h->kp.box_lo[1] = spawn->box_lo[1];
  h->kp.box_hi[0] = spawn->box_hi[0]; h->kp.box_hi[1] = spawn->box_hi[1];
  // per-env spawn cells: kept in the handle for the in-kernel auto-reset
  if (pos_dev) {
    const size_t n = (size_t)h->E * h->A * 2;
    if (!h->sp_pos_env && dalloc(h, &h->sp_pos_env, n)) return LNW_ENOMEM;
    HIPCHK(hipMemcpyAsync(h->sp_pos_env, pos_dev, n * sizeof(int32_t), hipMemcpyDeviceToDevice, st));
  }
  h->sp_pos_env_on = pos_dev != nullptr;
  KState s = make_state(h);
  reset_kernel<<<(h->E + 255) / 256, 256, 0, st>>>(h->kp, s, env_mask_dev);
  HIPCHK(hipGetLastError());
  return 0;
}

namespace {
// lnw_step's launch (lnw_step_seq makes one per step)
int step_launch(lnw_handle *h, void *actions_dev, int32_t action_dtype,
                const uint8_t *row_kind_dev, float *obs_blue_dev, float *obs_red_dev, float *rew_blue_dev,
                float *rew_red_dev, int32_t *done_dev, float *cog_dev, void *stream) {
  if (!h || !actions_dev) return fail(LNW_EINVAL, "null argument");
  if (!h->terrain) return fail(LNW_ESTATE, "lnw_load_terrain must be called first");
  if (action_dtype != LNW_ACT_F32 && action_dtype != LNW_ACT_F64 && action_dtype != LNW_ACT_I32)
    return fail(LNW_EINVAL, "bad action dtype");
  if (action_dtype == LNW_ACT_I32 && !h->params.discrete)
    return fail(LNW_EINVAL, "integer actions go with DISCRETE mode only");
  if (action_dtype == LNW_ACT_F32 && h->params.discrete)
    return fail(LNW_EINVAL, "DISCRETE mode takes int32 (ndarray) or float64 (list rows) actions");
  if ((obs_blue_dev == nullptr) != (obs_red_dev == nullptr))
    return fail(LNW_EINVAL, "observation outputs: both or neither");
  KParams k = h->kp;
  k.act_dtype = action_dtype;
  k.no_obs = obs_blue_dev == nullptr ? 1 : 0;
  k.dbg_skip = h->dbg_skip;
  k.store_wt = h->store_wt;
  KState s = make_state(h);
  k.qdirect = step_qdirect(h, k.epw) ? 1 : 0;
  size_t lds = step_launch_lds_bytes(h, k.epw);
  dim3 grid((h->E + k.epw - 1) / k.epw), block(WAVE);
  hipStream_t st = (hipStream_t)stream;
  // (medium ships: 5x5 windows and shorter rows, the runtime-size kernels only)
  bool generic = h->force_generic;
  const bool templated = k.los_mode != 2 && !generic && !h->has_medium && h->nb == h->nr && h->nb >= 2 && h->nb <= 4 &&
                         !(h->force_group && h->group_fits);
  const bool use_group = k.los_mode != 2 && !templated && !generic && !h->no_group && h->group_fits;
  // 4v4 at 64 envs per workgroup in LOS-table mode, whole units (the headline):
  // the units kernel (LNW_NO_UNITS keeps one unit per workgroup)
  const bool units = templated && h->nb == 4 && !h->contact && !h->no_units && h->units_fit && k.epw == EPW &&
                     k.los_mode == 0 && h->E % (EPW * UNITS) == 0 && !(h->dbg_skip & (1 | 2 | 512));
  // per-unit records (LNW_PROF) of the kernel launched below (the group kernel has its own grid)
  const unsigned nwg = use_group ? (unsigned)((h->E + GEPW - 1) / GEPW) : grid.x;
  if (h->prof) {
    const size_t slots = (size_t)nwg * PROF_SLOTS;
    if (slots > h->prof_cap) {
      HIPCHK(hipStreamSynchronize(st));
      if (h->d_prof) { (void)hipFree(h->d_prof); h->d_prof = nullptr; h->prof_cap = 0; }
      HIPCHK(hipMalloc(&h->d_prof, slots * sizeof(unsigned long long)));
      h->prof_cap = slots;
    }
    HIPCHK(hipMemsetAsync(h->d_prof, 0, slots * sizeof(unsigned long long), st));
    s.prof = h->d_prof;
  }
#define LNW_STEP(NB_, NR_, CW_, RW_)                                                             \
  step_kernel<NB_, NR_, CW_, RW_><<<grid, dim3(NB_ > 0 && EPW == WAVE ? 2 * WAVE : WAVE), lds, st>>>(k, s, actions_dev, row_kind_dev, obs_blue_dev, \
                                                 obs_red_dev, rew_blue_dev, rew_red_dev,        \
                                                 done_dev, cog_dev)
  const bool cw = h->contact;
  h->last_kernel = units ? LNW_KERNEL_UNITS
                   : k.los_mode == 2 ? LNW_KERNEL_REFLOS
                   : templated ? (cw ? LNW_KERNEL_TEAM_CONTACT : LNW_KERNEL_TEAM)
                   : use_group ? LNW_KERNEL_GROUP : LNW_KERNEL_GENERIC;
  if (units) {
    // 4 units of 64 envs per workgroup, one workgroup per CU (step_kernel UN)
    step_kernel<4, 4, false, false, UNITS><<<dim3(h->E / (EPW * UNITS)), dim3(2 * WAVE * UNITS),
                                             (size_t)UNITS * ((lds + 15) & ~(size_t)15), st>>>(
        k, s, actions_dev, row_kind_dev, obs_blue_dev, obs_red_dev, rew_blue_dev, rew_red_dev, done_dev,
        cog_dev);
  }
  else if (k.los_mode == 2) LNW_STEP(0, 0, false, true);  // diagnostics: the reference's LOS work
  else if (templated && h->nb == 4) {
    // the contact variant: phase S split by side (step_kernel PS; LNW_NO_SPLIT_ROWS:
    // only for steps without rows, A/B)
    if (cw && k.los_mode == 0 && (k.no_obs || !h->no_split_rows))
      step_kernel<4, 4, true, false, 1, true><<<grid, dim3(2 * WAVE), lds, st>>>(
          k, s, actions_dev, row_kind_dev, obs_blue_dev, obs_red_dev, rew_blue_dev, rew_red_dev, done_dev, cog_dev);
    else if (cw) LNW_STEP(4, 4, true, false);
    else if (k.qdirect && k.epw * 4 > WAVE)  // two-slab direct rows (step_qdirect)
      step_kernel<4, 4, false, false, 1, false, true><<<grid, dim3(2 * WAVE), lds, st>>>(
          k, s, actions_dev, row_kind_dev, obs_blue_dev, obs_red_dev, rew_blue_dev, rew_red_dev, done_dev, cog_dev);
    else LNW_STEP(4, 4, false, false);
  }
  else if (templated && h->nb == 3) { if (cw) LNW_STEP(3, 3, true, false); else LNW_STEP(3, 3, false, false); }
  else if (templated && h->nb == 2) { if (cw) LNW_STEP(2, 2, true, false); else LNW_STEP(2, 2, false, false); }
  else if (use_group) {
    // runtime team sizes: GL lanes per env (lnw_group.inc)
    const GroupLds gl = group_lds(lds_layout(h->A, h->nb, h->nr, h->nmax, h->G * h->W16, h->G), h->G * h->W16,
                                  h->A, h->nb * h->nr, k.atan_odd != 0);
    const size_t glds = (size_t)gl.total;
    if (s.prof)
      fprintf(stderr, "[lnw prof] group kernel LDS %zu B (staged: target lists %d, dist_lz %d, bearing half table %d, pooled slopes %d)\n",
              glds, (int)(gl.tls >= 0), (int)(gl.dlz >= 0), (int)(gl.atab >= 0), (int)(gl.ms >= 0));
    step_group_kernel<<<dim3((h->E + GEPW - 1) / GEPW), dim3(GEPW * GL), glds, st>>>(
        k, s, actions_dev, row_kind_dev, obs_blue_dev, obs_red_dev, rew_blue_dev, rew_red_dev,
        done_dev, cog_dev);
  }
  else LNW_STEP(0, 0, false, false);
#undef LNW_STEP
  HIPCHK(hipGetLastError());
  if (s.prof) prof_report(h, st, (int)nwg);
  return 0;
}
}  // namespace

int lnw_step(lnw_handle *h, void *actions_dev, int32_t action_dtype, const uint8_t *row_kind_dev,
             float *obs_blue_dev, float *obs_red_dev, float *rew_blue_dev, float *rew_red_dev,
             int32_t *done_dev, float *cog_dev, void *stream) {
  return step_launch(h, actions_dev, action_dtype, row_kind_dev, obs_blue_dev, obs_red_dev, rew_blue_dev,
                     rew_red_dev, done_dev, cog_dev, stream);
}

int lnw_step_seq(lnw_handle *h, const lnw_seq *seq, void *actions_dev, int32_t action_dtype,
                 const uint8_t *row_kind_dev, float *obs_blue_dev, float *obs_red_dev, float *rew_blue_dev,
                 float *rew_red_dev, int32_t *done_dev, float *cog_dev, void *stream) {
  if (!h || !seq) return fail(LNW_EINVAL, "null argument");
  if (seq->steps < 1) return fail(LNW_EINVAL, "seq->steps must be >= 1");
  if (seq->act_step < 0 || seq->kind_step < 0 || seq->obs_blue_step < 0 || seq->obs_red_step < 0 ||
      seq->rew_blue_step < 0 || seq->rew_red_step < 0 || seq->done_step < 0 || seq->cog_step < 0)
    return fail(LNW_EINVAL, "negative step stride");
  // K launches back to back on the caller's stream. (Round 5 measured one launch
  // in which each workgroup ran its envs through the K steps: parity with K
  // launches at best, DESIGN.md "Action sequences in one call"; removed.)
  const long long asz = action_dtype == LNW_ACT_F64 ? 8 : 4, rsz = h->kp.rew_f64 ? 8 : 4;
  for (int k = 0; k < seq->steps; k++) {
    auto adv = [&](const void *p, long long stride, long long sz) {
      return p ? (void *)((char *)p + (long long)k * stride * sz) : nullptr;
    };
    if (int e = step_launch(h, adv(actions_dev, seq->act_step, asz), action_dtype,
                            (const uint8_t *)adv(row_kind_dev, seq->kind_step, 1),
                            (float *)adv(obs_blue_dev, seq->obs_blue_step, 4),
                            (float *)adv(obs_red_dev, seq->obs_red_step, 4),
                            (float *)adv(rew_blue_dev, seq->rew_blue_step, rsz),
                            (float *)adv(rew_red_dev, seq->rew_red_step, rsz),
                            (int32_t *)adv(done_dev, seq->done_step, 4), (float *)adv(cog_dev, seq->cog_step, rsz),
                            stream))
      return e;
  }
  return 0;
}

int lnw_observe(lnw_handle *h, int32_t agent, float *obs_blue_dev, float *obs_red_dev, void *stream) {
  return lnw_observe_ex(h, agent, obs_blue_dev, 0, obs_red_dev, 0, stream);
}

int lnw_observe_ex(lnw_handle *h, int32_t agent, float *obs_blue_dev, int64_t blue_env_stride,
                   float *obs_red_dev, int64_t red_env_stride, void *stream) {
  if (!h) return fail(LNW_EINVAL, "null handle");
  if (!h->terrain) return fail(LNW_ESTATE, "lnw_load_terrain must be called first");
  if (agent >= h->A || agent < LNW_OBS_RED) return fail(LNW_EINVAL, "bad agent selector");
  const int64_t row_b = (int64_t)h->nb * side_D(h->kp, 0), row_r = (int64_t)h->nr * side_D(h->kp, 1);
  if (blue_env_stride < 0 || red_env_stride < 0 || (blue_env_stride && (blue_env_stride < row_b || blue_env_stride % 4)) ||
      (red_env_stride && (red_env_stride < row_r || red_env_stride % 4)))
    return fail(LNW_EINVAL, "env stride: 0, or a multiple of 4 floats of at least the side's n * D");
  if (((uintptr_t)obs_blue_dev | (uintptr_t)obs_red_dev) & 15) return fail(LNW_EINVAL, "rows must be 16-B aligned");
  KState s = make_state(h);
  size_t lds = step_lds_bytes(h);
  dim3 grid((h->E + h->kp.epw - 1) / h->kp.epw), block(WAVE);
  hipStream_t st = (hipStream_t)stream;
  const bool tmpl = !h->force_generic && !h->has_medium && h->params.los_mode != 2 && h->nb == h->nr;
  const bool cw = h->contact;
  KParams k = h->kp;
  k.obs_stride[0] = blue_env_stride;
  k.obs_stride[1] = red_env_stride;
#define LNW_OBS(NB_, CW_)                                                                          \
  observe_kernel<NB_, NB_, CW_><<<grid, dim3(NB_ > 0 && CW_ ? 2 * WAVE : WAVE), lds, st>>>(k, s, agent, \
                                                                                    obs_blue_dev, obs_red_dev)
  if (tmpl && h->nb == 4) { if (cw) LNW_OBS(4, true); else LNW_OBS(4, false); }
  else if (tmpl && h->nb == 3) { if (cw) LNW_OBS(3, true); else LNW_OBS(3, false); }
  else if (tmpl && h->nb == 2) { if (cw) LNW_OBS(2, true); else LNW_OBS(2, false); }
  else LNW_OBS(0, false);
#undef LNW_OBS
  HIPCHK(hipGetLastError());
  return 0;
}

int lnw_state_field(lnw_handle *h, int32_t field, void **dev_ptr, int64_t *nbytes) {
  if (!h || !dev_ptr || !nbytes) return fail(LNW_EINVAL, "null argument");
  const int64_t E = h->E, A = h->A;
  switch (field) {
    case LNW_F_POS: *dev_ptr = h->pos; *nbytes = 4 * A * E; break;
    case LNW_F_RADAR: *dev_ptr = h->radar; *nbytes = 4 * A * E; break;
    case LNW_F_MISSILES: *dev_ptr = h->miss; *nbytes = A * E; break;
    case LNW_F_MKIND: *dev_ptr = h->mkind; *nbytes = A * E; break;
    case LNW_F_ALIVE: *dev_ptr = h->alive; *nbytes = A * E; break;
    case LNW_F_TYPE: *dev_ptr = h->type; *nbytes = A * E; break;
    case LNW_F_STEPS: *dev_ptr = h->steps; *nbytes = 4 * A * E; break;
    case LNW_F_DIST_LZ: *dev_ptr = h->dist_lz; *nbytes = 8 * A * E; break;
    case LNW_F_TL_CNT: *dev_ptr = h->tl_cnt; *nbytes = 2 * A * E; break;
    case LNW_F_TL: *dev_ptr = h->tl; *nbytes = 2 * A * h->T * E; break;
    case LNW_F_DUCT: *dev_ptr = h->duct; *nbytes = 8 * E; break;
    case LNW_F_ENV: *dev_ptr = h->envi; *nbytes = 4 * 8 * E; break;
    case LNW_F_RNG: *dev_ptr = h->rng; *nbytes = 8 * E; break;
    case LNW_F_ERR: *dev_ptr = h->err; *nbytes = 4 * E; break;
    default: return fail(LNW_EINVAL, "unknown state field");
  }
  return 0;
}

int lnw_tlist_cap(lnw_handle *h) { return h ? h->T : LNW_EINVAL; }

int lnw_step_kernel(lnw_handle *h) { return h ? h->last_kernel : LNW_EINVAL; }

// ---- whole-state snapshots (lnw_state_bytes / lnw_get_state / lnw_set_state)
// Snapshot layout: a 128-byte header (below), then the LNW_NFIELDS state
// fields in field order, then the spawn spec the in-kernel auto-reset reads
// (types, cells, randint flags: 64 x i32, 64 x 2 x i32, 64 x i32) and the
// per-env spawn cells ([E][A][2] i32, zeros when the last reset had none);
// every section starts on a 256-byte boundary.
namespace {
struct StateHeader {
  char magic[8];            // "LNWSTATE"
  uint32_t version;         // 1
  int32_t E, nb, nr, T, G;
  int32_t rng_mode;         // LNW_RNG_*
  int32_t pos_env_on;       // the auto-reset respawns on per-env cells
  uint64_t seed;
  uint64_t terrain_hash;    // FNV-1a of the grid loaded when the snapshot was taken
  int64_t total;            // snapshot bytes
  int32_t box_lo[2], box_hi[2];
  int32_t abi;              // LNW_ABI_VERSION
  uint8_t pad[128 - 8 - 4 - 7 * 4 - 3 * 8 - 4 * 4 - 4];
};
static_assert(sizeof(StateHeader) == 128, "state header is 128 bytes");

struct Section { void *dev; int64_t bytes; };

int state_sections(lnw_handle *h, std::vector<Section> &out) {
  out.clear();
  for (int f = 0; f < LNW_NFIELDS; f++) {
    void *p = nullptr;
    int64_t n = 0;
    if (int rc = lnw_state_field(h, f, &p, &n)) return rc;
    out.push_back({p, n});
  }
  out.push_back({h->sp_types, 64 * 4});
  out.push_back({h->sp_pos, 128 * 4});
  out.push_back({h->sp_randls, 64 * 4});
  out.push_back({h->sp_pos_env, (int64_t)h->E * h->A * 2 * 4});  // (may not be allocated yet)
  return 0;
}

inline int64_t sec_align(int64_t v) { return (v + 255) & ~(int64_t)255; }
}  // namespace

int64_t lnw_state_bytes(lnw_handle *h) {
  if (!h) return fail(LNW_EINVAL, "null handle");
  std::vector<Section> s;
  if (int rc = state_sections(h, s)) return rc;
  int64_t o = 256;
  for (const Section &x : s) o += sec_align(x.bytes);
  return o;
}

int lnw_get_state(lnw_handle *h, void *dst, int64_t nbytes, void *stream) {
  if (!h || !dst) return fail(LNW_EINVAL, "null argument");
  if (!h->terrain) return fail(LNW_ESTATE, "lnw_load_terrain must be called first");
  const int64_t total = lnw_state_bytes(h);
  if (nbytes < total) return fail(LNW_EINVAL, "snapshot buffer smaller than lnw_state_bytes()");
  HIPCHK(hipSetDevice(h->device));
  HIPCHK(hipStreamSynchronize((hipStream_t)stream));
  StateHeader hd;
  memset(&hd, 0, sizeof hd);
  memcpy(hd.magic, "LNWSTATE", 8);
  hd.version = 1;
  hd.E = h->E; hd.nb = h->nb; hd.nr = h->nr; hd.T = h->T; hd.G = h->G;
  hd.rng_mode = h->kp.rng_mode;
  hd.pos_env_on = h->sp_pos_env_on ? 1 : 0;
  hd.seed = h->kp.seed;
  hd.terrain_hash = h->terrain_hash;
  hd.total = total;
  for (int i = 0; i < 2; i++) { hd.box_lo[i] = h->kp.box_lo[i]; hd.box_hi[i] = h->kp.box_hi[i]; }
  hd.abi = LNW_ABI_VERSION;
  std::vector<Section> s;
  if (int rc = state_sections(h, s)) return rc;
  char *d = (char *)dst;
  char hbuf[256] = {0};
  memcpy(hbuf, &hd, sizeof hd);
  HIPCHK(hipMemcpy(d, hbuf, sizeof hbuf, hipMemcpyDefault));
  int64_t o = 256;
  for (const Section &x : s) {
    if (x.dev) {
      HIPCHK(hipMemcpy(d + o, x.dev, (size_t)x.bytes, hipMemcpyDefault));
    } else {  // per-env spawn cells never given: zeros (host or device destination)
      const std::vector<char> z((size_t)x.bytes, 0);
      HIPCHK(hipMemcpy(d + o, z.data(), (size_t)x.bytes, hipMemcpyDefault));
    }
    o += sec_align(x.bytes);
  }
  return 0;
}

int lnw_set_state(lnw_handle *h, const void *src, int64_t nbytes, void *stream) {
  if (!h || !src) return fail(LNW_EINVAL, "null argument");
  if (!h->terrain) return fail(LNW_ESTATE, "lnw_load_terrain must be called first");
  HIPCHK(hipSetDevice(h->device));
  HIPCHK(hipStreamSynchronize((hipStream_t)stream));
  if (nbytes < (int64_t)sizeof(StateHeader)) return fail(LNW_EINVAL, "snapshot too short");
  StateHeader hd;
  HIPCHK(hipMemcpy(&hd, src, sizeof hd, hipMemcpyDefault));
  if (memcmp(hd.magic, "LNWSTATE", 8) != 0 || hd.version != 1)
    return fail(LNW_EINVAL, "not an lnw state snapshot (bad magic or version)");
  if (hd.abi != LNW_ABI_VERSION)
    return fail(LNW_EINVAL, "snapshot was taken by a library of another ABI version");
  const int64_t total = lnw_state_bytes(h);
  if (hd.E != h->E || hd.nb != h->nb || hd.nr != h->nr || hd.T != h->T || hd.G != h->G || hd.total != total)
    return fail(LNW_EINVAL, "snapshot shape (envs, team sizes, grid) differs from this handle");
  if (hd.terrain_hash != h->terrain_hash) return fail(LNW_EINVAL, "snapshot was taken on another terrain");
  if (nbytes < total) return fail(LNW_EINVAL, "snapshot shorter than its header says");
  if (hd.rng_mode == LNW_RNG_TAPE && (!h->tape || !h->tape_off))
    return fail(LNW_ESTATE, "snapshot is in tape mode: bind the tape (lnw_set_rng) before restoring");
  if (hd.pos_env_on && !h->sp_pos_env && dalloc(h, &h->sp_pos_env, (size_t)h->E * h->A * 2)) return LNW_ENOMEM;
  std::vector<Section> s;
  if (int rc = state_sections(h, s)) return rc;
  const char *p = (const char *)src;
  // the spawn types decide the kernels and the row lengths (wc, has_medium):
  // validate them before anything is overwritten, apply them after
  int32_t types[64];
  {
    int64_t ot = 256;
    for (int i = 0; i < LNW_NFIELDS; i++) ot += sec_align(s[i].bytes);
    HIPCHK(hipMemcpy(types, p + ot, sizeof types, hipMemcpyDefault));
    if (int rc = apply_side_types(h, types, false)) return rc;
  }
  int64_t o = 256;
  for (const Section &x : s) {
    if (x.dev) HIPCHK(hipMemcpy(x.dev, p + o, (size_t)x.bytes, hipMemcpyDefault));
    o += sec_align(x.bytes);
  }
  apply_side_types(h, types, true);
  h->kp.rng_mode = hd.rng_mode;
  if (hd.rng_mode == LNW_RNG_PHILOX) h->kp.seed = hd.seed;
  for (int i = 0; i < 2; i++) { h->kp.box_lo[i] = hd.box_lo[i]; h->kp.box_hi[i] = hd.box_hi[i]; }
  h->sp_pos_env_on = hd.pos_env_on != 0;
  return 0;
}

int lnw_set_counters(lnw_handle *h, uint64_t *counters_dev) {
  if (!h) return fail(LNW_EINVAL, "null handle");
  h->ctr = (unsigned long long *)counters_dev;
  return 0;
}

int lnw_set_reward_dtype(lnw_handle *h, int32_t f64) {
  if (!h) return fail(LNW_EINVAL, "null handle");
  h->kp.rew_f64 = f64 != 0;
  return 0;
}

int lnw_set_variant(lnw_handle *h, int32_t contact) {
  if (!h) return fail(LNW_EINVAL, "null handle");
  h->contact = contact != 0;
  return 0;
}

int lnw_set_epw(lnw_handle *h, int32_t epw) {
  if (!h) return fail(LNW_EINVAL, "null handle");
  if (epw < 0 || epw > EPW) return fail(LNW_EINVAL, "epw must be 0 (automatic) or 1..64");
  if (!h->terrain) return fail(LNW_ESTATE, "lnw_load_terrain must be called first");
  h->kp.epw = epw ? epw : choose_epw(h);
  return h->kp.epw;
}

int lnw_los_batch(const uint8_t *grid_dev, int32_t G, const int16_t *pairs_dev, int64_t n,
                  int32_t move_thr, int32_t ew_thr, uint8_t *out_dev, void *stream) {
  if (!grid_dev || !pairs_dev || !out_dev) return fail(LNW_EINVAL, "null argument");
  if (n <= 0) return 0;
  const size_t lds = (size_t)G * ((G + 15) / 16) * 4;
  if (lds <= 64 * 1024 && ((uintptr_t)pairs_dev & 7) == 0) {  // (the LDS kernel reads a pair as 8 bytes)
    const long long per_block = (long long)(LB_THREADS / WAVE) * LB_RAYS_PER_WAVE;
    los_batch_kernel<<<(unsigned)((n + per_block - 1) / per_block), LB_THREADS, lds, (hipStream_t)stream>>>(
        grid_dev, G, pairs_dev, n, move_thr, ew_thr, out_dev);
  } else {
    los_batch_global_kernel<<<(unsigned)((n + 255) / 256), 256, 0, (hipStream_t)stream>>>(
        grid_dev, G, pairs_dev, n, move_thr, ew_thr, out_dev);
  }
  HIPCHK(hipGetLastError());
  return 0;
}

int lnw_astar_batch(const uint8_t *grid_dev, int32_t G, int32_t move_thr, const int8_t *types_dev,
                    const int16_t *start_dev, const int16_t *target_dev, int64_t n,
                    int16_t *plen_dev, int8_t *kind_dev, uint8_t *feasible_dev, void *stream) {
  if (!grid_dev || !types_dev || !start_dev || !target_dev || !plen_dev || !kind_dev || !feasible_dev)
    return fail(LNW_EINVAL, "null argument");
  if (n <= 0) return 0;
  astar_batch_kernel<<<(unsigned)((n + WAVE - 1) / WAVE), WAVE, 0, (hipStream_t)stream>>>(
      grid_dev, G, move_thr, types_dev, start_dev, target_dev, n, plen_dev, kind_dev, feasible_dev);
  HIPCHK(hipGetLastError());
  return 0;
}

int lnw_move_batch(lnw_handle *h, const int8_t *types_dev, const int16_t *pos_dev,
                   const double *act_dev, const uint8_t *is_f32_dev, int64_t n, int32_t *rounded_dev,
                   uint8_t *ok_dev, void *stream) {
  if (!h || !types_dev || !pos_dev || !act_dev || !is_f32_dev || !rounded_dev || !ok_dev)
    return fail(LNW_EINVAL, "null argument");
  if (!h->terrain) return fail(LNW_ESTATE, "lnw_load_terrain must be called first");
  if (n <= 0) return 0;
  KState s = make_state(h);
  move_batch_kernel<<<(unsigned)((n + WAVE - 1) / WAVE), WAVE, 0, (hipStream_t)stream>>>(
      h->kp, s, types_dev, pos_dev, act_dev, is_f32_dev, n, rounded_dev, ok_dev);
  HIPCHK(hipGetLastError());
  return 0;
}

int lnw_path_query(lnw_handle *h, const int8_t *types_dev, const int16_t *start_dev,
                   const int16_t *target_dev, int64_t n, uint8_t *out_dev, void *stream) {
  if (!h || !types_dev || !start_dev || !target_dev || !out_dev) return fail(LNW_EINVAL, "null argument");
  if (!h->terrain) return fail(LNW_ESTATE, "lnw_load_terrain must be called first");
  if (n <= 0) return 0;
  KState s = make_state(h);
  path_query_kernel<<<(unsigned)((n + WAVE - 1) / WAVE), WAVE, 0, (hipStream_t)stream>>>(
      h->kp, s, types_dev, start_dev, target_dev, n, out_dev);
  HIPCHK(hipGetLastError());
  return 0;
}

int lnw_los_query(lnw_handle *h, const int16_t *pairs_dev, int64_t n, uint8_t *out_dev, void *stream) {
  if (!h || !pairs_dev || !out_dev) return fail(LNW_EINVAL, "null argument");
  if (!h->terrain) return fail(LNW_ESTATE, "lnw_load_terrain must be called first");
  if (n <= 0) return 0;
  KState s = make_state(h);
  los_query_kernel<<<(unsigned)((n + 255) / 256), 256, 0, (hipStream_t)stream>>>(h->kp, s, pairs_dev, n, out_dev);
  HIPCHK(hipGetLastError());
  return 0;
}

int lnw_copy(void *dst, const void *src, int64_t nbytes, void *stream) {
  if (nbytes <= 0) return 0;
  if (!dst || !src) return fail(LNW_EINVAL, "null argument");
  HIPCHK(hipMemcpyAsync(dst, src, (size_t)nbytes, hipMemcpyDefault, (hipStream_t)stream));
  return 0;
}

int lnw_fill_uniform_f32(float *out_dev, int64_t n, uint64_t seed, uint64_t offset, void *stream) {
  if (!out_dev) return fail(LNW_EINVAL, "null argument");
  if (n <= 0) return 0;
  if (offset & 3) return fail(LNW_EINVAL, "offset must be a multiple of 4");
  long long nt = (n + 3) / 4;
  fill_uniform_kernel<<<(unsigned)((nt + 255) / 256), 256, 0, (hipStream_t)stream>>>(out_dev, n, seed, offset);
  HIPCHK(hipGetLastError());
  return 0;
}

}  // extern "C"
