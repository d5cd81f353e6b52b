/*
 * lnw.h — C-ABI of the MI355X-native batched littoral-warfare environment step.
 *
 * Drop-in boundary for the reference's environment API
 * (valauri/Littoral-Naval-Warfare-MARL):
 *
 *   lnw_create / lnw_load_terrain   replace Game.__init__ (game.py:107-158) and
 *                                   Game.define_grid_from_image (game.py:616-626)
 *   lnw_reset                       replaces Game.reset (game.py:528-613)
 *   lnw_step                        replaces Game.step (game.py:298-525) with
 *                                   Combatant/LandingShip.take_action
 *                                   (combatant.py:501-565, landingship.py:508-572)
 *                                   and Game.calculate_reward (game.py:214-295)
 *   lnw_observe                     replaces ship.get_obs() (combatant.py:90-233,
 *                                   landingship.py:94-239) as called by
 *                                   main.py:282, ppo.py:500, ddqn.py:296
 *   lnw_los_batch                   check_line_of_sight (combatant.py:436-456)
 *   lnw_move_batch                  continuous_to_discrete / value_to_coordinates +
 *                                   check_path / astar (combatant.py:289-489,689-704)
 *
 * Conventions
 *  - Every pointer argument named *_dev is a device pointer (HIP, gfx950); the
 *    caller owns action/observation/reward buffers, the handle owns the
 *    environment state and the terrain.
 *  - Work is enqueued on the caller's stream (hipStream_t passed as void*; NULL
 *    = the default stream). Nothing synchronises except lnw_create,
 *    lnw_load_terrain and lnw_destroy.
 *  - Every function returns 0 on success or a negative LNW_E* code; the message
 *    of the last failure on the calling thread is available from
 *    lnw_last_error(). Reference crash modes (ZeroDivisionError in an EW fix,
 *    round(nan), tape exhaustion) do not abort: they set per-environment bits in
 *    the err-flags array (LNW_ERRF_*).
 *  - A handle is not thread-safe; use one handle per device (per process).
 *
 * Layouts (E = n_envs, nb/nr = blue/red slots, A = nb+nr, D_side = 4*n_side+52,
 * or 4*n_side+28 for a side of medium ships: game.py:609-610 sizes a side's rows
 * by its fastest ship, (2*speed+1)^2 window cells):
 *  actions   [E][A][4]  f32 or f64 (continuous), or [E][A][4] i32 (discrete:
 *                       radar, salvo, move-index 0..49, unused) — mutated in
 *                       place where the reference mutates it (game.py:379)
 *  obs_blue  [E][nb][Db] f32, obs_red [E][nr][Dr] f32 (float32 of the reference's
 *                       float64 value; dead slots are zeros)
 *  rew_blue  [E][nb] f32, rew_red [E][nr] f32, done [E] i32 (1 running, 0 over),
 *  cog       [E] f32 (NaN where the reference returns None)
 *  rew_* and cog are float64 instead after lnw_set_reward_dtype(h, 1)
 */
#ifndef LNW_H
#define LNW_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LNW_ABI_VERSION 5

/* status codes */
#define LNW_OK 0
#define LNW_EINVAL (-1)
#define LNW_ENOMEM (-2)
#define LNW_EDEVICE (-3)
#define LNW_ESTATE (-4)
#define LNW_EUNSUPPORTED (-5)

/* ship types (Combatant "small"/"large"/"medium", LandingShip "ls";
 * combatant.py:60-88, landingship.py:61-92, game.py:184-212) */
#define LNW_SMALL 0
#define LNW_LARGE 1
#define LNW_LS 2
#define LNW_MEDIUM 3   /* speed 2, 8 missiles, mast 30, rcs 1, 5x5 observation window */

/* action dtypes / per-row value kinds (NumPy NEP 50 semantics) */
#define LNW_ACT_F32 0      /* whole buffer float32 (np.float32 rows)            */
#define LNW_ACT_F64 1      /* whole buffer float64 (np.float64 rows)            */
#define LNW_ACT_I32 2      /* discrete integer actions (DISCRETE=true)         */
#define LNW_KIND_PYFLOAT 1 /* row_kind values for an F64 buffer: python floats */
#define LNW_KIND_F32 2     /*   np.float32 row stored widened to f64           */
#define LNW_KIND_F64 3     /*   np.float64 row                                 */

/* rng modes */
#define LNW_RNG_PHILOX 0   /* production: Philox4x32-10 keyed by (seed, global env id) */
#define LNW_RNG_TAPE 1     /* parity: per-env recorded draws                           */

/* per-env error bits */
#define LNW_ERRF_ZERODIV 1u    /* combatant.py:274 ZeroDivisionError (fix skipped) */
#define LNW_ERRF_NAN_ROUND 2u  /* round(nan/inf) in a fix or a radar action        */
#define LNW_ERRF_TAPE 4u       /* tape exhausted                                   */
#define LNW_ERRF_MISSILES 8u   /* missile count outside the 0..8 hit table         */

/* observe selectors */
#define LNW_OBS_ALL (-1)   /* every live ship, blue then red (main.py:280-333) */
#define LNW_OBS_BLUE (-2)
#define LNW_OBS_RED (-3)

typedef struct lnw_handle lnw_handle;

/* Scenario flags: the reference's config.json keys (game.py:41-53,
 * combatant.py:33-38) that change step semantics. */
typedef struct lnw_params {
    int32_t discrete;        /* overall.discrete                       */
    int32_t landing_ops;     /* overall.landing_ops                    */
    int32_t aggressive;      /* overall.tactics == "aggressive"        */
    int32_t side_blue;       /* environment_setup.side == "blue"       */
    int32_t trained_red;     /* environment_setup.trained_red          */
    int32_t move_thr;        /* environment_setup.movement_threshold   */
    int32_t ew_thr;          /* environment_setup.ew_threshold         */
    int32_t lz_x, lz_y;      /* landing zone (game.py:590): (14, 82)   */
    double red_aggression;   /* environment_setup.red_aggression       */
    /* build-side knobs (not in the reference) */
    int32_t episode_steps;   /* auto-reset horizon (0 = never)          */
    int32_t auto_reset;      /* reset an env in-kernel when done==0 or at the horizon */
    int32_t los_mode;        /* 0 = precomputed LOS table, 1 = ray march,
                                2 = table + the reference's LOS work: every
                                own x opponent ray marched in full at each
                                get_obs and discarded (diagnostics)        */
    int32_t move_mode;       /* 0 = precomputed move table, 1 = direct A*  */
} lnw_params;

/* Spawn description used by lnw_reset and by in-kernel auto-reset.
 * types[A]: LNW_SMALL/LARGE/LS/MEDIUM (medium ships only as a whole side: the
 * reference's row assignment raises for a medium ship beside speed-3 ships,
 * game.py:344 / 381, so lnw_reset refuses that with LNW_EUNSUPPORTED);
 * pos[A][2]: spawn cell; rand_ls[A] != 0 draws the
 * cell with random.randint(98,99), random.randint(48,56) (game.py:589).
 * If box_lo/box_hi are set (box_hi[0] > box_lo[0]) every agent instead spawns on
 * a random water cell of that box (a build-side "melee" scenario, drawn from a
 * separate Philox stream so the game stream is unchanged). */
typedef struct lnw_spawn {
    int32_t types[64];
    int32_t pos[64][2];
    int32_t rand_ls[64];
    int32_t box_lo[2], box_hi[2];
} lnw_spawn;

/* ---- lifecycle ---------------------------------------------------------- */
int lnw_abi_version(void);
const char *lnw_last_error(void);

/* env_id_base: global id of this handle's first env (multi-GPU sharding keys the
 * RNG by global env id so trajectories do not depend on the GPU count). */
int lnw_create(const lnw_params *params, int32_t n_envs, int32_t nb, int32_t nr, int32_t device,
               int64_t env_id_base, lnw_handle **out);
int lnw_destroy(lnw_handle *h);

/* Upload the uint8 terrain (row-major [G][G], grid[x][y]) and build the device
 * structures: radar/EW bitmask, move-feasibility table, LOS table. Synchronous. */
int lnw_load_terrain(lnw_handle *h, const uint8_t *grid_host, int32_t G);

int lnw_set_rng(lnw_handle *h, int32_t mode, uint64_t seed, const double *tape_dev,
                const int64_t *tape_off_dev);

/* ---- environment API ---------------------------------------------------- */
/* env_mask_dev: [E] u8, nonzero = reset that env (NULL = all).
 * pos_dev: optional [E][A][2] i32 per-env spawn cells (overrides spawn->pos). It is
 * copied into the handle (stream-ordered), and the in-kernel auto-reset
 * (lnw_params.auto_reset) respawns every env on its own cells from then on; a
 * reset without pos_dev returns all envs to the shared spawn->pos. */
int lnw_reset(lnw_handle *h, const uint8_t *env_mask_dev, const lnw_spawn *spawn,
              const int32_t *pos_dev, void *stream);

/* obs_blue_dev and obs_red_dev both NULL: no observation rows are written
 * (the MAPPO rollout discards step()'s observations, ppo.py:577, and observes
 * afresh); every other effect of the step is unchanged. One NULL alone is
 * LNW_EINVAL. */
int lnw_step(lnw_handle *h, void *actions_dev, int32_t action_dtype, const uint8_t *row_kind_dev,
             float *obs_blue_dev, float *obs_red_dev, float *rew_blue_dev, float *rew_red_dev,
             int32_t *done_dev, float *cog_dev, void *stream);

/* K consecutive Game.step calls whose action arrays the caller has ahead of
 * time (an open-loop action sequence: scripted or replayed agents, benchmark
 * actions) — no reference counterpart beyond K calls of Game.step; results are
 * exactly those of K lnw_step calls, step k reading actions_dev + k *
 * seq->act_step elements (and row kinds + k * kind_step bytes) and writing its
 * outputs at the output pointers + k * the output strides (elements; a stride
 * 0 makes every step write the same rows, each step's outputs replacing the
 * previous step's as K separate calls would). It makes the K lnw_step
 * launches itself, back to back on the caller's stream. */
typedef struct lnw_seq {
  int32_t steps;               /* K >= 1 */
  int64_t act_step, kind_step; /* action elements / row-kind bytes between steps */
  int64_t obs_blue_step, obs_red_step, rew_blue_step, rew_red_step, done_step, cog_step;
} lnw_seq;
int lnw_step_seq(lnw_handle *h, const lnw_seq *seq, void *actions_dev, int32_t action_dtype,
                 const uint8_t *row_kind_dev, float *obs_blue_dev, float *obs_red_dev, float *rew_blue_dev,
                 float *rew_red_dev, int32_t *done_dev, float *cog_dev, void *stream);

/* agent >= 0: that agent (blue 0..nb-1, red nb..A-1) in every env;
 * LNW_OBS_ALL / LNW_OBS_BLUE / LNW_OBS_RED: every live ship of the selection,
 * in list order. Side effects as the reference (target lists, RNG draws). */
int lnw_observe(lnw_handle *h, int32_t agent, float *obs_blue_dev, float *obs_red_dev,
                void *stream);
/* lnw_observe with the rows of env e at obs + e * stride (floats; 0 = the
 * packed n * D; else a multiple of 4, at least n * D) and NULL for a side whose
 * rows nobody reads (its get_obs calls and their side effects still run):
 * the MAPPO rollout observes straight into its buffer (ppo.py:497-575). */
int lnw_observe_ex(lnw_handle *h, int32_t agent, float *obs_blue_dev, int64_t blue_env_stride,
                   float *obs_red_dev, int64_t red_env_stride, void *stream);

/* ---- state access (tests, facade, checkpoint) --------------------------- */
#define LNW_F_POS 0        /* [A][E] u32: x | y<<16                          */
#define LNW_F_RADAR 1      /* [A][E] i32                                     */
#define LNW_F_MISSILES 2   /* [A][E] u8  missile count                       */
#define LNW_F_MKIND 3      /* [A][E] u8  value kind of the missile count     */
#define LNW_F_ALIVE 4      /* [A][E] u8  list slot is not None               */
#define LNW_F_TYPE 5       /* [A][E] u8                                      */
#define LNW_F_STEPS 6      /* [A][E] i32 ship.steps_done                     */
#define LNW_F_DIST_LZ 7    /* [A][E] f64 LandingShip.distance_to_landing_zone */
#define LNW_F_TL_CNT 8     /* [A][E] u16 len(target_list)                    */
#define LNW_F_TL 9         /* [A][T][E] u16 x | y<<8                         */
#define LNW_F_DUCT 10      /* [E] f64                                        */
#define LNW_F_ENV 11       /* [8][E] i32: n_blue_left, n_red_left, steps_done,
                              blue_victory, red_victory, blue_engagements,
                              red_engagements, episode                      */
#define LNW_F_RNG 12       /* [E] u64 Philox counter or tape cursor          */
#define LNW_F_ERR 13       /* [E] u32 LNW_ERRF_* bits                        */
#define LNW_NFIELDS 14

/* Device pointer and byte size of one state field (valid until lnw_destroy). */
int lnw_state_field(lnw_handle *h, int32_t field, void **dev_ptr, int64_t *nbytes);

/* Whole-state snapshot (SURVEY.md §8(b) lnw_get_state / lnw_set_state; the
 * reference has no counterpart: its state is the Game object itself, and
 * checkpointing it means pickling that object). A snapshot holds every state
 * field above, the spawn spec and per-env spawn cells the in-kernel auto-reset
 * reads, the RNG mode and seed, and a header naming the handle's shape and a
 * hash of its terrain. lnw_set_state restores it into any handle of the same
 * shape (envs, team sizes, grid) and terrain — the same one later, or a fresh
 * one — after which stepping continues exactly as the saved handle would have.
 * A tape-mode snapshot restores the tape cursors only: bind the same tape with
 * lnw_set_rng first. dst / src: host or device memory of at least
 * lnw_state_bytes(h) bytes. Both wait for `stream` and copy synchronously. */
int64_t lnw_state_bytes(lnw_handle *h);
int lnw_get_state(lnw_handle *h, void *dst, int64_t nbytes, void *stream);
int lnw_set_state(lnw_handle *h, const void *src, int64_t nbytes, void *stream);

/* The step kernel the last lnw_step launched (build-side launch shape, no
 * reference counterpart; tests use it to know which code path they checked). */
#define LNW_KERNEL_NONE 0
#define LNW_KERNEL_GENERIC 1       /* one lane per env, runtime team sizes         */
#define LNW_KERNEL_TEAM 2          /* 2v2/3v3/4v4, one unit (<= 64 envs) per workgroup */
#define LNW_KERNEL_TEAM_CONTACT 3  /* the same, contact variant (lnw_set_variant)  */
#define LNW_KERNEL_UNITS 4         /* 4v4 headline: four 64-env units per workgroup */
#define LNW_KERNEL_GROUP 5         /* runtime team sizes, 16 lanes per env         */
#define LNW_KERNEL_REFLOS 6        /* los_mode 2 (the reference's LOS work)        */
int lnw_step_kernel(lnw_handle *h);
/* Target-list capacity T per agent (= max(nb,nr) + max(nb,nr)^2, never overflows). */
int lnw_tlist_cap(lnw_handle *h);
/* Environments per workgroup of the step / observe launches (build-side launch
 * shape, no reference counterpart). epw = 0 restores the automatic choice made
 * by lnw_load_terrain: 64 (one env per lane) unless E is too small to fill the
 * GPU, then fewer per workgroup. 1 <= epw <= 64 forces it (results do not depend
 * on it; tests use it to cover both launch shapes). Returns the epw in force, or
 * a negative LNW_E* code. */
int lnw_set_epw(lnw_handle *h, int32_t epw);

/* Step-kernel code variant for 2v2 / 3v3 / 4v4 (build-side, no reference
 * counterpart; results are identical either way). contact = 0 (default): the
 * variant tuned for envs whose fleets are mostly out of sensor range (the
 * quiet-workgroup path, BASELINE's reference spawns). contact = 1: get_obs
 * pair walk as bit masks over registers and two EW bearings per iteration,
 * faster when fleets are in contact every step (melee, MAPPO rollouts against
 * a closing red) but slower on the quiet path, which shares the kernel. */
int lnw_set_variant(lnw_handle *h, int32_t contact);

/* Work counters (diagnostics, no reference counterpart): while bound, the step
 * and observe kernels add to counters_dev[0] the LOS rays they ray-march
 * (queries outside the LOS table, or every query with los_mode = 1), to [1] the
 * Bresenham cells those rays visit (combatant.py:411-456) and to [2] the A*
 * searches they run (targets outside the move table, or move_mode = 1;
 * combatant.py:289-408), to [3] the EW bearings evaluated pooled across lanes:
 * by the contact variant in wave-pooled rounds (get_obs calls whose busiest
 * lane has more than two), by the group kernel (runtime team sizes) every
 * bearing of an opponent that gets a fix (spread over the env's 16 lanes).
 * counters_dev: [4] uint64 device array, or NULL to unbind. Costs one uniform
 * branch per march / search / pooled get_obs while unbound. */
int lnw_set_counters(lnw_handle *h, uint64_t *counters_dev);

/* Reward / cog output type of lnw_step. f64 = 0 (default): rew_blue, rew_red and
 * cog are float32 arrays; f64 = 1: they are float64 arrays (pass double* cast to
 * float*), the exact values the reference returns as Python floats
 * (game.py:214-295, 507-525) rather than their float32 rounding. */
int lnw_set_reward_dtype(lnw_handle *h, int32_t f64);

/* ---- unit kernels (parity tests, standalone use) ------------------------ */
/* LOS (radar thr = move_thr; EW thr): out[i] = bit0 radar clear | bit1 EW clear
 * for pairs[i] = (x1, y1, x2, y2), traced from (x1,y1) to (x2,y2); every cell of
 * the pairs must lie on the G x G grid. Rays march from the grid's 2-bit mask
 * staged in LDS per workgroup (G <= 512, pairs_dev 8-byte aligned), else from
 * HBM. */
int lnw_los_batch(const uint8_t *grid_dev, int32_t G, const int16_t *pairs_dev, int64_t n,
                  int32_t move_thr, int32_t ew_thr, uint8_t *out_dev, void *stream);
/* A*: plen[i] (-1 = None), kind[i] (0 goal, 1 timeout, 2 none), feasible[i]
 * (check_path) for ship type types[i] from start[i] to target[i]. */
int lnw_astar_batch(const uint8_t *grid_dev, int32_t G, int32_t move_thr, const int8_t *types_dev,
                    const int16_t *start_dev, const int16_t *target_dev, int64_t n,
                    int16_t *plen_dev, int8_t *kind_dev, uint8_t *feasible_dev, void *stream);
/* Continuous move target: rounded (x,y) and feasibility (can_move_to && check_path)
 * through the handle's structures (table or direct A* per params.move_mode). */
int lnw_move_batch(lnw_handle *h, const int8_t *types_dev, const int16_t *pos_dev,
                   const double *act_dev /* [n][2] */, const uint8_t *is_f32_dev, int64_t n,
                   int32_t *rounded_dev, uint8_t *ok_dev, void *stream);
/* check_path(start, target) through the handle's move table (params.move_mode 0,
 * targets within +-4) or the A* replica. start must lie inside the grid. */
int lnw_path_query(lnw_handle *h, const int8_t *types_dev, const int16_t *start_dev,
                   const int16_t *target_dev, int64_t n, uint8_t *out_dev, void *stream);
/* The handle's LOS query (table or march per params.los_mode). Together with
 * params.los_mode = 1 (every query marched) and 2 (the reference's full
 * own x opponent LOS work inside the step), this is what SURVEY.md §8(b)'s
 * lnw_debug_los (the full unpruned LOS matrix) was to provide: any pair set
 * can be queried through the step's own LOS path, bit-exact with
 * check_line_of_sight (combatant.py:436-456). */
int lnw_los_query(lnw_handle *h, const int16_t *pairs_dev, int64_t n, uint8_t *out_dev,
                  void *stream);

/* Stream-ordered byte copy (device<->device/host), for state access. */
int lnw_copy(void *dst, const void *src, int64_t nbytes, void *stream);

/* Philox U[0,1) float32 fill keyed by (seed, offset + i): synthetic actions. */
int lnw_fill_uniform_f32(float *out_dev, int64_t n, uint64_t seed, uint64_t offset,
                         void *stream);

/* ---- analytics side channels ----------------------
 * Device counterparts of Game.heatmap / coldmap / launch_sites / engagements /
 * blue_ew / red_ew (game.py:119-154; written at combatant.py:640-657 and
 * 146-150), accumulated over every env and step while bound. Each pointer may
 * be NULL (that channel is off); lnw_set_analytics(h, NULL) turns all off.
 * Maps are indexed [x * 100 + y] like the reference's 100x100 arrays (cells
 * outside them are skipped). Log records are 4 x uint32:
 *   engagement: env, step | side << 16 | missiles << 24, shooter x | y << 16,
 *               target x | y << 16          (every hit; missiles 0 = main gun)
 *   EW fix:     env, step | side << 16, observer x | y << 16,
 *               (uint16)fix_x | (uint16)fix_y << 16   (every finite EW fix)
 * with env the global env id, step the episode step (0-based) and side 0 blue /
 * 1 red. *_count are incremented atomically per record; records past *_cap are
 * counted but not stored. */
typedef struct lnw_analytics {
  uint32_t *heatmap;   /* [100*100] shooter cells of missile hits by the params.side side */
  uint32_t *coldmap;   /* [100*100] target cells of those hits */
  uint32_t *launch;    /* [2][100*100] missile-hit launch cells (blue, red) */
  uint32_t *eng_log;   /* [eng_cap][4] */
  uint32_t *eng_count; /* [1] */
  int64_t eng_cap;
  uint32_t *ew_log;    /* [ew_cap][4] */
  uint32_t *ew_count;  /* [1] */
  int64_t ew_cap;
} lnw_analytics;
int lnw_set_analytics(lnw_handle *h, const lnw_analytics *a);

/* ---- batched policy forward -------------------------
 * The convolutional head and LayerNorm of the reference actor (network.py:70-85:
 * conv 1->5, BatchNorm, ReLU, 2x2 max pool, conv 5->8, BatchNorm, ReLU, pool,
 * linear 8->12, LayerNorm over [head, obs[49:]]) for B observation rows of
 * obs_dim floats (the first 49 are the 7x7 window): out[B][n_in], n_in =
 * obs_dim - 37 (<= 64). params: 578 + 2 n_in floats packed by
 * lnw.rollout.BatchedActor.packed_features(). bn_running 0: per-row BatchNorm
 * statistics (the reference's training-mode one-state calls), 1: running. */
int lnw_actor_features(const float *params_dev, int32_t obs_dim, const float *obs_dev, int64_t B,
                       int32_t bn_running, float *out_dev /* [B][n_in] */, void *stream);

/* ---- fused rollout step of the MAPPO caller -----
 * lnw_policy_act replaces, per step and side, the reference rollout's actor
 * calls (ppo.py:497-575: MLP.forward per live ship, network.py:70-115, or
 * MLP.get_dist :117-152 for given actions) and the assembly of the action
 * array (ppo.py:515-577), for every env at once: conv head + LayerNorm + tanh
 * MLP + Normal heads, a keyed Philox sample clamped to [0, 1] (+ N(0, noise)),
 * its log-probability, then the f64 rows lnw_step takes (sunk ships 0), the
 * rollout buffer rows, scripted red rows (red_steps*.csv, ppo.py:560-566) and
 * the rows' value kinds (np.asarray of the step's rows, ppo.py:577).
 * params: BatchedActor.packed_policy() (lnw/rollout.py). One launch. */
typedef struct lnw_policy_args {
  const float *obs;            /* [E][n][D] this side's observation rows (16-B aligned) */
  int64_t E;
  int32_t n, D, own0, A;       /* ships of the side, row length, first agent slot, agents per env */
  const float *params;
  int32_t bn_running;          /* 0: per-row BatchNorm statistics (training-mode batch-1 calls) */
  int32_t forced;              /* 1: log-probabilities of forced_act (get_dist), no sampling */
  const float *forced_act;     /* rows of 4 floats: env e ship i at [e * fa_env_stride + 4 i] */
  int64_t fa_env_stride;
  float noise;                 /* > 0: + noise * N(0, 1) before the clamp */
  uint64_t seed;               /* keyed draws: Philox(seed) at slot (call * T + t) * 4 + which */
  const int64_t *call_dev;     /* rollout index, read on the device (NULL = 0) */
  int32_t T, t, which;
  int64_t row_base;            /* global id of row 0 (env_id_base * n) */
  const uint8_t *alive;        /* [A][E] the handle's LNW_F_ALIVE field */
  const uint8_t *live;         /* [E] episode still running (NULL: all) */
  float *obs_out;              /* NULL, or rollout rows: env e at obs_out + e * obs_env_stride */
  int64_t obs_env_stride;
  float *act_out, *logp_out;   /* NULL, or rollout rows of 4: env e ship i at e * act_env_stride + 4 i */
  int64_t act_env_stride;
  double *full;                /* [E][A][4] action array of lnw_step (this side's rows), or NULL */
  const double *script;        /* NULL, or scripted rows [script_n][script_steps][4] */
  int32_t script_n, script_steps, script_own0, script_cnt;
  uint8_t *kinds;              /* NULL, or [E][A] row kinds for lnw_step */
  int32_t kinds_f32_all_alive; /* 1: LNW_KIND_F32 rows when every ship is alive, else F64 */
  uint8_t *f32_out;            /* NULL, or env e at f32_out[e * f32_env_stride]: the rows are F32 */
  int64_t f32_env_stride;
  int64_t obs_in_env_stride;   /* floats between envs' rows in obs (0: n * D). obs_out == obs with
                                  obs_env_stride == this stride: the rows already sit in the rollout
                                  buffer (lnw_observe_ex wrote them there), and only the rows of
                                  envs whose episode ended (live == 0) are zeroed in place */
} lnw_policy_args;
int lnw_policy_act(const lnw_policy_args *args, void *stream);

/* After lnw_step: the rollout's bookkeeping of step t (ppo.py:598-641) and the
 * critic (Value, network.py:154-172) on the rows the actor saw: value (0 after
 * the episode ended), rewards (ditto), running flag, and live &= done != 0. */
typedef struct lnw_rollout_post_args {
  const float *obs;            /* rollout rows of step t: env e at obs + e * obs_env_stride, [n][D] */
  int64_t obs_env_stride, E;
  int32_t n, D;
  const float *critic;         /* BatchedCritic.packed(), or NULL (no value) */
  float *val;                  /* env e at val[e * val_env_stride] */
  int64_t val_env_stride;
  const void *rew;             /* [E][n_rew] lnw_step rewards (float32, or float64 if rew_f64) */
  int32_t rew_f64, n_rew;
  double *rew_out;             /* NULL, or env e at rew_out + e * rew_env_stride */
  int64_t rew_env_stride;
  const int32_t *done;         /* [E] lnw_step done */
  uint8_t *live;               /* [E] in/out */
  uint8_t *running;            /* NULL, or env e at running[e * running_env_stride] */
  int64_t running_env_stride;
  int32_t stop_at_done;        /* mask values / rewards after the episode ended, update live */
} lnw_rollout_post_args;
int lnw_rollout_post(const lnw_rollout_post_args *args, void *stream);

/* Host-side constants the kernels use (for tests): hit probability tables
 * 1-(1-p)^n for p in {0.45, 0.63}, n = 0..8, in float64 and float32. */
int lnw_hit_tables(double *tab64 /* [2][9] */, float *tab32 /* [2][9] */);

#ifdef __cplusplus
}
#endif
#endif /* LNW_H */
