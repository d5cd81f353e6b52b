/*
 * lnw_oracle.c — CPU restatement of the reference environment step.
 *
 * TEST INFRASTRUCTURE ONLY. This file is the parity oracle for the HIP path:
 * only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * it, and only as the checker (or the timed CPU baseline), never as the product.
 *
 * It is a single-environment, line-by-line restatement of the reference's
 * Python (valauri/Littoral-Naval-Warfare-MARL):
 *   game.py        Game.reset (528-613), Game.step (298-525),
 *                  Game.calculate_reward (214-295)
 *   combatant.py   get_obs (90-233), radar_range/ew_range (235-247),
 *                  calculate_bearing (249-263), calculate_fixed_position
 *                  (265-277), astar (289-379), check_path (382-408),
 *                  bresenham_line (411-433), check_line_of_sight (436-456),
 *                  continuous_to_discrete (459-476), can_move_to (482-489),
 *                  take_action (501-565), check_target (570-584),
 *                  fire_missile (587-668), calculate_hit_probability (672-680),
 *                  value_to_coordinates (689-704)
 *   landingship.py the LandingShip differences (speed 2, mast 30, rcs 0.9,
 *                  missiles 0, asymmetric 5x5 window 169-188, check_path
 *                  manhattan limit 393/406)
 * It is pinned by the golden vectors in tests/golden/ (captured from the
 * reference itself, see tests/golden/make_golden.py).
 *
 * NumPy-2 (NEP 50) dtype semantics of the reference are reproduced: a value's
 * "kind" (Python int, Python float, np.float32, np.float64) decides whether a
 * product is evaluated in float32 or float64.
 *
 * Build: gcc -O2 -ffp-contract=off -fno-fast-math -shared -fPIC (see Makefile).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ORC_MAX_AGENTS 64
#define ORC_TMAX 1024
#define ORC_NEUT_MAX 4096

/* value kinds (NEP 50 promotion lattice) */
enum { K_PYINT = 0, K_PYFLOAT = 1, K_F32 = 2, K_F64 = 3 };
/* ship types */
enum { T_SMALL = 0, T_LARGE = 1, T_LS = 2, T_MEDIUM = 3 };
/* error flags (reference crash modes, recorded instead of raising) */
enum {
    ORC_ERR_ZERODIV = 1,      /* combatant.py:274 ZeroDivisionError */
    ORC_ERR_NAN_ROUND = 2,    /* round(nan/inf) ValueError/OverflowError */
    ORC_ERR_TAPE = 4,         /* tape exhausted */
    ORC_ERR_TLIST = 8,        /* target list overflow */
    ORC_ERR_NEUT = 16,        /* neutralized list overflow */
};

typedef struct {
    int discrete, landing_ops, aggressive, side_blue, trained_red;
    double red_aggression;
    int move_thr, ew_thr;
    int lz_x, lz_y;
} orc_params;

typedef struct {
    int side, type, x, y, radar, alive, steps_done;
    double missiles;
    int mkind; /* kind of self.missiles */
    double dist_lz;
    int lz_x, lz_y;
    int tl_n;
    int tl[ORC_TMAX][2];
} orc_ship;

typedef struct {
    orc_params P;
    const uint8_t *grid;
    int G;
    int nb, nr;
    orc_ship s[ORC_MAX_AGENTS];
    double ducting;
    int n_blue_left, n_red_left, steps_done;
    int blue_victory, red_victory, blue_eng, red_eng;
    int neut_n[2];
    int neut[2][ORC_NEUT_MAX];
    /* rng */
    int rng_mode; /* 0 philox, 1 tape */
    const double *tape;
    int64_t tape_len, tape_pos;
    uint64_t seed, env_gid, ctr;
    uint32_t err;
} orc_env;

/* ------------------------------------------------------------------------ */
/* numeric helpers                                                           */
/* ------------------------------------------------------------------------ */
static const double PY_PI = 3.141592653589793;
/* CPython mathmodule.c: degrees(x) = x * (180/pi), radians(x) = x * (pi/180) */
static double py_degrees(double x) { return x * (180.0 / PY_PI); }
static double py_radians(double x) { return x * (PY_PI / 180.0); }
/* Python round()/np.round: half to even */
static double py_round(double x) { return nearbyint(x); }

static int kind_promote(int a, int b) {
    if (a == K_F64 || b == K_F64) return K_F64;
    if (a == K_F32 || b == K_F32) return K_F32;
    if (a == K_PYFLOAT || b == K_PYFLOAT) return K_PYFLOAT;
    return K_PYINT;
}

/* a*b evaluated in the promoted kind */
static double kmul(double a, int ka, double b, int kb, int *kout) {
    int k = kind_promote(ka, kb);
    *kout = k;
    if (k == K_F32) return (double)((float)a * (float)b);
    return a * b;
}

/* ------------------------------------------------------------------------ */
/* RNG: Philox4x32-10 production stream, or a recorded tape                  */
/* ------------------------------------------------------------------------ */
static void philox(uint32_t ctr[4], uint32_t key[2], uint32_t out[4]) {
    uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3];
    uint32_t k0 = key[0], k1 = key[1];
    for (int r = 0; r < 10; r++) {
        uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
        uint32_t n1 = (uint32_t)p1;
        uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        uint32_t n3 = (uint32_t)p0;
        c0 = n0; c1 = n1; c2 = n2; c3 = n3;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

static void rng_block(orc_env *e, uint32_t out[4]) {
    uint32_t ctr[4] = {(uint32_t)e->ctr, (uint32_t)(e->ctr >> 32), (uint32_t)e->env_gid,
                       (uint32_t)(e->env_gid >> 32)};
    uint32_t key[2] = {(uint32_t)e->seed, (uint32_t)(e->seed >> 32)};
    philox(ctr, key, out);
    e->ctr++;
}

static double u53(uint32_t a, uint32_t b) {
    return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6)) / 9007199254740992.0;
}

/* Portable ln(x), x in (0, 1]: only + - * / and frexp/ldexp, so CPU and GPU
 * produce identical bits when built without FP contraction. */
static double p_log(double x) {
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

/* Portable cos(2*pi*u), u in [0, 1) */
static double p_cos2pi(double u) {
    double t = u * 4.0;
    int q = (int)t;
    double r = t - (double)q;
    double th = r * 1.5707963267948966;
    double z = th * th;
    double c = 1.0 / 2432902008176640000.0;        /* 1/20! */
    c = c * -z + 1.0 / 6402373705728000.0;          /* 1/18! */
    c = c * -z + 1.0 / 20922789888000.0;            /* 1/16! */
    c = c * -z + 1.0 / 87178291200.0;               /* 1/14! */
    c = c * -z + 1.0 / 479001600.0;                 /* 1/12! */
    c = c * -z + 1.0 / 3628800.0;                   /* 1/10! */
    c = c * -z + 1.0 / 40320.0;
    c = c * -z + 1.0 / 720.0;
    c = c * -z + 1.0 / 24.0;
    c = c * -z + 1.0 / 2.0;
    c = c * -z + 1.0;
    double s = 1.0 / 51090942171709440000.0;        /* 1/21! */
    s = s * -z + 1.0 / 121645100408832000.0;        /* 1/19! */
    s = s * -z + 1.0 / 355687428096000.0;           /* 1/17! */
    s = s * -z + 1.0 / 1307674368000.0;             /* 1/15! */
    s = s * -z + 1.0 / 6227020800.0;                /* 1/13! */
    s = s * -z + 1.0 / 39916800.0;                  /* 1/11! */
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

static double tape_next(orc_env *e) {
    if (e->tape_pos >= e->tape_len) {
        e->err |= ORC_ERR_TAPE;
        return 0.0;
    }
    return e->tape[e->tape_pos++];
}

/* random.random() */
static double rng_uniform(orc_env *e) {
    if (e->rng_mode == 1) return tape_next(e);
    uint32_t o[4];
    rng_block(e, o);
    return u53(o[0], o[1]);
}

/* random.gauss(0, 1) */
static double rng_gauss(orc_env *e) {
    if (e->rng_mode == 1) return tape_next(e);
    uint32_t o[4];
    rng_block(e, o);
    double a = u53(o[0], o[1]), b = u53(o[2], o[3]);
    return sqrt(-2.0 * p_log(1.0 - a)) * p_cos2pi(b);
}

/* random.randint(a, b) */
static int rng_randint(orc_env *e, int a, int b) {
    if (e->rng_mode == 1) return (int)tape_next(e);
    double u = rng_uniform(e);
    return a + (int)floor(u * (double)(b - a + 1));
}

/* np.random.beta(1, 3): the minimum of three uniforms in production mode */
static double rng_beta13(orc_env *e) {
    if (e->rng_mode == 1) return tape_next(e);
    uint32_t o[4];
    rng_block(e, o);
    double m = ((double)o[0] + 0.5) * 2.3283064365386963e-10;
    double v1 = ((double)o[1] + 0.5) * 2.3283064365386963e-10;
    double v2 = ((double)o[2] + 0.5) * 2.3283064365386963e-10;
    if (v1 < m) m = v1;
    if (v2 < m) m = v2;
    return m;
}

/* ------------------------------------------------------------------------ */
/* ship attributes (combatant.py:60-88, landingship.py:61-92)                */
/* ------------------------------------------------------------------------ */
static int ship_speed(int t) { return (t == T_MEDIUM || t == T_LS) ? 2 : 3; }
static int ship_mast(int t) { return t == T_SMALL ? 15 : 30; }
static double ship_rcs(int t) {
    if (t == T_SMALL) return 0.7;
    if (t == T_LS) return 0.9;
    return 1.0;
}
static double ship_missiles0(int t) {
    if (t == T_LS) return 0.0;
    return t == T_SMALL ? 4.0 : 8.0;
}
/* missiles/(4 if small else 8) */
static double miss_norm(int t) { return t == T_SMALL ? 4.0 : 8.0; }

/* ------------------------------------------------------------------------ */
/* geometry: Bresenham LOS (combatant.py:411-456)                            */
/* ------------------------------------------------------------------------ */
int orc_bresenham_count(int x1, int y1, int x2, int y2) {
    int n = 0;
    int dx = abs(x2 - x1), dy = abs(y2 - y1);
    int sx = x1 > x2 ? -1 : 1, sy = y1 > y2 ? -1 : 1;
    int err = dx - dy;
    for (;;) {
        n++;
        if (x1 == x2 && y1 == y2) break;
        int e2 = 2 * err;
        if (e2 > -dy) { err -= dy; x1 += sx; }
        if (e2 < dx) { err += dx; y1 += sy; }
    }
    return n;
}

/* check_line_of_sight: 1 if every point has grid <= thr.
 * The reference builds the whole point list first and then scans it; the
 * cells visited are the same, and a point outside the grid is indexed with
 * numpy semantics (negative wraps) — never reached for in-grid endpoints. */
int orc_los(const uint8_t *grid, int G, int x1, int y1, int x2, int y2, int thr) {
    int dx = abs(x2 - x1), dy = abs(y2 - y1);
    int sx = x1 > x2 ? -1 : 1, sy = y1 > y2 ? -1 : 1;
    int err = dx - dy;
    for (;;) {
        if (grid[x1 * G + y1] > thr) return 0;
        if (x1 == x2 && y1 == y2) break;
        int e2 = 2 * err;
        if (e2 > -dy) { err -= dy; x1 += sx; }
        if (e2 < dx) { err += dx; y1 += sy; }
    }
    return 1;
}

/* ------------------------------------------------------------------------ */
/* A* (combatant.py:289-379), literal restatement incl. the list-mutation    */
/* quirks of `for index, item in enumerate(open_list): ... open_list.pop()`  */
/* ------------------------------------------------------------------------ */
typedef struct { int x, y, g, parent; double f; } onode;

#define ORC_POOL 4096
/* returns path length (>=1), or -1 for None; *kind: 0 goal, 1 timeout, 2 none.
 * path_ok: 1 if every path cell is <= thr (check_path's final scan). */
int orc_astar(const uint8_t *grid, int G, int thr, int speed, int sx, int sy, int ex, int ey,
              int *kind, int *path_ok) {
    static const int adj[8][2] = {{0, -1}, {0, 1}, {-1, 0}, {1, 0},
                                  {-1, -1}, {-1, 1}, {1, -1}, {1, 1}};
    onode pool[ORC_POOL];
    int npool = 0;
    int open[ORC_POOL];
    int nopen = 0;
    pool[npool] = (onode){sx, sy, 0, -1, 0.0};
    open[nopen++] = npool++;
    double max_distance = sqrt((double)((0 - speed) * (0 - speed) + (0 - speed) * (0 - speed)));
    int iterations = 0;
    int max_iterations = (speed * 2 + 1) * (speed * 2 + 1);
    int cur = -1;
    int res_node = -1;
    int k = 2;
    while (nopen > 0) {
        iterations++;
        if (iterations > max_iterations) {
            res_node = cur;
            k = 1;
            break;
        }
        cur = open[0];
        int ci = 0;
        int children[8], nch = 0;
        int found = 0;
        int it = 0;
        while (it < nopen) {
            int index = it;
            int item = open[it++];
            if (pool[item].f < pool[cur].f) { cur = item; ci = index; }
            /* open_list.pop(current_index) */
            for (int q = ci; q < nopen - 1; q++) open[q] = open[q + 1];
            nopen--;
            if (pool[cur].x == ex && pool[cur].y == ey) { found = 1; break; }
            nch = 0;
            for (int a = 0; a < 8; a++) {
                int nx = pool[cur].x + adj[a][0], ny = pool[cur].y + adj[a][1];
                if (nx > G - 1 || nx < 0 || ny > G - 1 || ny < 0) continue;
                if (grid[nx * G + ny] > thr) continue;
                children[nch++] = a;
            }
        }
        if (found) { res_node = cur; k = 0; break; }
        for (int c = 0; c < nch; c++) {
            int nx = pool[cur].x + adj[children[c]][0], ny = pool[cur].y + adj[children[c]][1];
            int g = pool[cur].g + 1;
            double h = sqrt((double)((nx - ex) * (nx - ex))) + (double)((ny - ey) * (ny - ey));
            double f = (double)g + h;
            double dd = sqrt((double)((nx - sx) * (nx - sx) + (ny - sy) * (ny - sy)));
            if (dd <= max_distance) {
                if (npool >= ORC_POOL) { *kind = 3; return -2; }
                pool[npool] = (onode){nx, ny, g, cur, f};
                open[nopen++] = npool++;
            }
        }
    }
    *kind = k;
    if (res_node < 0) { if (path_ok) *path_ok = 0; return -1; }
    int len = 0, ok = 1;
    for (int n = res_node; n >= 0; n = pool[n].parent) {
        len++;
        if (grid[pool[n].x * G + pool[n].y] > thr) ok = 0;
    }
    if (path_ok) *path_ok = ok;
    return len;
}

/* check_path (combatant.py:382-408; landingship.py:389-415) */
int orc_check_path(const uint8_t *grid, int G, int thr, int type, int ox, int oy, int dx_, int dy_) {
    int speed = ship_speed(type);
    int limit;
    if (type == T_LS)
        limit = abs(ox - dx_) + abs(oy - dy_) + 1;
    else
        limit = speed + 2;
    if (dx_ < 0 || dx_ > 99 || dy_ < 0 || dy_ > 99) return 0;
    int kind, ok;
    int len = orc_astar(grid, G, thr, speed, ox, oy, dx_, dy_, &kind, &ok);
    if (len < 0 || len > limit) return 0;
    return ok;
}

/* can_move_to (combatant.py:482-489): hard-coded 0..99 */
static int can_move_to(const uint8_t *grid, int G, int thr, int x, int y) {
    if (0 <= x && x < 100 && 0 <= y && y < 100) return grid[x * G + y] > thr ? 0 : 1;
    return 0;
}

/* continuous_to_discrete target arithmetic (combatant.py:459-471).
 * kind: K_F32 for np.float32 actions, K_F64/K_PYFLOAT for doubles.
 * Returns 0 when float_x or float_y is not finite: round() of it raises
 * (ValueError for nan, OverflowError for inf, combatant.py:470-471); the target
 * is then (-10^6, -10^6), never feasible. Finite targets beyond +-10^6 are just
 * out of the grid (Python rounds them to a big int). */
int orc_move_target(int px, int py, int speed, double a2, double a3, int kind, int *nx, int *ny) {
    double rx, ry;
    if (kind == K_F32) {
        float course = (float)(2.0 * PY_PI) * (float)a2;
        float dist = (float)speed * (float)a3;
        double deg = py_degrees((double)course);
        float dx = (float)cos(deg) * dist;
        float dy = (float)sin(deg) * dist;
        float fx = (float)px + dx;
        float fy = (float)py + dy;
        rx = (double)nearbyintf(fx);
        ry = (double)nearbyintf(fy);
    } else {
        double course = 2.0 * PY_PI * a2;
        double dist = (double)speed * a3;
        double deg = py_degrees(course);
        double dx = cos(deg) * dist;
        double dy = sin(deg) * dist;
        rx = py_round((double)px + dx);
        ry = py_round((double)py + dy);
    }
    if (!(fabs(rx) < 1.0e6) || !(fabs(ry) < 1.0e6)) {
        *nx = *ny = -1000000;
        return isfinite(rx) && isfinite(ry);
    }
    *nx = (int)rx;
    *ny = (int)ry;
    return 1;
}

/* floor division / modulo with Python semantics */
static int py_floordiv(int a, int b) { int q = a / b; if ((a % b != 0) && ((a < 0) != (b < 0))) q--; return q; }
static int py_mod(int a, int b) { int m = a % b; if (m != 0 && ((m < 0) != (b < 0))) m += b; return m; }

/* ------------------------------------------------------------------------ */
/* environment                                                               */
/* ------------------------------------------------------------------------ */
size_t orc_env_size(void) { return sizeof(orc_env); }

void orc_env_init(orc_env *e, const orc_params *P, const uint8_t *grid, int G, int nb, int nr) {
    memset(e, 0, sizeof(*e));
    e->P = *P;
    e->grid = grid;
    e->G = G;
    e->nb = nb;
    e->nr = nr;
}

void orc_set_rng(orc_env *e, int mode, uint64_t seed, uint64_t env_gid, uint64_t ctr,
                 const double *tape, int64_t tape_len, int64_t tape_pos) {
    e->rng_mode = mode;
    e->seed = seed;
    e->env_gid = env_gid;
    e->ctr = ctr;
    e->tape = tape;
    e->tape_len = tape_len;
    e->tape_pos = tape_pos;
}

/* Game.reset (game.py:528-613). types[A], pos[A][2]; rand_ls[A] = 1 draws the
 * landing-ship spawn with random.randint(98,99), randint(48,56) (game.py:589). */
void orc_reset(orc_env *e, const int *types, const int *pos, const int *rand_ls) {
    e->steps_done = 0;
    e->ducting = 1.0 + rng_beta13(e);
    e->blue_victory = 0;
    e->red_victory = 0;
    int A = e->nb + e->nr;
    for (int a = 0; a < A; a++) {
        orc_ship *s = &e->s[a];
        memset(s, 0, sizeof(*s));
        s->side = a < e->nb ? 0 : 1;
        s->type = types[a];
        s->x = pos[2 * a];
        s->y = pos[2 * a + 1];
        s->radar = 1;
        s->alive = 1;
        s->missiles = ship_missiles0(s->type);
        s->mkind = K_PYINT;
        s->lz_x = e->P.lz_x;
        s->lz_y = e->P.lz_y;
    }
    for (int a = 0; a < A; a++) {
        orc_ship *s = &e->s[a];
        if (rand_ls && rand_ls[a]) {
            int xs = rng_randint(e, 98, 99);
            int ys = rng_randint(e, 48, 56);
            s->x = xs;
            s->y = ys;
        }
        if (s->type == T_LS) {
            int ddx = s->x - s->lz_x, ddy = s->y - s->lz_y;
            s->dist_lz = sqrt((double)(ddx * ddx + ddy * ddy));
        }
    }
    e->n_blue_left = e->nb;
    e->n_red_left = e->nr;
}

void orc_set_ducting(orc_env *e, double d) { e->ducting = d; }

/* radar_range / ew_range (combatant.py:235-247) */
static double base_d(int mast_a, int mast_b) {
    double d = sqrt((4.0 / 3.0) * 6370.0 * 2.0) *
               (sqrt((double)mast_a / 1000.0) + sqrt((double)mast_b / 1000.0));
    return d;
}
int orc_radar_range(double duct, int t_ship, int t_opp) {
    double d = base_d(ship_mast(t_ship), ship_mast(t_opp));
    d = d / 5.0;
    return (int)ceil(d * ship_rcs(t_opp) * duct);
}
int orc_ew_range(double duct, int t_ship, int t_opp) {
    double d = base_d(ship_mast(t_ship), ship_mast(t_opp));
    d = (d / 5.0) * duct;
    d = 2.0 * d;
    return (int)ceil(d);
}

/* numpy mean of a float64 list (pairwise_sum for n >= 8) */
static double np_mean(const double *v, int n) {
    double res;
    if (n < 8) {
        res = 0.0;
        for (int i = 0; i < n; i++) res += v[i];
    } else if (n <= 128) {
        double r[8];
        for (int j = 0; j < 8; j++) r[j] = v[j];
        int i;
        for (i = 8; i < n - (n % 8); i += 8)
            for (int j = 0; j < 8; j++) r[j] += v[i + j];
        res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; i++) res += v[i];
    } else {
        res = 0.0; /* not reachable: <= ORC_MAX_AGENTS bearings */
        for (int i = 0; i < n; i++) res += v[i];
    }
    return res / (double)n;
}

/* get_obs (combatant.py:90-233 / landingship.py:94-239). Writes D values. */
static void get_obs(orc_env *e, int a, double *out) {
    orc_ship *me = &e->s[a];
    int G = e->G;
    int own0 = me->side == 0 ? 0 : e->nb, nown = me->side == 0 ? e->nb : e->nr;
    int opp0 = me->side == 0 ? e->nb : 0, nopp = me->side == 0 ? e->nr : e->nb;
    me->tl_n = 0;
    int obs_n = 0;
    int obs_xy[ORC_MAX_AGENTS][2];
    /* electronic_bearings: insertion-ordered dict keyed by opponent */
    int b_order[ORC_MAX_AGENTS], b_norder = 0;
    int b_cnt[ORC_MAX_AGENTS];
    int b_ship[ORC_MAX_AGENTS][ORC_MAX_AGENTS];
    double b_val[ORC_MAX_AGENTS][ORC_MAX_AGENTS];
    memset(b_cnt, 0, sizeof(b_cnt));
    for (int i = own0; i < own0 + nown; i++) {
        orc_ship *sh = &e->s[i];
        if (!sh->alive) continue;
        for (int j = opp0; j < opp0 + nopp; j++) {
            orc_ship *op = &e->s[j];
            if (!op->alive) continue;
            if (!orc_los(e->grid, G, sh->x, sh->y, op->x, op->y, e->P.move_thr)) continue;
            int ddx = op->x - sh->x, ddy = op->y - sh->y;
            double dist = sqrt((double)(ddx * ddx + ddy * ddy));
            int seen;
            if (me->radar == 1) {
                if (dist < (double)orc_radar_range(e->ducting, sh->type, op->type)) {
                    seen = 0;
                    for (int q = 0; q < obs_n; q++)
                        if (obs_xy[q][0] == op->x && obs_xy[q][1] == op->y) seen = 1;
                    if (!seen) { obs_xy[obs_n][0] = op->x; obs_xy[obs_n][1] = op->y; obs_n++; }
                }
            }
            seen = 0;
            for (int q = 0; q < obs_n; q++)
                if (obs_xy[q][0] == op->x && obs_xy[q][1] == op->y) seen = 1;
            if (dist < 4.0 && !seen) { obs_xy[obs_n][0] = op->x; obs_xy[obs_n][1] = op->y; obs_n++; }
            if (dist < (double)orc_ew_range(e->ducting, sh->type, op->type) && op->radar == 1 &&
                orc_los(e->grid, G, sh->x, sh->y, op->x, op->y, e->P.ew_thr)) {
                seen = 0;
                for (int q = 0; q < obs_n; q++)
                    if (obs_xy[q][0] == op->x && obs_xy[q][1] == op->y) seen = 1;
                if (!seen) {
                    /* calculate_bearing (combatant.py:249-263) */
                    double bearing = py_degrees(atan2((double)ddy, (double)ddx));
                    double distortion = rng_gauss(e);
                    if (bearing + distortion < 0)
                        bearing = bearing + distortion + 360.0;
                    else
                        bearing = bearing + distortion;
                    int jj = j - opp0;
                    if (b_cnt[jj] == 0) b_order[b_norder++] = jj;
                    b_ship[jj][b_cnt[jj]] = i;
                    b_val[jj][b_cnt[jj]] = bearing;
                    b_cnt[jj]++;
                }
            }
        }
    }
    /* EW fixes (combatant.py:128-150) */
    int fix_n = 0;
    int fix_xy[ORC_MAX_AGENTS][2];
    for (int o = 0; o < b_norder; o++) {
        int jj = b_order[o];
        int n = b_cnt[jj];
        if (n > 1) {
            double ex[ORC_MAX_AGENTS], ey[ORC_MAX_AGENTS];
            int ne = 0, bad = 0;
            for (int q = 0; q + 1 < n; q++) {
                orc_ship *s1 = &e->s[b_ship[jj][q]], *s2 = &e->s[b_ship[jj][q + 1]];
                double x1 = s1->x, y1 = s1->y, x2 = s2->x, y2 = s2->y;
                double m1 = tan(py_radians(b_val[jj][q]));
                double m2 = tan(py_radians(b_val[jj][q + 1]));
                if (m1 - m2 == 0.0) { bad = 1; break; }
                double x3 = (m1 * x1 - m2 * x2 + y2 - y1) / (m1 - m2);
                double y3 = m1 * (x3 - x1) + y1;
                ex[ne] = x3;
                ey[ne] = y3;
                ne++;
            }
            if (bad) { e->err |= ORC_ERR_ZERODIV; continue; }
            double mx = np_mean(ex, ne), my = np_mean(ey, ne);
            if (!isfinite(mx) || !isfinite(my)) {
                /* round(nan) -> ValueError, round(inf) -> OverflowError */
                e->err |= ORC_ERR_NAN_ROUND;
                continue;
            }
            double rx = py_round(mx), ry = py_round(my);
            /* a fix outside the grid never becomes a target (combatant.py:158) */
            fix_xy[fix_n][0] = (rx >= 0.0 && rx < (double)G) ? (int)rx : -1;
            fix_xy[fix_n][1] = (ry >= 0.0 && ry < (double)G) ? (int)ry : -1;
            fix_n++;
        }
    }
    for (int q = 0; q < obs_n; q++) {
        if (me->tl_n >= ORC_TMAX) { e->err |= ORC_ERR_TLIST; break; }
        me->tl[me->tl_n][0] = obs_xy[q][0];
        me->tl[me->tl_n][1] = obs_xy[q][1];
        me->tl_n++;
    }
    for (int f = 0; f < fix_n; f++) {
        int x = fix_xy[f][0], y = fix_xy[f][1];
        if (0 <= x && x < G && 0 <= y && y < G) {
            for (int j = opp0; j < opp0 + nopp; j++) {
                orc_ship *op = &e->s[j];
                if (!op->alive) continue;
                int ddx = op->x - x, ddy = op->y - y;
                if (sqrt((double)(ddx * ddx + ddy * ddy)) < 2.0) {
                    if (me->tl_n >= ORC_TMAX) { e->err |= ORC_ERR_TLIST; break; }
                    me->tl[me->tl_n][0] = x;
                    me->tl[me->tl_n][1] = y;
                    me->tl_n++;
                }
            }
        }
    }
    /* observation vector */
    int D = nown * 4 + 49 + 3;
    for (int q = 0; q < D; q++) out[q] = 0.0;
    int idx = 0;
    if (me->type == T_LS) {
        int speed = 2;
        int sx = me->x - speed, sy = me->y - speed;
        int W = (speed + 1) * 2 + 1;
        for (int x = sx; x < sx + W; x++)
            for (int y = sy; y < sy + W; y++) {
                if (x == sx || y == sy || x == sx + (speed + 1) * 2 || y == sy + (speed + 1) * 2)
                    continue;
                if (0 <= x && x < 100 && 0 <= y && y < 100)
                    out[idx++] = (double)e->grid[x * G + y] / 255.0;
                else
                    out[idx++] = 0.0;
            }
    } else {
        int speed = ship_speed(me->type);
        int sx = me->x - speed, sy = me->y - speed;
        for (int x = sx; x < sx + speed * 2 + 1; x++)
            for (int y = sy; y < sy + speed * 2 + 1; y++) {
                if (0 <= x && x < 100 && 0 <= y && y < 100)
                    out[idx++] = (double)e->grid[x * G + y] / 255.0;
                else
                    out[idx++] = 0.0;
            }
    }
    out[idx++] = (double)me->x / (double)G;
    out[idx++] = (double)me->y / (double)G;
    out[idx++] = (double)me->radar;
    out[idx++] = me->missiles / miss_norm(me->type);
    for (int i = own0; i < own0 + nown; i++) {
        orc_ship *sh = &e->s[i];
        if (sh->alive) {
            if (i != a) {
                out[idx++] = (double)sh->x / (double)G;
                out[idx++] = (double)sh->y / (double)G;
                out[idx++] = (double)sh->radar;
                out[idx++] = sh->missiles / miss_norm(sh->type);
            }
        } else {
            idx += 4;
        }
    }
    out[idx++] = (double)me->tl_n;
    out[idx++] = me->type == T_LS ? 1.0 : 0.0;
    out[idx] = e->ducting / 2.0;
}

/* check_target (combatant.py:570-584): first live opponent within 3.5 */
static int check_target(orc_env *e, int side, int tx, int ty) {
    int opp0 = side == 0 ? e->nb : 0, nopp = side == 0 ? e->nr : e->nb;
    for (int j = opp0; j < opp0 + nopp; j++) {
        orc_ship *op = &e->s[j];
        if (!op->alive) continue;
        int ddx = op->x - tx, ddy = op->y - ty;
        if (sqrt((double)(ddx * ddx + ddy * ddy)) <= 3.5) return j;
    }
    return -1;
}

static void neutralize(orc_env *e, int side_of_target, int idx) {
    if (e->neut_n[side_of_target] >= ORC_NEUT_MAX) { e->err |= ORC_ERR_NEUT; return; }
    e->neut[side_of_target][e->neut_n[side_of_target]++] = idx;
}

/* fire_missile (combatant.py:587-668). salvo has kind ks. */
static int fire_missile(orc_env *e, int a, int tx, int ty, double salvo, int ks) {
    orc_ship *me = &e->s[a];
    int hit = 0;
    int t = check_target(e, me->side, tx, ty);
    if (t < 0) return 0;
    orc_ship *tg = &e->s[t];
    int ddx = tg->x - me->x, ddy = tg->y - me->y;
    if (sqrt((double)(ddx * ddx + ddy * ddy)) < 2.0) {
        hit = 1; /* main gun */
    } else {
        if (me->missiles == 0.0) return 0;
        int detected = 1;
        double detected_prob = tg->radar == 1 ? 0.345 - 0.1 : 0.345 + 0.1;
        if (rng_uniform(e) < detected_prob) detected = 0;
        double hit_prob = detected ? 0.45 : 0.63;
        double num_msl;
        int kn;
        if (!e->P.discrete) {
            double prod = kmul(me->missiles, me->mkind, salvo, ks, &kn);
            if (kn == K_F32)
                num_msl = (double)nearbyintf((float)prod);
            else
                num_msl = nearbyint(prod);
            if (kn == K_PYINT || kn == K_PYFLOAT) kn = K_F64; /* np.round -> np.float64 */
        } else {
            num_msl = me->type == T_SMALL ? salvo : salvo * 2.0;
            kn = K_PYINT;
        }
        if (num_msl > me->missiles) { num_msl = me->missiles; kn = me->mkind; }
        me->missiles = me->missiles - num_msl;
        me->mkind = kind_promote(me->mkind, kn);
        /* calculate_hit_probability: 1 - (1-p)**n, n of kind kn */
        double u2 = rng_uniform(e);
        if (kn == K_F32) {
            float pn = powf((float)(1.0 - hit_prob), (float)num_msl);
            float prob = 1.0f - pn;
            if ((float)u2 < prob) hit = 1;
        } else {
            double prob = 1.0 - pow(1.0 - hit_prob, num_msl);
            if (u2 < prob) hit = 1;
        }
    }
    if (hit) neutralize(e, tg->side, t - (tg->side == 0 ? 0 : e->nb));
    return hit;
}

/* take_action (combatant.py:501-565). act[4] with per-row kind. */
static void take_action(orc_env *e, int a, const double *act, int kind, double *obs, int *moved,
                        int *engage_out, int *n_destroyed) {
    orc_ship *me = &e->s[a];
    const uint8_t *grid = e->grid;
    int G = e->G, thr = e->P.move_thr;
    double rad_action = act[0];
    double engagement;
    int keng;
    if (e->P.discrete) { engagement = py_round(act[1]); keng = K_PYINT; }
    else { engagement = act[1]; keng = kind; }
    /* new position */
    int feasible = 0, nx = 0, ny = 0;
    if (!e->P.discrete) {
        if (!orc_move_target(me->x, me->y, ship_speed(me->type), act[2], act[3], kind, &nx, &ny))
            e->err |= ORC_ERR_NAN_ROUND;  /* round(nan/inf), combatant.py:470 */
        if (can_move_to(grid, G, thr, nx, ny) &&
            orc_check_path(grid, G, thr, me->type, me->x, me->y, nx, ny))
            feasible = 1;
    } else {
        int v = (int)act[2];
        int x = py_floordiv(v, 7), y = py_mod(v, 7);
        if (0 <= me->x - 3 + x && me->x - 3 + x < G && 0 <= me->y - 3 + y && me->y - 3 + y < G) {
            nx = me->x - 3 + x;
            ny = me->y - 3 + y;
            if (orc_check_path(grid, G, thr, me->type, me->x, me->y, nx, ny)) feasible = 1;
        }
    }
    int kthr;
    double thr_v = kmul(engagement, keng, me->missiles, me->mkind, &kthr);
    double engagement_threshold = kthr == K_F32 ? (double)nearbyintf((float)thr_v) : nearbyint(thr_v);
    if (!isfinite(engagement_threshold)) {
        /* round(nan/inf) of engagement * missiles raises (combatant.py:528): flagged,
         * and the ship then does not engage */
        e->err |= ORC_ERR_NAN_ROUND;
        engagement_threshold = 0.0;
    }
    int engage = engagement_threshold > 0;
    int destroyed = 0;
    if (engage && me->tl_n > 0) {
        for (int q = 0; q < me->tl_n; q++) {
            /* check_target result only feeds the always-true
             * `target not in neutralized_units` test */
            if (fire_missile(e, a, me->tl[q][0], me->tl[q][1], engagement, keng)) destroyed++;
        }
    }
    if (me->side == 0) e->blue_eng += destroyed; else e->red_eng += destroyed;
    if (!isfinite(rad_action)) { e->err |= ORC_ERR_NAN_ROUND; me->radar = 0; }
    else me->radar = (int)py_round(rad_action);
    if (feasible) { me->x = nx; me->y = ny; }
    get_obs(e, a, obs);
    *moved = feasible;
    *engage_out = engage;
    *n_destroyed = destroyed;
}

/* calculate_reward (game.py:214-295) */
static double calculate_reward(orc_env *e, int a, int movement, int engage, int n_hit) {
    orc_ship *u = &e->s[a];
    double reward = 0.0;
    u->steps_done += 1;
    if (u->tl_n > 0) reward += (double)(u->tl_n * 3);
    if (movement) reward += 1.0;
    else reward = fmax(reward - 0.5, 0.0);
    if (u->tl_n > 0 && !engage) reward = reward / 2.0;
    else if (u->tl_n > 0 && engage && n_hit == 0) reward += 0.5;
    reward += (double)(n_hit * 10);
    if (u->side == 1 && u->type != T_LS && !e->P.aggressive) {
        if (u->steps_done > 14) {
            if (u->x < 19 || u->x > 55 || u->y < 40 || u->y > 70) reward = fmax(reward - 2.0, 0.0);
            else reward += 1.0;
        }
    }
    if (u->side == 1 && e->P.aggressive && u->type != T_LS) {
        int fx = 15, fy = 60;
        double nom = fmax(sqrt((double)((u->x - fx) * (u->x - fx) + (u->y - fy) * (u->y - fy))), 1.0);
        double den = (sqrt((4.0 / 3.0) * 6370.0 * 2.0) *
                      (sqrt((double)ship_mast(u->type) / 1000.0) + sqrt(15.0 / 1000.0))) / 5.0;
        double d = (1.0 / (nom / den)) * 1.0;
        reward += d;
    }
    if (u->type == T_LS) {
        int ddx = u->x - u->lz_x, ddy = u->y - u->lz_y;
        double dl = sqrt((double)(ddx * ddx + ddy * ddy));
        if (dl > 0) {
            if (dl < u->dist_lz) { reward += 1.0; u->dist_lz = dl; }
            else reward -= 1.0;
        } else {
            reward += 100.0;
        }
        if (dl == 0) reward += 100.0;
        else reward += log10(100.0 / dl) * 5.0;
    }
    return reward;
}

/* Game.step (game.py:298-525).
 * act: [A][4] doubles; kinds: per-row K_* (NULL = all K_F64); act is updated in
 * place where the reference mutates it (game.py:379).
 * obs_b [nb][Db], obs_r [nr][Dr], rew_b [nb], rew_r [nr]; returns done. */
int orc_step(orc_env *e, double *act, const int *kinds, double *obs_b, double *obs_r, double *rew_b,
             double *rew_r, double *cog) {
    int nb = e->nb, nr = e->nr;
    int Db = nb * 4 + 52, Dr = nr * 4 + 52;
    e->neut_n[0] = e->neut_n[1] = 0;
    for (int q = 0; q < nb * Db; q++) obs_b[q] = 0.0;
    for (int q = 0; q < nr * Dr; q++) obs_r[q] = 0.0;
    int done = 1;
    int alive0[ORC_MAX_AGENTS];
    for (int a = 0; a < nb + nr; a++) alive0[a] = e->s[a].alive;
    int blue_hits = 0, red_hits = 0;
    int eng_b[ORC_MAX_AGENTS] = {0}, eng_r[ORC_MAX_AGENTS] = {0};
    double bsx = 0, bsy = 0, rsx = 0, rsy = 0;
    int nbp = 0, nrp = 0;
    for (int a = 0; a < nb; a++) {
        if (!alive0[a]) { rew_b[a] = 0.0; continue; }
        orc_ship *s = &e->s[a];
        if (e->P.side_blue) { bsx += s->x; bsy += s->y; nbp++; }
        int mv, eg, nd;
        int k = kinds ? kinds[a] : K_F64;
        take_action(e, a, act + 4 * a, k, obs_b + a * Db, &mv, &eg, &nd);
        double r = calculate_reward(e, a, mv, eg, nd);
        if (e->P.side_blue) { if (nd > 0) eng_b[a] = 1; }
        else { if (eg) eng_b[a] = 1; }
        blue_hits += nd;
        rew_b[a] = r;
    }
    for (int a = 0; a < nr; a++) {
        int g = nb + a;
        if (!alive0[g]) { rew_r[a] = 0.0; continue; }
        orc_ship *s = &e->s[g];
        rsx += s->x; rsy += s->y; nrp++;
        int k = kinds ? kinds[g] : K_F64;
        int mv, eg, nd;
        if (!e->P.trained_red) {
            if (rng_uniform(e) < e->P.red_aggression) {
                double v = rng_uniform(e);
                if (k == K_F32) v = (double)(float)v;
                else if (k == K_PYINT) v = trunc(v);
                act[4 * g + 1] = v;
            }
            take_action(e, g, act + 4 * g, k, obs_r + a * Dr, &mv, &eg, &nd);
            double r = calculate_reward(e, g, mv, eg, nd);
            if (eg) eng_r[a] = 1;
            red_hits += nd;
            rew_r[a] = r;
        } else {
            take_action(e, g, act + 4 * g, k, obs_r + a * Dr, &mv, &eg, &nd);
            double r = calculate_reward(e, g, mv, eg, nd);
            red_hits += nd;
            if (nd > 1) eng_r[a] = 1;
            rew_r[a] = r;
        }
    }
    int blue_new_losses = e->neut_n[0];
    e->n_blue_left -= blue_new_losses;
    int red_new_losses = e->neut_n[1];
    e->n_red_left -= red_new_losses;
    int no_blue = e->n_blue_left == 0, no_red = e->n_red_left == 0;
    for (int a = 0; a < nb; a++)
        if (!eng_b[a] && alive0[a]) rew_b[a] += (double)(blue_hits * 2);
    for (int a = 0; a < nr; a++)
        if (!eng_r[a] && alive0[nb + a]) rew_r[a] += (double)(red_hits * 2);
    if (!e->P.aggressive) {
        if (blue_new_losses > 0)
            for (int a = 0; a < nb; a++) rew_b[a] = fmax(rew_b[a] - (double)(blue_new_losses * 5), 0.0);
        if (red_new_losses > 0)
            for (int a = 0; a < nr; a++) rew_r[a] = fmax(rew_r[a] - (double)(red_new_losses * 5), 0.0);
    }
    if (no_blue && !no_red) {
        done = 0;
        if (!e->P.aggressive) for (int a = 0; a < nb; a++) rew_b[a] = rew_b[a] - rew_b[a];
        for (int a = 0; a < nr; a++) rew_r[a] += 100.0;
        e->red_victory++;
    }
    if (no_red && !no_blue) {
        done = 0;
        for (int a = 0; a < nb; a++) rew_b[a] += 100.0;
        if (!e->P.aggressive) for (int a = 0; a < nr; a++) rew_r[a] = rew_r[a] - rew_r[a];
        e->blue_victory++;
    }
    if (no_blue && no_red) {
        done = 0;
        for (int a = 0; a < nb; a++) rew_b[a] += 10.0;
        for (int a = 0; a < nr; a++) rew_r[a] += 10.0;
    }
    if (e->P.landing_ops) {
        int rem = 0;
        for (int a = 0; a < nr; a++)
            if (e->s[nb + a].alive && e->s[nb + a].type == T_LS) rem++;
        if (!rem) {
            done = 0;
            for (int a = 0; a < nb; a++) rew_b[a] += 100.0;
            for (int a = 0; a < nr; a++) rew_r[a] = rew_r[a] - rew_r[a];
            e->blue_victory++;
        } else {
            for (int a = 0; a < nr; a++) {
                orc_ship *s = &e->s[nb + a];
                if (s->alive && s->type == T_LS && s->lz_x == s->x && s->lz_y == s->y) {
                    done = 0;
                    for (int q = 0; q < nb; q++) rew_b[q] = rew_b[q] - rew_b[q];
                    for (int q = 0; q < nr; q++) rew_r[q] += 100.0;
                    e->blue_victory++;
                }
            }
        }
    }
    e->steps_done++;
    for (int q = 0; q < e->neut_n[0]; q++) e->s[e->neut[0][q]].alive = 0;
    for (int q = 0; q < e->neut_n[1]; q++) e->s[nb + e->neut[1][q]].alive = 0;
    if (nbp > 0 && nrp > 0) {
        double bx = bsx / nbp, by = bsy / nbp, rx = rsx / nrp, ry = rsy / nrp;
        *cog = sqrt((bx - rx) * (bx - rx) + (by - ry) * (by - ry));
    } else {
        *cog = NAN;
    }
    return done;
}

/* ship.get_obs() for one agent (callers: main.py:282, ppo.py:500, ddqn.py:296) */
void orc_observe(orc_env *e, int a, double *out) { get_obs(e, a, out); }

/* ------------------------------------------------------------------------ */
/* state access                                                              */
/* ------------------------------------------------------------------------ */
void orc_get_agents(const orc_env *e, int *pos, int *radar, double *missiles, int *mkind, int *alive,
                    int *steps, double *dist_lz, int *tl_cnt) {
    for (int a = 0; a < e->nb + e->nr; a++) {
        const orc_ship *s = &e->s[a];
        pos[2 * a] = s->x;
        pos[2 * a + 1] = s->y;
        radar[a] = s->radar;
        missiles[a] = s->missiles;
        mkind[a] = s->mkind;
        alive[a] = s->alive;
        steps[a] = s->steps_done;
        dist_lz[a] = s->dist_lz;
        tl_cnt[a] = s->tl_n;
    }
}

int orc_get_tlist(const orc_env *e, int a, int *xy, int cap) {
    const orc_ship *s = &e->s[a];
    int n = s->tl_n < cap ? s->tl_n : cap;
    for (int q = 0; q < n; q++) { xy[2 * q] = s->tl[q][0]; xy[2 * q + 1] = s->tl[q][1]; }
    return s->tl_n;
}

void orc_get_env(const orc_env *e, int *out /* 9 ints */, double *ducting, uint32_t *err,
                 int64_t *tape_pos, uint64_t *ctr) {
    out[0] = e->n_blue_left; out[1] = e->n_red_left; out[2] = e->steps_done;
    out[3] = e->blue_victory; out[4] = e->red_victory; out[5] = e->blue_eng; out[6] = e->red_eng;
    out[7] = e->neut_n[0]; out[8] = e->neut_n[1];
    *ducting = e->ducting;
    *err = e->err;
    *tape_pos = e->tape_pos;
    *ctr = e->ctr;
}

/* set an agent's state (tests / state injection) */
void orc_set_agent(orc_env *e, int a, int type, int x, int y, int radar, double missiles, int mkind,
                   int alive, int steps, double dist_lz) {
    orc_ship *s = &e->s[a];
    s->side = a < e->nb ? 0 : 1;
    s->type = type; s->x = x; s->y = y; s->radar = radar; s->missiles = missiles;
    s->mkind = mkind; s->alive = alive; s->steps_done = steps; s->dist_lz = dist_lz;
    s->lz_x = e->P.lz_x; s->lz_y = e->P.lz_y;
}

/* ------------------------------------------------------------------------ */
/* batch helpers for tests                                                   */
/* ------------------------------------------------------------------------ */
void orc_los_batch(const uint8_t *grid, int G, const int16_t *pairs, int64_t n, int thr, uint8_t *out) {
    for (int64_t i = 0; i < n; i++)
        out[i] = (uint8_t)orc_los(grid, G, pairs[4 * i], pairs[4 * i + 1], pairs[4 * i + 2],
                                  pairs[4 * i + 3], thr);
}

void orc_astar_batch(const uint8_t *grid, int G, int thr, const int8_t *cls, const int16_t *st,
                     const int16_t *tg, int64_t n, int16_t *plen, int8_t *kind, uint8_t *feas) {
    static const int types[3] = {T_SMALL, T_LS, T_MEDIUM};
    for (int64_t i = 0; i < n; i++) {
        int t = types[cls[i]];
        int k, ok;
        plen[i] = (int16_t)orc_astar(grid, G, thr, ship_speed(t), st[2 * i], st[2 * i + 1], tg[2 * i],
                                     tg[2 * i + 1], &k, &ok);
        kind[i] = (int8_t)k;
        feas[i] = (uint8_t)orc_check_path(grid, G, thr, t, st[2 * i], st[2 * i + 1], tg[2 * i],
                                          tg[2 * i + 1]);
    }
}

/* continuous move: rounded target + feasibility (can_move_to && check_path) */
void orc_move_batch(const uint8_t *grid, int G, int thr, const int8_t *cls, const uint8_t *is_f32,
                    const int16_t *pos, const double *act, int64_t n, int32_t *rounded, uint8_t *ok) {
    static const int types[2] = {T_SMALL, T_LS};
    for (int64_t i = 0; i < n; i++) {
        int t = types[cls[i]];
        int nx, ny;
        orc_move_target(pos[2 * i], pos[2 * i + 1], ship_speed(t), act[2 * i], act[2 * i + 1],
                        is_f32[i] ? K_F32 : K_F64, &nx, &ny);
        rounded[2 * i] = nx;
        rounded[2 * i + 1] = ny;
        ok[i] = (uint8_t)(can_move_to(grid, G, thr, nx, ny) &&
                          orc_check_path(grid, G, thr, t, pos[2 * i], pos[2 * i + 1], nx, ny));
    }
}

/* feasibility of a move to an explicit target for each start (A* table rows):
 * out[s*W*W + (dx+R)*W + (dy+R)] for offsets in [-R, R]^2 */
void orc_move_table(const uint8_t *grid, int G, int thr, int type, int R, const int32_t *starts,
                    int64_t ns, uint8_t *out) {
    int W = 2 * R + 1;
    for (int64_t s = 0; s < ns; s++) {
        int sx = starts[2 * s], sy = starts[2 * s + 1];
        for (int dx = -R; dx <= R; dx++)
            for (int dy = -R; dy <= R; dy++) {
                int tx = sx + dx, ty = sy + dy;
                out[s * W * W + (dx + R) * W + (dy + R)] =
                    (uint8_t)(can_move_to(grid, G, thr, tx, ty) &&
                              orc_check_path(grid, G, thr, type, sx, sy, tx, ty));
            }
    }
}

/* Philox stream check helper */
void orc_philox(uint64_t seed, uint64_t ctr, uint64_t gid, uint32_t *out) {
    uint32_t c[4] = {(uint32_t)ctr, (uint32_t)(ctr >> 32), (uint32_t)gid, (uint32_t)(gid >> 32)};
    uint32_t k[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    philox(c, k, out);
}

/* ------------------------------------------------------------------------ */
/* CPU baseline driver (bench.py cpu_baseline leg): n_envs environments      */
/* stepped one after another for n_steps each with U[0,1) float32 actions,   */
/* auto-reset when done == 0 or after `horizon` steps. Returns steps run.    */
/* ------------------------------------------------------------------------ */
int64_t orc_bench_range(const orc_params *P, const uint8_t *grid, int G, int nb, int nr,
                        const int *types, const int *pos, int env0, int n_envs, int n_steps,
                        int horizon, uint64_t seed);

int64_t orc_bench(const orc_params *P, const uint8_t *grid, int G, int nb, int nr, const int *types,
                  const int *pos, int n_envs, int n_steps, int horizon, uint64_t seed) {
    return orc_bench_range(P, grid, G, nb, nr, types, pos, 0, n_envs, n_steps, horizon, seed);
}

/* CPU-baseline driver over global env ids [env0, env0 + n_envs): no shared
 * mutable state, so disjoint ranges can run on concurrent threads. */
int64_t orc_bench_range(const orc_params *P, const uint8_t *grid, int G, int nb, int nr,
                        const int *types, const int *pos, int env0, int n_envs, int n_steps,
                        int horizon, uint64_t seed) {
    int A = nb + nr;
    orc_env *e = (orc_env *)malloc(sizeof(orc_env));
    double *act = (double *)malloc(sizeof(double) * 4 * A);
    int *kinds = (int *)malloc(sizeof(int) * A);
    double *ob = (double *)malloc(sizeof(double) * nb * (4 * nb + 52));
    double *orr = (double *)malloc(sizeof(double) * nr * (4 * nr + 52));
    double rb[ORC_MAX_AGENTS], rr[ORC_MAX_AGENTS], cog;
    int64_t steps = 0;
    for (int a = 0; a < A; a++) kinds[a] = K_F32;
    for (int env = env0; env < env0 + n_envs; env++) {
        orc_env_init(e, P, grid, G, nb, nr);
        orc_set_rng(e, 0, seed, (uint64_t)env, 0, NULL, 0, 0);
        orc_reset(e, types, pos, NULL);
        uint64_t actr = 0;
        for (int s = 0; s < n_steps; s++) {
            for (int a = 0; a < A; a++) {
                uint32_t o[4];
                orc_philox(seed ^ 0x9E3779B97F4A7C15ull, actr++, (uint64_t)env, o);
                for (int k = 0; k < 4; k++) act[4 * a + k] = (double)((float)(o[k] >> 8) * 5.9604644775390625e-08f);
            }
            int done = orc_step(e, act, kinds, ob, orr, rb, rr, &cog);
            steps++;
            if (done == 0 || e->steps_done >= horizon) orc_reset(e, types, pos, NULL);
        }
    }
    free(e); free(act); free(kinds); free(ob); free(orr);
    return steps;
}

/* ------------------------------------------------------------------------ */
/* Full-size parity driver (tests/test_gpu_fullsize.py only): the global    */
/* envs [env0, env0 + n) of an E-env batch, Philox-seeded by global env id, */
/* stepped S times with float32 actions acts[S][E][A][4] (row kind K_F32),  */
/* auto-reset after done == 0 or `horizon` steps as the device does         */
/* (lnw_kernels.hip phase W). Per (step, env) it records a 64-bit hash of   */
/* the float32 observations, sum_k bits(obs[k]) * mult[k] mod 2^64 over the */
/* blue rows then the red rows, and the float32 rewards, done and cog, so a */
/* 65 536-env batch is checked without holding its observations.            */
/* pos: [E][A][2] when pos_per_env, else [A][2]. Disjoint ranges may run on */
/* concurrent threads.                                                      */
/* ------------------------------------------------------------------------ */
void orc_fullsize_range(const orc_params *P, const uint8_t *grid, int G, int nb, int nr,
                        const int *types, const int *pos, int pos_per_env, const int *rand_ls,
                        uint64_t seed, int64_t E, int64_t env0, int64_t n, int S, int horizon,
                        const float *acts, const uint64_t *mult, uint64_t *hash, float *rew,
                        int32_t *done_out, float *cog_out, float *acts_after) {
    int A = nb + nr, Db = 4 * nb + 52, Dr = 4 * nr + 52;
    orc_env *e = (orc_env *)malloc(sizeof(orc_env));
    double *act = (double *)malloc(sizeof(double) * 4 * A);
    int *kinds = (int *)malloc(sizeof(int) * A);
    double *ob = (double *)malloc(sizeof(double) * nb * Db);
    double *orr = (double *)malloc(sizeof(double) * nr * Dr);
    double rb[ORC_MAX_AGENTS], rr[ORC_MAX_AGENTS], cog;
    for (int a = 0; a < A; a++) kinds[a] = K_F32;
    for (int64_t env = env0; env < env0 + n; env++) {
        const int *p = pos_per_env ? pos + env * A * 2 : pos;
        orc_env_init(e, P, grid, G, nb, nr);
        orc_set_rng(e, 0, seed, (uint64_t)env, 0, NULL, 0, 0);
        orc_reset(e, types, p, rand_ls);
        for (int s = 0; s < S; s++) {
            const float *ar = acts + ((int64_t)s * E + env) * A * 4;
            for (int q = 0; q < 4 * A; q++) act[q] = (double)ar[q];
            int done = orc_step(e, act, kinds, ob, orr, rb, rr, &cog);
            uint64_t h = 0;
            int k = 0;
            for (int q = 0; q < nb * Db; q++, k++) {
                float f = (float)ob[q];
                uint32_t w;
                memcpy(&w, &f, 4);
                h += (uint64_t)w * mult[k];
            }
            for (int q = 0; q < nr * Dr; q++, k++) {
                float f = (float)orr[q];
                uint32_t w;
                memcpy(&w, &f, 4);
                h += (uint64_t)w * mult[k];
            }
            int64_t se = (int64_t)s * E + env;
            hash[se] = h;
            if (acts_after)  /* the action rows as the step left them (game.py:379 write-back) */
                for (int q = 0; q < 4 * A; q++) acts_after[se * A * 4 + q] = (float)act[q];
            for (int a = 0; a < nb; a++) rew[se * A + a] = (float)rb[a];
            for (int a = 0; a < nr; a++) rew[se * A + nb + a] = (float)rr[a];
            done_out[se] = done;
            cog_out[se] = (float)cog;
            if (done == 0 || e->steps_done >= horizon) orc_reset(e, types, p, rand_ls);
        }
    }
    free(e); free(act); free(kinds); free(ob); free(orr);
}

/* ------------------------------------------------------------------------ */
/* Full-size rollout driver (tests/test_gpu_rollout_fullsize.py only): the  */
/* env side of a MAPPO rollout (ppo.py:497-577) for the global envs [env0,  */
/* env0 + n) of an E-env batch. Every step s: ship.get_obs() of every live  */
/* ship, blue then red (their side effects: target lists, EW gauss draws),  */
/* then Game.step on the action array acts[s][E][A][4] (doubles, row kinds  */
/* kinds[s][E][A], as the device policy wrote them). Per (step, env): the   */
/* 64-bit hash of the float32 blue observation rows (sum bits * mult mod    */
/* 2^64, zero rows for sunk ships), the blue rewards (double) and done;     */
/* auto-reset after done == 0 or `horizon` steps as the device does.       */
/* ------------------------------------------------------------------------ */
void orc_rollout_range(const orc_params *P, const uint8_t *grid, int G, int nb, int nr,
                       const int *types, const int *pos, int pos_per_env, uint64_t seed, int64_t E,
                       int64_t env0, int64_t n, int S, int horizon, const double *acts,
                       const uint8_t *kinds_in, const uint64_t *mult, uint64_t *hash, double *rew,
                       int32_t *done_out) {
    int A = nb + nr, Db = 4 * nb + 52, Dr = 4 * nr + 52;
    orc_env *e = (orc_env *)malloc(sizeof(orc_env));
    double *act = (double *)malloc(sizeof(double) * 4 * A);
    int *kinds = (int *)malloc(sizeof(int) * A);
    double *row = (double *)malloc(sizeof(double) * (Db > Dr ? Db : Dr));
    double *ob = (double *)malloc(sizeof(double) * nb * Db);
    double *orr = (double *)malloc(sizeof(double) * nr * Dr);
    double rb[ORC_MAX_AGENTS], rr[ORC_MAX_AGENTS], cog;
    for (int64_t env = env0; env < env0 + n; env++) {
        const int *p = pos_per_env ? pos + env * A * 2 : pos;
        orc_env_init(e, P, grid, G, nb, nr);
        orc_set_rng(e, 0, seed, (uint64_t)env, 0, NULL, 0, 0);
        orc_reset(e, types, p, NULL);
        for (int s = 0; s < S; s++) {
            const int64_t se = (int64_t)s * E + env;
            uint64_t h = 0;
            for (int a = 0; a < A; a++) {
                if (!e->s[a].alive) continue;
                memset(row, 0, sizeof(double) * (Db > Dr ? Db : Dr));
                get_obs(e, a, row);
                if (a < nb)
                    for (int q = 0; q < Db; q++) {
                        float f = (float)row[q];
                        uint32_t w;
                        memcpy(&w, &f, 4);
                        h += (uint64_t)w * mult[a * Db + q];
                    }
            }
            hash[se] = h;
            memcpy(act, acts + se * A * 4, sizeof(double) * 4 * A);
            for (int a = 0; a < A; a++) kinds[a] = kinds_in[se * A + a];
            int done = orc_step(e, act, kinds, ob, orr, rb, rr, &cog);
            for (int a = 0; a < nb; a++) rew[se * nb + a] = rb[a];
            done_out[se] = done;
            if (done == 0 || e->steps_done >= horizon) orc_reset(e, types, p, NULL);
        }
    }
    free(e); free(act); free(kinds); free(row); free(ob); free(orr);
}
