"""ctypes binding of the CPU parity oracle (oracle/lnw_oracle.c).

TEST INFRASTRUCTURE: imported only by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg. Never part of the product path.
"""
import ctypes as C
import json
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
ORACLE_SO = os.path.join(ORACLE_DIR, "liblnw_oracle.so")
GOLDEN = os.environ.get("LNW_GOLDEN_DIR", os.path.join(ROOT, "tests", "golden"))

K_PYINT, K_PYFLOAT, K_F32, K_F64 = 0, 1, 2, 3
T_SMALL, T_LARGE, T_LS, T_MEDIUM = 0, 1, 2, 3


class OrcParams(C.Structure):
    _fields_ = [("discrete", C.c_int), ("landing_ops", C.c_int), ("aggressive", C.c_int),
                ("side_blue", C.c_int), ("trained_red", C.c_int),
                ("red_aggression", C.c_double), ("move_thr", C.c_int), ("ew_thr", C.c_int),
                ("lz_x", C.c_int), ("lz_y", C.c_int)]


def build_oracle():
    src = os.path.join(ORACLE_DIR, "lnw_oracle.c")
    if (not os.path.exists(ORACLE_SO)) or os.path.getmtime(ORACLE_SO) < os.path.getmtime(src):
        subprocess.check_call(["make", "-s", "-C", ORACLE_DIR])
    return ORACLE_SO


_lib = None


def lib():
    global _lib
    if _lib is None:
        build_oracle()
        L = C.CDLL(ORACLE_SO)
        P = C.c_void_p
        L.orc_env_size.restype = C.c_size_t
        L.orc_los.restype = C.c_int
        L.orc_astar.restype = C.c_int
        L.orc_check_path.restype = C.c_int
        L.orc_radar_range.restype = C.c_int
        L.orc_radar_range.argtypes = [C.c_double, C.c_int, C.c_int]
        L.orc_ew_range.restype = C.c_int
        L.orc_ew_range.argtypes = [C.c_double, C.c_int, C.c_int]
        L.orc_step.restype = C.c_int
        L.orc_step.argtypes = [P, P, P, P, P, P, P, P]
        L.orc_set_rng.argtypes = [P, C.c_int, C.c_uint64, C.c_uint64, C.c_uint64, P,
                                  C.c_int64, C.c_int64]
        L.orc_set_ducting.argtypes = [P, C.c_double]
        L.orc_env_init.argtypes = [P, P, P, C.c_int, C.c_int, C.c_int]
        L.orc_reset.argtypes = [P, P, P, P]
        L.orc_observe.argtypes = [P, C.c_int, P]
        L.orc_get_agents.argtypes = [P] * 9
        L.orc_get_tlist.argtypes = [P, C.c_int, P, C.c_int]
        L.orc_get_tlist.restype = C.c_int
        L.orc_get_env.argtypes = [P] * 6
        L.orc_set_agent.argtypes = [P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_double,
                                    C.c_int, C.c_int, C.c_int, C.c_double]
        L.orc_los_batch.argtypes = [P, C.c_int, P, C.c_int64, C.c_int, P]
        L.orc_astar_batch.argtypes = [P, C.c_int, C.c_int, P, P, P, C.c_int64, P, P, P]
        L.orc_move_batch.argtypes = [P, C.c_int, C.c_int, P, P, P, P, C.c_int64, P, P]
        L.orc_move_table.argtypes = [P, C.c_int, C.c_int, C.c_int, C.c_int, P, C.c_int64, P]
        L.orc_philox.argtypes = [C.c_uint64, C.c_uint64, C.c_uint64, P]
        L.orc_fullsize_range.argtypes = [P, P, C.c_int, C.c_int, C.c_int, P, P, C.c_int, P,
                                         C.c_uint64, C.c_int64, C.c_int64, C.c_int64, C.c_int,
                                         C.c_int, P, P, P, P, P, P, P]
        L.orc_rollout_range.argtypes = [P, P, C.c_int, C.c_int, C.c_int, P, P, C.c_int,
                                        C.c_uint64, C.c_int64, C.c_int64, C.c_int64, C.c_int,
                                        C.c_int, P, P, P, P, P, P]
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


def los_batch(grid, pairs, thr):
    grid = np.ascontiguousarray(grid, np.uint8)
    pairs = np.ascontiguousarray(pairs, np.int16)
    out = np.zeros(len(pairs), np.uint8)
    lib().orc_los_batch(_p(grid), grid.shape[0], _p(pairs), len(pairs), thr, _p(out))
    return out


def astar_batch(grid, cls, start, target, thr=74):
    grid = np.ascontiguousarray(grid, np.uint8)
    cls = np.ascontiguousarray(cls, np.int8)
    st = np.ascontiguousarray(start, np.int16)
    tg = np.ascontiguousarray(target, np.int16)
    n = len(cls)
    plen = np.zeros(n, np.int16)
    kind = np.zeros(n, np.int8)
    feas = np.zeros(n, np.uint8)
    lib().orc_astar_batch(_p(grid), grid.shape[0], thr, _p(cls), _p(st), _p(tg), n, _p(plen),
                          _p(kind), _p(feas))
    return plen, kind, feas


def move_batch(grid, cls, is_f32, pos, act, thr=74):
    grid = np.ascontiguousarray(grid, np.uint8)
    cls = np.ascontiguousarray(cls, np.int8)
    f32 = np.ascontiguousarray(is_f32, np.uint8)
    pos = np.ascontiguousarray(pos, np.int16)
    act = np.ascontiguousarray(act, np.float64)
    n = len(cls)
    rounded = np.zeros((n, 2), np.int32)
    ok = np.zeros(n, np.uint8)
    lib().orc_move_batch(_p(grid), grid.shape[0], thr, _p(cls), _p(f32), _p(pos), _p(act), n,
                         _p(rounded), _p(ok))
    return rounded, ok


def move_table(grid, type_code, R, starts, thr=74):
    grid = np.ascontiguousarray(grid, np.uint8)
    starts = np.ascontiguousarray(starts, np.int32)
    W = 2 * R + 1
    out = np.zeros((len(starts), W, W), np.uint8)
    lib().orc_move_table(_p(grid), grid.shape[0], thr, type_code, R, _p(starts), len(starts),
                         _p(out))
    return out


def philox(seed, ctr, gid):
    out = np.zeros(4, np.uint32)
    lib().orc_philox(seed, ctr, gid, _p(out))
    return out


class OracleEnv:
    """One reference environment (Game + its ships) in the C oracle."""

    def __init__(self, grid, nb, nr, *, discrete=False, landing_ops=False, aggressive=True,
                 side_blue=True, trained_red=True, red_aggression=0.4, move_thr=74, ew_thr=70,
                 lz=(14, 82)):
        L = lib()
        self.grid = np.ascontiguousarray(grid, np.uint8)
        self.G = self.grid.shape[0]
        self.nb, self.nr = nb, nr
        self.A = nb + nr
        self.Db, self.Dr = 4 * nb + 52, 4 * nr + 52
        self.params = OrcParams(int(discrete), int(landing_ops), int(aggressive), int(side_blue),
                                int(trained_red), float(red_aggression), move_thr, ew_thr,
                                lz[0], lz[1])
        self.buf = C.create_string_buffer(L.orc_env_size())
        self.e = C.cast(self.buf, C.c_void_p)
        L.orc_env_init(self.e, C.byref(self.params), _p(self.grid), self.G, nb, nr)
        self._tape = None

    def set_tape(self, tape, pos=0):
        self._tape = np.ascontiguousarray(tape, np.float64)
        lib().orc_set_rng(self.e, 1, 0, 0, 0, _p(self._tape), len(self._tape), pos)

    def set_philox(self, seed, env_gid, ctr=0):
        lib().orc_set_rng(self.e, 0, seed, env_gid, ctr, None, 0, 0)

    def reset(self, types, pos, rand_ls=None):
        t = np.ascontiguousarray(types, np.int32)
        # a side's row length follows its fastest ship (game.py:595-610): a side
        # of medium ships (speed 2) has 5x5 windows, rows of 4n + 28 floats
        self.Db_out = 4 * self.nb + (28 if (t[:self.nb] == T_MEDIUM).all() else 52)
        self.Dr_out = 4 * self.nr + (28 if (t[self.nb:] == T_MEDIUM).all() else 52)
        p = np.ascontiguousarray(pos, np.int32).reshape(-1)
        r = np.ascontiguousarray(rand_ls if rand_ls is not None else np.zeros(self.A), np.int32)
        lib().orc_reset(self.e, _p(t), _p(p), _p(r))

    def set_ducting(self, d):
        lib().orc_set_ducting(self.e, d)

    def step(self, actions, kinds=None):
        act = np.ascontiguousarray(np.array(actions, np.float64).reshape(self.A, 4))
        k = None if kinds is None else np.ascontiguousarray(kinds, np.int32)
        ob = np.zeros((self.nb, self.Db))
        orr = np.zeros((self.nr, self.Dr))
        rb = np.zeros(self.nb)
        rr = np.zeros(self.nr)
        cog = np.zeros(1)
        done = lib().orc_step(self.e, _p(act), None if k is None else _p(k), _p(ob), _p(orr),
                              _p(rb), _p(rr), _p(cog))
        Db, Dr = getattr(self, "Db_out", self.Db), getattr(self, "Dr_out", self.Dr)
        assert not ob[:, Db:].any() and not orr[:, Dr:].any()
        return dict(obs_blue=ob[:, :Db], obs_red=orr[:, :Dr], rew_blue=rb, rew_red=rr, done=done,
                    cog=cog[0], actions_after=act)

    def observe(self, a):
        out = np.zeros(self.Db if a < self.nb else self.Dr)
        lib().orc_observe(self.e, a, _p(out))
        D = getattr(self, "Db_out", self.Db) if a < self.nb else getattr(self, "Dr_out", self.Dr)
        assert not out[D:].any()
        return out[:D]

    def agents(self):
        A = self.A
        pos = np.zeros((A, 2), np.int32)
        radar = np.zeros(A, np.int32)
        miss = np.zeros(A)
        mk = np.zeros(A, np.int32)
        alive = np.zeros(A, np.int32)
        steps = np.zeros(A, np.int32)
        dlz = np.zeros(A)
        tl = np.zeros(A, np.int32)
        lib().orc_get_agents(self.e, _p(pos), _p(radar), _p(miss), _p(mk), _p(alive), _p(steps),
                             _p(dlz), _p(tl))
        return dict(pos=pos, radar=radar, missiles=miss, mkind=mk, alive=alive, steps_done=steps,
                    dist_lz=dlz, tl_cnt=tl)

    def tlist(self, a, cap=1024):
        xy = np.zeros((cap, 2), np.int32)
        n = lib().orc_get_tlist(self.e, a, _p(xy), cap)
        return [tuple(v) for v in xy[:min(n, cap)]]

    def env_state(self):
        out = np.zeros(9, np.int32)
        d = np.zeros(1)
        err = np.zeros(1, np.uint32)
        tp = np.zeros(1, np.int64)
        ctr = np.zeros(1, np.uint64)
        lib().orc_get_env(self.e, _p(out), _p(d), _p(err), _p(tp), _p(ctr))
        keys = ["n_blue_left", "n_red_left", "steps_done", "blue_victory", "red_victory",
                "blue_eng", "red_eng", "neut_blue", "neut_red"]
        st = {k: int(v) for k, v in zip(keys, out)}
        st.update(ducting=float(d[0]), err=int(err[0]), tape_pos=int(tp[0]), ctr=int(ctr[0]))
        return st


# ---------------------------------------------------------------------------
# golden fixtures
# ---------------------------------------------------------------------------
def fullsize(grid, nb, nr, types, pos, acts, mult, seed, horizon, *, pos_per_env=False,
             rand_ls=None, landing_ops=False, trained_red=True, acts_after=False, threads=None):
    """orc_fullsize_range over all E envs of acts [S, E, A, 4] (float32) on a
    thread pool (ctypes releases the GIL; ranges are disjoint): per (step, env)
    the observation hash (sum bits * mult mod 2^64), float32 rewards [S, E, A],
    done [S, E] and cog [S, E]; with acts_after=True also the action rows as
    each step left them [S, E, A, 4] (an untrained red's salvo write-back)."""
    from concurrent.futures import ThreadPoolExecutor
    L = lib()
    S, E, A = acts.shape[:3]
    grid = np.ascontiguousarray(grid, np.uint8)
    acts = np.ascontiguousarray(acts, np.float32)
    types = np.ascontiguousarray(types, np.int32)
    pos = np.ascontiguousarray(pos, np.int32)
    mult = np.ascontiguousarray(mult, np.uint64)
    rls = np.ascontiguousarray(rand_ls if rand_ls is not None else np.zeros(A), np.int32)
    P = OrcParams(0, int(landing_ops), 1, 1, int(trained_red), 0.4, 74, 70, 14, 82)
    hsh = np.zeros((S, E), np.uint64)
    rew = np.zeros((S, E, A), np.float32)
    done = np.zeros((S, E), np.int32)
    cog = np.zeros((S, E), np.float32)
    aft = np.zeros((S, E, A, 4), np.float32) if acts_after else None
    threads = threads or min(16, os.cpu_count() or 1)
    chunk = (E + threads - 1) // threads

    def run(i):
        e0 = i * chunk
        n = max(0, min(chunk, E - e0))
        if n:
            L.orc_fullsize_range(C.byref(P), _p(grid), grid.shape[0], nb, nr, _p(types), _p(pos),
                                 int(pos_per_env), _p(rls), seed, E, e0, n, S, horizon,
                                 _p(acts), _p(mult), _p(hsh), _p(rew), _p(done), _p(cog),
                                 _p(aft) if aft is not None else None)
    with ThreadPoolExecutor(threads) as ex:
        list(ex.map(run, range(threads)))
    if acts_after:
        return hsh, rew, done, cog, aft
    return hsh, rew, done, cog


def rollout_env(grid, nb, nr, types, pos, acts, kinds, mult, seed, horizon, *, pos_per_env=False,
                trained_red=False, threads=None):
    """orc_rollout_range over all E envs: the env side of a MAPPO rollout
    (ppo.py:497-577) on the action arrays a device rollout stepped, acts
    [S, E, A, 4] float64 with row kinds [S, E, A]. Per (step, env): the hash of
    the blue get_obs rows taken before the step (sum bits * mult mod 2^64, mult
    over nb * (4 nb + 52) floats), the blue rewards [S, E, nb] (float64) and
    done [S, E]."""
    from concurrent.futures import ThreadPoolExecutor
    L = lib()
    S, E, A = acts.shape[:3]
    grid = np.ascontiguousarray(grid, np.uint8)
    acts = np.ascontiguousarray(acts, np.float64)
    kinds = np.ascontiguousarray(kinds, np.uint8)
    types = np.ascontiguousarray(types, np.int32)
    pos = np.ascontiguousarray(pos, np.int32)
    mult = np.ascontiguousarray(mult, np.uint64)
    P = OrcParams(0, 0, 1, 1, int(trained_red), 0.4, 74, 70, 14, 82)
    hsh = np.zeros((S, E), np.uint64)
    rew = np.zeros((S, E, nb), np.float64)
    done = np.zeros((S, E), np.int32)
    threads = threads or min(16, os.cpu_count() or 1)
    chunk = (E + threads - 1) // threads

    def run(i):
        e0 = i * chunk
        n = max(0, min(chunk, E - e0))
        if n:
            L.orc_rollout_range(C.byref(P), _p(grid), grid.shape[0], nb, nr, _p(types), _p(pos),
                                int(pos_per_env), seed, E, e0, n, S, horizon, _p(acts), _p(kinds),
                                _p(mult), _p(hsh), _p(rew), _p(done))
    with ThreadPoolExecutor(threads) as ex:
        list(ex.map(run, range(threads)))
    return hsh, rew, done


def load_fixture(name, golden_dir=GOLDEN):
    d = np.load(os.path.join(golden_dir, name), allow_pickle=False)
    return {k: d[k] for k in d.files}


def episode_meta(fx):
    return json.loads(str(fx["meta"]))


def fixture_kinds(fx, meta, step):
    """Per-row value kinds of the recorded actions."""
    A = fx["actions"].shape[1]
    if meta["flags"]["DISCRETE"]:
        # list rows (ddqn.py:396): the salvo rewrite stays a float (K_PYFLOAT);
        # an integer ndarray truncates it (K_PYINT)
        return np.full(A, K_PYFLOAT if meta.get("list_rows") else K_PYINT, np.int32)
    rf = fx["row_f32"][step]
    if meta["dtype"] == "f32":
        return np.full(A, K_F32, np.int32)
    if meta.get("mixed_rows"):
        return np.where(rf == 1, K_F32, K_PYFLOAT).astype(np.int32)
    return np.full(A, K_F64, np.int32)
