"""Golden-vector generator for the littoral env step (TEST INFRASTRUCTURE ONLY).

Runs only in the build container, where the read-only reference is mounted at
/root/reference. It imports the reference's own ``game.py`` / ``combatant.py`` /
``landingship.py`` (through the stub recipe of SURVEY.md §8c) and records inputs
and outputs as small ``.npz`` fixtures in this directory. Nothing here ships to
the GPU box as code; the fixtures are data. The product path never reads them.

Recorded fixtures
-----------------
grids.npz       terrain grids as built by ``Game.define_grid_from_image``
                (game.py:616-626) at G=100 and G=200.
los.npz         ``Combatant.check_line_of_sight`` radar/EW bits and the
                ``bresenham_line`` point count (combatant.py:411-456).
astar.npz       ``Combatant.astar`` / ``LandingShip.astar`` path length and
                termination kind plus ``check_path`` feasibility
                (combatant.py:289-408, landingship.py:296-415).
moves.npz       ``continuous_to_discrete`` targets (combatant.py:459-476) for
                float64 and float32 actions, and ``value_to_coordinates``
                (combatant.py:689-704).
ranges.npz      ``radar_range`` / ``ew_range`` (combatant.py:235-247).
ep_<name>.npz   full episodes through ``Game.reset`` / ``Game.step``
                (game.py:298-613) with every RNG draw recorded (tape), both
                sides' observations and rewards (captured from ``step``'s
                locals with sys.settrace — no reference code is copied), and
                the per-agent state after every step.

Usage:  python tests/golden/make_golden.py [--quick] [episodes|los|...]
        (LNW_GOLDEN_ONLY=ep1,ep2 limits the episode fixtures written)
"""
import contextlib
import io
import json
import math
import os
import random
import sys
import types

import numpy as np

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))
ASSETS = ["config.json", "red_steps.csv", "red_steps2.csv", "red_steps3.csv",
          "balt_mod_400x400_2.png"]

TYPE_CODE = {"small": 0, "large": 1, "ls": 2, "medium": 3}
# LNW_GOLDEN_ONLY=name1,name2 regenerates only those episode fixtures
ONLY_SCENARIOS = [n for n in os.environ.get("LNW_GOLDEN_ONLY", "").split(",") if n]


# ----------------------------------------------------------------------------
# reference import harness (SURVEY.md §8c recipe)
# ----------------------------------------------------------------------------
def import_reference(workdir="/tmp/lnw_golden_run"):
    os.makedirs(workdir, exist_ok=True)
    for f in ASSETS:
        dst = os.path.join(workdir, f)
        if not os.path.exists(dst):
            os.symlink(os.path.join(REF, f), dst)
    os.chdir(workdir)
    for name in ["skimage", "skimage.draw", "wandb", "IPython", "IPython.display",
                 "torchviz"]:
        sys.modules.setdefault(name, types.ModuleType(name))
    sys.modules["skimage.draw"].line = lambda *a, **k: None
    sys.modules["IPython.display"].clear_output = lambda *a, **k: None
    sys.modules["torchviz"].make_dot = lambda *a, **k: None
    from PIL import Image
    if not hasattr(Image, "ANTIALIAS"):
        Image.ANTIALIAS = Image.LANCZOS
    if REF not in sys.path:
        sys.path.insert(0, REF)
    import game
    import combatant
    import landingship
    return game, combatant, landingship


class TapeRNG:
    """Stands in for the ``random`` module inside the reference modules and
    records every value it hands out, in call order (kinds: 0 random(),
    1 gauss(), 2 randint(), 3 numpy beta(1,3))."""

    def __init__(self, seed):
        self.r = random.Random(seed)
        self.vals = []
        self.kinds = []

    def random(self):
        v = self.r.random()
        self.vals.append(v)
        self.kinds.append(0)
        return v

    def gauss(self, mu=0.0, sigma=1.0):
        v = self.r.gauss(mu, sigma)
        self.vals.append(v)
        self.kinds.append(1)
        return v

    def randint(self, a, b):
        v = self.r.randint(a, b)
        self.vals.append(float(v))
        self.kinds.append(2)
        return v

    def beta(self, a, b):
        v = float(np.random.default_rng(self.r.getrandbits(32)).beta(a, b))
        self.vals.append(v)
        self.kinds.append(3)
        return v


@contextlib.contextmanager
def quiet():
    with contextlib.redirect_stdout(io.StringIO()):
        yield


# ----------------------------------------------------------------------------
# fixtures: grids, LOS, A*, moves, ranges
# ----------------------------------------------------------------------------
def make_grids(game):
    env = game.Game()
    env.define_grid_from_image("balt_mod_400x400_2.png", 100)
    g100 = np.array(env.grid, dtype=np.uint8)
    env.define_grid_from_image("balt_mod_400x400_2.png", 200)
    g200 = np.array(env.grid, dtype=np.uint8)
    np.savez_compressed(os.path.join(OUT, "grids.npz"), grid100=g100, grid200=g200)
    return g100, g200


def _probe_ship(game, combatant, grid, cls="small"):
    env = game.Game()
    env.grid = grid
    env.ducting_factor = 1.5
    if cls == "ls":
        import landingship
        return landingship.LandingShip("red", "ls", (0, 0), (14, 82), env), env
    return combatant.Combatant("blue", cls, (0, 0), [], env), env


def make_los(game, combatant, g100, g200, quick):
    rng = np.random.default_rng(1234)
    rows = []
    for gi, grid in ((0, g100), (1, g200)):
        G = grid.shape[0]
        ship, _ = _probe_ship(game, combatant, grid)
        n_rand = (4000 if quick else (60000 if gi == 0 else 25000))
        o = rng.integers(0, G, size=(n_rand, 2))
        d = rng.integers(0, G, size=(n_rand, 2))
        pairs = [np.concatenate([o, d], 1)]
        # dense local neighbourhoods (the sensor ranges are <= 37 cells)
        n_org = 8 if quick else (120 if gi == 0 else 40)
        R = 14 if gi == 0 else 40
        for _ in range(n_org):
            ox, oy = rng.integers(0, G, size=2)
            for dx in range(-R, R + 1, 1 if gi == 0 else 3):
                for dy in range(-R, R + 1, 1 if gi == 0 else 3):
                    x, y = ox + dx, oy + dy
                    if 0 <= x < G and 0 <= y < G:
                        pairs.append(np.array([[ox, oy, x, y]]))
        # coast-hugging pairs (origins next to land)
        land = np.argwhere(grid > 70)
        k = 500 if quick else 15000
        sel = land[rng.integers(0, len(land), size=k)]
        o = np.clip(sel + rng.integers(-3, 4, size=(k, 2)), 0, G - 1)
        d = np.clip(o + rng.integers(-30, 31, size=(k, 2)), 0, G - 1)
        pairs.append(np.concatenate([o, d], 1))
        P = np.concatenate(pairs, 0).astype(np.int64)
        for (x1, y1, x2, y2) in P:
            a, b = (int(x1), int(y1)), (int(x2), int(y2))
            r = ship.check_line_of_sight(a, b, "radar")
            e = ship.check_line_of_sight(a, b, "ew")
            n = len(ship.bresenham_line(a[0], a[1], b[0], b[1]))
            rows.append((gi, a[0], a[1], b[0], b[1], int(r), int(e), n))
    A = np.array(rows, dtype=np.int32)
    np.savez_compressed(os.path.join(OUT, "los.npz"), grid_id=A[:, 0].astype(np.int8),
                        pairs=A[:, 1:5].astype(np.int16), radar=A[:, 5].astype(np.uint8),
                        ew=A[:, 6].astype(np.uint8), npts=A[:, 7].astype(np.int16))
    print("los cases", len(A))


def make_astar(game, combatant, g100, g200, quick):
    rng = np.random.default_rng(777)
    rows = []
    for gi, grid in ((0, g100), (1, g200)):
        G = grid.shape[0]
        for ci, cls in enumerate(("small", "ls", "medium")):
            if gi == 1 and cls == "medium":
                continue
            ship, env = _probe_ship(game, combatant, grid, cls)
            n_start = 20 if quick else (1100 if gi == 0 else 250)
            land = np.argwhere(grid > 74)
            water = np.argwhere(grid <= 74)
            # bias towards coasts: water cells within 3 cells of land
            near = land[rng.integers(0, len(land), size=n_start)] + rng.integers(-3, 4, size=(n_start, 2))
            near = np.clip(near, 0, min(G, 100) - 1)
            starts = np.concatenate([
                near[: n_start // 2],
                water[rng.integers(0, len(water), size=n_start // 3)],
                rng.integers(0, min(G, 100), size=(n_start - n_start // 2 - n_start // 3, 2)),
            ])
            for (sx, sy) in starts:
                sx, sy = int(sx), int(sy)
                tgts = [(sx + dx, sy + dy) for dx in range(-4, 5) for dy in range(-4, 5)]
                for _ in range(6):
                    tgts.append((sx + int(rng.integers(-30, 31)), sy + int(rng.integers(-30, 31))))
                for (tx, ty) in tgts:
                    path = ship.astar(grid, (sx, sy), (tx, ty))
                    if path is None:
                        plen, kind = -1, 2
                    else:
                        plen = len(path)
                        kind = 0 if tuple(path[-1]) == (tx, ty) else 1
                    feas = ship.check_path((sx, sy), (tx, ty))
                    rows.append((gi, ci, sx, sy, tx, ty, plen, kind, int(feas)))
    A = np.array(rows, dtype=np.int32)
    np.savez_compressed(os.path.join(OUT, "astar.npz"), grid_id=A[:, 0].astype(np.int8),
                        cls=A[:, 1].astype(np.int8), start=A[:, 2:4].astype(np.int16),
                        target=A[:, 4:6].astype(np.int16), plen=A[:, 6].astype(np.int16),
                        kind=A[:, 7].astype(np.int8), feasible=A[:, 8].astype(np.uint8))
    print("astar cases", len(A))


def make_moves(game, combatant, g100, quick):
    rng = np.random.default_rng(99)
    rows = []
    specials = np.array([0.0, 0.5, 1.0, 0.25, 0.125, 0.75, 1 / 3, 2 / 3, 1e-9, 0.9999999,
                         -0.25, 1.5, 2.0, -1.0, 0.0625, 0.375])
    n = 3000 if quick else 20000
    for ci, cls in enumerate(("small", "ls")):
        ship, env = _probe_ship(game, combatant, g100, cls)
        water = np.argwhere(g100 <= 74)
        seen = []
        orig = ship.can_move_to

        def rec(x, y, _o=orig):
            seen.append((x, y))
            return _o(x, y)
        ship.can_move_to = rec
        for dt in (np.float64, np.float32):
            pos = water[rng.integers(0, len(water), size=n)]
            a = rng.random((n, 2))
            a[: n // 8] = rng.choice(specials, size=(n // 8, 2))
            a = a.astype(dt)
            for (px, py), (a2, a3) in zip(pos, a):
                ship.position = (int(px), int(py))
                seen.clear()
                with quiet():
                    res = ship.continuous_to_discrete(np.array([a2, a3], dtype=dt))
                nx, ny = seen[0]
                if res is False:
                    rx, ry, ok = -9999, -9999, 0
                else:
                    rx, ry, ok = res[0], res[1], 1
                rows.append((ci, 1 if dt == np.float32 else 0, int(px), int(py),
                             float(a2), float(a3), int(nx), int(ny), ok, rx, ry))
    A = np.array([r[:4] + r[6:] for r in rows], dtype=np.int32)
    acts = np.array([r[4:6] for r in rows], dtype=np.float64)
    # discrete: value_to_coordinates for a Combatant (LandingShip has none)
    ship, env = _probe_ship(game, combatant, g100, "small")
    water = np.argwhere(g100 <= 74)
    drows = []
    for (px, py) in water[rng.integers(0, len(water), size=(200 if quick else 2500))]:
        ship.position = (int(px), int(py))
        for v in range(50):
            res = ship.value_to_coordinates(v)
            drows.append((int(px), int(py), v) + ((1, res[0], res[1]) if res is not False
                                                   else (0, -9999, -9999)))
    D = np.array(drows, dtype=np.int32)
    np.savez_compressed(os.path.join(OUT, "moves.npz"), cls=A[:, 0].astype(np.int8),
                        is_f32=A[:, 1].astype(np.uint8), pos=A[:, 2:4].astype(np.int16),
                        act=acts, rounded=A[:, 4:6].astype(np.int32),
                        ok=A[:, 6].astype(np.uint8), result=A[:, 7:9].astype(np.int32),
                        disc=D)
    print("move cases", len(A), "discrete", len(D))


def make_ranges(game, combatant, landingship, g100):
    env = game.Game()
    env.grid = g100
    ships = [combatant.Combatant("blue", "small", (0, 0), [], env),
             combatant.Combatant("red", "large", (0, 0), [], env),
             landingship.LandingShip("red", "ls", (0, 0), (14, 82), env),
             combatant.Combatant("red", "medium", (0, 0), [], env)]
    ducts = [1.0, 1.0 + 1e-12, 1.25, 1.5, 1.75, 1.9999999, 1.3333333333333333]
    ducts += list(1.0 + np.random.default_rng(5).beta(1, 3, size=200))
    R = np.zeros((len(ducts), 4, 4, 2), dtype=np.int32)
    for k, d in enumerate(ducts):
        env.ducting_factor = d
        for i, a in enumerate(ships):
            for j, b in enumerate(ships):
                R[k, i, j, 0] = a.radar_range(a, b)
                R[k, i, j, 1] = a.ew_range(a, b)
    np.savez_compressed(os.path.join(OUT, "ranges.npz"), ducting=np.array(ducts), ranges=R)


# ----------------------------------------------------------------------------
# episodes
# ----------------------------------------------------------------------------
REF_BLUE = [(6, 61), (10, 81), (8, 70), (11, 58)]
REF_RED4 = [(98, 48), (98, 52), (98, 56), (96, 52)]
MELEE_BOXES = [((40, 57), (40, 65)), ((30, 60), (55, 80)), ((60, 85), (55, 80))]
# "split" spawns: the sides start 15-35 cells apart (inside EW range, mostly
# outside radar range), which exercises bearings and EW fixes
SPLIT_BOXES = [(((30, 45), (40, 60)), ((55, 70), (45, 65))),
               (((40, 55), (30, 45)), ((40, 55), (55, 75))),
               (((20, 40), (60, 80)), ((50, 70), (60, 80)))]


def _water_in_box(grid, rng, box, n):
    (x0, x1), (y0, y1) = box
    cells = [(x, y) for x in range(x0, x1) for y in range(y0, y1) if grid[x, y] <= 74]
    idx = rng.integers(0, len(cells), size=n)
    return [cells[i] for i in idx]


def _capture_step(game, env, action):
    cap = {}
    code = game.Game.step.__code__

    def local(fr, ev, arg):
        if ev == "return":
            for k in ("blue_rewards", "red_rewards", "observations", "red_observations",
                      "done", "cog_dist"):
                cap[k] = fr.f_locals.get(k)
        return local

    def glob(fr, ev, arg):
        if ev == "call" and fr.f_code is code:
            return local
        return None
    sys.settrace(glob)
    try:
        with quiet():
            ret = env.step(action)
    finally:
        sys.settrace(None)
    return ret, cap


def _snapshot(env, ships_all, nb):
    """State of every agent slot (blue then red) after a step/observe."""
    A = len(ships_all)
    pos = np.zeros((A, 2), np.int32)
    radar = np.zeros(A, np.int32)
    miss = np.zeros(A, np.float64)
    alive = np.zeros(A, np.uint8)
    steps = np.zeros(A, np.int32)
    dlz = np.zeros(A, np.float64)
    tl = []
    lists = list(env.blue_ships) + list(env.red_ships)
    for a, s in enumerate(ships_all):
        pos[a] = s.position
        radar[a] = s.radar_transmission
        miss[a] = float(s.missiles)
        alive[a] = 1 if lists[a] is not None else 0
        steps[a] = s.steps_done
        dlz[a] = getattr(s, "distance_to_landing_zone", 0.0)
        tl.append([tuple(int(v) for v in t) for t in s.target_list])
    return pos, radar, miss, alive, steps, dlz, tl


def run_scenario(game, combatant, landingship, name, grids, *, nb_types, nr_types,
                 spawn="ref", n_ep=4, steps=40, flags=None, dtype="f64",
                 act_lo=0.0, act_hi=1.0, observe=False, grid_id=0, seed=0,
                 random_ls=0, mixed_rows=False, analytics=False, list_rows=False):
    if ONLY_SCENARIOS and name not in ONLY_SCENARIOS:
        return
    flags = dict(flags or {})
    F = dict(DISCRETE=False, LANDING_OPS=False, TACTICS="aggressive", SIDE="blue",
             TRAINED_RED=True, RED_AGGRESSION=0.4, N_RED_LANDINGSHIP=random_ls)
    F.update(flags)
    game.RED_AGGRESSION = F["RED_AGGRESSION"]
    game.N_RED_LANDINGSHIP = F["N_RED_LANDINGSHIP"]
    game.SIDE = F["SIDE"]
    combatant.CUR_SIDE = F["SIDE"]  # the same config key (combatant.py:38, landingship.py:39)
    landingship.CUR_SIDE = F["SIDE"]
    game.TRAINED_RED = F["TRAINED_RED"]
    game.DISCRETE = F["DISCRETE"]
    combatant.DISCRETE = F["DISCRETE"]
    landingship.DISCRETE = F["DISCRETE"]
    game.LANDING_OPS = F["LANDING_OPS"]
    game.TACTICS = F["TACTICS"]
    game.COA_PATH = False
    grid = grids[grid_id]
    rng = np.random.default_rng(seed)
    tape = TapeRNG(seed + 17)
    game.random = tape
    combatant.random = tape
    landingship.random = tape
    np_beta = np.random.beta
    np.random.beta = tape.beta

    nb, nr0 = len(nb_types), len(nr_types)
    rec = dict(actions=[], actions_after=[], row_f32=[], obs_blue=[], obs_red=[],
               rew_blue=[], rew_red=[], done=[], cog=[], pos=[], radar=[], missiles=[],
               alive=[], steps_done=[], dist_lz=[], n_left=[], tape_pos=[], tl_cnt=[],
               tl_xy=[], ep_index=[], victories=[], engagements=[], pre_obs=[],
               pre_obs_valid=[], pre_tl_cnt=[], pre_tl_xy=[], pre_tape_pos=[])
    ep_meta = []
    crashes = []
    # analytics side channels (game.py:119-154, combatant.py:146-150, 640-657):
    # engagement / EW records tagged with (episode, step), maps per episode
    ana = dict(eng=[], ew=[], heat=[], cold=[], launch=[])
    try:
        for ep in range(n_ep):
            env = game.Game()
            tape_start = len(tape.vals)
            blue, red = [], []
            if spawn == "ref":
                bpos = REF_BLUE[:nb]
                rpos = REF_RED4[:nr0]
            elif spawn == "split":
                bbox, rbox = SPLIT_BOXES[ep % len(SPLIT_BOXES)]
                bpos = _water_in_box(grid, rng, bbox, nb)
                rpos = _water_in_box(grid, rng, rbox, nr0)
            else:
                box = MELEE_BOXES[ep % len(MELEE_BOXES)]
                bpos = _water_in_box(grid, rng, box, nb)
                rpos = _water_in_box(grid, rng, box, nr0)
            env.grid = grid  # so ship constructors see the grid
            for t, p in zip(nb_types, bpos):
                blue.append(combatant.Combatant("blue", t, p, [], env) if t != "ls" else
                            landingship.LandingShip("blue", "ls", p, (14, 82), env))
            for t, p in zip(nr_types, rpos):
                red.append(combatant.Combatant("red", t, p, [], env) if t != "ls" else
                           landingship.LandingShip("red", "ls", p, (14, 82), env))
            with quiet():
                env.reset(nb, nr0 + random_ls, grid=grid, blue_ships=blue, red_ships=red)
            ships_all = list(env.blue_ships) + list(env.red_ships)
            A = len(ships_all)
            nr = A - nb
            types = [TYPE_CODE[s.ship_type] for s in ships_all]
            spawn_pos = [tuple(s.position) for s in ships_all]
            meta = dict(ep=ep, types=types, spawn=spawn_pos, ducting=env.ducting_factor,
                        tape_start=tape_start, nb=nb, nr=nr,
                        Db=env.observation_space, Dr=env.red_observation_space,
                        first_step=len(rec["done"]))
            n_eng = n_bew = n_rew = 0

            def ana_step(s):
                nonlocal n_eng, n_bew, n_rew
                for e in env.engagements[n_eng:]:
                    (sx, sy), (tx, ty), msl = e
                    ana["eng"].append((ep, s, sx, sy, tx, ty, int(msl)))
                for side, lst, n0 in ((0, env.blue_ew, n_bew), (1, env.red_ew, n_rew)):
                    for (ox, oy), (fx, fy) in lst[n0:]:
                        ana["ew"].append((ep, s, side, ox, oy, int(fx), int(fy)))
                n_eng, n_bew, n_rew = len(env.engagements), len(env.blue_ew), len(env.red_ew)

            for s in range(steps):
                # ---- optional caller-side observe (main.py:280-333 pattern)
                pre_obs = np.zeros((A, max(meta["Db"], meta["Dr"])), np.float32)
                pre_valid = np.zeros(A, np.uint8)
                rec["pre_tape_pos"].append(len(tape.vals) - tape_start)
                if observe:
                    lists = list(env.blue_ships) + list(env.red_ships)
                    for a, sh in enumerate(lists):
                        if sh is not None:
                            with quiet():
                                o = sh.get_obs()
                            pre_obs[a, :len(o)] = o
                            pre_valid[a] = 1
                _, _, _, _, _, _, ptl = _snapshot(env, ships_all, nb)
                rec["pre_obs"].append(pre_obs)
                rec["pre_obs_valid"].append(pre_valid)
                rec["pre_tl_cnt"].append([len(t) for t in ptl])
                rec["pre_tl_xy"].append(ptl)
                # ---- actions
                if F["DISCRETE"]:
                    act = np.stack([rng.integers(0, 2, size=A), rng.integers(0, 5, size=A),
                                    rng.integers(0, 50, size=A)], 1).astype(np.int64)
                    act = np.concatenate([act, np.zeros((A, 1), np.int64)], 1)
                    # ddqn.py:396 passes a list of 3-int lists; an ndarray otherwise
                    call_act = ([[int(v) for v in row[:3]] for row in act] if list_rows
                                else act.copy())
                    row_f32 = np.zeros(A, np.uint8)
                else:
                    act = rng.uniform(act_lo, act_hi, size=(A, 4))
                    if dtype == "f32":
                        act = act.astype(np.float32)
                        call_act = act.copy()
                        row_f32 = np.ones(A, np.uint8)
                    elif mixed_rows:
                        row_f32 = (rng.random(A) < 0.5).astype(np.uint8)
                        call_act = [np.asarray(act[a], dtype=np.float32) if row_f32[a]
                                    else [float(v) for v in act[a]] for a in range(A)]
                        act = np.array([np.asarray(r, dtype=np.float64) for r in call_act])
                    else:
                        call_act = act.copy()
                        row_f32 = np.zeros(A, np.uint8)
                rec["actions"].append(np.asarray(act, dtype=np.float64))
                rec["row_f32"].append(row_f32)
                ret, cap = _capture_step(game, env, call_act)
                after = np.zeros((A, 4))
                for a, r in enumerate(call_act):
                    after[a, :len(r)] = np.asarray(r, dtype=np.float64)
                rec["actions_after"].append(after)
                ob = np.zeros((nb, meta["Db"]), np.float32)
                ob[:, :] = np.asarray(cap["observations"])[0]
                orr = np.zeros((nr, meta["Dr"]), np.float32)
                orr[:, :] = np.asarray(cap["red_observations"])[0]
                rec["obs_blue"].append(ob)
                rec["obs_red"].append(orr)
                rec["rew_blue"].append(np.array(cap["blue_rewards"], np.float64))
                rec["rew_red"].append(np.array(cap["red_rewards"], np.float64))
                rec["done"].append(int(cap["done"]))
                rec["cog"].append(np.nan if cap["cog_dist"] is None else float(cap["cog_dist"]))
                pos, radar, miss, alive, stp, dlz, tl = _snapshot(env, ships_all, nb)
                rec["pos"].append(pos)
                rec["radar"].append(radar)
                rec["missiles"].append(miss)
                rec["alive"].append(alive)
                rec["steps_done"].append(stp)
                rec["dist_lz"].append(dlz)
                rec["n_left"].append((env.n_blue_left, env.n_red_left))
                rec["tape_pos"].append(len(tape.vals) - tape_start)
                rec["tl_cnt"].append([len(t) for t in tl])
                rec["tl_xy"].append(tl)
                rec["ep_index"].append(ep)
                rec["victories"].append((env.blue_victory, env.red_victory))
                rec["engagements"].append((env.blue_engagements, env.red_engagements))
                if analytics:
                    ana_step(s)
                if cap["done"] == 0:
                    break
            if analytics:
                ana["heat"].append(np.array(env.heatmap, np.int32))
                ana["cold"].append(np.array(env.coldmap, np.int32))
                L = np.zeros((2, 100, 100), np.int32)
                for k, side in enumerate(("blue", "red")):
                    for (x, y) in env.launch_sites[side]:
                        L[k, x, y] += 1
                ana["launch"].append(L)
            meta["n_steps"] = len(rec["done"]) - meta["first_step"]
            meta["tape_end"] = len(tape.vals)
            ep_meta.append(meta)
    except (ZeroDivisionError, ValueError, OverflowError) as exc:  # reference crash modes
        crashes.append(repr(exc))
        print("  crash in", name, repr(exc))
    finally:
        np.random.beta = np_beta

    # drop a partially recorded (crashed) episode
    n_ok = sum(m["n_steps"] for m in ep_meta if "n_steps" in m)
    ep_meta = [m for m in ep_meta if "n_steps" in m]
    for k in rec:
        rec[k] = rec[k][:n_ok]

    def ragged(lst):
        cnt = np.array([[len(t) for t in row] for row in lst], np.int32)
        flat = [xy for row in lst for t in row for xy in t]
        return cnt, np.array(flat, np.int16).reshape(-1, 2)

    tl_cnt, tl_xy = ragged(rec["tl_xy"])
    ptl_cnt, ptl_xy = ragged(rec["pre_tl_xy"])
    meta_all = dict(name=name, flags=F, grid_id=grid_id, dtype=dtype, observe=observe,
                    episodes=ep_meta, crashes=crashes, mixed_rows=mixed_rows, list_rows=list_rows,
                    landing_zone=(14, 82), episode_steps=steps)
    out = dict(
        meta=np.array(json.dumps(meta_all)),
        tape=np.array(tape.vals, np.float64), tape_kind=np.array(tape.kinds, np.int8),
        actions=np.array(rec["actions"]), actions_after=np.array(rec["actions_after"]),
        row_f32=np.array(rec["row_f32"], np.uint8),
        obs_blue=np.array(rec["obs_blue"], np.float32),
        obs_red=np.array(rec["obs_red"], np.float32),
        rew_blue=np.array(rec["rew_blue"]), rew_red=np.array(rec["rew_red"]),
        done=np.array(rec["done"], np.int32), cog=np.array(rec["cog"]),
        pos=np.array(rec["pos"], np.int16), radar=np.array(rec["radar"], np.int32),
        missiles=np.array(rec["missiles"]), alive=np.array(rec["alive"], np.uint8),
        steps_done=np.array(rec["steps_done"], np.int32), dist_lz=np.array(rec["dist_lz"]),
        n_left=np.array(rec["n_left"], np.int32), tape_pos=np.array(rec["tape_pos"], np.int32),
        tl_cnt=tl_cnt, tl_xy=tl_xy, victories=np.array(rec["victories"], np.int32),
        engagements=np.array(rec["engagements"], np.int32),
        ep_index=np.array(rec["ep_index"], np.int32),
        pre_tape_pos=np.array(rec["pre_tape_pos"], np.int32),
    )
    if analytics:
        n_ep_ok = len(ep_meta)
        eng = [r for r in ana["eng"] if r[0] < n_ep_ok]
        ew = [r for r in ana["ew"] if r[0] < n_ep_ok]
        out.update(ana_eng=np.array(eng, np.int32).reshape(-1, 7),
                   ana_ew=np.array(ew, np.int32).reshape(-1, 7),
                   ana_heat=np.array(ana["heat"][:n_ep_ok], np.int32).reshape(-1, 100, 100),
                   ana_cold=np.array(ana["cold"][:n_ep_ok], np.int32).reshape(-1, 100, 100),
                   ana_launch=np.array(ana["launch"][:n_ep_ok], np.int32).reshape(-1, 2, 100, 100))
    if observe:
        out.update(pre_obs=np.array(rec["pre_obs"], np.float32),
                   pre_obs_valid=np.array(rec["pre_obs_valid"], np.uint8),
                   pre_tl_cnt=ptl_cnt, pre_tl_xy=ptl_xy)
    np.savez_compressed(os.path.join(OUT, f"ep_{name}.npz"), **out)
    print(f"episode fixture {name}: {len(ep_meta)} episodes, {n_ok} steps, "
          f"{len(tape.vals)} draws, crashes={crashes}")


def make_episodes(game, combatant, landingship, grids, quick):
    q = (lambda n: max(1, n // 4)) if quick else (lambda n: n)
    S4, R4 = ["small"] * 4, ["large"] * 4
    run_scenario(game, combatant, landingship, "2v2_ref", grids, nb_types=S4[:2],
                 nr_types=R4[:2], spawn="ref", n_ep=q(3), seed=1)
    run_scenario(game, combatant, landingship, "4v4_ref", grids, nb_types=S4, nr_types=R4,
                 spawn="ref", n_ep=q(3), seed=2)
    run_scenario(game, combatant, landingship, "4v4_melee_f64", grids, nb_types=S4,
                 nr_types=R4, spawn="melee", n_ep=q(12), seed=3)
    run_scenario(game, combatant, landingship, "4v4_melee_f32", grids, nb_types=S4,
                 nr_types=R4, spawn="melee", n_ep=q(12), seed=4, dtype="f32")
    run_scenario(game, combatant, landingship, "4v4_split_f64", grids, nb_types=S4,
                 nr_types=R4, spawn="split", n_ep=q(9), seed=16)
    run_scenario(game, combatant, landingship, "4v4_split_f32_observe", grids, nb_types=S4,
                 nr_types=R4, spawn="split", n_ep=q(9), seed=17, dtype="f32", observe=True)
    run_scenario(game, combatant, landingship, "4v4_melee_mixed", grids, nb_types=S4,
                 nr_types=R4, spawn="melee", n_ep=q(6), seed=5, mixed_rows=True)
    run_scenario(game, combatant, landingship, "3v2ls_landing", grids, nb_types=S4[:3],
                 nr_types=["large", "large"], spawn="ref", n_ep=q(3), seed=6, random_ls=1,
                 flags=dict(LANDING_OPS=True))
    run_scenario(game, combatant, landingship, "3v3ls_landing_melee", grids,
                 nb_types=S4[:3], nr_types=["large", "large", "ls"], spawn="melee",
                 n_ep=q(8), seed=7, flags=dict(LANDING_OPS=True))
    run_scenario(game, combatant, landingship, "4v4_defensive", grids, nb_types=S4,
                 nr_types=R4, spawn="melee", n_ep=q(6), seed=8,
                 flags=dict(TACTICS="defensive"))
    run_scenario(game, combatant, landingship, "4v4_side_red", grids, nb_types=S4,
                 nr_types=R4, spawn="melee", n_ep=q(6), seed=9, flags=dict(SIDE="red"))
    run_scenario(game, combatant, landingship, "4v4_untrained_red", grids, nb_types=S4,
                 nr_types=R4, spawn="melee", n_ep=q(6), seed=10,
                 flags=dict(TRAINED_RED=False))
    run_scenario(game, combatant, landingship, "4v4_discrete", grids, nb_types=S4,
                 nr_types=R4, spawn="melee", n_ep=q(6), seed=11, flags=dict(DISCRETE=True))
    run_scenario(game, combatant, landingship, "4v4_discrete_lists", grids, nb_types=S4,
                 nr_types=R4, spawn="melee", n_ep=q(6), seed=18, list_rows=True,
                 flags=dict(DISCRETE=True, TRAINED_RED=False))
    run_scenario(game, combatant, landingship, "4v4_observe", grids, nb_types=S4,
                 nr_types=R4, spawn="melee", n_ep=q(6), seed=12, observe=True)
    run_scenario(game, combatant, landingship, "4v4_wild", grids, nb_types=S4, nr_types=R4,
                 spawn="melee", n_ep=q(6), seed=13, act_lo=-0.6, act_hi=1.6)
    run_scenario(game, combatant, landingship, "8v10ls_g200", grids, nb_types=["small"] * 8,
                 nr_types=["large"] * 8, spawn="melee", n_ep=q(3), seed=14, random_ls=2,
                 grid_id=1, flags=dict(LANDING_OPS=True))
    run_scenario(game, combatant, landingship, "8v8_g200_observe", grids,
                 nb_types=["small"] * 8, nr_types=["large"] * 6 + ["ls"] * 2, spawn="melee",
                 n_ep=q(3), seed=15, grid_id=1, observe=True)
    # the "medium" Combatant (combatant.py:64-80: speed 2, 8 missiles, mast 30,
    # rcs 1; game.py:193-198). A side's row length follows its fastest ship
    # (game.py:595-610), and a medium row is 4n + 5x5 + 3 floats, so only a side
    # made of medium ships runs (mixed with speed-3 ships the row assignment at
    # game.py:344 raises ValueError)
    M = ["medium"] * 4
    run_scenario(game, combatant, landingship, "3v3_medium_melee_observe", grids,
                 nb_types=M[:3], nr_types=M[:3], spawn="melee", n_ep=q(8), seed=19, observe=True)
    run_scenario(game, combatant, landingship, "4v2_medium_split_f32", grids, nb_types=M,
                 nr_types=["large", "small"], spawn="split", n_ep=q(6), seed=20, dtype="f32")
    run_scenario(game, combatant, landingship, "2v4_medium_discrete", grids, nb_types=S4[:2],
                 nr_types=M, spawn="melee", n_ep=q(6), seed=24, flags=dict(DISCRETE=True))
    run_scenario(game, combatant, landingship, "3v3_medium_untrained_red", grids, nb_types=M[:3],
                 nr_types=M[:3], spawn="melee", n_ep=q(6), seed=25, flags=dict(TRAINED_RED=False))


def main():
    quick = "--quick" in sys.argv
    if not os.path.isdir(REF):
        print("reference not present; nothing to do")
        return
    game, combatant, landingship = import_reference()
    g100, g200 = make_grids(game)
    grids = [g100, g200]
    only = [a for a in sys.argv[1:] if not a.startswith("--")]
    if not only or "ranges" in only:
        make_ranges(game, combatant, landingship, g100)
    if not only or "los" in only:
        make_los(game, combatant, g100, g200, quick)
    if not only or "moves" in only:
        make_moves(game, combatant, g100, quick)
    if not only or "astar" in only:
        make_astar(game, combatant, g100, g200, quick)
    if not only or "episodes" in only:
        make_episodes(game, combatant, landingship, grids, quick)
    if "--analytics" in sys.argv or "analytics" in only:
        make_analytics_episodes(game, combatant, landingship, grids, quick)


def make_analytics_episodes(game, combatant, landingship, grids, quick):
    """Episodes with the analytics side channels recorded."""
    q = (lambda n: max(2, n // 3)) if quick else (lambda n: n)
    S4, R4 = ["small"] * 4, ["large"] * 4
    run_scenario(game, combatant, landingship, "ana_melee", grids, nb_types=S4, nr_types=R4,
                 spawn="melee", n_ep=q(8), seed=21, analytics=True)
    run_scenario(game, combatant, landingship, "ana_melee_red", grids, nb_types=S4, nr_types=R4,
                 spawn="melee", n_ep=q(6), seed=22, analytics=True, flags=dict(SIDE="red"))
    run_scenario(game, combatant, landingship, "ana_split_observe", grids, nb_types=S4,
                 nr_types=R4, spawn="split", n_ep=q(6), seed=23, analytics=True, observe=True)


if __name__ == "__main__":
    main()
