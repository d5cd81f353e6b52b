"""Parity of the HIP path (liblnw.so through the C-ABI) against the golden
vectors and the CPU oracle. Needs an MI355X.

Bar (BASELINE.json north_star): bit-exact occlusion/visibility masks, move
validity, positions, target lists, RNG consumption and observations
(float32 of the reference's float64); rewards and cog within 1e-5 absolute
(rtol = 0; the golden replays read them as float64, lnw_set_reward_dtype).
"""
import glob
import os

import numpy as np
import pytest
import torch

from _oracle import (GOLDEN, OracleEnv, astar_batch, episode_meta, load_fixture, los_batch,
                     move_batch)

pytestmark = pytest.mark.gpu

EPISODES = sorted(os.path.basename(p) for p in glob.glob(os.path.join(GOLDEN, "ep_*.npz")))
REW_TOL = 1e-5


@pytest.fixture(scope="module")
def grids():
    g = load_fixture("grids.npz")
    return [g["grid100"], g["grid200"]]


@pytest.fixture(scope="module")
def lib():
    import lnw
    from lnw import _abi
    return _abi.load()


_KEEP = []


def _dev(a):
    """Device copy that stays alive until the next test (a raw pointer taken from
    a temporary would let the caching allocator hand its block to the next
    argument before the kernel runs)."""
    t = torch.from_numpy(np.ascontiguousarray(a)).cuda()
    _KEEP.append(t)
    return t


@pytest.fixture(autouse=True)
def _release():
    yield
    torch.cuda.synchronize()
    _KEEP.clear()


def _p(t):
    import ctypes
    return ctypes.c_void_p(t.data_ptr())


# ---------------------------------------------------------------------------
# unit kernels
# ---------------------------------------------------------------------------
def test_los_batch_golden(lib, grids):
    fx = load_fixture("los.npz")
    for gi in (0, 1):
        m = fx["grid_id"] == gi
        g = _dev(grids[gi])
        pairs = _dev(fx["pairs"][m].astype(np.int16))
        out = torch.zeros(int(m.sum()), dtype=torch.uint8, device="cuda")
        assert lib.lnw_los_batch(_p(g), grids[gi].shape[0], _p(pairs), int(m.sum()), 74, 70,
                                 _p(out), None) == 0
        o = out.cpu().numpy()
        assert np.array_equal(o & 1, fx["radar"][m])
        assert np.array_equal((o >> 1) & 1, fx["ew"][m])


def test_los_batch_vs_oracle_random(lib, grids):
    rng = np.random.default_rng(0)
    for gi in (0, 1):
        G = grids[gi].shape[0]
        n = 400000
        P = rng.integers(0, G, size=(n, 4)).astype(np.int16)
        near = P[: n // 2]
        near[:, 2:] = np.clip(near[:, :2] + rng.integers(-40, 41, size=(n // 2, 2)), 0, G - 1)
        g = _dev(grids[gi])
        out = torch.zeros(n, dtype=torch.uint8, device="cuda")
        lib.lnw_los_batch(_p(g), G, _p(_dev(P)), n, 74, 70, _p(out), None)
        o = out.cpu().numpy()
        assert np.array_equal(o & 1, los_batch(grids[gi], P, 74))
        assert np.array_equal((o >> 1) & 1, los_batch(grids[gi], P, 70))


def test_los_batch_large_grid_and_ragged(lib):
    """lnw_los_batch beyond the LDS-staged size (G = 600: the 2-bit mask would
    take 90 KB, so the one-lane HBM kernel runs), at the largest staged size
    (G = 512: 64 KB of LDS) and with ray counts that leave a wave's queue
    partly filled (1, 63, 1 025 rays), against the oracle."""
    rng = np.random.default_rng(5)
    for G, n in ((600, 20000), (512, 20000), (100, 1), (100, 63), (100, 1025)):
        grid = rng.integers(0, 120, size=(G, G)).astype(np.uint8)
        P = rng.integers(0, G, size=(n, 4)).astype(np.int16)
        P[: n // 2, 2:] = np.clip(P[: n // 2, :2] + rng.integers(-40, 41, size=(n // 2, 2)), 0, G - 1)
        out = torch.full((n,), 255, dtype=torch.uint8, device="cuda")
        assert lib.lnw_los_batch(_p(_dev(grid)), G, _p(_dev(P)), n, 74, 70, _p(out), None) == 0
        o = out.cpu().numpy()
        assert np.array_equal(o & 1, los_batch(grid, P, 74)), G
        assert np.array_equal((o >> 1) & 1, los_batch(grid, P, 70)), G
        assert not np.any(o >> 2), G
    # a pairs buffer 2 bytes into its allocation (not 8-byte aligned: the HBM kernel)
    G, n = 100, 5000
    grid = rng.integers(0, 120, size=(G, G)).astype(np.uint8)
    P = rng.integers(0, G, size=(n, 4)).astype(np.int16)
    buf = torch.zeros(4 * n + 1, dtype=torch.int16, device="cuda")
    buf[1:] = torch.from_numpy(P.reshape(-1)).cuda()
    out = torch.zeros(n, dtype=torch.uint8, device="cuda")
    assert lib.lnw_los_batch(_p(_dev(grid)), G, _p(buf[1:]), n, 74, 70, _p(out), None) == 0
    o = out.cpu().numpy()
    assert np.array_equal(o & 1, los_batch(grid, P, 74))
    assert np.array_equal((o >> 1) & 1, los_batch(grid, P, 70))


def test_astar_batch_golden(lib, grids):
    fx = load_fixture("astar.npz")
    for gi in (0, 1):
        m = fx["grid_id"] == gi
        n = int(m.sum())
        # fixture classes: 0 small (speed 3), 1 ls (speed 2), 2 medium (speed 2)
        cls = fx["cls"][m]
        keep = np.ones(len(cls), bool)
        assert gi == 1 or (cls == 2).any()  # the medium cases are there (grid 100)
        types = np.choose(cls, [0, 2, 3]).astype(np.int8)
        st, tg = fx["start"][m][keep], fx["target"][m][keep]
        k = int(keep.sum())
        plen = torch.zeros(k, dtype=torch.int16, device="cuda")
        kind = torch.zeros(k, dtype=torch.int8, device="cuda")
        feas = torch.zeros(k, dtype=torch.uint8, device="cuda")
        g = _dev(grids[gi])
        assert lib.lnw_astar_batch(_p(g), grids[gi].shape[0], 74, _p(_dev(types)), _p(_dev(st)),
                                   _p(_dev(tg)), k, _p(plen), _p(kind), _p(feas), None) == 0
        assert np.array_equal(plen.cpu().numpy(), fx["plen"][m][keep])
        assert np.array_equal(kind.cpu().numpy(), fx["kind"][m][keep])
        assert np.array_equal(feas.cpu().numpy(), fx["feasible"][m][keep])


@pytest.mark.parametrize("gi", [0, 1])
@pytest.mark.parametrize("move_mode", [0, 1])
def test_move_table_exhaustive(lib, grids, gi, move_mode):
    """check_path for every start cell x every target offset in [-4,4]^2 (the
    move table's window) for Combatant, LandingShip and the medium Combatant
    (speed 2): table (move_mode 0) and A* replica (move_mode 1) against the
    oracle."""
    from lnw.batched import BatchedGame
    from lnw.config import Scenario
    grid = grids[gi]
    G = grid.shape[0]
    g = BatchedGame(64, ["small"], ["large"], scenario=Scenario(move_mode=move_mode), grid=grid)
    cells = np.array([(x, y) for x in range(G) for y in range(G)], np.int32)
    if gi == 1:
        cells = cells[::5]
    off = np.array([(dx, dy) for dx in range(-4, 5) for dy in range(-4, 5)], np.int32)
    st = np.repeat(cells, 81, axis=0)
    tg = st + np.tile(off, (len(cells), 1))
    n = len(st)
    for tcode, ocls in ((0, 0), (2, 1), (3, 2)):
        _, _, ref = astar_batch(grid, np.full(n, ocls, np.int8), st, tg)
        out = torch.zeros(n, dtype=torch.uint8, device="cuda")
        assert lib.lnw_path_query(g.h, _p(_dev(np.full(n, tcode, np.int8))),
                                  _p(_dev(st.astype(np.int16))), _p(_dev(tg.astype(np.int16))),
                                  n, _p(out), None) == 0
        o = out.cpu().numpy()
        bad = int((o != ref).sum())
        assert bad == 0, f"{bad} check_path mismatches (type {tcode}, move_mode {move_mode})"
    g.close()


def test_move_batch_golden(lib, grids):
    from lnw.batched import BatchedGame
    from lnw.config import Scenario
    fx = load_fixture("moves.npz")
    for move_mode in (0, 1):
        g = BatchedGame(64, ["small"], ["large"], scenario=Scenario(move_mode=move_mode),
                        grid=grids[0])
        n = len(fx["cls"])
        types = np.where(fx["cls"] == 1, 2, 0).astype(np.int8)
        rounded = torch.zeros((n, 2), dtype=torch.int32, device="cuda")
        ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
        assert lib.lnw_move_batch(g.h, _p(_dev(types)), _p(_dev(fx["pos"].astype(np.int16))),
                                  _p(_dev(fx["act"])), _p(_dev(fx["is_f32"])), n, _p(rounded),
                                  _p(ok), None) == 0
        assert np.array_equal(rounded.cpu().numpy(), fx["rounded"])
        assert np.array_equal(ok.cpu().numpy(), fx["ok"])
        g.close()


def test_move_batch_vs_oracle_random(lib, grids):
    """2M random continuous moves (f64 and f32 rows, in- and out-of-range
    actions): device cos/sin (ocml) vs glibc must round to the same cell."""
    from lnw.batched import BatchedGame
    from lnw.config import Scenario
    rng = np.random.default_rng(7)
    n = 2_000_000
    g = BatchedGame(64, ["small"], ["large"], scenario=Scenario(), grid=grids[0])
    water = np.argwhere(grids[0] <= 74)
    pos = water[rng.integers(0, len(water), size=n)].astype(np.int16)
    act = rng.uniform(-0.25, 1.5, size=(n, 2))
    f32 = (rng.random(n) < 0.5).astype(np.uint8)
    act[f32 == 1] = act[f32 == 1].astype(np.float32).astype(np.float64)
    cls = (rng.random(n) < 0.2).astype(np.int8)
    types = np.where(cls == 1, 2, 0).astype(np.int8)
    rounded = torch.zeros((n, 2), dtype=torch.int32, device="cuda")
    ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
    lib.lnw_move_batch(g.h, _p(_dev(types)), _p(_dev(pos)), _p(_dev(act)), _p(_dev(f32)), n,
                       _p(rounded), _p(ok), None)
    r_ref, ok_ref = move_batch(grids[0], cls, f32, pos, act)
    r = rounded.cpu().numpy()
    mism = int((r != r_ref).any(axis=1).sum())
    assert mism == 0, f"{mism} of {n} move targets differ from the oracle"
    assert np.array_equal(ok.cpu().numpy(), ok_ref)
    g.close()


@pytest.mark.parametrize("gi", [0, 1])
def test_los_table_vs_march(lib, grids, gi):
    """LOS table (precomputed at load_terrain) == ray march == oracle for pairs
    inside and outside the table window."""
    from lnw.batched import BatchedGame
    from lnw.config import Scenario
    grid = grids[gi]
    G = grid.shape[0]
    rng = np.random.default_rng(11 + gi)
    n = 1_000_000
    o = rng.integers(0, G, size=(n, 2))
    d = np.clip(o + rng.integers(-45, 46, size=(n, 2)), 0, G - 1)
    P = np.concatenate([o, d], 1).astype(np.int16)
    ref_r = los_batch(grid, P, 74)
    ref_e = los_batch(grid, P, 70)
    for los_mode in (0, 1):
        g = BatchedGame(64, ["small"], ["large"], scenario=Scenario(los_mode=los_mode), grid=grid)
        out = torch.zeros(n, dtype=torch.uint8, device="cuda")
        assert lib.lnw_los_query(g.h, _p(_dev(P)), n, _p(out), None) == 0
        o_ = out.cpu().numpy()
        assert np.array_equal(o_ & 1, ref_r)
        # the step's query may stop at the first radar-blocked cell: EW is only
        # consulted when radar LOS is clear (combatant.py:110,119)
        clear = ref_r == 1
        assert np.array_equal(((o_ >> 1) & 1)[clear], ref_e[clear])
        g.close()


def test_hit_tables_match_numpy(lib):
    import ctypes
    t64 = np.zeros(18)
    t32 = np.zeros(18, np.float32)
    lib.lnw_hit_tables(t64.ctypes.data_as(ctypes.c_void_p), t32.ctypes.data_as(ctypes.c_void_p))
    for h, p in enumerate((0.45, 0.63)):
        for n in range(9):
            assert t64[h * 9 + n] == 1 - (1 - p) ** np.float64(n)
            assert t32[h * 9 + n] == 1 - (1 - p) ** np.float32(n)


def test_device_sqrt_is_correctly_rounded(lib, grids):
    """Rewards use sqrt of integer squared distances (game.py:268,276); the
    reward path relies on IEEE sqrt. Checked through the cog/reward parity tests;
    here directly through torch on the same device for every d2 < 80001."""
    d2 = torch.arange(0, 80001, dtype=torch.float64, device="cuda")
    assert np.array_equal(torch.sqrt(d2).cpu().numpy(), np.sqrt(np.arange(0, 80001.0)))


# ---------------------------------------------------------------------------
# full episodes, tape mode
# ---------------------------------------------------------------------------
def _cmp_episode(name, grids, los_mode, move_mode, contact=False):
    from _gpu_replay import replay_gpu
    fx = load_fixture(name)
    meta = episode_meta(fx)
    cnt, xy = fx["tl_cnt"], fx["tl_xy"]
    offs = np.concatenate([[0], np.cumsum(cnt.reshape(-1))])
    checked = 0
    for kind, info, g, res in replay_gpu(fx, grids, los_mode, move_mode, contact):
        if kind == "reset":
            ds = g.env_state()["ducting"]
            for e, em in enumerate(meta["episodes"]):
                assert ds[e] == em["ducting"], f"{name} env {e} ducting"
            st = g.agents()
            for e, em in enumerate(meta["episodes"]):
                sp = np.array(em["spawn"])
                assert np.array_equal(np.stack([st["x"][e], st["y"][e]], 1), sp), f"{name} spawn"
            continue
        s, rows = info
        if kind == "observe":
            ob, orr = res
            nb = meta["episodes"][0]["nb"]
            for e, i in rows:
                for a in range(fx["pre_obs_valid"].shape[1]):
                    if not fx["pre_obs_valid"][i, a]:
                        continue
                    got = ob[e, a] if a < nb else orr[e, a - nb]
                    ref = fx["pre_obs"][i, a, :len(got)]
                    assert np.array_equal(got, ref), f"{name} pre-obs step {i} agent {a}"
            continue
        st = g.agents()
        es = g.env_state()
        A = st["x"].shape[1]
        for e, i in rows:
            ctx = f"{name} env {e} step {i}"
            assert np.array_equal(res["obs_blue"][e], fx["obs_blue"][i]), f"{ctx} obs_blue"
            assert np.array_equal(res["obs_red"][e], fx["obs_red"][i]), f"{ctx} obs_red"
            assert res["rew_blue"].dtype == np.float64
            np.testing.assert_allclose(res["rew_blue"][e], fx["rew_blue"][i], rtol=0,
                                       atol=REW_TOL, err_msg=ctx)
            np.testing.assert_allclose(res["rew_red"][e], fx["rew_red"][i], rtol=0,
                                       atol=REW_TOL, err_msg=ctx)
            assert res["done"][e] == fx["done"][i], ctx
            c = fx["cog"][i]
            if np.isnan(c):
                assert np.isnan(res["cog"][e]), ctx
            else:
                assert abs(res["cog"][e] - c) <= 1e-5, ctx
            assert np.array_equal(res["actions_after"][e].astype(np.float64),
                                  fx["actions_after"][i].astype(res["actions_after"].dtype)
                                  .astype(np.float64)), f"{ctx} mutated actions"
            pos = np.stack([st["x"][e], st["y"][e]], 1)
            assert np.array_equal(pos, fx["pos"][i]), f"{ctx} pos"
            assert np.array_equal(st["radar"][e], fx["radar"][i]), f"{ctx} radar"
            assert np.array_equal(st["missiles"][e].astype(np.float64), fx["missiles"][i]), f"{ctx} missiles"
            assert np.array_equal(st["alive"][e], fx["alive"][i]), f"{ctx} alive"
            assert np.array_equal(st["steps_done"][e], fx["steps_done"][i]), f"{ctx} steps"
            assert np.array_equal(st["dist_lz"][e], fx["dist_lz"][i]), f"{ctx} dist_lz"
            assert np.array_equal(st["tl_cnt"][e], fx["tl_cnt"][i]), f"{ctx} tl_cnt"
            assert [es["n_blue_left"][e], es["n_red_left"][e]] == list(fx["n_left"][i]), ctx
            assert [es["blue_victory"][e], es["red_victory"][e]] == list(fx["victories"][i]), ctx
            assert es["rng"][e] == fx["tape_pos"][i], f"{ctx} rng draws"
            assert es["err"][e] == 0, f"{ctx} err flags {es['err'][e]}"
            tls = g.tlists(e)
            for a in range(A):
                k = i * A + a
                ref = [tuple(int(v) for v in t) for t in xy[offs[k]:offs[k + 1]]]
                assert tls[a] == ref, f"{ctx} tlist agent {a}"
            checked += 1
        del st
    assert checked == len(fx["done"])
    return checked


@pytest.mark.parametrize("name", EPISODES)
def test_episode_gpu_tape(name, grids):
    _cmp_episode(name, grids, los_mode=0, move_mode=0)


@pytest.mark.parametrize("name", EPISODES)
def test_episode_gpu_tape_contact_variant(name, grids):
    """Every golden episode through the contact variant of the step kernel
    (lnw_set_variant: bit-mask pair walk, two bearings per iteration)."""
    _cmp_episode(name, grids, los_mode=0, move_mode=0, contact=True)


@pytest.mark.parametrize("name", ["ep_4v4_melee_f64.npz", "ep_4v4_split_f64.npz",
                                  "ep_8v10ls_g200.npz", "ep_4v4_wild.npz",
                                  "ep_3v3_medium_melee_observe.npz"])
def test_episode_gpu_tape_march_astar(name, grids):
    """Same episodes with the LOS ray march and the direct A* instead of the
    precomputed tables."""
    if not os.path.exists(os.path.join(GOLDEN, name)):
        pytest.skip("fixture absent")
    _cmp_episode(name, grids, los_mode=1, move_mode=1)


@pytest.mark.parametrize("contact", [False, True])
@pytest.mark.parametrize("name", ["ep_ana_melee.npz", "ep_ana_melee_red.npz",
                                  "ep_ana_split_observe.npz"])
def test_analytics_replay(name, contact, grids):
    """Analytics side channels (lnw_set_analytics) against the reference's
    heatmap / coldmap / launch_sites / engagements / blue_ew / red_ew recorded
    over the same tape-mode episodes (make_golden.py make_analytics_episodes),
    through both step-kernel variants (the contact variant's pooled bearings
    record the EW fixes from the lane that finishes them)."""
    from _gpu_replay import replay_gpu
    fx = load_fixture(name)
    n_steps = np.array([em["n_steps"] for em in episode_meta(fx)["episodes"]])
    g = None
    counting = False
    for kind, info, g, res in replay_gpu(fx, grids, contact=contact):
        if kind == "reset":
            g.enable_analytics(eng_cap=4096, ew_cap=4096)
            if contact and not counting:
                g.count_work(True)
                counting = True
    torch.cuda.synchronize()
    if contact and "melee" in name:  # the pooled path ran
        assert g.work_counts()["pooled_bearings"] > 0
    an = g.analytics()
    assert an["engagements_total"] <= 4096 and an["ew_total"] <= 4096
    np.testing.assert_array_equal(an["heatmap"].cpu().numpy(), fx["ana_heat"].sum(0))
    np.testing.assert_array_equal(an["coldmap"].cpu().numpy(), fx["ana_cold"].sum(0))
    np.testing.assert_array_equal(an["launch"].cpu().numpy(), fx["ana_launch"].sum(0))
    eng = an["engagements"].cpu().numpy()
    eng = eng[eng[:, 1] < n_steps[eng[:, 0]]]  # steps past an episode's end replay idle
    got = sorted(tuple(int(v) for v in r[[0, 1, 3, 4, 5, 6, 7]]) for r in eng)
    want = sorted(tuple(int(v) for v in r) for r in fx["ana_eng"])
    assert got == want
    ew = an["ew_fixes"].cpu().numpy()
    ew = ew[ew[:, 1] < n_steps[ew[:, 0]]]
    got = sorted(tuple(int(v) for v in r) for r in ew)
    want = sorted(tuple(int(v) for v in r) for r in fx["ana_ew"])
    assert got == want
    g.disable_analytics()
    g.close()


def test_shard_invariance(grids):
    """Env sharding: two handles holding global envs [0,32) and [32,64) produce
    exactly the trajectories of one handle holding [0,64) (RNG keyed by global
    env id; melee box spawns drawn per global id too)."""
    from lnw.batched import BatchedGame
    from lnw.config import Scenario
    sc = Scenario(landing_ops=False, auto_reset=True, episode_steps=40)
    box = ((40, 40), (57, 65))
    pos = [(6, 61), (10, 81), (8, 70), (11, 58), (98, 48), (98, 52), (98, 56), (96, 52)]
    full = BatchedGame(64, ["small"] * 4, ["large"] * 4, scenario=sc, grid=grids[0], seed=5)
    assert full.set_epw(64) == 64  # one full two-wave workgroup: rows emitted during phase S
    parts = [BatchedGame(32, ["small"] * 4, ["large"] * 4, scenario=sc, grid=grids[0], seed=5,
                         env_id_base=b) for b in (0, 32)]
    for g in [full] + parts:
        g.reset(positions=pos, box=box)
    rng = np.random.default_rng(0)
    for s in range(60):
        act = torch.from_numpy(rng.random((64, 8, 4)).astype(np.float32)).cuda()
        of = {k: v.cpu().numpy().copy() for k, v in full.step(act.clone()).items()}
        op = [{k: v.cpu().numpy().copy() for k, v in g.step(act[32 * i:32 * (i + 1)].clone()).items()}
              for i, g in enumerate(parts)]
        for k in of:
            merged = np.concatenate([op[0][k], op[1][k]])
            assert np.array_equal(of[k], merged, equal_nan=True), (s, k)
    for g in [full] + parts:
        g.close()


def _melee_positions(grid, E, nb, nr, seed, box_b=(30, 45, 40, 60), box_r=(55, 70, 45, 65)):
    rng = np.random.default_rng(seed)
    water = lambda x0, x1, y0, y1: [(x, y) for x in range(x0, x1) for y in range(y0, y1)
                                    if grid[x, y] <= 74]
    wb, wr = water(*box_b), water(*box_r)
    return np.array([[wb[i] for i in rng.integers(0, len(wb), nb)] +
                     [wr[i] for i in rng.integers(0, len(wr), nr)] for _ in range(E)], np.int32)


@pytest.mark.parametrize("epw,contact", [(64, False), (16, False), (1, False), (64, True), (16, True)])
def test_philox_4v4_vs_oracle_launch_shapes(grids, epw, contact):
    """4v4 split spawns (fire, EW bearings and fixes happen) in production
    (Philox) mode, 128 envs, with the step launched at 64 / 16 / 1 envs per
    workgroup (64: the two-wave emission path; 16, 1: phase O after phase S),
    every output bit-exact against the CPU oracle stepping the same envs."""
    import _oracle
    from lnw.batched import BatchedGame
    from lnw.config import Scenario
    grid = grids[0]
    E, S = 128, 10
    g = BatchedGame(E, ["small"] * 4, ["large"] * 4, scenario=Scenario(landing_ops=False),
                    grid=grid, seed=11)
    assert g.set_epw(epw) == epw
    g.set_variant(contact)
    pos = _melee_positions(grid, E, 4, 4, seed=epw)
    g.reset(positions=pos[0], pos_per_env=torch.from_numpy(pos))
    oracles = []
    for e in range(E):
        o = _oracle.OracleEnv(grid, 4, 4)
        o.set_philox(11, e)
        o.reset([0] * 4 + [1] * 4, pos[e])
        oracles.append(o)
    rng = np.random.default_rng(epw + 100)
    for s in range(S):
        act = rng.random((E, 8, 4)).astype(np.float32)
        out = g.step(torch.from_numpy(act).cuda())
        ob, orr = out["obs_blue"].cpu().numpy(), out["obs_red"].cpu().numpy()
        rb, rr = out["rew_blue"].cpu().numpy(), out["rew_red"].cpu().numpy()
        dn = out["done"].cpu().numpy()
        for e in range(E):
            r = oracles[e].step(act[e], np.full(8, _oracle.K_F32, np.int32))
            assert np.array_equal(ob[e], r["obs_blue"].astype(np.float32)), (s, e, "obs_blue")
            assert np.array_equal(orr[e], r["obs_red"].astype(np.float32)), (s, e, "obs_red")
            assert np.allclose(rb[e], r["rew_blue"], rtol=0, atol=REW_TOL), (s, e, "rew_blue")
            assert np.allclose(rr[e], r["rew_red"], rtol=0, atol=REW_TOL), (s, e, "rew_red")
            assert dn[e] == r["done"], (s, e, "done")
    g.close()


def test_contact_pooled_bearings(grids):
    """Contact variant at melee spawns (every get_obs has EW bearings): the
    wave-pooled bearing rounds (finish_obs_t) run — the work counter says so —
    and give the same trajectories as the per-lane loop (LNW_DEBUG_SKIP bit 17)
    and as the default variant; a sample of envs is checked against the oracle."""
    import os
    import _oracle
    from lnw.batched import BatchedGame
    from lnw.config import Scenario
    grid = grids[0]
    E, S = 1024, 6
    pos = _melee_positions(grid, E, 4, 4, seed=5)
    rng = np.random.default_rng(7)
    acts = [rng.random((E, 8, 4)).astype(np.float32) for _ in range(S)]
    outs = []
    for contact, skip in ((True, "0"), (True, str(1 << 17)), (False, "0")):
        os.environ["LNW_DEBUG_SKIP"] = skip
        try:
            g = BatchedGame(E, ["small"] * 4, ["large"] * 4, scenario=Scenario(landing_ops=False),
                            grid=grid, seed=21)
        finally:
            os.environ.pop("LNW_DEBUG_SKIP")
        g.set_variant(contact)
        g.reset(positions=pos[0], pos_per_env=torch.from_numpy(pos))
        g.count_work(True)
        traj = [{k: v.cpu().numpy().copy() for k, v in g.step(torch.from_numpy(a).cuda()).items()}
                for a in acts]
        torch.cuda.synchronize()
        outs.append((traj, g.work_counts()))
        g.close()
    assert outs[0][1]["pooled_bearings"] > 0, outs[0][1]
    assert outs[1][1]["pooled_bearings"] == 0 and outs[2][1]["pooled_bearings"] == 0
    for traj, _ in outs[1:]:
        for s in range(S):
            for k in traj[s]:
                assert np.array_equal(outs[0][0][s][k], traj[s][k], equal_nan=True), (s, k)
    for e in range(0, E, 97):
        o = _oracle.OracleEnv(grid, 4, 4)
        o.set_philox(21, e)
        o.reset([0] * 4 + [1] * 4, pos[e])
        for s in range(S):
            r = o.step(acts[s][e], np.full(8, _oracle.K_F32, np.int32))
            out = outs[0][0][s]
            assert np.array_equal(out["obs_blue"][e], r["obs_blue"].astype(np.float32)), (s, e)
            assert np.array_equal(out["obs_red"][e], r["obs_red"].astype(np.float32)), (s, e)
            assert np.allclose(out["rew_blue"][e], r["rew_blue"], rtol=0, atol=REW_TOL), (s, e)
            assert out["done"][e] == r["done"], (s, e)


def test_config4_launch_shape_invariance(grids):
    """Config 4 shape (8 small blue vs 8 large + 2 LandingShip red, landing ops,
    200x200 grid, box spawns): the automatic envs-per-workgroup choice, 64 and 1
    give identical trajectories (observations, rewards, done, cog)."""
    from lnw.batched import BatchedGame
    from lnw.config import Scenario
    sc = Scenario(landing_ops=True, auto_reset=True, episode_steps=40)
    E = 256
    games = []
    for epw in (0, 64, 1):
        g = BatchedGame(E, ["small"] * 8, ["large"] * 8 + ["ls"] * 2, scenario=sc, grid=grids[1],
                        seed=3)
        g.set_epw(epw)
        g.reset(positions=[(0, 0)] * 18, rand_ls=[0] * 16 + [1, 1], box=((20, 60), (80, 140)))
        games.append(g)
    assert games[0].epw < 64  # 256 envs cannot fill the GPU at 64 per workgroup
    rng = np.random.default_rng(1)
    for s in range(50):
        act = torch.from_numpy(rng.random((E, 18, 4)).astype(np.float32)).cuda()
        outs = [{k: v.cpu().numpy().copy() for k, v in g.step(act.clone()).items()} for g in games]
        for o in outs[1:]:
            for k in outs[0]:
                assert np.array_equal(outs[0][k], o[k], equal_nan=True), (s, k)
    for g in games:
        g.close()


REF_SPAWNS = [(6, 61), (10, 81), (8, 70), (11, 58), (98, 48), (98, 52), (98, 56), (96, 52)]


@pytest.mark.parametrize("trained_red", [True, False])
def test_quiet_path_vs_oracle(grids, trained_red):
    """Quiet workgroups (lnw_quiet.inc): 128 envs at 64 per workgroup in Philox
    mode; workgroup 0 holds reference spawns (quiet: no sensor contact, phase Q
    + whole-block emission), workgroup 1 half reference, half split spawns (not
    quiet: phase S). Every output bit-exact against the CPU oracle; with an
    untrained red also its random salvos (game.py:375-379: the draws and the
    in-place action writes)."""
    import _oracle
    from lnw.batched import BatchedGame
    from lnw.config import Scenario
    grid = grids[0]
    E, S = 128, 14
    g = BatchedGame(E, ["small"] * 4, ["large"] * 4,
                    scenario=Scenario(landing_ops=False, trained_red=trained_red),
                    grid=grid, seed=21)
    assert g.set_epw(64) == 64
    pos = np.array([REF_SPAWNS] * E, np.int32)
    pos[96:] = _melee_positions(grid, 32, 4, 4, seed=4)
    g.reset(positions=pos[0], pos_per_env=torch.from_numpy(pos))
    oracles = []
    for e in range(E):
        o = _oracle.OracleEnv(grid, 4, 4, trained_red=trained_red)
        o.set_philox(21, e)
        o.reset([0] * 4 + [1] * 4, pos[e])
        oracles.append(o)
    rng = np.random.default_rng(8)
    for s in range(S):
        act = rng.random((E, 8, 4)).astype(np.float32)
        act_dev = torch.from_numpy(act).cuda()
        out = g.step(act_dev)
        act_after = act_dev.cpu().numpy()
        ob, orr = out["obs_blue"].cpu().numpy(), out["obs_red"].cpu().numpy()
        rb, rr = out["rew_blue"].cpu().numpy(), out["rew_red"].cpu().numpy()
        dn, cg = out["done"].cpu().numpy(), out["cog"].cpu().numpy()
        for e in range(E):
            r = oracles[e].step(act[e], np.full(8, _oracle.K_F32, np.int32))
            assert np.array_equal(act_after[e], r["actions_after"].astype(np.float32)), (s, e, "actions")
            assert np.array_equal(ob[e], r["obs_blue"].astype(np.float32)), (s, e, "obs_blue")
            assert np.array_equal(orr[e], r["obs_red"].astype(np.float32)), (s, e, "obs_red")
            assert np.allclose(rb[e], r["rew_blue"], rtol=0, atol=REW_TOL), (s, e, "rew_blue")
            assert np.allclose(rr[e], r["rew_red"], rtol=0, atol=REW_TOL), (s, e, "rew_red")
            assert dn[e] == r["done"], (s, e, "done")
            assert abs(cg[e] - r["cog"]) <= 1e-5 or (np.isnan(cg[e]) and np.isnan(r["cog"])), (s, e)
    g.close()


@pytest.mark.parametrize("E,trained_red", [(256, True), (256, False), (8192, True), (4133, False)])
@pytest.mark.parametrize("spawns", ["reference", "mixed"])
def test_quiet_path_vs_phase_s_long(grids, spawns, trained_red, E, monkeypatch):
    """The bench workload shape (auto-reset, 40-step episodes, Philox) over 90
    steps, four launch shapes with identical results (observations, rewards,
    done, cog, written-back actions, final state): 64 envs per workgroup (quiet
    path where it applies), 16 and 8 envs per workgroup (the quiet path in
    partial two-wave workgroups with wave 1 storing every row straight from
    registers: the small-E launch shapes), and 64 per workgroup with
    the quiet path disabled (LNW_DEBUG_SKIP bit 9: phase S everywhere). E = 8 192
    is config 3's per-GPU shard; 4 133 leaves a ragged last workgroup. "mixed":
    every second group of 64 envs spawns (and re-spawns) in the melee box."""
    from lnw import _abi
    from lnw.batched import BatchedGame
    from lnw.config import Scenario
    sc = Scenario(landing_ops=False, auto_reset=True, episode_steps=40, trained_red=trained_red)
    pos = np.array([REF_SPAWNS] * E, np.int32)
    if spawns == "mixed":
        for w in range(1, (E + 63) // 64, 2):
            n = min(64, E - 64 * w)
            pos[64 * w:64 * w + n] = _melee_positions(grids[0], n, 4, 4, seed=w)
    games = []
    for epw, skip in ((64, None), (16, None), (8, None), (64, "512")):
        if skip:
            monkeypatch.setenv("LNW_DEBUG_SKIP", skip)  # read once, by lnw_create
        g = BatchedGame(E, ["small"] * 4, ["large"] * 4, scenario=sc, grid=grids[0], seed=9)
        monkeypatch.delenv("LNW_DEBUG_SKIP", raising=False)
        assert g.set_epw(epw) == epw
        g.reset(positions=REF_SPAWNS, pos_per_env=torch.from_numpy(pos))
        games.append(g)
    rng = np.random.default_rng(2)
    for s in range(90):
        act = torch.from_numpy(rng.random((E, 8, 4)).astype(np.float32)).cuda()
        acts = [act.clone() for _ in games]
        outs = [{k: v.cpu().numpy().copy() for k, v in g.step(a).items()} for g, a in zip(games, acts)]
        for o in outs[1:]:
            for k in outs[0]:
                assert np.array_equal(outs[0][k], o[k], equal_nan=True), (s, k)
        for a in acts[1:]:
            assert torch.equal(acts[0], a), (s, "actions written back")
    sts = [g.env_state() for g in games]
    for st in sts[1:]:
        for k in sts[0]:
            assert np.array_equal(sts[0][k], st[k], equal_nan=True), k
    for f in range(_abi.F_TL):  # per-agent fields (target-list contents: via counts)
        a = games[0].get(f).cpu().numpy()
        for g in games[1:]:
            assert np.array_equal(a, g.get(f).cpu().numpy(), equal_nan=True), f
    for g in games:
        g.close()


@pytest.mark.parametrize("duct", [2.9, 4.5])
def test_philox_long_sensor_ranges_vs_oracle(grids, duct):
    """Ducting far above the reference's 1+Beta(1,3) < 2 (set through the state
    API) stretches EW ranges past the 40-cell LOS-table / bearing-table window:
    the batched LOS prefetch falls back to the ray march and the deferred
    bearings to the device atan2 for those pairs. 64 envs (one full two-wave
    workgroup), sides 20-50 cells apart, Philox mode, bit-exact against the CPU
    oracle with the same ducting."""
    import _oracle
    from lnw._abi import F_DUCT
    from lnw.batched import BatchedGame
    from lnw.config import Scenario
    grid = grids[0]
    E, S = 64, 8
    g = BatchedGame(E, ["small"] * 4, ["large"] * 4, scenario=Scenario(landing_ops=False),
                    grid=grid, seed=5)
    assert g.set_epw(64) == 64
    pos = _melee_positions(grid, E, 4, 4, seed=int(duct * 10), box_b=(20, 35, 35, 65),
                           box_r=(60, 75, 35, 65))
    g.reset(positions=pos[0], pos_per_env=torch.from_numpy(pos))
    g.set(F_DUCT, torch.full((E,), duct, dtype=torch.float64))
    oracles = []
    for e in range(E):
        o = _oracle.OracleEnv(grid, 4, 4)
        o.set_philox(5, e)
        o.reset([0] * 4 + [1] * 4, pos[e])
        o.set_ducting(duct)
        oracles.append(o)
    rng = np.random.default_rng(int(duct * 100))
    for s in range(S):
        act = rng.random((E, 8, 4)).astype(np.float32)
        out = g.step(torch.from_numpy(act).cuda())
        ob, orr = out["obs_blue"].cpu().numpy(), out["obs_red"].cpu().numpy()
        rb, rr = out["rew_blue"].cpu().numpy(), out["rew_red"].cpu().numpy()
        for e in range(E):
            r = oracles[e].step(act[e], np.full(8, _oracle.K_F32, np.int32))
            assert np.array_equal(ob[e], r["obs_blue"].astype(np.float32)), (s, e, "obs_blue")
            assert np.array_equal(orr[e], r["obs_red"].astype(np.float32)), (s, e, "obs_red")
            assert np.allclose(rb[e], r["rew_blue"], rtol=0, atol=REW_TOL), (s, e, "rew_blue")
            assert np.allclose(rr[e], r["rew_red"], rtol=0, atol=REW_TOL), (s, e, "rew_red")
    st = g.env_state()
    for e in range(E):
        assert st["err"][e] == oracles[e].env_state()["err"], e
    g.close()


@pytest.mark.parametrize("trained_red", [True, False])
@pytest.mark.parametrize("mode", ["f64_mixed_kinds", "i32_discrete"])
def test_quiet_path_dtypes_vs_oracle(grids, mode, trained_red):
    """The quiet path with float64 action rows of mixed value kinds (Python
    float / np.float32 / np.float64 rows, NEP 50) and with DISCRETE int32
    actions, trained and untrained red: 128 envs at 64 per workgroup (workgroup
    0 quiet, workgroup 1 half in contact), Philox mode, outputs and the
    written-back action rows bit-exact against the CPU oracle."""
    import _oracle
    from lnw.batched import BatchedGame
    from lnw.config import Scenario
    grid = grids[0]
    E, S = 128, 12
    discrete = mode == "i32_discrete"
    g = BatchedGame(E, ["small"] * 4, ["large"] * 4,
                    scenario=Scenario(landing_ops=False, trained_red=trained_red, discrete=discrete),
                    grid=grid, seed=31)
    assert g.set_epw(64) == 64
    pos = np.array([REF_SPAWNS] * E, np.int32)
    pos[96:] = _melee_positions(grid, 32, 4, 4, seed=6)
    g.reset(positions=pos[0], pos_per_env=torch.from_numpy(pos))
    oracles = []
    for e in range(E):
        o = _oracle.OracleEnv(grid, 4, 4, trained_red=trained_red, discrete=discrete)
        o.set_philox(31, e)
        o.reset([0] * 4 + [1] * 4, pos[e])
        oracles.append(o)
    rng = np.random.default_rng(17 + int(trained_red))
    for s in range(S):
        if discrete:
            act = np.stack([rng.integers(0, 2, (E, 8)), rng.integers(0, 2, (E, 8)),
                            rng.integers(0, 50, (E, 8)), np.zeros((E, 8), np.int64)], -1).astype(np.int32)
            # integer rows: the oracle truncates a random salvo written into
            # them, as an int ndarray does (the golden discrete fixtures' calls)
            kinds = np.full((E, 8), _oracle.K_PYINT, np.uint8)
            at = torch.from_numpy(act).cuda()
            out = g.step(at)
        else:
            act = rng.random((E, 8, 4))
            kinds = rng.choice([_oracle.K_PYFLOAT, _oracle.K_F32, _oracle.K_F64], (E, 8)).astype(np.uint8)
            f32 = kinds == _oracle.K_F32
            act[f32] = act[f32].astype(np.float32)
            at = torch.from_numpy(act).cuda()
            out = g.step(at, torch.from_numpy(kinds).cuda())
        act_after = at.cpu().numpy()
        ob, orr = out["obs_blue"].cpu().numpy(), out["obs_red"].cpu().numpy()
        rb, rr = out["rew_blue"].cpu().numpy(), out["rew_red"].cpu().numpy()
        dn = out["done"].cpu().numpy()
        for e in range(E):
            r = oracles[e].step(act[e], kinds[e].astype(np.int32))
            assert np.array_equal(act_after[e], r["actions_after"].astype(act.dtype)), (s, e, "actions")
            assert np.array_equal(ob[e], r["obs_blue"].astype(np.float32)), (s, e, "obs_blue")
            assert np.array_equal(orr[e], r["obs_red"].astype(np.float32)), (s, e, "obs_red")
            assert np.allclose(rb[e], r["rew_blue"], rtol=0, atol=REW_TOL), (s, e, "rew_blue")
            assert np.allclose(rr[e], r["rew_red"], rtol=0, atol=REW_TOL), (s, e, "rew_red")
            assert dn[e] == r["done"], (s, e, "done")
    g.close()


def test_work_counters(grids):
    """lnw_set_counters: the table path at the reference spawns marches no ray
    and runs no A*; the unpruned mode (los_mode 1, move_mode 1) marches every
    pair get_obs tests and runs an A* per live ship per step; results do not
    change with the counters bound."""
    from lnw.batched import BatchedGame
    from lnw.config import Scenario
    E = 256
    counts = {}
    for mode in (0, 1, 2):
        sc = Scenario(landing_ops=False, auto_reset=True, los_mode=mode, move_mode=mode % 2)
        g = BatchedGame(E, ["small"] * 4, ["large"] * 4, scenario=sc, grid=grids[0], seed=3)
        g.reset(positions=REF_SPAWNS)
        rng = np.random.default_rng(1)
        acts = [torch.from_numpy(rng.random((E, 8, 4)).astype(np.float32)).cuda() for _ in range(6)]
        ref = [{k: v.clone() for k, v in g.step(a.clone()).items()} for a in acts[:3]]
        g.set_rng(3)  # the same draws again (the reset draws the ducting)
        g.reset(positions=REF_SPAWNS)
        g.count_work(True)
        for a, r in zip(acts[:3], ref):
            out = g.step(a.clone())
            for k in r:
                assert torch.equal(out[k], r[k]) or torch.allclose(out[k], r[k], equal_nan=True), k
        torch.cuda.synchronize()
        counts[mode] = g.work_counts()
        g.count_work(False)
        g.close()
    assert counts[0] == dict(rays_marched=0, cells_marched=0, astar_searches=0,
                             pooled_bearings=0), counts[0]
    c = counts[1]
    # at most one A* per live ship per step (8 ships x 3 steps x E); at these
    # spawns the march mode's range pruning leaves no pair to march
    assert 0 < c["astar_searches"] <= 8 * 3 * E, c
    assert c["rays_marched"] == c["cells_marched"] == 0, c
    # los_mode 2 (the reference's LOS work): 8 get_obs x 4 x 4 pairs per env-step,
    # every ray in full; the reference measured 85.9 cells per ray at these spawns
    # 
    c = counts[2]
    assert c["rays_marched"] == 128 * 3 * E and c["astar_searches"] == 0, c
    assert 70 < c["cells_marched"] / c["rays_marched"] < 100, c


def test_result_altering_debug_bits_refused(grids, monkeypatch):
    """The shipped library refuses LNW_DEBUG_SKIP bits that change results
    (section skips, replaced arithmetic): lnw_create fails loudly. The
    timing-only bits (9: no quiet path, 17: per-lane bearings) are accepted."""
    from lnw import _abi
    from lnw.batched import BatchedGame
    from lnw.config import Scenario
    for bits in ("1", str(1 << 16), str(1 << 21), str((1 << 9) | (1 << 20))):
        monkeypatch.setenv("LNW_DEBUG_SKIP", bits)
        with pytest.raises(_abi.LnwError, match="diagnostics build"):
            BatchedGame(64, ["small"] * 4, ["large"] * 4, scenario=Scenario(landing_ops=False),
                        grid=grids[0], seed=1)
    monkeypatch.setenv("LNW_DEBUG_SKIP", str((1 << 9) | (1 << 17)))
    g = BatchedGame(64, ["small"] * 4, ["large"] * 4, scenario=Scenario(landing_ops=False),
                    grid=grids[0], seed=1)
    g.close()


def test_prof_group_kernel_grid(grids, monkeypatch):
    """LNW_PROF with the runtime-size group kernel, whose grid (E / 32
    workgroups) is larger than the epw-64 step grid: the timestamp buffer is
    sized by the launched grid (and regrown when a later launch needs more),
    and the profiled launch gives the same results as an unprofiled one."""
    from lnw.batched import BatchedGame
    from lnw.config import Scenario
    sc = Scenario(landing_ops=True, auto_reset=True, episode_steps=40)
    E = 2048
    games = []
    for prof in (True, False):
        if prof:
            monkeypatch.setenv("LNW_PROF", "1")
        g = BatchedGame(E, ["small"] * 8, ["large"] * 8 + ["ls"] * 2, scenario=sc, grid=grids[1],
                        seed=3)
        monkeypatch.delenv("LNW_PROF", raising=False)
        assert g.set_epw(64) == 64
        g.reset(positions=[(0, 0)] * 18, rand_ls=[0] * 16 + [1, 1], box=((20, 60), (80, 140)))
        games.append(g)
    rng = np.random.default_rng(4)
    for s in range(4):
        act = torch.from_numpy(rng.random((E, 18, 4)).astype(np.float32)).cuda()
        outs = [{k: v.cpu().numpy().copy() for k, v in g.step(act.clone()).items()} for g in games]
        for k in outs[0]:
            assert np.array_equal(outs[0][k], outs[1][k], equal_nan=True), (s, k)
        if s == 1:
            assert games[0].set_epw(8) == 8 and games[1].set_epw(8) == 8  # larger step grid
    for g in games:
        g.close()
