"""Pin the CPU oracle (oracle/lnw_oracle.c) against golden vectors captured from
the reference itself (tests/golden/make_golden.py). CPU-only.

Bar: bit-exact for LOS bits, A* lengths/kinds, move targets/validity, ranges,
positions, target lists, RNG consumption and f32-cast observations; rewards and
cog within 1e-9 (they come out bit-exact in practice).
"""
import glob
import os

import numpy as np
import pytest

from _oracle import (GOLDEN, K_F32, K_F64, OracleEnv, astar_batch, episode_meta,
                     fixture_kinds, load_fixture, los_batch, move_batch)
import _oracle

EPISODES = sorted(os.path.basename(p) for p in glob.glob(os.path.join(GOLDEN, "ep_*.npz")))


@pytest.fixture(scope="module")
def grids():
    g = load_fixture("grids.npz")
    return [g["grid100"], g["grid200"]]


def test_grid_fixture(grids):
    g100, g200 = grids
    assert g100.shape == (100, 100) and g100.dtype == np.uint8
    assert g200.shape == (200, 200)
    # 3838 cells > 74 and 3987 cells > 70 at G=100
    assert int((g100 > 74).sum()) == 3838
    assert int((g100 > 70).sum()) == 3987


def test_los_golden(grids):
    fx = load_fixture("los.npz")
    for gi in (0, 1):
        m = fx["grid_id"] == gi
        pairs = fx["pairs"][m]
        r = los_batch(grids[gi], pairs, 74)
        e = los_batch(grids[gi], pairs, 70)
        assert np.array_equal(r, fx["radar"][m]), f"radar LOS mismatch grid {gi}"
        assert np.array_equal(e, fx["ew"][m]), f"ew LOS mismatch grid {gi}"
    # point count of the Bresenham line
    lib = _oracle.lib()
    P = fx["pairs"][:5000]
    n = [lib.orc_bresenham_count(int(a), int(b), int(c), int(d)) for a, b, c, d in P]
    assert np.array_equal(np.array(n), fx["npts"][:5000])


def test_astar_golden(grids):
    fx = load_fixture("astar.npz")
    for gi in (0, 1):
        m = fx["grid_id"] == gi
        plen, kind, feas = astar_batch(grids[gi], fx["cls"][m], fx["start"][m], fx["target"][m])
        assert np.array_equal(plen, fx["plen"][m])
        assert np.array_equal(kind, fx["kind"][m])
        assert np.array_equal(feas, fx["feasible"][m])


def test_moves_golden(grids):
    fx = load_fixture("moves.npz")
    rounded, ok = move_batch(grids[0], fx["cls"], fx["is_f32"], fx["pos"], fx["act"])
    assert np.array_equal(rounded, fx["rounded"])
    assert np.array_equal(ok, fx["ok"])
    res = fx["result"]
    m = fx["ok"] == 1
    assert np.array_equal(rounded[m], res[m])


def test_discrete_moves_golden(grids):
    fx = load_fixture("moves.npz")
    D = fx["disc"]
    g = grids[0]
    lib = _oracle.lib()
    for px, py, v, ok, rx, ry in D[:20000]:
        x, y = v // 7, v % 7
        tx, ty = px - 3 + x, py - 3 + y
        inb = 0 <= tx < 100 and 0 <= ty < 100
        got = inb and lib.orc_check_path(_oracle._p(g), 100, 74, 0, int(px), int(py), int(tx),
                                         int(ty))
        assert bool(got) == bool(ok)
        if ok:
            assert (tx, ty) == (rx, ry)


def test_ranges_golden():
    fx = load_fixture("ranges.npz")
    lib = _oracle.lib()
    for k, d in enumerate(fx["ducting"]):
        for i in range(4):
            for j in range(4):
                assert lib.orc_radar_range(float(d), i, j) == fx["ranges"][k, i, j, 0]
                assert lib.orc_ew_range(float(d), i, j) == fx["ranges"][k, i, j, 1]


def replay_oracle(fx, grids):
    """Replay a golden episode fixture through the oracle; yield (step, fixture
    index, oracle outputs, oracle env) per step."""
    meta = episode_meta(fx)
    F = meta["flags"]
    grid = grids[meta["grid_id"]]
    for em in meta["episodes"]:
        nb, nr = em["nb"], em["nr"]
        env = OracleEnv(grid, nb, nr, discrete=F["DISCRETE"], landing_ops=F["LANDING_OPS"],
                        aggressive=F["TACTICS"] == "aggressive", side_blue=F["SIDE"] == "blue",
                        trained_red=F["TRAINED_RED"], red_aggression=F["RED_AGGRESSION"])
        tape = fx["tape"][em["tape_start"]:em["tape_end"]]
        env.set_tape(tape)
        types = np.array(em["types"], np.int32)
        spawn = np.array(em["spawn"], np.int32)
        rand_ls = np.zeros(nb + nr, np.int32)
        if F["N_RED_LANDINGSHIP"] > 0:
            rand_ls[nb + nr - F["N_RED_LANDINGSHIP"]:] = 1
        env.reset(types, spawn, rand_ls)
        yield ("reset", em, env)
        for s in range(em["n_steps"]):
            i = em["first_step"] + s
            pre = None
            if meta["observe"]:
                pre = {}
                st = env.agents()
                for a in range(nb + nr):
                    if st["alive"][a]:
                        pre[a] = env.observe(a)
            kinds = fixture_kinds(fx, meta, i)
            out = env.step(fx["actions"][i], kinds)
            yield ("step", (s, i, out, pre), env)


@pytest.mark.parametrize("name", EPISODES)
def test_episode_golden(name, grids):
    fx = load_fixture(name)
    meta = episode_meta(fx)
    n_checked = 0
    for kind, payload, env in replay_oracle(fx, grids):
        if kind == "reset":
            em = payload
            st = env.agents()
            assert np.array_equal(st["pos"], np.array(em["spawn"])), "spawn"
            assert env.env_state()["ducting"] == em["ducting"], "ducting"
            continue
        s, i, out, pre = payload
        ctx = f"{name} step {i}"
        es = env.env_state()
        assert es["err"] == 0, ctx
        if pre is not None:
            tape_pos_pre = fx["pre_tape_pos"][i]
            for a, o in pre.items():
                assert fx["pre_obs_valid"][i, a] == 1, ctx
                ref = fx["pre_obs"][i, a, :len(o)]
                assert np.array_equal(o.astype(np.float32), ref), f"{ctx} pre-obs agent {a}"
        assert np.array_equal(out["obs_blue"].astype(np.float32), fx["obs_blue"][i]), f"{ctx} obs_blue"
        assert np.array_equal(out["obs_red"].astype(np.float32), fx["obs_red"][i]), f"{ctx} obs_red"
        np.testing.assert_allclose(out["rew_blue"], fx["rew_blue"][i], rtol=0, atol=1e-9, err_msg=ctx)
        np.testing.assert_allclose(out["rew_red"], fx["rew_red"][i], rtol=0, atol=1e-9, err_msg=ctx)
        assert out["done"] == fx["done"][i], ctx
        c = fx["cog"][i]
        if np.isnan(c):
            assert np.isnan(out["cog"]), ctx
        else:
            assert abs(out["cog"] - c) <= 1e-9, ctx
        assert np.array_equal(out["actions_after"], fx["actions_after"][i]), f"{ctx} mutated actions"
        st = env.agents()
        assert np.array_equal(st["pos"], fx["pos"][i]), f"{ctx} pos"
        assert np.array_equal(st["radar"], fx["radar"][i]), f"{ctx} radar"
        assert np.array_equal(st["missiles"], fx["missiles"][i]), f"{ctx} missiles"
        assert np.array_equal(st["alive"], fx["alive"][i]), f"{ctx} alive"
        assert np.array_equal(st["steps_done"], fx["steps_done"][i]), f"{ctx} steps_done"
        assert np.array_equal(st["dist_lz"], fx["dist_lz"][i]), f"{ctx} dist_lz"
        assert np.array_equal(st["tl_cnt"], fx["tl_cnt"][i]), f"{ctx} tl_cnt"
        assert [es["n_blue_left"], es["n_red_left"]] == list(fx["n_left"][i]), ctx
        assert [es["blue_victory"], es["red_victory"]] == list(fx["victories"][i]), ctx
        assert es["tape_pos"] == fx["tape_pos"][i], f"{ctx} rng draws"
        n_checked += 1
    # target-list contents (ragged), checked on the final state of each step
    assert n_checked == len(fx["done"])


@pytest.mark.parametrize("name", EPISODES)
def test_episode_tlists_golden(name, grids):
    fx = load_fixture(name)
    cnt, xy = fx["tl_cnt"], fx["tl_xy"]
    offs = np.concatenate([[0], np.cumsum(cnt.reshape(-1))])
    for kind, payload, env in replay_oracle(fx, grids):
        if kind != "step":
            continue
        s, i, out, pre = payload
        A = cnt.shape[1]
        for a in range(A):
            k = i * A + a
            ref = [tuple(v) for v in xy[offs[k]:offs[k + 1]]]
            assert env.tlist(a) == ref, f"{name} step {i} agent {a}"


@pytest.mark.parametrize("name", ["3v3_scripted", "4v2ls_trained", "4v4_trained_contact",
                                  "4v4_melee_done", "2v2_trained_breaks"])
def test_rollout_fixture_env_trajectory(name, grids):
    """The env side of the recorded reference rollouts (PPO.rollout,
    make_rollout_golden.py) through the oracle: each step observes every live
    ship (blue then red, ppo.py:497-575), then steps the recorded action array
    in its np.asarray kind (ppo.py:577). Observations the actor saw, rewards
    and the tape consumption must match."""
    import json
    fx = load_fixture(f"rollout_{name}.npz")
    meta = json.loads(str(fx["meta"]))
    nb, A = meta["nb"], meta["A"]
    for e, em in enumerate(meta["episodes"]):
        env = OracleEnv(grids[0], nb, A - nb, landing_ops=meta["landing_ops"],
                        trained_red=meta["trained_red"])
        tape = fx["tape"][em["tape_start"]:em["tape_end"]]
        env.set_tape(tape)
        rand_ls = [0] * (A - meta["n_ls"]) + [1] * meta["n_ls"]
        env.reset(np.array(em["types"], np.int32), np.array(em["spawn"], np.int32),
                  np.array(rand_ls, np.int32))
        assert env.env_state()["ducting"] == em["ducting"]
        for t in range(meta["n_steps"][e]):
            st = env.agents()
            for a in range(A):
                if st["alive"][a]:
                    o = env.observe(a)
                    if a < nb:
                        assert np.array_equal(o.astype(np.float32), fx["batch_obs"][e, t, a]), (e, t, a)
                elif a < nb:
                    assert not fx["batch_obs"][e, t, a].any()
            kind = K_F32 if fx["act_f32"][e, t] else K_F64
            out = env.step(fx["act"][e, t], np.full(A, kind, np.int32))
            np.testing.assert_allclose(out["rew_blue"], fx["rew"][e, t], rtol=0, atol=1e-12)
            assert out["done"] == fx["done"][e, t]
        assert env.env_state()["tape_pos"] == len(tape)
