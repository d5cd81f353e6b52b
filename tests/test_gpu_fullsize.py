"""Parity at BASELINE.json's full sizes (configs 2, 3 per GPU and 4): every env
of the batch checked against the CPU oracle, in production (Philox) mode, over
45 steps so the 40-step horizon's in-kernel auto-reset is crossed.

Holding 65 536 envs' observations for every step on the host is not needed:
per (step, env) both sides reduce the float32 observations to a 64-bit hash,
sum_k bits(obs[k]) * mult[k] mod 2^64 (mult: random odd 31-bit constants), the
device with torch int64 arithmetic (wrapping), the oracle in C
(oracle/lnw_oracle.c orc_fullsize_range). A single flipped bit anywhere in an
env's rows changes its hash. Rewards (float32, tolerance 1e-5), done and cog are
compared in full. Needs an MI355X.
"""
import numpy as np
import pytest
import torch

import _oracle

pytestmark = pytest.mark.gpu

REW_TOL = 1e-5
REF_SPAWNS = [(6, 61), (10, 81), (8, 70), (11, 58), (98, 48), (98, 52), (98, 56), (96, 52)]


def _mult(n, seed=99):
    return (np.random.default_rng(seed).integers(0, 1 << 30, n, dtype=np.int64) * 2 + 1)


def _gpu_run(g, acts, mult):
    """Step g through acts [S, E, A, 4]; per step the observation hashes, rewards,
    done and cog as host arrays."""
    S, E = acts.shape[:2]
    mt = torch.from_numpy(mult).cuda()
    hs, rews, dones, cogs = [], [], [], []
    for s in range(S):
        out = g.step(torch.from_numpy(acts[s]).cuda())
        w = torch.cat([out["obs_blue"].reshape(E, -1), out["obs_red"].reshape(E, -1)], 1)
        w = w.contiguous().view(torch.int32).to(torch.int64) & 0xFFFFFFFF
        hs.append((w * mt).sum(1).cpu().numpy().view(np.uint64))
        rews.append(torch.cat([out["rew_blue"].reshape(E, -1), out["rew_red"].reshape(E, -1)],
                              1).cpu().numpy())
        dones.append(out["done"].cpu().numpy().copy())
        cogs.append(out["cog"].cpu().numpy().copy())
    torch.cuda.synchronize()
    return np.stack(hs), np.stack(rews), np.stack(dones), np.stack(cogs)


def _compare(gpu, orc, label):
    gh, gr, gd, gc = gpu
    oh, orw, od, oc = orc
    bad = np.argwhere(gh != oh)
    assert bad.size == 0, f"{label}: {len(bad)} (step, env) observation hashes differ, first {bad[:4].tolist()}"
    assert np.array_equal(gd, od), f"{label}: done differs at {np.argwhere(gd != od)[:4].tolist()}"
    assert np.allclose(gr, orw, rtol=0, atol=REW_TOL), \
        f"{label}: rewards differ at {np.argwhere(~np.isclose(gr, orw, rtol=0, atol=REW_TOL))[:4].tolist()}"
    assert np.allclose(gc, oc, rtol=0, atol=1e-5, equal_nan=True), f"{label}: cog differs"


def _grids():
    g = _oracle.load_fixture("grids.npz")
    return g["grid100"], g["grid200"]


def _water_positions(grid, E, boxes, seed):
    """Per env, per agent a water cell drawn uniformly from that agent's box."""
    rng = np.random.default_rng(seed)
    out = np.zeros((E, len(boxes), 2), np.int32)
    for a, (x0, x1, y0, y1) in enumerate(boxes):
        cells = np.argwhere(grid[x0:x1, y0:y1] <= 74) + np.array([x0, y0])
        out[:, a] = cells[rng.integers(0, len(cells), E)]
    return out


def test_fullsize_config3_reference_spawns():
    """Config 3 per GPU: 65 536 4v4 envs at the reference spawns (the bench
    workload: quiet workgroups throughout), 45 steps, every env vs the oracle."""
    from lnw.batched import BatchedGame
    from lnw.config import Scenario
    grid = _grids()[0]
    E, S, seed = 65536, 45, 1234
    sc = Scenario(landing_ops=False, auto_reset=True, episode_steps=40)
    g = BatchedGame(E, ["small"] * 4, ["large"] * 4, scenario=sc, grid=grid, seed=seed)
    g.reset(positions=REF_SPAWNS)
    acts = np.random.default_rng(5).random((S, E, 8, 4), dtype=np.float32)
    mult = _mult(4 * 68 + 4 * 68)
    gpu = _gpu_run(g, acts, mult)
    assert int((g.env_state()["err"] != 0).sum()) == 0
    g.close()
    orc = _oracle.fullsize(grid, 4, 4, [0] * 4 + [1] * 4, np.array(REF_SPAWNS), acts, mult, seed, 40)
    _compare(gpu, orc, "config3")
    assert (gpu[2][39] == 1).all()  # horizon reached, envs reset in-kernel after step 40


@pytest.mark.parametrize("contact", [False, True])
def test_fullsize_config2_contact_spawns(contact):
    """Config 2 size (4 096 4v4 envs) with the sides 10-40 cells apart, so
    firing, hits, EW bearings and fixes happen every step (phase S workgroups),
    45 steps, every env vs the oracle."""
    from lnw.batched import BatchedGame
    from lnw.config import Scenario
    grid = _grids()[0]
    E, S, seed = 4096, 45, 77
    pos = _water_positions(grid, E, [(30, 45, 40, 60)] * 4 + [(55, 70, 45, 65)] * 4, seed=3)
    sc = Scenario(landing_ops=False, auto_reset=True, episode_steps=40)
    g = BatchedGame(E, ["small"] * 4, ["large"] * 4, scenario=sc, grid=grid, seed=seed)
    g.set_variant(contact)  # both step-kernel variants (lnw_set_variant)
    g.reset(positions=pos[0], pos_per_env=torch.from_numpy(pos))
    acts = np.random.default_rng(6).random((S, E, 8, 4), dtype=np.float32)
    mult = _mult(4 * 68 + 4 * 68, seed=7)
    gpu = _gpu_run(g, acts, mult)
    assert int((g.env_state()["err"] != 0).sum()) == 0
    g.close()
    orc = _oracle.fullsize(grid, 4, 4, [0] * 4 + [1] * 4, pos, acts, mult, seed, 40,
                           pos_per_env=True)
    _compare(gpu, orc, "config2-contact")
    assert (gpu[2] == 0).any()  # some episodes end in a victory (done == 0) and reset


def test_fullsize_config4():
    """Config 4: 8 192 envs, 8 small blue vs 8 large + 2 LandingShip red
    (landing ops, LandingShip spawns drawn by randint as game.py:587-591) on the
    200x200 grid, per-env water spawns in x in [20, 60), y in [80, 140), 42 steps,
    every env vs the oracle."""
    from lnw.batched import BatchedGame
    from lnw.config import Scenario
    grid = _grids()[1]
    E, S, seed = 8192, 42, 21
    A = 18
    pos = _water_positions(grid, E, [(20, 60, 80, 140)] * A, seed=4)
    rand_ls = [0] * 16 + [1, 1]
    sc = Scenario(landing_ops=True, auto_reset=True, episode_steps=40)
    g = BatchedGame(E, ["small"] * 8, ["large"] * 8 + ["ls"] * 2, scenario=sc, grid=grid, seed=seed)
    g.reset(positions=pos[0], rand_ls=rand_ls, pos_per_env=torch.from_numpy(pos))
    acts = np.random.default_rng(8).random((S, E, A, 4), dtype=np.float32)
    mult = _mult(8 * 84 + 10 * 92, seed=9)
    gpu = _gpu_run(g, acts, mult)
    assert int((g.env_state()["err"] != 0).sum()) == 0
    g.close()
    orc = _oracle.fullsize(grid, 8, 10, [0] * 8 + [1] * 8 + [2] * 2, pos, acts, mult, seed, 40,
                           pos_per_env=True, rand_ls=rand_ls, landing_ops=True)
    _compare(gpu, orc, "config4")
