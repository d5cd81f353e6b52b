"""The headline units kernel (step_kernel<4, 4, false, false, 4>: four 64-env
units per 512-thread workgroup, DESIGN.md "Units kernel") checked directly
against the CPU oracle, with quiet and loud units mixed inside every workgroup.

The units kernel runs only for 4v4, 64 envs per workgroup, the default variant
and E a multiple of 256 (lnw_kernels.hip lnw_step). Here E = 512 is two
workgroups; each holds units at the reference spawns (quiet: phase Q and the
shared observation-pass queue), units at melee spawns (loud: phase S inside the
same workgroup) and a unit with both kinds of env (loud as a whole). 45 Philox
steps cross the 40-step horizon's in-kernel auto-reset, and melee episodes end
in victories (done == 0) and respawn on their own cells. Every env is compared
with orc_fullsize_range (oracle/lnw_oracle.c) bit for bit: observation hashes,
done, the action rows as the step left them (an untrained red's salvo
write-back, game.py:375-379); rewards and cog within 1e-5. Needs an MI355X.
"""
import numpy as np
import pytest
import torch

import _oracle

pytestmark = pytest.mark.gpu

REW_TOL = 1e-5
REF_SPAWNS = [(6, 61), (10, 81), (8, 70), (11, 58), (98, 48), (98, 52), (98, 56), (96, 52)]
# unit kinds per workgroup (E = 512: two workgroups of four 64-env units)
LAYOUT = [["ref", "melee", "ref", "mixed"], ["melee", "ref", "mixed", "ref"]]


def _mult(n, seed=99):
    return (np.random.default_rng(seed).integers(0, 1 << 30, n, dtype=np.int64) * 2 + 1)


def _melee(grid, n, seed):
    rng = np.random.default_rng(seed)
    wb = np.argwhere(grid[30:45, 40:60] <= 74) + np.array([30, 40])
    wr = np.argwhere(grid[55:70, 45:65] <= 74) + np.array([55, 45])
    return np.concatenate([wb[rng.integers(0, len(wb), (n, 4))], wr[rng.integers(0, len(wr), (n, 4))]],
                          1).astype(np.int32)


def _positions(grid):
    pos = np.array([REF_SPAWNS] * 512, np.int32)
    for w, kinds in enumerate(LAYOUT):
        for u, kind in enumerate(kinds):
            e0 = 256 * w + 64 * u
            if kind == "melee":
                pos[e0:e0 + 64] = _melee(grid, 64, seed=e0)
            elif kind == "mixed":
                pos[e0 + 32:e0 + 64] = _melee(grid, 32, seed=e0)
    return pos


@pytest.mark.parametrize("trained_red", [True, False])
def test_units_kernel_vs_oracle(trained_red):
    from lnw import _abi
    from lnw.batched import BatchedGame
    from lnw.config import Scenario
    grid = _oracle.load_fixture("grids.npz")["grid100"]
    E, S, seed = 512, 45, 4242
    pos = _positions(grid)
    sc = Scenario(landing_ops=False, auto_reset=True, episode_steps=40, trained_red=trained_red)
    g = BatchedGame(E, ["small"] * 4, ["large"] * 4, scenario=sc, grid=grid, seed=seed)
    assert g.set_epw(64) == 64
    g.reset(positions=REF_SPAWNS, pos_per_env=torch.from_numpy(pos))
    acts = np.random.default_rng(12 + trained_red).random((S, E, 8, 4), dtype=np.float32)
    mult = _mult(2 * 4 * 68, seed=5)
    mt = torch.from_numpy(mult).cuda()
    hs, rews, dones, cogs, after = [], [], [], [], []
    for s in range(S):
        a = torch.from_numpy(acts[s]).cuda()
        out = g.step(a)
        assert g.step_kernel() == _abi.KERNEL_UNITS, "the units kernel must be the one under test"
        w = torch.cat([out["obs_blue"].reshape(E, -1), out["obs_red"].reshape(E, -1)], 1)
        w = w.contiguous().view(torch.int32).to(torch.int64) & 0xFFFFFFFF
        hs.append((w * mt).sum(1).cpu().numpy().view(np.uint64))
        rews.append(torch.cat([out["rew_blue"], out["rew_red"]], 1).cpu().numpy())
        dones.append(out["done"].cpu().numpy().copy())
        cogs.append(out["cog"].cpu().numpy().copy())
        after.append(a.cpu().numpy())
    torch.cuda.synchronize()
    assert int((g.env_state()["err"] != 0).sum()) == 0
    g.close()
    oh, orw, od, oc, oa = _oracle.fullsize(grid, 4, 4, [0] * 4 + [1] * 4, pos, acts, mult, seed, 40,
                                           pos_per_env=True, trained_red=trained_red,
                                           acts_after=True)
    gh, gr, gd, gc, ga = map(np.stack, (hs, rews, dones, cogs, after))
    bad = np.argwhere(gh != oh)
    assert bad.size == 0, f"{len(bad)} (step, env) observation hashes differ, first {bad[:6].tolist()}"
    assert np.array_equal(gd, od), np.argwhere(gd != od)[:6].tolist()
    assert np.array_equal(ga, oa), np.argwhere((ga != oa).any(-1))[:6].tolist()
    assert np.allclose(gr, orw, rtol=0, atol=REW_TOL)
    assert np.allclose(gc, oc, rtol=0, atol=1e-5, equal_nan=True)
    # what the layout is for: loud units fought (victories) and quiet ones ran
    # to the horizon, in both workgroups
    for w in range(2):
        for u, kind in enumerate(LAYOUT[w]):
            blk = gd[:, 256 * w + 64 * u:256 * w + 64 * (u + 1)]
            if kind == "ref":
                assert (blk == 1).all(), (w, u)
            elif kind == "melee":
                assert (blk == 0).any(), (w, u)
    if not trained_red:  # the scripted salvos were written back in both kinds of unit
        assert not np.array_equal(ga[:, :, 4:], acts[:, :, 4:])
