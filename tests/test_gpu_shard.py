"""The metric's real per-GPU path at N = 8 and config 2: 8 192 and 4 096 4v4 envs
on one GPU take the small-workgroup quiet direct mode (16 envs per workgroup,
quiet_step_t in csrc/lnw_quiet.inc, DESIGN.md "Direct mode for small
workgroups"); 16 384 envs (config 3's shard at N = 4) take it with 32 envs per
workgroup, the rows written in two slabs of 16 envs. Checked directly against the CPU oracle (orc_fullsize_range,
oracle/lnw_oracle.c) with the default envs-per-workgroup choice:

* "reference": every env at the reference spawns (game.py:560-585), the
  bench's workload: every workgroup quiet every step;
* "mixed": a melee block (sides 10-40 cells apart: fire, hits, EW fixes,
  victories) in every other 16-env workgroup, so quiet direct-mode workgroups
  and phase-S workgroups run side by side in one launch.

45 Philox steps cross the 40-step horizon's in-kernel auto-reset (and, in the
melee blocks, victory resets on the per-env cells), with a trained and an
untrained (scripted-salvo) red. Every env is compared bit for bit:
observation hashes, done and the action rows as the step left them (the
untrained red's salvo write-back, game.py:375-379); rewards and cog within
1e-5. Needs an MI355X."""
import numpy as np
import pytest
import torch

import _oracle

pytestmark = pytest.mark.gpu

REW_TOL = 1e-5
REF_SPAWNS = [(6, 61), (10, 81), (8, 70), (11, 58), (98, 48), (98, 52), (98, 56), (96, 52)]


def _mult(n, seed=99):
    return (np.random.default_rng(seed).integers(0, 1 << 30, n, dtype=np.int64) * 2 + 1)


def _melee(grid, n, seed):
    rng = np.random.default_rng(seed)
    wb = np.argwhere(grid[30:45, 40:60] <= 74) + np.array([30, 40])
    wr = np.argwhere(grid[55:70, 45:65] <= 74) + np.array([55, 45])
    return np.concatenate([wb[rng.integers(0, len(wb), (n, 4))], wr[rng.integers(0, len(wr), (n, 4))]],
                          1).astype(np.int32)


@pytest.mark.parametrize("trained_red", [True, False])
@pytest.mark.parametrize("layout", ["reference", "mixed"])
@pytest.mark.parametrize("E", [8192, 4096, 16384])
def test_shard_quiet_direct_vs_oracle(E, layout, trained_red):
    from lnw import _abi
    from lnw.batched import BatchedGame
    from lnw.config import Scenario
    grid = _oracle.load_fixture("grids.npz")["grid100"]
    S, seed = 45, 900 + E // 1024 + 2 * trained_red
    pos = np.array([REF_SPAWNS] * E, np.int32)
    if layout == "mixed":
        blocks = np.arange(E).reshape(-1, 32)[:, 16:].reshape(-1)   # every other 16-env workgroup
        pos[blocks] = _melee(grid, len(blocks), seed=E)
    sc = Scenario(landing_ops=False, auto_reset=True, episode_steps=40, trained_red=trained_red)
    g = BatchedGame(E, ["small"] * 4, ["large"] * 4, scenario=sc, grid=grid, seed=seed)
    # the default choice: 16 envs per workgroup at 8 192 / 4 096 (one slab), 32 at
    # 16 384 (config 3 at N = 4: wave 1 writes the rows in two slabs of 16 envs)
    assert g.epw == (32 if E == 16384 else 16)
    g.reset(positions=REF_SPAWNS, pos_per_env=torch.from_numpy(pos))
    acts = np.random.default_rng(31 + trained_red).random((S, E, 8, 4), dtype=np.float32)
    mult = _mult(2 * 4 * 68, seed=13)
    mt = torch.from_numpy(mult).cuda()
    hs, rews, dones, cogs, after = [], [], [], [], []
    for s in range(S):
        a = torch.from_numpy(acts[s]).cuda()
        out = g.step(a)
        assert g.step_kernel() == _abi.KERNEL_TEAM
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
                                           pos_per_env=True, trained_red=trained_red, acts_after=True)
    gh, gr, gd, gc, ga = map(np.stack, (hs, rews, dones, cogs, after))
    bad = np.argwhere(gh != oh)
    assert bad.size == 0, f"{len(bad)} (step, env) observation hashes differ, first {bad[:6].tolist()}"
    assert np.array_equal(gd, od), np.argwhere(gd != od)[:6].tolist()
    assert np.array_equal(ga, oa), np.argwhere((ga != oa).any(-1))[:6].tolist()
    assert np.allclose(gr, orw, rtol=0, atol=REW_TOL)
    assert np.allclose(gc, oc, rtol=0, atol=1e-5, equal_nan=True)
    assert (gd[39] == 1).all() if layout == "reference" else (gd == 0).any()
    if not trained_red:  # the scripted salvos were written back
        assert not np.array_equal(ga[:, :, 4:], acts[:, :, 4:])
