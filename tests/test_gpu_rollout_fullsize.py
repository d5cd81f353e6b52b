"""Config 5's env side at its full size: a 32 768-env MAPPO rollout
(lnw.rollout.Rollout, the fused HIP path the bench times: lnw_observe_ex,
lnw_policy_act, lnw_step without rows, lnw_rollout_post) checked env by env
against the CPU oracle stepping the same action arrays.

The rollout records each step's float64 action array and row kinds as
lnw_policy_act wrote them (blue actor rows, the scripted red rows of
red_steps*.csv, zeros for sunk ships; Rollout.record_actions). The oracle
(orc_rollout_range, oracle/lnw_oracle.c) replays the env side of ppo.py:497-577
on them: get_obs of every live ship, blue then red (target lists and EW gauss
draws included), then Game.step. Compared per (step, env) where the rollout is
still running: the hash of the blue observation rows the policy read (bit for
bit), the blue rewards (1e-5) and the running flags (an env stops after its
first done == 0, ppo.py:640). Two consecutive 40-step rollouts cross the
horizon's in-kernel auto-reset. Needs an MI355X."""
import numpy as np
import pytest
import torch

import _oracle

pytestmark = pytest.mark.gpu

REF_SPAWNS = [(6, 61), (10, 81), (8, 70), (11, 58), (98, 48), (98, 52), (98, 56), (96, 52)]


def _melee(grid, n, seed):
    rng = np.random.default_rng(seed)
    wb = np.argwhere(grid[30:45, 40:60] <= 74) + np.array([30, 40])
    wr = np.argwhere(grid[55:70, 45:65] <= 74) + np.array([55, 45])
    return np.concatenate([wb[rng.integers(0, len(wb), (n, 4))], wr[rng.integers(0, len(wr), (n, 4))]],
                          1).astype(np.int32)


@pytest.mark.parametrize("strided", [False, True])
@pytest.mark.parametrize("layout", ["reference", "mixed"])
def test_rollout_env_side_vs_oracle(layout, strided, monkeypatch):
    from lnw import rollout as R
    from lnw.batched import BatchedGame
    from lnw.config import Scenario
    monkeypatch.setattr(R, "STRIDED_POLICY_INPUT", strided)
    grid = _oracle.load_fixture("grids.npz")["grid100"]
    E, T, seed, nb = 32768, 40, 77, 4
    pos = np.array([REF_SPAWNS] * E, np.int32)
    if layout == "mixed":  # melee spawns in every other 64-env block: contact from step 0
        blocks = np.arange(E).reshape(-1, 128)[:, 64:].reshape(-1)
        pos[blocks] = _melee(grid, len(blocks), seed=5)
    # bench.mappo_rollout's scenario, actor, critic and sampling
    sc = Scenario(landing_ops=False, tactics="aggressive", side="blue", trained_red=False,
                  auto_reset=True, episode_steps=40)
    g = BatchedGame(E, ["small"] * 4, ["large"] * 4, scenario=sc, grid=grid, seed=seed)
    g.set_variant(True)
    torch.manual_seed(0)
    actor = R.BatchedActor.for_obs(g.Db).cuda()
    critic = R.BatchedCritic(g.Db * g.nb).cuda()
    r = R.Rollout(g, actor, critic, steps=T, noise=0.05, seed=5)
    r.record_actions = True
    g.reset(positions=REF_SPAWNS, pos_per_env=torch.from_numpy(pos))
    D = g.Db
    mult = (np.random.default_rng(3).integers(0, 1 << 30, nb * D, dtype=np.int64) * 2 + 1)
    mt = torch.from_numpy(mult).cuda()
    hs, rews, runs, acts, kinds = [], [], [], [], []
    for rep in range(2):
        b = r.run()
        w = b["obs"].reshape(E, T, nb * D).view(torch.int32).to(torch.int64) & 0xFFFFFFFF
        hs.append((w * mt).sum(2).t().cpu().numpy().view(np.uint64))        # [T, E]
        rews.append(b["rewards"].transpose(0, 1).cpu().numpy())              # [T, E, nb]
        runs.append(b["running"].t().cpu().numpy())                           # [T, E]
        acts.append(b["step_actions"].transpose(0, 1).cpu().numpy())         # [T, E, A, 4]
        kinds.append(b["step_kinds"].transpose(0, 1).cpu().numpy())          # [T, E, A]
    torch.cuda.synchronize()
    assert int((g.env_state()["err"] != 0).sum()) == 0
    g.close()
    gh, gr, grun = (np.concatenate(x) for x in (hs, rews, runs))
    oh, orw, od = _oracle.rollout_env(grid, 4, 4, [0] * 4 + [1] * 4, pos, np.concatenate(acts),
                                      np.concatenate(kinds), mult, seed, 40, pos_per_env=True)
    # running flags: each rollout starts all-running; an env stops after its first done == 0
    orun = np.ones_like(grun)
    for rep in range(2):
        for t in range(1, T):
            s = rep * T + t
            orun[s] = orun[s - 1] & (od[s - 1] != 0)
    assert np.array_equal(grun, orun), np.argwhere(grun != orun)[:6].tolist()
    m = grun.astype(bool)
    bad = np.argwhere((gh != oh) & m)
    assert bad.size == 0, f"{len(bad)} running (step, env) observation hashes differ, first {bad[:6].tolist()}"
    assert np.allclose(gr[m], orw[m], rtol=0, atol=1e-5)
    assert not gr[~m].any()  # masked steps hold zeros, as the reference's buffers after its break
    if layout == "mixed":  # what the layout is for: fights ended episodes inside a rollout
        assert not m.all()
