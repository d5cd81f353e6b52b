"""Config 5 pinned to the reference's own MAPPO rollout:
lnw.rollout.Rollout on the device against fixtures recorded from
`PPO.rollout` (ppo.py:421-671) by tests/golden/make_rollout_golden.py.

Each recorded rollout episode is one device env, replayed in tape mode (every
random / gauss / randint / beta draw of the reference), with the reference's
actor / critic / red-actor weights and its sampled actor outputs replayed
(`forced_actions`; torch's sampler draws are not the env's). Both rollout
implementations: the fused HIP kernels (lnw_policy_act / lnw_rollout_post) and
the torch ops. Checked per env
and step: the observations the actor saw (bit-exact float32), the action
array's value kind after np.asarray (ppo.py:577), rewards (float64, 1e-5),
log-probabilities and critic values (float32 network arithmetic on another
device: 1e-4 / 1e-5), reward-to-go (ppo.py:645-659) and the learner's GAE
(ppo.py:695-714 on the flattened batch, evaluated on the device) within 1e-5
relative, and the RNG tape consumed draw for draw up to the step that ends the
episode. `4v4_melee_done` has episodes that end before step 40 (done == 0 and
the reference's `break`, ppo.py:640-641): the masking after it is checked
against what the reference leaves in its buffers."""
import json
import os

import numpy as np
import pytest
import torch

from _oracle import GOLDEN, load_fixture

pytestmark = pytest.mark.gpu

NAMES = {0: "small", 1: "large", 2: "ls"}


@pytest.mark.parametrize("impl", ["hip", "torch"])
@pytest.mark.parametrize("name", ["3v3_scripted", "4v2ls_trained", "4v4_trained_contact",
                                  "4v4_melee_done", "2v2_trained_breaks"])
def test_rollout_matches_reference(name, impl):
    _rollout_case(name, impl)


@pytest.mark.parametrize("strided", [True, False])
@pytest.mark.parametrize("name", ["4v4_trained_contact", "4v4_melee_done"])
def test_rollout_contact_variant_matches_reference(name, strided, monkeypatch):
    """The contact variant's kernels on the same recorded rollouts, without a
    per-step callback: the rollout's fast path (steps without rows, whose phase S
    splits by side, and the two-wave observe), tape mode, with the policy reading
    its rows where lnw_observe_ex left them in the rollout buffer (strided) or
    from the game's packed buffer. The draw counters are checked through every
    value the draws feed (a finished env's later draws belong to no reference
    episode, so the final counter is not compared)."""
    from lnw import rollout
    monkeypatch.setattr(rollout, "STRIDED_POLICY_INPUT", strided)
    _rollout_case(name, "hip", contact=True)


def _rollout_case(name, impl, contact=False):
    from lnw.batched import BatchedGame
    from lnw.config import Scenario
    from lnw.rollout import BatchedActor, BatchedCritic, Rollout, gae
    fx = load_fixture(f"rollout_{name}.npz")
    meta = json.loads(str(fx["meta"]))
    eps, R, T, nb = meta["episodes"], meta["R"], meta["T"], meta["nb"]
    types = eps[0]["types"]
    A = len(types)
    grid = load_fixture("grids.npz")["grid100"]
    sc = Scenario(landing_ops=meta["landing_ops"], trained_red=meta["trained_red"],
                  tactics="aggressive", side="blue", auto_reset=False)
    g = BatchedGame(R, [NAMES[t] for t in types[:nb]], [NAMES[t] for t in types[nb:]],
                    scenario=sc, grid=grid, reward_dtype=torch.float64)
    if contact:
        g.set_variant(True)
    tapes = [fx["tape"][e["tape_start"]:e["tape_end"]] for e in eps]
    offs = np.concatenate([[0], np.cumsum([len(t) for t in tapes])]).astype(np.int64)
    g.set_tape(np.concatenate(tapes), offs)
    rand_ls = [0] * (A - meta["n_ls"]) + [1] * meta["n_ls"]
    pos = np.array([e["spawn"] for e in eps], np.int32)
    g.reset(positions=pos[0], rand_ls=rand_ls, pos_per_env=torch.from_numpy(pos))
    st = g.agents()
    assert np.array_equal(np.stack([st["x"], st["y"]], 2), pos), "spawn cells (LS drawn)"
    assert np.array_equal(g.env_state()["ducting"], [e["ducting"] for e in eps]), "ducting"

    def weights(pre):
        return {k[len(pre):]: fx[k] for k in fx if k.startswith(pre)}

    actor = BatchedActor.for_obs(g.Db).load_reference(weights("actor.")).cuda()
    critic = BatchedCritic(g.Db * nb).load_reference(weights("critic.")).cuda()
    red_actor = None
    if meta["trained_red"]:
        red_actor = BatchedActor.for_obs(g.Dr).load_reference(weights("red_actor.")).cuda()
    r = Rollout(g, actor, critic, steps=T, red="actor" if red_actor is not None else "script",
                red_actor=red_actor, gamma=meta["gamma"], impl=impl)
    rng_after = []  # every env's draw counter after each step (the tape position)
    out = r.run(forced_actions=torch.from_numpy(fx["act"]).cuda(),
                on_step=None if contact else (lambda t, o: rng_after.append(g.env_state()["rng"].copy())))
    torch.cuda.synchronize()
    run = out["running"].cpu().numpy()
    n_steps = np.array(meta["n_steps"])
    assert np.array_equal(run.sum(1), n_steps)
    if name == "4v4_melee_done":  # episodes that end early: the `break` at ppo.py:640-641
        assert (n_steps < T).sum() >= 3, n_steps
    if name == "2v2_trained_breaks":  # breaks mid-rollout after float32 steps
        assert ((n_steps >= 5) & (n_steps <= 35)).sum() >= 3, n_steps
        assert fx["act_f32"].sum() >= 40
    # after an episode's `break` the device buffers hold zeros, like the reference's
    np.testing.assert_array_equal(out["obs"].cpu().numpy(), fx["batch_obs"])
    np.testing.assert_array_equal(out["f32_step"].cpu().numpy() & run, fx["act_f32"].astype(bool))
    np.testing.assert_allclose(out["rewards"].cpu().numpy(), fx["rew"], rtol=0, atol=1e-5)
    np.testing.assert_allclose(out["log_probs"].cpu().numpy(), fx["batch_log_probs"], rtol=0,
                               atol=1e-4)
    vals = out["values"].cpu().numpy()
    np.testing.assert_allclose(vals[:, :, None, None].repeat(nb, 2), fx["batch_values"], rtol=0,
                               atol=1e-5)
    rtg = out["rtg"].cpu().numpy()
    np.testing.assert_allclose(rtg, fx["batch_rtg"][..., 0], rtol=1e-5, atol=1e-5)
    # the learner's advantage (ppo.py:336) on the flattened batch, computed on
    # the device: values from the device critic (zero after the break, as the
    # reference's buffer), reward-to-go from the device buffer (float32, as
    # ppo.py:665 converts it)
    flat_v = out["values"][:, :, None].expand(R, T, nb).reshape(1, -1)
    assert flat_v.is_cuda and out["rtg"].is_cuda
    adv = gae(out["rtg"].float().reshape(1, -1), flat_v, meta["gamma"])
    assert adv.is_cuda
    np.testing.assert_allclose(adv.cpu().numpy().reshape(-1), fx["learner_gae"].reshape(-1),
                               rtol=1e-5, atol=1e-5)
    # every env consumed exactly its episode's draws by the step that ended it
    # (draws a finished env makes afterwards belong to no reference episode)
    if not contact:
        used = np.array([rng_after[n - 1][e] for e, n in enumerate(n_steps)])
        assert np.array_equal(used, [len(t) for t in tapes]), (used, [len(t) for t in tapes])
    g.close()
