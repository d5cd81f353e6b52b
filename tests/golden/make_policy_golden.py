#!/usr/bin/env python3
"""Golden vectors for the batched actor / critic / GAE of lnw.rollout.

Imports the reference's network.py and ppo.py through the stub harness of
make_golden.py (this container only) and records, for seeded
random weights and inputs:
  * MLP (network.py:38-152): per-sample train-mode calls as the PPO rollout
    makes them (ppo.py:504-512, one state at a time, BatchNorm in training mode):
    head outputs (normal mean / std, via forward hooks), get_dist log_prob and
    entropy for given actions; and the same in eval mode (running statistics);
  * Value (network.py:154-172) on batched global states (ppo.py:599-600);
  * PPO.gae (ppo.py:695-714) on 1-D reward / value sequences.
Writes tests/golden/policy.npz (weights as arrays keyed by state_dict name).

usage: python tests/golden/make_policy_golden.py
"""
import copy
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import make_golden  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "policy.npz")


def random_obs(rng, n, D):
    """Observation rows shaped like Combatant.get_obs (combatant.py:163-233):
    49 window values grid/255, then own / teammate x, y in [0,1), radar 0/1,
    missile fractions, target count, LS flag, ducting/2."""
    o = np.zeros((n, D), np.float32)
    o[:, :49] = rng.integers(0, 256, (n, 49)) / 255.0
    k = 49
    while k + 4 <= D - 3:
        o[:, k:k + 2] = rng.random((n, 2))
        o[:, k + 2] = rng.integers(0, 2, n)
        o[:, k + 3] = rng.integers(0, 5, n) / 4.0
        k += 4
    o[:, D - 3] = rng.integers(0, 6, n)
    o[:, D - 2] = 0.0
    o[:, D - 1] = (1.0 + rng.random(n)) / 2.0
    return o


def main():
    make_golden.import_reference()
    import torch
    import network
    import ppo
    torch.manual_seed(0)
    rng = np.random.default_rng(0)
    D, nb, n = 68, 4, 48
    actor = network.MLP(D - 49 + 12, 4)
    sd = {k: v.detach().cpu().numpy().copy() for k, v in actor.state_dict().items()}
    obs = random_obs(rng, n, D)
    acts = rng.random((n, 4)).astype(np.float32)
    cap = {}
    actor.normal_head.register_forward_hook(lambda m, i, o: cap.__setitem__("mean", torch.tanh(o)))
    actor.log_std_head.register_forward_hook(lambda m, i, o: cap.__setitem__("std", torch.exp(o)))

    def per_sample(model):
        mean, std, lp, ent = [], [], [], []
        for i in range(n):
            l, e = model.get_dist(torch.tensor(obs[i]), torch.tensor(acts[i]))
            mean.append(cap["mean"].detach().numpy().reshape(-1))
            std.append(cap["std"].detach().numpy().reshape(-1))
            lp.append(l.detach().numpy().reshape(-1))
            ent.append(e.detach().numpy().reshape(-1))
        return [np.stack(a).astype(np.float32) for a in (mean, std, lp, ent)]

    ev = copy.deepcopy(actor)
    ev.normal_head.register_forward_hook(lambda m, i, o: cap.__setitem__("mean", torch.tanh(o)))
    ev.log_std_head.register_forward_hook(lambda m, i, o: cap.__setitem__("std", torch.exp(o)))
    ev.eval()
    with torch.no_grad():
        ev_mean, ev_std, ev_lp, ev_ent = per_sample(ev)
    actor.train()
    tr_mean, tr_std, tr_lp, tr_ent = per_sample(actor)

    critic = network.Value(D * nb)
    csd = {k: v.detach().cpu().numpy().copy() for k, v in critic.state_dict().items()}
    cop = random_obs(rng, 8 * nb, D).reshape(8, nb * D)
    with torch.no_grad():
        val = critic(torch.tensor(cop)).numpy()

    T = 40
    rew = rng.normal(0, 5, (6, T)).astype(np.float32)
    vals = rng.normal(0, 5, (6, T)).astype(np.float32)
    gae = np.stack([ppo.PPO.gae(None, torch.tensor(rew[i]), torch.tensor(vals[i])).cpu().numpy()
                    for i in range(6)])
    out = dict(obs=obs, acts=acts, tr_mean=tr_mean, tr_std=tr_std, tr_lp=tr_lp, tr_ent=tr_ent,
               ev_mean=ev_mean, ev_std=ev_std, ev_lp=ev_lp, ev_ent=ev_ent, cop=cop, value=val,
               gae_rew=rew, gae_val=vals, gae=gae, gamma=np.float64(ppo.GAMMA))
    out.update({"actor." + k: v for k, v in sd.items()})
    out.update({"critic." + k: v for k, v in csd.items()})
    np.savez_compressed(OUT, **out)
    print("wrote", OUT, {k: v.shape for k, v in out.items() if not k.startswith(("actor.", "critic."))})


if __name__ == "__main__":
    main()
