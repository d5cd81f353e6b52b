"""On-device MAPPO rollout pieces around the batched step (SURVEY.md §8(f) rows
1-3): the reference's actor / critic evaluated for every (env, ship) at once,
rollout storage as [E, T, ...] device tensors, the reference's reward-to-go and
GAE as batched tensor ops, and the scripted red action profiles as a device
table. Observations never leave the GPU.

Reference: ppo.py:421-671 (rollout), network.py:38-172 (MLP, Value),
ppo.py:645-659 (reward-to-go), ppo.py:695-714 (gae), game.py:173-182 and
536-542 (red_steps*.csv profiles).
"""
import os

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.distributions import Normal

from .batched import BatchedGame

DATA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data")
WINDOW = 49  # the 7x7 terrain window at the head of a Combatant observation


class BatchedActor(nn.Module):
    """network.py:38-152 `MLP` for a [B, D] batch of observations.

    Same submodules, parameter names and initialisation as the reference, so a
    reference `state_dict` loads as is (`load_reference`). The reference is a
    batch-1 network: it flattens the conv head over the batch and concatenates
    along dim 0 (network.py:83), and the PPO rollout calls it one state at a time
    with BatchNorm in training mode (ppo.py:504-512), i.e. with statistics of that
    single sample. `bn="sample"` reproduces exactly that for every row (instance
    statistics with the BatchNorm affine parameters); `bn="running"` is the
    eval-mode network (running statistics). Running statistics are not updated.
    """

    def __init__(self, n_inputs, n_outputs):
        super().__init__()
        self.conv1 = nn.Conv2d(1, 5, 3, 1, padding=1)
        self.norm1 = nn.BatchNorm2d(5)
        self.pool = nn.MaxPool2d(2, 2)
        self.conv2 = nn.Conv2d(5, 8, 3, 1, padding=1)
        self.norm2 = nn.BatchNorm2d(8)
        self.pool2 = nn.MaxPool2d(2, 2)
        self.convhead = nn.Linear(8, 12, bias=True)
        self.layernorm = nn.LayerNorm(n_inputs)
        self.fc1 = nn.Linear(n_inputs, 64, bias=True)
        self.fc2 = nn.Linear(64, 64, bias=True)
        self.fc3 = nn.Linear(64, 32, bias=True)
        self.normal_head = nn.Linear(32, n_outputs, bias=False)
        self.log_std_head = nn.Linear(32, n_outputs, bias=False)
        for m in (self.fc1, self.fc2, self.fc3, self.normal_head, self.log_std_head):
            nn.init.xavier_uniform_(m.weight)
        self.logstd = nn.Parameter(torch.zeros(()))  # present in the reference, unused there too

    @classmethod
    def for_obs(cls, obs_dim, n_outputs=4):
        """The reference sizing: n_inputs = obs_dim - 7*7 + 12 (ppo.py:78, 446)."""
        return cls(obs_dim - WINDOW + 12, n_outputs)

    def load_reference(self, state_dict):
        """Load a reference MLP state_dict (tensors or arrays)."""
        sd = {k: torch.as_tensor(np.asarray(v)) for k, v in state_dict.items()}
        if "logstd" not in sd:
            sd["logstd"] = torch.zeros(())
        self.load_state_dict({k: v.reshape(self.state_dict()[k].shape) for k, v in sd.items()})
        return self

    def packed_features(self):
        """Parameters in lnw_actor_features' order (csrc/lnw_actor.hip): conv1
        w, b; norm1 w, b, running mean, var; conv2 w, b; norm2 w, b, running
        mean, var; convhead w, b; layernorm w, b (578 + 2 n_in floats)."""
        parts = [self.conv1.weight, self.conv1.bias, self.norm1.weight, self.norm1.bias,
                 self.norm1.running_mean, self.norm1.running_var, self.conv2.weight,
                 self.conv2.bias, self.norm2.weight, self.norm2.bias, self.norm2.running_mean,
                 self.norm2.running_var, self.convhead.weight, self.convhead.bias,
                 self.layernorm.weight, self.layernorm.bias]
        return torch.cat([p.detach().reshape(-1).float() for p in parts]).contiguous()

    def features(self, obs, bn="sample"):
        """network.py:70-85 up to the LayerNorm -> [B, n_in]: the HIP kernel
        for device tensors (lnw_actor_features), torch ops for host tensors."""
        B = obs.shape[0]
        if obs.is_cuda:
            from . import _abi
            L = _abi.load()
            obs = obs.contiguous().float()
            n_in = self.layernorm.normalized_shape[0]
            out = torch.empty((B, n_in), dtype=torch.float32, device=obs.device)
            params = self.packed_features()
            _abi.check(L.lnw_actor_features(params.data_ptr(), obs.shape[1], obs.data_ptr(), B,
                                            0 if bn == "sample" else 1, out.data_ptr(),
                                            torch.cuda.current_stream(obs.device).cuda_stream))
            return out
        z = obs[:, :WINDOW].reshape(B, 1, 7, 7)
        z = self.pool(F.relu(self._bn(self.norm1, self.conv1(z), bn)))
        z = self.pool2(F.relu(self._bn(self.norm2, self.conv2(z), bn)))
        z = self.convhead(torch.flatten(z, 1))
        return self.layernorm(torch.cat((z, obs[:, WINDOW:]), 1))

    @staticmethod
    def _bn(m, z, bn):
        if bn == "sample":
            return F.instance_norm(z, weight=m.weight, bias=m.bias, eps=m.eps)
        return F.batch_norm(z, m.running_mean, m.running_var, m.weight, m.bias, False, 0.0, m.eps)

    def heads(self, obs, bn="sample"):
        """(normal mean, normal std) for every row of obs [B, D]."""
        x = self.features(obs, bn)
        x = torch.tanh(self.fc1(x))
        x = torch.tanh(self.fc2(x))
        x = torch.tanh(self.fc3(x))
        return torch.tanh(self.normal_head(x)), torch.exp(self.log_std_head(x))

    def forward(self, obs, noise=None, bn="sample", generator=None, eps=None, noise_eps=None):
        """network.py:70-115 for every row: sample N(mean, std), add N(0, noise)
        exploration noise, clamp to [0, 1], log-probabilities of the clamped
        actions. Returns (actions, log_probs, ok) where ok marks rows without
        NaN heads (the reference returns (None, None) for those). `eps` /
        `noise_eps`: given standard-normal draws [B, n_outputs] instead of
        drawing from `generator` (keyed_normal: shard-invariant rollouts)."""
        mean, std = self.heads(obs, bn)
        ok = ~(torch.isnan(mean).any(1) | torch.isnan(std).any(1))
        mean_s = torch.where(ok[:, None], mean, torch.zeros_like(mean))
        std_s = torch.where(ok[:, None], std, torch.ones_like(std))
        dist = Normal(mean_s, std_s, validate_args=False)  # no host sync (graph capture)
        if eps is None:
            eps = torch.randn(mean.shape, generator=generator, device=mean.device, dtype=mean.dtype)
        actions = mean_s + std_s * eps
        if noise is not None:
            if noise_eps is None:
                noise_eps = torch.randn(mean.shape, generator=generator, device=mean.device,
                                        dtype=mean.dtype)
            actions = actions + noise * noise_eps
        actions = torch.clamp(actions, 0, 1)
        return actions, dist.log_prob(actions), ok

    def get_dist(self, obs, actions, bn="sample"):
        """network.py:117-152: (log_probs, entropies) of given actions."""
        mean, std = self.heads(obs, bn)
        dist = Normal(mean, std)
        return dist.log_prob(actions), dist.entropy()


class BatchedCritic(nn.Module):
    """network.py:154-172 `Value` (already batched in the reference): the
    centralised critic over the concatenated observations of one side."""

    def __init__(self, n_inputs):
        super().__init__()
        self.fc1 = nn.Linear(n_inputs, 32, bias=True)
        self.fc2 = nn.Linear(32, 64, bias=True)
        self.fc3 = nn.Linear(64, 64, bias=True)
        self.fc4 = nn.Linear(64, 1)
        for m in (self.fc1, self.fc2, self.fc3, self.fc4):
            nn.init.xavier_uniform_(m.weight)

    def load_reference(self, state_dict):
        self.load_state_dict({k: torch.as_tensor(np.asarray(v)) for k, v in state_dict.items()})
        return self

    def forward(self, x):
        x = torch.flatten(x, 1)
        x = torch.tanh(self.fc1(x))
        x = torch.tanh(self.fc2(x))
        x = torch.tanh(self.fc3(x))
        return self.fc4(x)


def keyed_normal(row0, rows, cols, seed, slot, device):
    """Standard-normal draws [rows, cols] for global rows row0 .. row0+rows-1,
    a pure function of (seed, slot, global row, column): Philox uniforms
    (lnw_fill_uniform_f32, the bench's action generator) at absolute counter
    slot * 2^40 + row * 2 * cols + k, then Box-Muller. A rank holding global
    envs [lo, hi) draws exactly the values one rank holding all envs draws for
    them, so a sharded rollout samples what an unsharded one does."""
    from . import _abi
    L = _abi.load()
    per = 2 * cols
    u = torch.empty((rows, per), dtype=torch.float32, device=device)
    off = (int(slot) << 40) + int(row0) * per
    _abi.check(L.lnw_fill_uniform_f32(u.data_ptr(), rows * per, int(seed), off,
                                      torch.cuda.current_stream(device).cuda_stream))
    r = torch.sqrt(-2.0 * torch.log1p(-u[:, :cols]))  # 1 - u in (0, 1]
    return r * torch.cos((2.0 * np.pi) * u[:, cols:])


def red_script_table(device="cuda", dtype=torch.float64):
    """The scripted red profiles (red_steps.csv, red_steps2.csv, red_steps3.csv;
    game.py:173-182) as a device tensor [3, 40, 4] = [red ship, step, action].
    float64: the reference's CSV rows are Python floats (game.py:181), so a step
    that contains one runs in float64 (np.asarray upcast, ppo.py:577)."""
    return torch.as_tensor(np.load(os.path.join(DATA, "red_steps.npy")), dtype=dtype, device=device)


def red_script_actions(table, step, n_red):
    """Red actions of one step for untrained red (ppo.py:560-565): profile i for
    red ship i < 3; ships beyond the three profiles, and steps past the 40 rows,
    get zero actions (the reference indexes past its lists there)."""
    out = torch.zeros((n_red, 4), dtype=table.dtype, device=table.device)
    if step < table.shape[1]:
        k = min(n_red, table.shape[0])
        out[:k] = table[:k, step]
    return out


def reference_rtg(rewards, gamma):
    """ppo.py:645-659 reward-to-go for rollouts rewards [R, T, n] (one rollout
    per leading index), as the reference computes it. The loop walks the steps
    in reverse and the ships in order, `discounted_reward += gamma * r`, and
    appends the accumulator after every term; the reward buffer has a trailing
    dim of 1, so after the first term the accumulator is a 1-element ndarray
    updated in place and every appended entry is that same array. Every element
    of the result is therefore gamma * (sum of the rollout's rewards), summed in
    that order. Returned as float64 [R, T, n], like the reference's buffer."""
    R, T, n = rewards.shape
    rev = torch.flip(rewards.to(torch.float64), dims=[1]).reshape(R, T * n)
    total = torch.cumsum(gamma * rev, dim=1)[:, -1]
    return total[:, None, None].expand(R, T, n).contiguous()


def discounted_rtg(rewards, gamma):
    """Per-ship discounted return G_t = r_t + gamma * G_{t+1} over [R, T, n]
    (what the reference's loop is meant to compute; not used by it)."""
    out = torch.zeros_like(rewards, dtype=torch.float64)
    acc = torch.zeros_like(rewards[:, 0], dtype=torch.float64)
    for t in reversed(range(rewards.shape[1])):
        acc = rewards[:, t].to(torch.float64) + gamma * acc
        out[:, t] = acc
    return out


def gae(rewards, values, gamma, lambda_=0.95):
    """ppo.py:695-714 `PPO.gae`, batched over leading dims (the sequence runs
    along the last dim), same operation order. The reference learner calls it
    on the reward-to-go and critic values of a minibatch, treating the sampled
    rows as the sequence (ppo.py:336)."""
    returns = torch.zeros_like(rewards)
    n = rewards.shape[-1]
    g = torch.zeros_like(rewards[..., 0])
    for i in reversed(range(n)):
        if i < n - 1:
            delta = rewards[..., i] + gamma * values[..., i + 1] - values[..., i]
            g = delta + gamma * lambda_ * g
        else:
            delta = rewards[..., i] - values[..., i]
            g = delta
        returns[..., i] = g + values[..., i]
    return returns


class Rollout:
    """Batched MAPPO rollout (ppo.py:421-671, side being trained = blue): env e
    plays one rollout episode; all E envs advance together. Every step t:

      1. observe (ppo.py:497-575): `ship.get_obs()` of every live ship, blue
         then red, with its side effects (target lists, EW gauss draws) — one
         lnw_observe launch; rows of sunk ships are zeros (compiled_picture);
      2. the actor acts for every live blue ship (training-mode BatchNorm on a
         batch-1 call = per-row statistics, bn="sample"); red acts from the
         scripted profiles (untrained red, ppo.py:563-566) or the red actor in
         eval mode (ppo.py:569-572, red_bn="running"); sunk ships act
         np.zeros(4) (ppo.py:515, 574);
      3. the step runs on what `np.asarray(actions_for_step)` makes of those
         rows (ppo.py:577): a float32 array when every row is an actor output
         (all ships alive, red actor-driven), else float64 (a CSV row of Python
         floats or a np.zeros(4) row upcasts it) — per env, through a float64
         buffer with per-row value kinds (include/lnw.h);
      4. the critic scores the concatenated blue observations (ppo.py:598-605).

    Rewards are kept in float64 (the reference's floats). With `stop_at_done`
    an env's steps after its first done == 0 are masked out (observations,
    actions, log-probabilities, values and rewards zero, `running` False), as
    the reference `break`s and leaves its buffers at zero.

    Differences from the reference loop, by design:
      * it observes the env it steps; ppo.py:497 calls get_obs on self.env, a
        Game that rollout() never steps (a reference bug);
      * exploration: the reference's parameter noise and adaptive noise ratio
        (ppo.py:466-482, 586-596) belong to the learner; `noise` adds a fixed
        N(0, noise) term like MLP.forward's `noise` argument;
      * sunk ships' action rows are stored as zeros (the reference stores the
        previous ship's `action` variable there, ppo.py:516-517).

    `keyed_seed`: sampling draws come from keyed_normal (Philox keyed by the
    global env id, the rollout index and the step) instead of a torch
    generator, so a rollout sharded over ranks by env_id_base samples exactly
    what one rank over all envs samples (eager runs; a captured graph freezes
    the keys of the capture).

    `observe="step"` reuses the step's own output rows instead of a fresh
    observe (one launch less per step, but not the reference's draw order).
    `run(forced_actions=...)` replays given actor outputs [E, T, A, 4] instead of
    sampling (log-probabilities from get_dist): parity against recorded
    reference rollouts (tests/golden/make_rollout_golden.py).
    """

    def __init__(self, game: BatchedGame, actor, critic=None, steps=40, red="script",
                 red_actor=None, noise=None, bn="sample", red_bn="running", gamma=0.99,
                 stop_at_done=True, observe="fresh", keyed_seed=None):
        if observe not in ("fresh", "step"):
            raise ValueError("observe must be 'fresh' or 'step'")
        self.keyed_seed, self._calls = keyed_seed, 0
        self.g, self.actor, self.critic = game, actor, critic
        self.T, self.red, self.red_actor = int(steps), red, red_actor
        self.noise, self.bn, self.red_bn = noise, bn, red_bn
        self.gamma, self.stop_at_done, self.observe = float(gamma), stop_at_done, observe
        self.table = red_script_table(game.device) if red == "script" else None

    @torch.no_grad()
    def run(self, generator=None, forced_actions=None, on_step=None):
        """One rollout of T steps from the envs' current state. `on_step(t, out)`
        is called after step t's launch with the step outputs (device tensors),
        where ppo.py:620-638 does its per-step bookkeeping and logging; it must
        not be given while capturing a graph if it synchronises."""
        from ._abi import F_ALIVE, LNW_KIND_F32, LNW_KIND_F64
        g = self.g
        E, nb, nr, A, D = g.E, g.nb, g.nr, g.A, g.Db
        dev = g.device
        T = self.T
        obs = torch.zeros((E, T, nb, D), dtype=torch.float32, device=dev)
        acts = torch.zeros((E, T, nb, 4), dtype=torch.float32, device=dev)
        logp = torch.zeros((E, T, nb, 4), dtype=torch.float32, device=dev)
        rew = torch.zeros((E, T, nb), dtype=torch.float64, device=dev)
        val = torch.zeros((E, T), dtype=torch.float32, device=dev)
        running = torch.ones((E, T), dtype=torch.bool, device=dev)
        f32_step = torch.zeros((E, T), dtype=torch.bool, device=dev)
        full = torch.zeros((E, A, 4), dtype=torch.float64, device=dev)
        red_actor_rows = self.red != "script" and self.red_actor is not None
        if self.observe == "step":
            g.observe(-1)
        live = torch.ones(E, dtype=torch.bool, device=dev)
        call = self._calls
        self._calls += 1
        base = g.env_id_base

        def draws(t, which, n_side):
            """keyed draws for this step: which 0/1 blue sample / noise, 2 red"""
            if self.keyed_seed is None:
                return None
            slot = ((call * T + t) * 4 + which)
            return keyed_normal(base * n_side, E * n_side, 4, self.keyed_seed, slot, dev)

        for t in range(T):
            if self.observe == "fresh":
                g.observe(-1)
            cur, cur_red = g.obs_blue, g.obs_red
            alive = g.get(F_ALIVE).t().bool()  # [E, A], slots not None
            ab = alive[:, :nb, None]
            # rows an env fills after its episode ended stay zero, as the
            # reference's buffers do after its `break` (ppo.py:640-641)
            keep = ab & live[:, None, None] if self.stop_at_done else ab
            obs[:, t] = torch.where(live[:, None, None], cur, torch.zeros((), device=dev)) \
                if self.stop_at_done else cur
            if forced_actions is not None:
                a = forced_actions[:, t, :nb].to(torch.float32)
                lp, _ = self.actor.get_dist(cur.reshape(E * nb, D), a.reshape(E * nb, 4),
                                            bn=self.bn)
            else:
                a, lp, _ = self.actor(cur.reshape(E * nb, D), noise=self.noise, bn=self.bn,
                                      generator=generator, eps=draws(t, 0, nb),
                                      noise_eps=draws(t, 1, nb) if self.noise is not None else None)
            a = torch.where(ab, a.reshape(E, nb, 4), torch.zeros((), device=dev))
            acts[:, t] = torch.where(keep, a, torch.zeros((), device=dev))
            logp[:, t] = torch.where(keep, lp.reshape(E, nb, 4), torch.zeros((), device=dev))
            full[:, :nb] = a
            ar = alive[:, nb:, None]
            if self.red == "script":
                full[:, nb:] = torch.where(ar, red_script_actions(self.table, t, nr),
                                           torch.zeros((), dtype=torch.float64, device=dev))
            elif self.red_actor is not None:
                if forced_actions is not None:
                    ra = forced_actions[:, t, nb:].to(torch.float32)
                else:
                    ra, _, _ = self.red_actor(cur_red.reshape(E * nr, g.Dr), bn=self.red_bn,
                                              generator=generator, eps=draws(t, 2, nr))
                full[:, nb:] = torch.where(ar, ra.reshape(E, nr, 4),
                                           torch.zeros((), device=dev)).double()
            else:
                full[:, nb:] = 0
            # np.asarray(actions_for_step): float32 only if every row is float32
            f32 = alive.all(1) if red_actor_rows else torch.zeros(E, dtype=torch.bool, device=dev)
            f32_step[:, t] = f32
            kinds = torch.where(f32, LNW_KIND_F32, LNW_KIND_F64).to(torch.uint8)[:, None]
            if self.critic is not None:
                v = self.critic(cur.reshape(E, nb * D)).reshape(E)
                val[:, t] = torch.where(live, v, torch.zeros((), device=dev)) if self.stop_at_done else v
            out = g.step(full, kinds.expand(E, A).contiguous())
            running[:, t] = live
            r = out["rew_blue"].to(torch.float64)
            rew[:, t] = torch.where(live[:, None], r, torch.zeros_like(r)) if self.stop_at_done else r
            if self.stop_at_done:
                live = live & (out["done"] != 0)
            if on_step is not None:
                on_step(t, out)
        rtg = reference_rtg(rew, self.gamma)
        # the learner's advantage is gae(rtg, values) on a sampled minibatch
        # (ppo.py:336), left to the caller as in the reference
        return dict(obs=obs, actions=acts, log_probs=logp, rewards=rew, values=val,
                    running=running, f32_step=f32_step, rtg=rtg)

    def capture(self, generator=None):
        """Record one whole rollout (T steps of actor, red, critic, step kernel and
        buffer writes, then reward-to-go and GAE) as a HIP graph, so `replay()`
        launches its ~30 kernels per step without host work in between. One eager
        rollout runs first on a side stream (lazy initialisation, GEMM heuristics)
        and advances the envs; reset before replaying. The graph freezes the
        step launch's parameters (scenario, spawn spec) and the buffers it
        returns: `replay()` overwrites them in place."""
        dev = self.g.device
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            self.run(generator)
        torch.cuda.current_stream(dev).wait_stream(side)
        graph = torch.cuda.CUDAGraph()
        if generator is not None:
            graph.register_generator_state(generator)
        with torch.cuda.graph(graph):
            out = self.run(generator)
        self._graph, self._graph_out = graph, out
        return out

    def replay(self):
        """One rollout from the envs' current state through the captured graph."""
        self._graph.replay()
        return self._graph_out
