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

    def packed_policy(self):
        """Every parameter lnw_policy_act reads (csrc/lnw_actor.hip), in its order:
        packed_features() zero-padded to a multiple of 4 floats; the biases b1
        [64], b2 [64], b3 [32]; then the MFMA A-operand fragments of fc1 (n_in
        zero-padded to 32 columns, 64 when n_in > 32), fc2, fc3 and the heads
        (normal_head rows 0-3, log_std_head rows 4-7, zero rows to 16) for
        v_mfma_f32_16x16x32_bf16 with each weight split exactly into three
        bfloat16 terms (w = hi + mid + lo, round-to-nearest each): per layer three
        planes (hi, mid, lo) of bf16x8 [n-tile][k-pair p][lane], element j =
        W[16 nt + lane % 16][32 p + 16 (j // 4) + 4 (lane // 16) + j % 4] (the k
        order the kernel's chained layers sum in), stored as raw bits, two per
        float."""
        n_in = self.layernorm.normalized_shape[0]
        dev = self.fc1.weight.device

        def frags(w, k_pad, n_pad):
            wp = torch.zeros((n_pad, k_pad), dtype=torch.float32, device=dev)
            wp[:w.shape[0], :w.shape[1]] = w.detach().float()
            nt, qp = n_pad // 16, k_pad // 32
            # [nt][m][p][half][g][v] -> [nt][p][lane = 16 g + m][j = 4 half + v]
            x = wp.reshape(nt, 16, qp, 2, 4, 4).permute(0, 2, 4, 1, 3, 5).reshape(nt, qp, 64, 8)
            hi = x.to(torch.bfloat16)
            r = x - hi.float()
            mid = r.to(torch.bfloat16)
            lo = (r - mid.float()).to(torch.bfloat16)
            return torch.stack([hi, mid, lo]).contiguous().reshape(-1).view(torch.float32)

        conv = self.packed_features()
        conv = torch.cat([conv, torch.zeros((-conv.numel()) % 4, device=dev)])
        k1 = 32 if n_in <= 32 else 64
        heads = torch.cat([self.normal_head.weight, self.log_std_head.weight], 0)
        parts = [conv, self.fc1.bias, self.fc2.bias, self.fc3.bias,
                 frags(self.fc1.weight, k1, 64), frags(self.fc2.weight, 64, 64),
                 frags(self.fc3.weight, 64, 32), frags(heads, 32, 16)]
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

    def packed(self, n_ships, obs_dim):
        """Parameters in lnw_rollout_post's order (csrc/lnw_actor.hip): the MFMA
        A-operand fragments of fc1 per ship (its obs_dim inputs zero-padded to
        a multiple of 16), b1; fc2 fragments, b2; fc3 fragments, b3; fc4 w
        [64], b (+ 3 zeros). Fragments: float4 [n-tile][k-quad][lane] =
        W[16 nt + lane % 16][16 q + 4 (lane // 16) + 0..3] (BatchedActor.packed_policy)."""
        dev = self.fc1.weight.device

        def frags(w, k_pad, n_pad):
            wp = torch.zeros((n_pad, k_pad), dtype=torch.float32, device=dev)
            wp[:w.shape[0], :w.shape[1]] = w.detach().float()
            return wp.reshape(n_pad // 16, 16, k_pad // 16, 4, 4).permute(0, 2, 3, 1, 4).reshape(-1)

        dq = (obs_dim + 15) // 16
        w1 = self.fc1.weight.detach().float().reshape(32, n_ships, obs_dim)
        f1 = torch.cat([frags(w1[:, i], 16 * dq, 32) for i in range(n_ships)])
        parts = [f1, self.fc1.bias, frags(self.fc2.weight, 32, 64), self.fc2.bias,
                 frags(self.fc3.weight, 64, 64), self.fc3.bias, self.fc4.weight.reshape(-1),
                 self.fc4.bias, torch.zeros(3, device=dev)]
        return torch.cat([p.detach().reshape(-1).float() for p in parts]).contiguous()

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


# The rollout's fast path observes into the buffer directly and the policy
# reads the rows there (obs_in_env_stride); off: the rows go to the game's
# packed observation buffer and the policy copies them.
STRIDED_POLICY_INPUT = True


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

    impl="hip" (default) runs a step as four launches: lnw_observe, the fused
    policy kernel (lnw_policy_act: conv head, MLP, heads, keyed sample, log-
    probability, the action array with scripted red rows and row kinds, and
    the rollout rows; a second launch for a red actor), lnw_step, and
    lnw_rollout_post (critic, rewards, running / live flags). impl="torch" is
    the same rollout as batched torch ops (the features kernel + hipBLASLt
    GEMMs + ~45 small kernels per step), kept as the reference implementation
    the fused path is tested against.

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

    Sampling: keyed draws (keyed_normal: Philox keyed by the seed, the global
    row, the rollout index and the step), so a rollout sharded over ranks by
    env_id_base samples exactly what one rank over all envs samples. The
    rollout index lives in a device counter (`call_index`) that every rollout
    advances — inside a captured graph too, so each replay draws fresh values.
    The hip impl always samples this way (seed `keyed_seed`, else `seed`); the
    torch impl does when `keyed_seed` is given, else it draws from the torch
    `generator` passed to run().

    `observe="step"` reuses the step's own output rows instead of a fresh
    observe (one launch less per step, but not the reference's draw order).
    `run(forced_actions=...)` replays given actor outputs [E, T, A, 4] instead of
    sampling (log-probabilities from get_dist): parity against recorded
    reference rollouts (tests/golden/make_rollout_golden.py).
    """

    def __init__(self, game: BatchedGame, actor, critic=None, steps=40, red="script",
                 red_actor=None, noise=None, bn="sample", red_bn="running", gamma=0.99,
                 stop_at_done=True, observe="fresh", keyed_seed=None, impl="hip", seed=0):
        if observe not in ("fresh", "step"):
            raise ValueError("observe must be 'fresh' or 'step'")
        if impl not in ("hip", "torch"):
            raise ValueError("impl must be 'hip' or 'torch'")
        self.keyed_seed, self.impl, self.seed = keyed_seed, impl, int(seed)
        self.g, self.actor, self.critic = game, actor, critic
        self.T, self.red, self.red_actor = int(steps), red, red_actor
        self.noise, self.bn, self.red_bn = noise, bn, red_bn
        self.gamma, self.stop_at_done, self.observe = float(gamma), stop_at_done, observe
        self.table = red_script_table(game.device) if red == "script" else None
        # diagnostics / parity: keep each step's action array and row kinds as
        # the policy wrote them (before the step's in-place salvo write-back)
        # in the returned buffers ("step_actions" [E, T, A, 4] float64,
        # "step_kinds" [E, T, A]); hip impl only
        self.record_actions = False
        # rollout index of the keyed draws, on the device (advanced by run())
        self._call = torch.zeros(1, dtype=torch.int64, device=game.device)

    def call_index(self, value=None):
        """The device rollout counter the keyed draws are keyed by (read, or set
        to `value`)."""
        if value is not None:
            self._call.fill_(int(value))
        return int(self._call.item())

    @torch.no_grad()
    def run(self, generator=None, forced_actions=None, on_step=None):
        """One rollout of T steps from the envs' current state. `on_step(t, out)`
        is called after step t's launch with the step outputs (device tensors),
        where ppo.py:620-638 does its per-step bookkeeping and logging; it must
        not be given while capturing a graph if it synchronises."""
        if self.impl == "hip":
            return self._run_hip(forced_actions, on_step)
        return self._run_torch(generator, forced_actions, on_step)

    def _buffers(self, fill=True):
        """The rollout's storage. fill=False (the HIP path): uninitialised, since
        every element is written each step — the observe writes every ship's row
        (a sunk ship's as zeros), the policy zeroes the rows, actions and
        log-probabilities of envs whose episode ended and writes each env's
        float32 flag, lnw_rollout_post writes every value, reward and running
        flag (masked ones as zeros) — so the 1.4 GB observation buffer of a
        32 768-env rollout is not zero-filled first (≈7 µs per step)."""
        g = self.g
        E, nb, A, D, T, dev = g.E, g.nb, g.A, g.Db, self.T, g.device
        z = torch.zeros if fill else torch.empty
        return dict(obs=z((E, T, nb, D), dtype=torch.float32, device=dev),
                    actions=z((E, T, nb, 4), dtype=torch.float32, device=dev),
                    log_probs=z((E, T, nb, 4), dtype=torch.float32, device=dev),
                    rewards=z((E, T, nb), dtype=torch.float64, device=dev),
                    values=z((E, T), dtype=torch.float32, device=dev),
                    running=(torch.ones if fill else torch.empty)((E, T), dtype=torch.bool, device=dev),
                    f32_step=z((E, T), dtype=torch.bool, device=dev))

    def _run_hip(self, forced_actions, on_step):
        import ctypes as C
        from . import _abi
        from ._abi import F_ALIVE, PolicyArgs, RolloutPostArgs
        L = _abi.load()
        g = self.g
        E, nb, nr, A, Db, Dr, T = g.E, g.nb, g.nr, g.A, g.Db, g.Dr, self.T
        dev = g.device
        b = self._buffers(fill=False)
        obs, acts, logp, rew, val, running, f32s = (b[k] for k in ("obs", "actions", "log_probs", "rewards",
                                                                "values", "running", "f32_step"))
        full = torch.zeros((E, A, 4), dtype=torch.float64, device=dev)
        kinds = torch.full((E, A), _abi.LNW_KIND_F64, dtype=torch.uint8, device=dev)
        live = torch.ones(E, dtype=torch.bool, device=dev)
        red_actor_rows = self.red != "script" and self.red_actor is not None
        ap = self.actor.packed_policy()
        cp = self.critic.packed(nb, Db) if self.critic is not None else None
        if cp is None:  # (no critic: nothing writes the values, which are zeros)
            val.zero_()
        rap = self.red_actor.packed_policy() if red_actor_rows else None
        fa = None
        if forced_actions is not None:
            fa = forced_actions.to(device=dev, dtype=torch.float32).contiguous()
            assert fa.shape == (E, T, A, 4)
        alive_p, _ = g._field(F_ALIVE)
        if self.record_actions:
            b["step_actions"] = torch.zeros((E, T, A, 4), dtype=torch.float64, device=dev)
            b["step_kinds"] = torch.zeros((E, T, A), dtype=torch.uint8, device=dev)
        seed = int(self.keyed_seed if self.keyed_seed is not None else self.seed) & (2**64 - 1)
        stream = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        P = lambda t_: t_.data_ptr()  # noqa: E731
        f4, f8 = 4, 8
        table = self.table.contiguous() if self.table is not None else None
        rew_f64 = int(g.rew_blue.dtype == torch.float64)
        # fresh observations with no per-step callback: the blue rows go straight
        # into the rollout buffer (lnw_observe_ex; the policy zeroes ended envs'
        # rows in place), red's only where a red actor reads them, and the step
        # writes none (ppo.py:577 discards them). g.obs_blue is not updated then.
        direct = self.observe == "fresh" and on_step is None
        # (STRIDED_POLICY_INPUT: the policy reads the rows in the buffer itself)
        strided = direct and STRIDED_POLICY_INPUT
        if self.observe == "step":
            g.observe(-1)
        for t in range(T):
            row_t = P(obs) + t * nb * Db * f4  # the rollout buffer's rows of step t
            red_rows = P(g.obs_red) if red_actor_rows else None
            if strided:
                g.observe_into(-1, row_t, T * nb * Db, red_rows, 0)
            elif direct:
                g.observe_into(-1, P(g.obs_blue), 0, red_rows, 0)
            elif self.observe == "fresh":
                g.observe(-1)
            pa = PolicyArgs()
            pa.obs, pa.E, pa.n, pa.D, pa.own0, pa.A = (row_t if strided else P(g.obs_blue)), E, nb, Db, 0, A
            pa.obs_in_env_stride = T * nb * Db if strided else 0
            pa.params, pa.bn_running = P(ap), int(self.bn == "running")
            if fa is not None:
                pa.forced, pa.forced_act, pa.fa_env_stride = 1, P(fa) + t * A * 4 * f4, T * A * 4
            pa.noise = float(self.noise) if self.noise is not None else 0.0
            pa.seed, pa.call_dev, pa.T, pa.t, pa.which = seed, P(self._call), T, t, 0
            pa.row_base = g.env_id_base * nb
            pa.alive = alive_p
            pa.live = P(live) if self.stop_at_done else None
            pa.obs_out, pa.obs_env_stride = row_t, T * nb * Db
            pa.act_out, pa.logp_out = P(acts) + t * nb * 4 * f4, P(logp) + t * nb * 4 * f4
            pa.act_env_stride = T * nb * 4
            pa.full = P(full)
            if table is not None:
                pa.script, pa.script_n, pa.script_steps = P(table), table.shape[0], table.shape[1]
                pa.script_own0, pa.script_cnt = nb, nr
            pa.kinds, pa.kinds_f32_all_alive = P(kinds), int(red_actor_rows)
            pa.f32_out, pa.f32_env_stride = P(f32s) + t, T
            _abi.check(L.lnw_policy_act(C.byref(pa), stream))
            if red_actor_rows:
                ra = PolicyArgs()
                ra.obs, ra.E, ra.n, ra.D, ra.own0, ra.A = P(g.obs_red), E, nr, Dr, nb, A
                ra.params, ra.bn_running = P(rap), int(self.red_bn == "running")
                if fa is not None:
                    ra.forced, ra.forced_act, ra.fa_env_stride = 1, P(fa) + (t * A + nb) * 4 * f4, T * A * 4
                ra.seed, ra.call_dev, ra.T, ra.t, ra.which = seed, P(self._call), T, t, 2
                ra.row_base, ra.alive, ra.full = g.env_id_base * nr, alive_p, P(full)
                _abi.check(L.lnw_policy_act(C.byref(ra), stream))
            if self.record_actions:
                b["step_actions"][:, t] = full
                b["step_kinds"][:, t] = kinds
            out = g.step(full, kinds, obs=not direct)
            pp = RolloutPostArgs()
            pp.obs, pp.obs_env_stride, pp.E, pp.n, pp.D = pa.obs_out, T * nb * Db, E, nb, Db
            if cp is not None:
                pp.critic, pp.val, pp.val_env_stride = P(cp), P(val) + t * f4, T
            pp.rew, pp.rew_f64, pp.n_rew = P(out["rew_blue"]), rew_f64, nb
            pp.rew_out, pp.rew_env_stride = P(rew) + t * nb * f8, T * nb
            pp.done, pp.live = P(out["done"]), P(live)
            pp.running, pp.running_env_stride = P(running) + t, T
            pp.stop_at_done = int(bool(self.stop_at_done))
            _abi.check(L.lnw_rollout_post(C.byref(pp), stream))
            if on_step is not None:
                on_step(t, out)
        self._call += 1
        rtg = reference_rtg(rew, self.gamma)
        b["rtg"] = rtg
        return b

    def _run_torch(self, generator, forced_actions, on_step):
        from ._abi import F_ALIVE, LNW_KIND_F32, LNW_KIND_F64
        g = self.g
        E, nb, nr, A, D = g.E, g.nb, g.nr, g.A, g.Db
        dev = g.device
        T = self.T
        b = self._buffers()
        obs, acts, logp, rew, val, running, f32_step = (b[k] for k in (
            "obs", "actions", "log_probs", "rewards", "values", "running", "f32_step"))
        full = torch.zeros((E, A, 4), dtype=torch.float64, device=dev)
        red_actor_rows = self.red != "script" and self.red_actor is not None
        if self.observe == "step":
            g.observe(-1)
        live = torch.ones(E, dtype=torch.bool, device=dev)
        base = g.env_id_base
        call = self._call  # device counter; keyed draws read it on the host here

        def draws(t, which, n_side):
            """keyed draws for this step: which 0/1 blue sample / noise, 2 red"""
            if self.keyed_seed is None:
                return None
            slot = ((int(call.item()) * T + t) * 4 + which)
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
        self._call += 1
        # the learner's advantage is gae(rtg, values) on a sampled minibatch
        # (ppo.py:336), left to the caller as in the reference
        b["rtg"] = reference_rtg(rew, self.gamma)
        return b

    def capture(self, generator=None):
        """Record one whole rollout (T steps of actor, red, critic, step kernel,
        buffer writes and reward-to-go) as a HIP graph, so `replay()` launches
        its kernels without host work in between. One eager rollout runs first
        on a side stream (lazy initialisation, GEMM heuristics) and advances the
        envs; reset before replaying. The graph freezes the step launch's
        parameters (scenario, spawn spec) and the buffers it returns: `replay()`
        overwrites them in place. The rollout counter the keyed draws read is a
        device tensor the graph advances, so every replay draws fresh values;
        the torch impl with a `generator` registers it with the graph instead
        (torch's graph-safe generator offsets). The torch impl with
        `keyed_seed` cannot be captured (its keyed draws take the counter on the
        host) and refuses."""
        if self.impl == "torch" and self.keyed_seed is not None:
            raise RuntimeError("Rollout(impl='torch', keyed_seed=...) cannot be captured: its keyed "
                               "draws would be frozen at the capture's rollout index; use impl='hip'")
        dev = self.g.device
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            self.run(generator)
        torch.cuda.current_stream(dev).wait_stream(side)
        graph = torch.cuda.CUDAGraph()
        if generator is not None and self.impl == "torch":
            graph.register_generator_state(generator)
        with torch.cuda.graph(graph):
            out = self.run(generator)
        self._graph, self._graph_out = graph, out
        return out

    def replay(self):
        """One rollout from the envs' current state through the captured graph."""
        self._graph.replay()
        return self._graph_out
