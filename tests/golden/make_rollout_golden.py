#!/usr/bin/env python3
"""Golden vectors for the batched MAPPO rollout (lnw.rollout.Rollout) taken from
the reference's own `PPO.rollout` (ppo.py:421-671). TEST INFRASTRUCTURE ONLY:
runs in the build container, where /root/reference is mounted, through the
stub harness of make_golden.py.

What runs is the reference loop as written, with three substitutions:
  * `ppo.Game` returns the PPO's own env, so the loop observes the env it
    steps (ppo.py:497 observes `self.env`, which rollout() never steps — the
    reference bug lnw.rollout.Rollout documents);
  * the Python `random` module of game/combatant/landingship and numpy's
    `np.random.beta` are a recording tape (make_golden.TapeRNG), so the device
    can replay every draw;
  * parameter noise is off (`add_param_noise = False`): the actor each step is
    the seeded one whose weights are stored here.

Recorded per scenario (R rollout episodes = R device envs):
  per episode  tape slice, ducting, spawn cells (landing ship drawn);
  per step     the array handed to step() (its dtype: float32 or float64 after
               np.asarray, ppo.py:577), rewards, done, cog;
  rollout()'s  batch_obs, batch_log_probs, batch_values, batch_rewards_to_go;
  learner      PPO.gae (ppo.py:695-714) on the flattened reward-to-go and
               values, the way ppo.py:336 feeds it (here the whole batch in
               order instead of a sampled minibatch);
  weights      actor / critic / red actor state_dicts.

usage: python tests/golden/make_rollout_golden.py [NAME ...]   (writes rollout_*.npz)
"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import make_golden  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))
TYPE_CODE = make_golden.TYPE_CODE


def run(name, *, n_blue, n_red, n_ls, landing_ops, trained_red, R, T, seed, boxes=None):
    game, combatant, landingship = make_golden.import_reference()
    import torch
    import network  # noqa: F401
    import ppo
    game.N_RED_LANDINGSHIP = n_ls
    game.LANDING_OPS = landing_ops
    game.TRAINED_RED = trained_red
    game.SIDE = "blue"
    game.TACTICS = "aggressive"
    game.DISCRETE = combatant.DISCRETE = landingship.DISCRETE = False
    combatant.CUR_SIDE = landingship.CUR_SIDE = "blue"
    ppo.TRAINED_RED = trained_red
    ppo.SIDE = "blue"
    ppo.WANDA = False
    tape = make_golden.TapeRNG(seed)
    game.random = combatant.random = landingship.random = tape
    np_beta = np.random.beta
    np.random.beta = tape.beta
    try:
        env = game.Game()
        marks, rec = [], dict(act=[], f32=[], rew=[], done=[], cog=[], ep=[])
        eps = []
        real_reset, real_step = env.reset, env.step
        rng = np.random.default_rng(seed)
        grid = np.load(os.path.join(OUT, "grids.npz"))["grid100"]

        def reset(*a, **k):
            marks.append(len(tape.vals))
            if boxes is not None:
                # 4v4 exists only through reset(..., blue_ships, red_ships)
                # (SURVEY.md §3.2): fresh ships on water cells of two boxes
                env.grid = grid
                k = dict(k, grid=grid,
                         blue_ships=[combatant.Combatant("blue", "small", p, [], env) for p in
                                     make_golden._water_in_box(grid, rng, boxes[0], n_blue)],
                         red_ships=[combatant.Combatant("red", "large", p, [], env) for p in
                                    make_golden._water_in_box(grid, rng, boxes[1], n_red)])
            out = real_reset(*a, **k)
            ships = list(env.blue_ships) + list(env.red_ships)
            eps.append(dict(tape_start=marks[-1], ducting=env.ducting_factor,
                            spawn=[tuple(int(v) for v in s.position) for s in ships],
                            types=[TYPE_CODE[s.ship_type] for s in ships]))
            return out

        def step(action):
            arr = np.asarray(action)
            rec["act"].append(np.array(arr, np.float64))
            rec["f32"].append(arr.dtype == np.float32)
            obs, reward, done, cog = real_step(action)
            rec["rew"].append([float(r) for r in reward])
            rec["done"].append(int(done))
            rec["cog"].append(np.nan if cog is None else float(cog))
            # eps[0]: the reset before PPO(env); eps[1]: rollout()'s pre-loop reset
            rec["ep"].append(len(eps) - 3)
            return obs, reward, done, cog

        env.reset, env.step = reset, step
        with make_golden.quiet():
            env.reset(n_blue, n_red)
        torch.manual_seed(seed)
        agent = ppo.PPO(env, torch.device("cpu"))
        agent.add_param_noise = False
        weights = {}
        for pre, net in (("actor.", agent.actor), ("critic.", agent.critic),
                         ("red_actor.", agent.red_actor)):
            weights.update({pre + k: v.detach().cpu().numpy().copy()
                            for k, v in net.state_dict().items()})
        ppo.Game = lambda: env
        with make_golden.quiet():
            b_obs, b_act, b_lp, b_rtg, lens, b_gs, b_val = agent.rollout(R, T, 0.0)
        end = len(tape.vals)
        nb = len(env.blue_ships)
        rtg_flat = b_rtg.reshape(R * T * nb, 1)
        val_flat = b_val.detach().reshape(R * T * nb, 1)
        learner_gae = agent.gae(rtg_flat, val_flat).detach().cpu().numpy()
    finally:
        np.random.beta = np_beta
    eps = eps[2:]
    for i, e in enumerate(eps):
        e["tape_end"] = eps[i + 1]["tape_start"] if i + 1 < len(eps) else end
    A = len(eps[0]["types"])
    steps = np.array(rec["ep"])
    n_steps = [int((steps == i).sum()) for i in range(R)]
    act = np.zeros((R, T, A, 4))
    f32 = np.zeros((R, T), np.uint8)
    rew = np.zeros((R, T, nb))
    done = np.ones((R, T), np.int32)
    cog = np.full((R, T), np.nan)
    k = 0
    for i in range(R):
        for t in range(n_steps[i]):
            act[i, t], f32[i, t] = rec["act"][k], rec["f32"][k]
            rew[i, t], done[i, t], cog[i, t] = rec["rew"][k], rec["done"][k], rec["cog"][k]
            k += 1
    meta = dict(name=name, n_blue=n_blue, n_red=n_red, n_ls=n_ls, landing_ops=landing_ops,
                boxes=boxes,
                trained_red=trained_red, R=R, T=T, nb=nb, A=A, episodes=eps, n_steps=n_steps,
                gamma=float(agent.gamma), Db=env.observation_space, Dr=env.red_observation_space)
    out = dict(meta=np.array(json.dumps(meta)), tape=np.array(tape.vals, np.float64),
               act=act, act_f32=f32, rew=rew, done=done, cog=cog,
               batch_obs=b_obs.detach().cpu().numpy(), batch_log_probs=b_lp.detach().cpu().numpy(),
               batch_values=b_val.detach().cpu().numpy(), batch_rtg=b_rtg.detach().cpu().numpy(),
               learner_gae=learner_gae, **weights)
    path = os.path.join(OUT, f"rollout_{name}.npz")
    np.savez_compressed(path, **out)
    print(f"{path}: {R} episodes, steps {n_steps}, {len(tape.vals)} draws, "
          f"float32 steps {int(f32.sum())} / {int(sum(n_steps))}, done at "
          f"{[int(np.argmin(done[i])) if (done[i] == 0).any() else None for i in range(R)]}")


def main(only=None):
    """All scenarios, or only the names given on the command line."""
    if not os.path.isdir(make_golden.REF):
        print("reference not present; nothing to do")
        return
    if only is not None:
        return _main_only(only)
    _main_only(None)


def _main_only(only):
    # untrained (scripted CSV) red, 3v3 at the reference spawns (game.py:551-585)
    if only is None or "3v3_scripted" in only:
        run("3v3_scripted", n_blue=3, n_red=3, n_ls=0, landing_ops=False, trained_red=False,
            R=6, T=40, seed=31)
    # trained red (red actor in eval mode) with a landing ship and landing ops
    if only is None or "4v2ls_trained" in only:
        run("4v2ls_trained", n_blue=4, n_red=2, n_ls=1, landing_ops=True, trained_red=True,
            R=6, T=40, seed=32)
    # config 5's 4v4 through reset(..., blue_ships, red_ships), fleets 15-30 cells
    # apart, trained red: fire, sunk ships (float64 steps) and EW every episode
    if only is None or "4v4_trained_contact" in only:
        run("4v4_trained_contact", n_blue=4, n_red=4, n_ls=0, landing_ops=False, trained_red=True,
            R=8, T=40, seed=33, boxes=(((30, 45), (40, 60)), ((55, 70), (45, 65))))
    if only is None or "4v4_melee_done" in only:
        # fleets 0-16 cells apart (the melee box): sinkings end most episodes
        # before step 40 (done == 0, the `break` at ppo.py:640-641)
        run("4v4_melee_done", n_blue=4, n_red=4, n_ls=0, landing_ops=False, trained_red=True,
            R=8, T=40, seed=34, boxes=(((40, 48), (44, 56)), ((48, 56), (48, 60))))
    if only is None or "2v2_trained_breaks" in only:
        # 2v2 fleets 8-20 cells apart, trained red: episodes that run with every
        # ship alive for a while (float32 action arrays, ppo.py:577) and then end
        # mid-rollout (done == 0 at steps 7-10: the `break`, ppo.py:640-641),
        # beside episodes that end at once and ones that reach step 40
        run("2v2_trained_breaks", n_blue=2, n_red=2, n_ls=0, landing_ops=False, trained_red=True,
            R=12, T=40, seed=62, boxes=(((37, 43), (45, 53)), ((51, 57), (47, 55))))


if __name__ == "__main__":
    main(sys.argv[1:] or None)
