#!/usr/bin/env python3
"""Golden vectors for the reference's crash modes (TEST INFRASTRUCTURE ONLY).

The reference raises inside ``Game.step`` on a few inputs; the build defines
them as per-env error bits instead (include/lnw.h LNW_ERRF_*) and keeps
stepping. This script runs the reference itself (make_golden.py's import
harness) on constructed episodes and records, per case, the
step at which it raised, the exception type and the reference function and
line that raised it, plus every step's outputs before that. The tape RNG
hands out a fixed list of values in call order (any draw kind), so the same
list replays on the oracle and on the GPU.

Cases:
  equal_bearings  two blue ships on one line to a radiating red ship: equal EW
                  bearings, m1 == m2 (combatant.py:274 ZeroDivisionError)
  nan_fix         the same with NaN gauss draws: NaN fixes, round(np.mean)
                  (combatant.py:146 ValueError)
  nan_move / inf_move / nan_move_f32   a NaN or inf move component
                  (continuous_to_discrete, combatant.py:470)
  nan_engagement / inf_engagement      a NaN or inf engagement value
                  (round(engagement * missiles), combatant.py:528)
  nan_radar       a NaN radar action (round(rad_action), combatant.py:558)
  huge_move       a huge but finite move: no crash (the target is off-grid)

usage: python tests/golden/make_crash_golden.py   (writes crash_modes.npz)
"""
import json
import os
import sys
import traceback

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import make_golden  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))
STEPS = 4
A = 8
# (x0, y0) red ship 0; blue 0 and 1 at 5 and 10 cells down the diagonal (open water)
LINE = [(45, 47), (40, 42), (10, 81), (8, 70), (50, 52), (98, 48), (98, 56), (96, 52)]
REF = make_golden.REF_BLUE + make_golden.REF_RED4


class ListRNG:
    """random / numpy.random.beta stand-in: the next value of a fixed list for
    every draw, whatever its kind (the device tape semantics)."""

    def __init__(self, vals):
        self.vals = list(vals)
        self.i = 0

    def _next(self):
        v = self.vals[self.i]
        self.i += 1
        return v

    def random(self):
        return self._next()

    def gauss(self, mu=0.0, sigma=1.0):
        return mu + sigma * self._next()

    def randint(self, a, b):
        return int(self._next())

    def beta(self, a, b):
        return self._next()


def base_actions(dtype=np.float64):
    """Nobody moves or fires; red radars on, blue radars off."""
    act = np.zeros((STEPS, A, 4), dtype)
    act[:, 4:, 0] = 1
    act[:, :, 1] = 0.0
    act[:, :, 2] = 0.25
    act[:, :, 3] = 0.5
    return act


def cases():
    const = [0.3] + [0.25] * 4000
    out = []
    act = base_actions()
    act[:, :, 3] = 0.0
    out.append(("equal_bearings", LINE, act, const))
    out.append(("nan_fix", LINE, act.copy(), [0.3] + [float("nan")] * 4000))
    for name, k, v, dt in (("nan_move", 2, np.nan, np.float64), ("inf_move", 3, np.inf, np.float64),
                           ("nan_move_f32", 2, np.nan, np.float32),
                           ("nan_engagement", 1, np.nan, np.float64),
                           ("inf_engagement", 1, np.inf, np.float64),
                           ("nan_radar", 0, np.nan, np.float64), ("huge_move", 3, 1e300, np.float64)):
        a = base_actions(dt)
        a[1, 2, k] = v  # blue ship 2, step 1
        out.append((name, REF, a, const))
    return out


def run_case(game, combatant, landingship, name, pos, acts, tape):
    # Game() draws a ducting factor of its own (game.py:116) before reset draws
    # the episode's (game.py:531): the tape starts at reset, as make_golden's does
    rng = ListRNG([0.5] + list(tape))
    game.random = combatant.random = landingship.random = rng
    np_beta = np.random.beta
    np.random.beta = rng.beta
    rec = dict(obs_blue=[], obs_red=[], rew_blue=[], rew_red=[], done=[], tape_pos=[])
    crash = None
    try:
        env = game.Game()
        grid = np.load(os.path.join(OUT, "grids.npz"))["grid100"]
        env.grid = grid
        blue = [combatant.Combatant("blue", "small", p, [], env) for p in pos[:4]]
        red = [combatant.Combatant("red", "large", p, [], env) for p in pos[4:]]
        with make_golden.quiet():
            env.reset(4, 4, grid=grid, blue_ships=blue, red_ships=red)
        for s in range(STEPS):
            call = acts[s].copy()
            try:
                _, cap = make_golden._capture_step(game, env, call)
            except (ZeroDivisionError, ValueError, OverflowError) as exc:
                tb = [f for f in traceback.extract_tb(exc.__traceback__)
                      if f.filename.startswith(make_golden.REF)]
                last = tb[-1]
                crash = dict(step=s, exc=type(exc).__name__, func=last.name,
                             file=os.path.basename(last.filename), line=last.lineno)
                break
            rec["obs_blue"].append(np.asarray(cap["observations"], np.float32)[0])
            rec["obs_red"].append(np.asarray(cap["red_observations"], np.float32)[0])
            rec["rew_blue"].append(np.array(cap["blue_rewards"], np.float64))
            rec["rew_red"].append(np.array(cap["red_rewards"], np.float64))
            rec["done"].append(int(cap["done"]))
            rec["tape_pos"].append(rng.i - 1)
    finally:
        np.random.beta = np_beta
    return rec, crash


def main():
    game, combatant, landingship = make_golden.import_reference()
    game.RED_AGGRESSION = 0.4
    game.N_RED_LANDINGSHIP = 0
    game.SIDE = "blue"
    combatant.CUR_SIDE = landingship.CUR_SIDE = "blue"
    game.TRAINED_RED = True
    game.DISCRETE = combatant.DISCRETE = landingship.DISCRETE = False
    game.LANDING_OPS = False
    game.TACTICS = "aggressive"
    game.COA_PATH = False
    meta, arrays = [], {}
    for name, pos, acts, tape in cases():
        rec, crash = run_case(game, combatant, landingship, name, pos, acts, tape)
        n = len(rec["done"])
        meta.append(dict(name=name, pos=[list(map(int, p)) for p in pos], crash=crash, ok_steps=n,
                         dtype=str(acts.dtype)))
        arrays[f"{name}_actions"] = acts.astype(np.float64)
        arrays[f"{name}_tape"] = np.array(tape, np.float64)
        for k, v in rec.items():
            arrays[f"{name}_{k}"] = np.array(v)
        print(f"{name}: {n} clean steps, crash {crash}")
    np.savez_compressed(os.path.join(OUT, "crash_modes.npz"), meta=np.array(json.dumps(meta)),
                        **arrays)


if __name__ == "__main__":
    main()
