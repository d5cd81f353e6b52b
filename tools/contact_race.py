#!/usr/bin/env python3
"""Diagnostics: test_fullsize_config2_contact_spawns[True]'s workload (4 096 4v4
envs in contact, 45 steps, the contact variant) run R times on the same inputs:
per run the (step, env) pairs whose observation hash, rewards or done differ from
the oracle, with the env's lane (env % 64) and workgroup (env // 64), and
whether the runs agree with each other.
usage: python tools/contact_race.py [R] [variant 0|1]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# RACE_PKG=dir: an older host package to pair with an older LNW_LIB build (A/B)
sys.path[:0] = [ROOT, os.environ.get("RACE_PKG", os.path.join(ROOT, "littoral-naval-warfare-marl_amd")),
                os.path.join(ROOT, "tests")]


def main():
    import numpy as np
    import torch
    import _oracle
    from test_gpu_fullsize import _grids, _water_positions, _mult, _gpu_run
    from lnw.batched import BatchedGame
    from lnw.config import Scenario
    R = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    variant = bool(int(sys.argv[2])) if len(sys.argv) > 2 else True
    grid = _grids()[0]
    E, S, seed = 4096, 45, 77
    pos = _water_positions(grid, E, [(30, 45, 40, 60)] * 4 + [(55, 70, 45, 65)] * 4, seed=3)
    acts = np.random.default_rng(6).random((S, E, 8, 4), dtype=np.float32)
    mult = _mult(4 * 68 + 4 * 68, seed=7)
    oh, orw, od, oc = _oracle.fullsize(grid, 4, 4, [0] * 4 + [1] * 4, pos, acts, mult, seed, 40,
                                       pos_per_env=True)
    print("oracle done", flush=True)
    def run_rows(g):  # _gpu_run plus every step's rows kept on the host
        mt = torch.from_numpy(mult).cuda()
        hs, rews, dones, rows = [], [], [], []
        for s in range(S):
            out = g.step(torch.from_numpy(acts[s]).cuda())
            w = torch.cat([out["obs_blue"].reshape(E, -1), out["obs_red"].reshape(E, -1)], 1)
            rows.append(w.cpu().numpy().reshape(E, 8, -1))
            wi = w.contiguous().view(torch.int32).to(torch.int64) & 0xFFFFFFFF
            hs.append((wi * mt).sum(1).cpu().numpy().view(np.uint64))
            rews.append(torch.cat([out["rew_blue"].reshape(E, -1), out["rew_red"].reshape(E, -1)],
                                  1).cpu().numpy())
            dones.append(out["done"].cpu().numpy().copy())
        return np.stack(hs), np.stack(rews), np.stack(dones), np.stack(rows)

    first = None
    good_rows = None
    dumps = {}
    for r in range(R):
        # RACE_SKIP_BITS=b: LNW_DEBUG_SKIP for runs >= 1 (diagnostics build via LNW_LIB,
        # e.g. 33554432 = bit 25: write_obs_t without its per-pass store wait)
        if os.environ.get("RACE_SKIP_BITS"):
            if r == 0:
                os.environ.pop("LNW_DEBUG_SKIP", None)
            else:
                os.environ["LNW_DEBUG_SKIP"] = os.environ["RACE_SKIP_BITS"]
        # RACE_REF_NOSPLIT=1: run 0 on the emission path (LNW_NO_SPLIT_ROWS), the reference rows
        if os.environ.get("RACE_REF_NOSPLIT"):
            if r == 0:
                os.environ["LNW_NO_SPLIT_ROWS"] = "1"
            else:
                os.environ.pop("LNW_NO_SPLIT_ROWS", None)
        sc = Scenario(landing_ops=False, auto_reset=True, episode_steps=40)
        g = BatchedGame(E, ["small"] * 4, ["large"] * 4, scenario=sc, grid=grid, seed=seed)
        g.set_variant(variant)
        g.reset(positions=pos[0], pos_per_env=torch.from_numpy(pos))
        gh, gr, gd, rows = run_rows(g)
        kern = g.step_kernel()
        g.close()
        bad = np.argwhere(gh != oh)
        badr = np.argwhere(~np.isclose(gr, orw, rtol=0, atol=1e-5).all(2))
        badd = np.argwhere(gd != od)
        first_step = {}
        for s, e in bad.tolist():
            first_step.setdefault(e, s)
        envs = sorted(first_step)
        print(f"run {r} kernel {kern}: {len(bad)} hash, {len(badr)} reward, {len(badd)} done mismatches;"
              f" envs {envs[:12]} first steps {[first_step[e] for e in envs[:12]]}"
              f" lanes {sorted(set(e % 64 for e in envs))[:16]} workgroups {sorted(set(e // 64 for e in envs))[:8]}",
              flush=True)
        if len(bad) == 0 and good_rows is None:
            good_rows = rows
        if len(bad) and good_rows is not None and os.environ.get("RACE_DUMP"):
            # RACE_DUMP=path: the rows of every workgroup with a wrong (step, env), as
            # written and as they should be (the first clean run), for the offline
            # source attribution of each wrong float4 (tools/race_chunks.py)
            keys = sorted({(s_, e // 64) for s_, e in bad.tolist()})[:48]
            dumps.setdefault("got", []).extend(rows[s_, 64 * w:64 * w + 64] for s_, w in keys)
            dumps.setdefault("want", []).extend(good_rows[s_, 64 * w:64 * w + 64] for s_, w in keys)
            dumps.setdefault("key", []).extend((r, s_, w) for s_, w in keys)
        if len(bad) and good_rows is not None:
            for s_, e in bad[:3].tolist():
                for a in range(8):
                    x, y = rows[s_, e, a], good_rows[s_, e, a]
                    d = np.nonzero(x.view(np.int32) != y.view(np.int32))[0]
                    if len(d) == 0:
                        continue
                    print(f"  step {s_} env {e} agent {a}: {len(d)} elements differ at {d[:12].tolist()};"
                          f" got {x[d[:6]].tolist()} want {y[d[:6]].tolist()}", flush=True)
                    # the wrong row: some other (env, agent) row of this step or the step before?
                    for s2 in (s_, s_ - 1):
                        if s2 < 0:
                            continue
                        m = np.nonzero((good_rows[s2].view(np.int32) == x.view(np.int32)).all(-1))
                        if len(m[0]):
                            print(f"    equals good row (step {s2}, env, agent) {list(zip(m[0].tolist(), m[1].tolist()))[:4]}",
                                  flush=True)
        if first is None:
            first = gh
        else:
            print(f"  vs run 0: {int((gh != first).sum())} (step, env) hashes differ", flush=True)
    if dumps:
        np.savez_compressed(os.environ["RACE_DUMP"], got=np.stack(dumps["got"]), want=np.stack(dumps["want"]),
                            key=np.array(dumps["key"], np.int64))
        print(f"dumped {len(dumps['key'])} (run, step, workgroup) blocks to {os.environ['RACE_DUMP']}",
              flush=True)


if __name__ == "__main__":
    main()
