"""The oracle's full-size driver (orc_fullsize_range, used by
tests/test_gpu_fullsize.py) against the per-env OracleEnv stepping of the same
envs: same trajectories, auto-reset at the horizon, and the observation hash
sum_k bits(float32 obs[k]) * mult[k] mod 2^64 recomputed in numpy. CPU only."""
import numpy as np

import _oracle


def _hash(ob, orr, mult):
    w = np.concatenate([ob.astype(np.float32).ravel(), orr.astype(np.float32).ravel()])
    return int(np.sum(w.view(np.uint32).astype(np.uint64) * mult.astype(np.uint64),
                      dtype=np.uint64))


def test_fullsize_driver_matches_per_env_oracle():
    g = _oracle.load_fixture("grids.npz")["grid100"]
    E, S, seed, horizon = 12, 23, 5, 10
    rng = np.random.default_rng(0)
    water = np.argwhere(g[30:70, 40:65] <= 74) + np.array([30, 40])
    pos = water[rng.integers(0, len(water), (E, 8))].astype(np.int32)
    acts = rng.random((S, E, 8, 4), dtype=np.float32)
    mult = rng.integers(0, 1 << 30, 8 * 68, dtype=np.int64) * 2 + 1
    types = [0] * 4 + [1] * 4
    hsh, rew, done, cog = _oracle.fullsize(g, 4, 4, types, pos, acts, mult, seed, horizon,
                                           pos_per_env=True, threads=3)
    resets = 0
    for e in range(E):
        o = _oracle.OracleEnv(g, 4, 4, landing_ops=False)
        o.set_philox(seed, e)
        o.reset(types, pos[e])
        for s in range(S):
            r = o.step(acts[s, e], np.full(8, _oracle.K_F32, np.int32))
            assert hsh[s, e] == _hash(r["obs_blue"], r["obs_red"], mult), (s, e)
            assert np.array_equal(rew[s, e], np.concatenate([r["rew_blue"], r["rew_red"]]).astype(np.float32))
            assert done[s, e] == r["done"]
            assert np.array_equal(cog[s, e], np.float32(r["cog"]), equal_nan=True)
            if r["done"] == 0 or o.env_state()["steps_done"] >= horizon:
                o.reset(types, pos[e])
                resets += 1
    assert resets >= E * (S // horizon)
