"""The reference's crash modes on the HIP path (the build must
define them). Game.step raises on a ZeroDivisionError in an EW fix
(combatant.py:274) and on round() of NaN / inf: a fix (:146), a move target
(:470), an engagement threshold (:528), a radar action (:558). The build sets
the env's error bit instead (LNW_ERRF_ZERODIV / LNW_ERRF_NAN_ROUND) and keeps
stepping: the ship whose round() raised does not move / engage / radiate, a
fix whose slopes are equal is skipped. These tests compare the GPU with the
oracle on every output, the error bits and the state, through the crash step
and the steps after it, on every step kernel:
  * the reference-pinned episodes of tests/golden/crash_modes.npz (tape mode;
    tests/test_oracle_crash_cpu.py pins the oracle to the reference's raises);
  * random action rows with NaN / +-inf / huge entries injected, reference and
    melee spawns, Philox mode (the quiet path sends such rows to phase S)."""
import numpy as np
import pytest
import torch

import _oracle
from test_oracle_crash_cpu import EXC_BIT, FX, META

pytestmark = pytest.mark.gpu

REW_TOL = 1e-5
CASES = sorted(META)
# variant -> (contact variant, environment knobs read at lnw_create, envs, epw, kernel code)
VARIANTS = {
    "units": (False, {}, 256, 64, 4),
    "team": (False, {"LNW_NO_UNITS": "1"}, 72, 0, 2),
    "contact": (True, {}, 72, 0, 3),
    "group": (False, {"LNW_FORCE_GROUP": "1"}, 72, 0, 5),
    "generic": (False, {"LNW_FORCE_GENERIC": "1"}, 72, 0, 1),
}


@pytest.fixture(scope="module")
def grid():
    return np.load(_oracle.GOLDEN + "/grids.npz")["grid100"]


def _game(grid, variant, monkeypatch, E):
    from lnw.batched import BatchedGame
    from lnw.config import Scenario
    contact, knobs, _, epw, _ = VARIANTS[variant]
    for k, v in knobs.items():
        monkeypatch.setenv(k, v)
    g = BatchedGame(E, ["small"] * 4, ["large"] * 4, scenario=Scenario(landing_ops=False), grid=grid,
                    reward_dtype=torch.float64, seed=1234)
    for k in knobs:
        monkeypatch.delenv(k)
    g.set_variant(contact)
    if epw:
        assert g.set_epw(epw) == epw
    return g


def _compare(g, res, oracles, act_after, s, ctx):
    st, es = g.agents(), g.env_state()
    for e, o in enumerate(oracles):
        r = o.step_result
        c = f"{ctx} env {e} step {s}"
        assert np.array_equal(res["obs_blue"][e], r["obs_blue"].astype(np.float32)), f"{c} obs_blue"
        assert np.array_equal(res["obs_red"][e], r["obs_red"].astype(np.float32)), f"{c} obs_red"
        assert np.allclose(res["rew_blue"][e], r["rew_blue"], rtol=0, atol=REW_TOL), f"{c} rew_blue"
        assert np.allclose(res["rew_red"][e], r["rew_red"], rtol=0, atol=REW_TOL), f"{c} rew_red"
        assert res["done"][e] == r["done"], f"{c} done"
        ost, oag = o.env_state(), o.agents()
        assert es["err"][e] == ost["err"], f"{c} err bits {es['err'][e]} vs oracle {ost['err']}"
        assert np.array_equal(np.stack([st["x"][e], st["y"][e]], 1), oag["pos"]), f"{c} pos"
        assert np.array_equal(st["radar"][e], oag["radar"]), f"{c} radar"
        assert np.array_equal(st["alive"][e], oag["alive"]), f"{c} alive"
        assert np.array_equal(st["tl_cnt"][e], oag["tl_cnt"]), f"{c} tl_cnt"
        a_ref = r["actions_after"].astype(act_after.dtype)
        assert np.array_equal(act_after[e], a_ref, equal_nan=True), f"{c} actions after"
    return es


@pytest.mark.parametrize("variant", list(VARIANTS))
def test_crash_fixtures_vs_oracle(grid, variant, monkeypatch):
    """Every reference-pinned crash episode as parallel envs (env e runs case
    e % 9; its own tape and spawns), 4 steps: the raising step and the steps
    after it equal the oracle's, and the raising step carries the bit the
    reference's exception maps to."""
    E = VARIANTS[variant][2]
    g = _game(grid, variant, monkeypatch, E)
    names = [CASES[e % len(CASES)] for e in range(E)]
    tapes = [FX[f"{n}_tape"] for n in names]
    offs = np.concatenate([[0], np.cumsum([len(t) for t in tapes])]).astype(np.int64)
    g.set_tape(np.concatenate(tapes), offs)
    pos = np.array([META[n]["pos"] for n in names], np.int32)
    g.reset(positions=pos[0], pos_per_env=torch.from_numpy(pos))
    oracles = []
    for e, n in enumerate(names):
        o = _oracle.OracleEnv(grid, 4, 4)
        o.set_tape(FX[f"{n}_tape"])
        o.reset([0] * 4 + [1] * 4, pos[e])
        oracles.append(o)
    kinds = np.array([[_oracle.K_F32 if META[n]["dtype"] == "float32" else _oracle.K_F64] * 8 for n in names],
                     np.uint8)
    first_err = {}
    for s in range(4):
        act = np.stack([FX[f"{n}_actions"][s] for n in names])
        at = torch.from_numpy(act).cuda()
        out = g.step(at, torch.from_numpy(kinds).cuda())
        torch.cuda.synchronize()
        assert g.step_kernel() == VARIANTS[variant][4]
        res = {k: v.cpu().numpy() for k, v in out.items()}
        for e, o in enumerate(oracles):
            o.step_result = o.step(act[e], kinds[e].astype(np.int32))
        es = _compare(g, res, oracles, at.cpu().numpy(), s, f"{variant}")
        for e, n in enumerate(names):
            assert es["rng"][e] == oracles[e].env_state()["tape_pos"], f"{variant} env {e} step {s} draws"
            if es["err"][e] and e not in first_err:
                first_err[e] = (s, int(es["err"][e]))
    for e, n in enumerate(names):
        crash = META[n]["crash"]
        if crash is None:
            assert e not in first_err, (n, first_err.get(e))
        else:
            assert first_err.get(e) == (crash["step"], EXC_BIT[crash["exc"]]), (n, first_err.get(e), crash)
    g.close()


@pytest.mark.parametrize("dtype", ["f32", "f64"])
@pytest.mark.parametrize("variant", list(VARIANTS))
def test_nonfinite_action_rows_vs_oracle(grid, variant, dtype, monkeypatch):
    """Random action rows with NaN, +-inf and huge finite entries in every
    component (about 3 % of rows), half the envs at the reference spawns (the
    quiet path, whose test sends non-finite rows to phase S) and half in
    contact, 10 Philox steps: every output, error bit and state field equal to
    the oracle's."""
    from test_gpu_parity import REF_SPAWNS, _melee_positions
    E = VARIANTS[variant][2]
    g = _game(grid, variant, monkeypatch, E)
    pos = np.array([REF_SPAWNS] * E, np.int32)
    pos[E // 2:] = _melee_positions(grid, E - E // 2, 4, 4, seed=11)
    g.reset(positions=pos[0], pos_per_env=torch.from_numpy(pos))
    oracles = []
    for e in range(E):
        o = _oracle.OracleEnv(grid, 4, 4)
        o.set_philox(1234, e)
        o.reset([0] * 4 + [1] * 4, pos[e])
        oracles.append(o)
    rng = np.random.default_rng(5 + (dtype == "f32"))
    bad_vals = np.array([np.nan, np.inf, -np.inf, 1e35, -1e35, 3e38])
    npdt = np.float32 if dtype == "f32" else np.float64
    kind = _oracle.K_F32 if dtype == "f32" else _oracle.K_F64
    flagged = 0
    for s in range(10):
        act = rng.random((E, 8, 4)).astype(npdt)
        hit = rng.random((E, 8)) < 0.03
        comp = rng.integers(0, 4, (E, 8))
        vals = bad_vals[rng.integers(0, len(bad_vals), (E, 8))]
        nonfin = bad_vals[rng.integers(0, 3, (E, 8))]
        for e, a in zip(*np.nonzero(hit)):
            # (a radar action gets NaN / inf only: the build keeps radar in int32, so a
            # finite |round(a0)| >= 2^31 is clamped where the reference keeps a Python int;
            # DESIGN.md, "Crash modes")
            act[e, a, comp[e, a]] = nonfin[e, a] if comp[e, a] == 0 else vals[e, a]
        at = torch.from_numpy(act).cuda()
        out = g.step(at)
        torch.cuda.synchronize()
        res = {k: v.cpu().numpy() for k, v in out.items()}
        for e, o in enumerate(oracles):
            o.step_result = o.step(act[e].astype(np.float64), np.full(8, kind, np.int32))
        es = _compare(g, res, oracles, at.cpu().numpy(), s, f"{variant}/{dtype}")
        flagged = int((es["err"] != 0).sum())
    assert flagged > 0  # the injected rows did raise somewhere
    g.close()
