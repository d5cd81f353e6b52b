"""The reference's crash modes, pinned (CPU): tests/golden/crash_modes.npz holds
constructed episodes run through the reference itself (make_crash_golden.py),
with the step at which Game.step raised, the exception and the reference line.
The oracle must step every clean step exactly as the reference did, and flag
the raising step with the build's error bit (include/lnw.h LNW_ERRF_*):
ZeroDivisionError in an EW fix (combatant.py:274) -> LNW_ERRF_ZERODIV;
ValueError / OverflowError of round() on a NaN / inf fix (:146), move target
(:470), engagement threshold (:528) or radar action (:558) -> LNW_ERRF_NAN_ROUND.
The GPU path is compared with the oracle on the same episodes, crash steps and
the steps after them included, in tests/test_gpu_crash_modes.py."""
import json

import numpy as np
import pytest

import _oracle

ERRF_ZERODIV, ERRF_NAN_ROUND = 1, 2
EXC_BIT = {"ZeroDivisionError": ERRF_ZERODIV, "ValueError": ERRF_NAN_ROUND,
           "OverflowError": ERRF_NAN_ROUND}


def crash_cases():
    fx = np.load(_oracle.GOLDEN + "/crash_modes.npz")
    return fx, {m["name"]: m for m in json.loads(str(fx["meta"]))}


FX, META = crash_cases()


def oracle_run(grid, m, fx):
    """Steps case m through the oracle; per step (outputs, err bits, tape position)."""
    name = m["name"]
    o = _oracle.OracleEnv(grid, 4, 4)
    o.set_tape(fx[f"{name}_tape"])
    o.reset([0] * 4 + [1] * 4, np.array(m["pos"], np.int32))
    kind = _oracle.K_F32 if m["dtype"] == "float32" else _oracle.K_F64
    out = []
    for a in fx[f"{name}_actions"]:
        r = o.step(a, np.full(8, kind, np.int32))
        st = o.env_state()
        out.append((r, st["err"], st["tape_pos"]))
    return out


@pytest.mark.parametrize("name", sorted(META))
def test_oracle_flags_reference_crash(name):
    grid = np.load(_oracle.GOLDEN + "/grids.npz")["grid100"]
    m = META[name]
    res = oracle_run(grid, m, FX)
    crash = m["crash"]
    clean = m["ok_steps"]
    for s in range(clean):  # the steps the reference completed: identical, no flag
        r, err, tp = res[s]
        assert err == 0, (name, s)
        assert np.array_equal(r["obs_blue"].astype(np.float32), FX[f"{name}_obs_blue"][s]), (name, s)
        assert np.array_equal(r["obs_red"].astype(np.float32), FX[f"{name}_obs_red"][s]), (name, s)
        assert np.allclose(r["rew_blue"], FX[f"{name}_rew_blue"][s], rtol=0, atol=1e-5), (name, s)
        assert np.allclose(r["rew_red"], FX[f"{name}_rew_red"][s], rtol=0, atol=1e-5), (name, s)
        assert r["done"] == FX[f"{name}_done"][s] and tp == FX[f"{name}_tape_pos"][s], (name, s)
    if crash is None:
        assert clean == len(res) and all(e == 0 for _, e, _ in res)
        return
    assert crash["step"] == clean
    err = res[clean][1]
    assert err == EXC_BIT[crash["exc"]], (name, crash, err)


def test_crash_fixture_covers_every_site():
    """The fixture pins one raising site per crash mode the build defines."""
    sites = {(m["crash"]["file"], m["crash"]["line"], m["crash"]["exc"])
             for m in META.values() if m["crash"]}
    assert {("combatant.py", 274, "ZeroDivisionError"), ("combatant.py", 146, "ValueError"),
            ("combatant.py", 470, "ValueError"), ("combatant.py", 470, "OverflowError"),
            ("combatant.py", 528, "ValueError"), ("combatant.py", 528, "OverflowError"),
            ("combatant.py", 558, "ValueError")} <= sites
    assert META["huge_move"]["crash"] is None
