"""The reference-compatible Game facade (lnw.game) used the way ppo.py / main.py
use game.Game: per-ship get_obs() then step(list of action rows), checked
step by step against the CPU oracle stepping the same environment."""
import random

import numpy as np
import pytest
import torch

import _oracle

pytestmark = pytest.mark.gpu


def _oracle_for(game):
    sc = game.scenario
    o = _oracle.OracleEnv(np.asarray(game.grid, np.uint8), len(game.blue_ships),
                          len(game.red_ships), discrete=sc.discrete, landing_ops=sc.landing_ops,
                          aggressive=sc.tactics == "aggressive", side_blue=sc.side == "blue",
                          trained_red=sc.trained_red, red_aggression=sc.red_aggression)
    return o


@pytest.mark.parametrize("seed,blue_type", [(0, "small"), (1, "small"), (2, "small"), (3, "medium")])
def test_facade_rollout_matches_oracle(seed, blue_type, tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)  # no config.json / PNG here: defaults + packaged grid
    from lnw.game import Game, ShipSpec
    random.seed(seed)
    np.random.seed(seed)
    g = Game()
    g.scenario.landing_ops = False
    g.scenario.n_red_landingship = 0
    blue = [ShipSpec("blue", blue_type, p) for p in [(36, 50), (40, 52), (38, 47), (42, 44)]]
    red = [ShipSpec("red", "large", p) for p in [(58, 55), (60, 60), (62, 52), (57, 64)]]
    state = random.getstate()
    g.reset(4, 4, blue_ships=blue, red_ships=red)
    # replicate the facade's seeds: it draws its Philox seed from `random` at reset
    random.setstate(state)
    seed63 = random.getrandbits(63)
    o = _oracle_for(g)
    o.set_philox(seed63, 0)
    o.reset([_oracle.T_MEDIUM if blue_type == "medium" else 0] * 4 + [1] * 4,
            [s.position for s in blue + red])
    if blue_type == "medium":  # a side of medium ships: 5x5 windows, rows of 4n + 28 (game.py:609)
        assert g.observation_space == 4 * 4 + 28 and g.red_observation_space == 4 * 4 + 52
        assert all(s.speed == 2 for s in g.blue_ships)
    o.set_ducting(g.ducting_factor)
    rng = np.random.default_rng(seed)
    for step in range(25):
        for i, ship in enumerate(g.blue_ships):
            if ship is not None:
                got = ship.get_obs()
                ref = o.observe(i)
                assert np.array_equal(got.astype(np.float32), ref.astype(np.float32)), (step, i)
                assert ship.target_list == o.tlist(i)
        acts = [rng.random(4).astype(np.float32) for _ in range(8)]
        obs, rew, done, cog = g.step(acts)
        r = o.step(np.array(acts, np.float64), np.full(8, _oracle.K_F32, np.int32))
        assert np.array_equal(obs[0].astype(np.float32), r["obs_blue"].astype(np.float32)), step
        np.testing.assert_allclose(rew, r["rew_blue"], rtol=0, atol=1e-5)
        assert done == r["done"]
        if cog is None:
            assert np.isnan(r["cog"])
        else:
            assert abs(cog - r["cog"]) < 1e-5
        st = o.agents()
        for i, ship in enumerate(g.blue_ships + g.red_ships):
            assert (ship is None) == (st["alive"][i] == 0)
            if ship is not None:
                assert ship.position == tuple(st["pos"][i])
                assert ship.missiles == st["missiles"][i]
        if done == 0:
            break
    g.close()


def test_facade_default_reset_and_shapes(tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    from lnw.game import Game
    g = Game()
    g.reset(3, 2)  # shipped config: 3 blue, 2 red + 1 landing ship (random spawn)
    assert len(g.blue_ships) == 3 and len(g.red_ships) == 3
    assert g.red_ships[-1].ship_type == "ls"
    assert g.observation_space == 3 * 4 + 52 and g.red_observation_space == 3 * 4 + 52
    ls = g.red_ships[-1]
    assert ls.position[0] in (98, 99) and 48 <= ls.position[1] <= 56
    obs, rew, done, cog = g.step([np.zeros(4, np.float32)] * 6)
    assert obs.shape == (1, 3, g.observation_space) and len(rew) == 3
    g.close()


def test_facade_analytics_side_channels(tmp_path, monkeypatch):
    """engagements / launch_sites / heatmap / coldmap / blue_ew / red_ew are
    filled from the device analytics logs with the reference's relations:
    every hit is an engagement (blue_/red_engagements count them), missile hits
    are launch sites, the heatmap counts the trained side's missile hits."""
    monkeypatch.chdir(tmp_path)
    from lnw.game import Game, ShipSpec
    random.seed(4)
    np.random.seed(4)
    g = Game()
    g.scenario.landing_ops = False
    g.scenario.n_red_landingship = 0
    blue = [ShipSpec("blue", "small", p) for p in [(36, 50), (40, 52), (38, 47), (42, 44)]]
    red = [ShipSpec("red", "large", p) for p in [(58, 55), (60, 60), (62, 52), (57, 64)]]
    rng = np.random.default_rng(4)
    for ep in range(6):
        g.reset(4, 4, blue_ships=blue, red_ships=red)
        for step in range(40):
            for ship in g.blue_ships:
                if ship is not None:
                    ship.get_obs()
            obs, rew, done, cog = g.step([rng.random(4).astype(np.float32) for _ in range(8)])
            if done == 0:
                break
    # the engagement counters accumulate across resets, as the reference's do
    assert len(g.engagements) == g.blue_engagements + g.red_engagements > 0
    missile = [e for e in g.engagements if e[2] > 0]
    assert len(g.launch_sites["blue"]) + len(g.launch_sites["red"]) == len(missile)
    assert g.heatmap.sum() == len(g.launch_sites["blue"]) == g.coldmap.sum()
    assert len(g.blue_ew) + len(g.red_ew) > 0
    for (ox, oy), (fx, fy) in g.blue_ew + g.red_ew:
        assert 0 <= ox < 100 and 0 <= oy < 100
    g.close()


@pytest.mark.parametrize("trained_red", [True, False])
def test_facade_discrete_ddqn_pattern(trained_red, tmp_path, monkeypatch):
    """DISCRETE mode through the facade the way ddqn.py:296-396 drives it:
    get_obs() per live ship, then step() on a list of 3-int rows [rad, msl,
    mov] (mov = value_to_coordinates index 0..49, combatant.py:689-704; [0, 0, 0]
    for sunk ships). With untrained red the step rewrites red salvo entries in
    place (game.py:375-379): the list element becomes the drawn float and
    round() of it decides the engagement; the facade hands it back in the
    caller's lists. Every step checked against the oracle in DISCRETE mode
    (K_PYFLOAT row kind = list rows: the rewrite is stored untruncated)."""
    monkeypatch.chdir(tmp_path)
    from lnw.game import Game, ShipSpec
    random.seed(11)
    np.random.seed(11)
    g = Game()
    sc = g.scenario
    sc.discrete, sc.landing_ops, sc.n_red_landingship = True, False, 0
    sc.trained_red = trained_red
    blue = [ShipSpec("blue", "small", p) for p in [(36, 50), (40, 52), (38, 47)]]
    red = [ShipSpec("red", "large", p) for p in [(50, 55), (52, 60), (54, 52)]]
    state = random.getstate()
    g.reset(3, 3, blue_ships=blue, red_ships=red)
    assert g.observation_space == 3 * 4 + 52
    random.setstate(state)
    seed63 = random.getrandbits(63)
    o = _oracle_for(g)
    o.set_philox(seed63, 0)
    o.reset([0] * 3 + [1] * 3, [s.position for s in blue + red])
    o.set_ducting(g.ducting_factor)
    rng = np.random.default_rng(5)
    mutated = 0
    for step in range(40):
        for i, ship in enumerate(g.blue_ships + g.red_ships):
            if ship is not None:
                got = ship.get_obs()
                assert np.array_equal(got.astype(np.float32), o.observe(i).astype(np.float32)), (step, i)
        acts = [[int(rng.integers(0, 2)), int(rng.integers(0, 5)), int(rng.integers(0, 50))]
                if ship is not None else [0, 0, 0] for ship in g.blue_ships + g.red_ships]
        sent = [list(r) for r in acts]
        obs, rew, done, cog = g.step(acts)
        r = o.step(np.array([row + [0] for row in sent], np.float64),
                   np.full(6, _oracle.K_PYFLOAT, np.int32))
        assert obs.shape == (1, 3, g.observation_space)
        assert np.array_equal(obs[0].astype(np.float32), r["obs_blue"].astype(np.float32)), step
        np.testing.assert_allclose(rew, r["rew_blue"], rtol=0, atol=1e-5)
        assert done == r["done"]
        # the in-place salvo rewrite reaches the caller's rows as a float
        after = r["actions_after"]
        for a in range(6):
            assert acts[a][1] == after[a, 1], (step, a)
            if acts[a][1] != sent[a][1]:
                assert isinstance(acts[a][1], float) and 0.0 <= acts[a][1] < 1.0
        mutated += sum(acts[a][1] != sent[a][1] for a in range(3, 6))
        st = o.agents()
        for i, ship in enumerate(g.blue_ships + g.red_ships):
            assert (ship is None) == (st["alive"][i] == 0)
            if ship is not None:
                assert ship.position == tuple(st["pos"][i])
        if done == 0:
            break
    if not trained_red:
        assert mutated > 0
    g.close()


def test_facade_visualize_and_coa_path(tmp_path, monkeypatch):
    """main.py:332 / 350 call env.visualize_grid() and env.visualize_heatmap()
    at the end of the test loop: both exist, keep the reference's side effects
    (imagen counter, engagements cleared, the reset inside visualize_heatmap)
    and write images. coa_path collects end-of-episode positions
    (game.py:489-498)."""
    monkeypatch.chdir(tmp_path)
    from lnw.game import Game
    random.seed(2)
    np.random.seed(2)
    g = Game()
    g.reset(3, 2)
    for s in range(45):
        obs, rew, done, cog = g.step([np.random.random(4).astype(np.float32) for _ in range(6)])
        if done == 0:
            break
    # the episode ends on done == 0 or at step episode_steps - 1: one coa entry per live ship
    assert len(g.coa_path["blue"]) + len(g.coa_path["red"]) + len(g.coa_path["ls"]) > 0
    g.engagements.append(((10, 10), (12, 12), 2))
    g.visualize_grid(path=str(tmp_path))
    assert g.imagen == 1 and g.engagements == []
    assert (tmp_path / "imagen0.png").exists()
    g.visualize_heatmap(g.heatmap, g.coldmap, path=str(tmp_path))
    assert (tmp_path / "heatmap.png").exists()
    assert g.steps_done == 0  # visualize_heatmap resets the game first (game.py:752)
    g.close()


def test_facade_visualize_medium_fleet(tmp_path, monkeypatch):
    """visualize_grid with a medium side (game.py:649-650, 659-660: medium
    combatants drawn at marker size 6) and a red LandingShip with its landing
    spot (game.py:663-666), after a few steps of main.py's test loop."""
    monkeypatch.chdir(tmp_path)
    from lnw.game import Game, ShipSpec
    random.seed(6)
    np.random.seed(6)
    g = Game()
    g.scenario.landing_ops, g.scenario.n_red_landingship = True, 1
    blue = [ShipSpec("blue", "medium", p) for p in [(36, 50), (40, 52), (38, 47)]]
    red = [ShipSpec("red", "large", p) for p in [(58, 55), (60, 60)]]
    g.reset(3, 2, blue_ships=blue, red_ships=red)   # + the scenario's landing ship
    assert [s.ship_type for s in g.blue_ships] == ["medium"] * 3
    assert g.red_ships[-1].ship_type == "ls"
    assert g.red_ships[-1].landing_spot == g.red_ships[-1].landing_zone
    n = len(g.blue_ships) + len(g.red_ships)
    for s in range(5):
        g.step([np.random.random(4).astype(np.float32) for _ in range(n)])
    g.visualize_grid(path=str(tmp_path))
    assert g.imagen == 1 and (tmp_path / "imagen0.png").exists()
    g.close()


_LAUNCHED = """\
import json, random, sys
import numpy as np
random.seed(3)
np.random.seed(3)
from game import Game
g = Game()
g.reset(3, 2)
rng = np.random.default_rng(3)
out = []
for s in range(12):
    for ship in g.blue_ships:
        if ship is not None:
            ship.get_obs()
    obs, rew, done, cog = g.step([rng.random(4).astype(np.float32) for _ in range(6)])
    out.append([obs.tolist(), rew, done, cog, type(g).__module__])
    if done == 0:
        break
g.close()
json.dump(out, open(sys.argv[1], "w"))
"""


def test_launcher_runs_caller_on_gpu(tmp_path, monkeypatch):
    """A caller script next to a decoy game.py that raises on import, run
    through `python -m lnw.run_reference`: it steps the
    HIP facade, and its outputs equal the same loop run in-process with the
    same seeds."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    pkg = os.path.join(root, "littoral-naval-warfare-marl_amd")
    d = tmp_path / "ref"
    d.mkdir()
    (d / "game.py").write_text("raise ImportError('decoy game.py imported')\n")
    (d / "caller.py").write_text(_LAUNCHED)
    out = tmp_path / "out.json"
    env = dict(os.environ, PYTHONPATH=pkg)
    r = subprocess.run([sys.executable, "-m", "lnw.run_reference", str(d / "caller.py"), str(out)],
                       cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    got = json.loads(out.read_text())
    monkeypatch.chdir(d)
    ns = {"__name__": "inproc"}
    monkeypatch.setattr(sys, "argv", ["caller.py", str(tmp_path / "in.json")])
    src = _LAUNCHED.replace("from game import Game", "from lnw.game import Game")
    exec(compile(src, "caller_inproc", "exec"), ns)
    want = json.loads((tmp_path / "in.json").read_text())
    assert len(got) == len(want) > 0
    for a, b in zip(got, want):
        assert a[4] == "lnw.game"
        assert a[:4] == b[:4]
