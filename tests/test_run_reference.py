"""The drop-in launcher (lnw.run_reference): a reference caller run through it
gets the MI355X facade from `from game import Game` (main.py:14, ppo.py:6,
ddqn.py:6) even though a game.py sits next to the script, which is where the
reference keeps its CPU game.py and where plain `python main.py` would look
first (sys.path[0] = the script's directory, ahead of PYTHONPATH)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "littoral-naval-warfare-marl_amd")
REF = "/root/reference"

DECOY = "raise ImportError('decoy game.py next to the script was imported')\n"

CALLER = """\
import json, os, sys
from game import Game
import game
import helper
json.dump({"game_module": Game.__module__, "game_file": game.__file__,
           "helper": helper.WHERE, "cwd": os.getcwd(), "argv": sys.argv,
           "config": open("config.json").read()}, open(sys.argv[1], "w"))
"""


def _launch(args, cwd, extra_env=None):
    env = dict(os.environ)
    env["PYTHONPATH"] = PKG
    env.update(extra_env or {})
    return subprocess.run([sys.executable, "-m", "lnw.run_reference"] + args, cwd=cwd,
                          env=env, capture_output=True, text=True, timeout=300)


def _caller_dir(tmp_path):
    d = tmp_path / "ref"
    d.mkdir()
    (d / "game.py").write_text(DECOY)
    (d / "helper.py").write_text("WHERE = 'script dir'\n")
    (d / "config.json").write_text('{"marker": 1}')
    (d / "caller.py").write_text(CALLER)
    return d


def test_launcher_binds_facade_over_decoy(tmp_path):
    d = _caller_dir(tmp_path)
    out = tmp_path / "out.json"
    elsewhere = tmp_path / "elsewhere"
    elsewhere.mkdir()
    # PYTHONPATH also names the decoy's directory: the launcher still wins
    r = _launch([str(d / "caller.py"), str(out), "x"], cwd=str(elsewhere),
                extra_env={"PYTHONPATH": PKG + os.pathsep + str(d)})
    assert r.returncode == 0, r.stderr
    res = json.loads(out.read_text())
    assert res["game_module"] == "lnw.game"
    assert os.path.dirname(os.path.abspath(res["game_file"])) == PKG
    assert res["helper"] == "script dir"          # other modules still from the script's dir
    assert os.path.realpath(res["cwd"]) == os.path.realpath(str(d))
    assert res["argv"] == [str(d / "caller.py"), str(out), "x"]
    assert res["config"] == '{"marker": 1}'


def test_plain_python_gets_the_decoy(tmp_path):
    """Why the launcher exists: the recipe `PYTHONPATH=pkg python caller.py`
    imports the game.py next to the script."""
    d = _caller_dir(tmp_path)
    env = dict(os.environ, PYTHONPATH=PKG)
    r = subprocess.run([sys.executable, str(d / "caller.py"), str(tmp_path / "o.json")],
                       cwd=str(d), env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and "decoy game.py" in r.stderr


def test_launcher_cwd_option_and_missing_script(tmp_path):
    d = _caller_dir(tmp_path)
    other = tmp_path / "other"
    other.mkdir()
    (other / "config.json").write_text('{"marker": 2}')
    out = tmp_path / "out.json"
    r = _launch(["--cwd", str(other), str(d / "caller.py"), str(out)], cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr
    res = json.loads(out.read_text())
    assert res["config"] == '{"marker": 2}' and res["game_module"] == "lnw.game"
    r = _launch([str(tmp_path / "nope.py")], cwd=str(tmp_path))
    assert r.returncode != 0 and "no such script" in r.stderr


@pytest.mark.skipif(not os.path.isdir(REF), reason="needs the reference checkout")
def test_reference_callers_resolve_to_facade(tmp_path):
    """The reference's own ppo.py and ddqn.py, next to the reference's own
    game.py (symlinked into a scratch directory, unchanged), imported by a
    caller run through the launcher: `ppo.Game` and `ddqn.Game` are the
    facade. Their optional imports (wandb, IPython, skimage, torchviz) are
    stubbed because this image lacks them."""
    d = tmp_path / "ref"
    d.mkdir()
    for f in os.listdir(REF):
        if f.endswith((".py", ".json", ".csv", ".png")):
            os.symlink(os.path.join(REF, f), d / f)
    (d / "lnw_check_callers.py").write_text(
        "import json, sys\nimport ppo, ddqn, game\n"
        "json.dump({'ppo': ppo.Game.__module__, 'ddqn': ddqn.Game.__module__,\n"
        "           'game': game.__file__}, open(sys.argv[1], 'w'))\n")
    out = tmp_path / "out.json"
    stubs = []
    for m in ("wandb", "IPython.display", "skimage.draw", "torchviz"):
        stubs += ["--stub", m]
    r = _launch(stubs + [str(d / "lnw_check_callers.py"), str(out)], cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads(out.read_text())
    assert res["ppo"] == "lnw.game" and res["ddqn"] == "lnw.game"
    assert os.path.dirname(os.path.abspath(res["game"])) == PKG
