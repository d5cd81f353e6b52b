"""Run a reference caller unchanged with `from game import Game` bound to the
MI355X facade.

    python -m lnw.run_reference /path/to/reference/main.py false false false
    python -m lnw.run_reference --stub wandb --stub IPython.display ppo_script.py ...

The reference's callers import the environment as `from game import Game`
(main.py:14, ppo.py:6, ddqn.py:6; main.py:18 also does `import game`). Run as
`python main.py`, Python puts the script's own directory at sys.path[0], ahead
of PYTHONPATH, so those imports would find the reference's CPU game.py next to
the script. This launcher stays in one process (no exec, no re-launch):

  1. sys.path becomes [this package's directory, the script's directory, ...]:
     `game` resolves to littoral-naval-warfare-marl_amd/game.py, every other
     reference module (network, ppo, ddqn, ...) still to the script's directory;
  2. `game` is imported here and kept in sys.modules, so a caller that edits
     sys.path later still gets the facade;
  3. cwd becomes the script's directory (the reference reads ./config.json,
     ./red_steps*.csv and the terrain PNG relative to cwd), unless --cwd is given;
  4. sys.argv is [script, args...] and the script runs as __main__ (runpy).

--stub NAME installs an empty module for NAME (and its parents) when NAME does
not import: the reference imports wandb, IPython.display, skimage.draw and
torchviz at top level (game.py:14,19,25, ppo.py:11, network.py:15,22) but its
environment path never calls them.
"""
import argparse
import importlib
import os
import runpy
import sys
import types

PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# attributes the reference reads from its stubbed optional modules at import
_STUB_ATTRS = {"IPython.display": {"clear_output": lambda *a, **k: None},
               "skimage.draw": {"line": None},
               "torchviz": {"make_dot": lambda *a, **k: None}}


def _stub(name):
    try:
        importlib.import_module(name)
        return
    except ImportError:
        pass
    parts = name.split(".")
    for i in range(1, len(parts) + 1):
        mod = ".".join(parts[:i])
        if mod not in sys.modules:
            m = types.ModuleType(mod)
            m.__lnw_stub__ = True
            for k, v in _STUB_ATTRS.get(mod, {}).items():
                setattr(m, k, v)
            sys.modules[mod] = m
            if i > 1:
                setattr(sys.modules[".".join(parts[:i - 1])], parts[i - 1], m)


def bind_game(script_dir):
    """Order sys.path as [package, script_dir, rest] and load the facade as
    the module `game`. Returns the module."""
    drop = {PKG, script_dir, "", "."}
    sys.path[:] = [PKG, script_dir] + [p for p in sys.path if os.path.abspath(p or ".") not in
                                       {os.path.abspath(d or ".") for d in drop}]
    old = sys.modules.get("game")
    if old is not None and os.path.dirname(os.path.abspath(getattr(old, "__file__", "") or "")) != PKG:
        del sys.modules["game"]
    game = importlib.import_module("game")
    from lnw.game import Game
    if game.Game is not Game:
        raise ImportError(f"`game` resolved to {game.__file__}, not the lnw facade")
    return game


def main(argv=None):
    ap = argparse.ArgumentParser(prog="python -m lnw.run_reference", description=__doc__.split("\n")[0])
    ap.add_argument("--stub", action="append", default=[],
                    help="install an empty module NAME when it does not import (repeatable)")
    ap.add_argument("--cwd", default=None, help="working directory (default: the script's directory)")
    ap.add_argument("script")
    ap.add_argument("args", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    script = os.path.abspath(a.script)
    if not os.path.isfile(script):
        ap.error(f"no such script: {a.script}")
    script_dir = os.path.dirname(script)
    for name in a.stub:
        _stub(name)
    bind_game(script_dir)
    os.chdir(a.cwd or script_dir)
    sys.argv = [script] + list(a.args)
    runpy.run_path(script, run_name="__main__")
    return 0


if __name__ == "__main__":
    sys.exit(main())
