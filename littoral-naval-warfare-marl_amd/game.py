"""Drop-in module for the reference's `from game import Game` (ppo.py:6,
ddqn.py:6, main.py:14): put littoral-naval-warfare-marl_amd/ on sys.path ahead
of the reference directory. The Game it exports steps on the MI355X."""
from lnw.game import Game, ShipProxy, ShipSpec  # noqa: F401
