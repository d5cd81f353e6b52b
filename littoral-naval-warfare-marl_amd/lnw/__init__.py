"""lnw — MI355X-native batched littoral naval-warfare environment step.

Drop-in for the environment of valauri/Littoral-Naval-Warfare-MARL
(game.py / combatant.py / landingship.py): hand-written HIP kernels for gfx950
behind the C-ABI in include/lnw.h, driven from PyTorch-ROCm.

    from lnw import BatchedGame      # batched surface (E envs per GPU)
    from lnw.game import Game        # reference-compatible Game facade
"""
from ._abi import LnwError, load  # noqa: F401
from .config import Scenario  # noqa: F401


def __getattr__(name):
    if name == "BatchedGame":
        from .batched import BatchedGame
        return BatchedGame
    raise AttributeError(name)
