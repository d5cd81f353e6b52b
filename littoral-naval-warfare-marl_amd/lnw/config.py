"""Scenario configuration: the reference's config.json keys that change the step
semantics (game.py:33-53, combatant.py:23-38), mapped onto the C-ABI's
lnw_params struct."""
import json
import os
from dataclasses import dataclass, asdict

from ._abi import Params


@dataclass
class Scenario:
    discrete: bool = False          # overall.discrete
    landing_ops: bool = True        # overall.landing_ops
    coa_path: bool = True           # overall.coa_path (game.py:489-498, facade only)
    tactics: str = "aggressive"     # overall.tactics
    side: str = "blue"              # environment_setup.side
    trained_red: bool = True        # environment_setup.trained_red
    red_aggression: float = 0.4     # environment_setup.red_aggression
    movement_threshold: int = 74    # environment_setup.movement_threshold
    ew_threshold: int = 70          # environment_setup.ew_threshold
    n_blue: int = 3                 # environment_setup.n_blue
    n_red: int = 2                  # environment_setup.n_red
    n_red_landingship: int = 1      # environment_setup.n_red_landingship
    episode_steps: int = 40         # hyperparameters.episode_steps
    landing_zone: tuple = (14, 82)  # game.py:590
    # build-side knobs
    auto_reset: bool = False
    los_mode: int = 0               # 0 LOS table, 1 ray march, 2 table + reference LOS work
    move_mode: int = 0              # 0 move table, 1 direct A*

    @classmethod
    def from_config(cls, path="config.json", **over):
        with open(path) as f:
            cfg = json.load(f)
        ov = cfg.get("overall", {})
        es = cfg.get("environment_setup", {})
        hp = cfg.get("hyperparameters", {})
        s = cls(discrete=bool(ov.get("discrete", False)),
                landing_ops=bool(ov.get("landing_ops", True)),
                coa_path=bool(ov.get("coa_path", True)),
                tactics=ov.get("tactics", "aggressive"), side=es.get("side", "blue"),
                trained_red=bool(es.get("trained_red", True)),
                red_aggression=float(es.get("red_aggression", 0.4)),
                movement_threshold=int(es.get("movement_threshold", 74)),
                ew_threshold=int(es.get("ew_threshold", 70)),
                n_blue=int(es.get("n_blue", 3)), n_red=int(es.get("n_red", 2)),
                n_red_landingship=int(es.get("n_red_landingship", 1)),
                episode_steps=int(hp.get("episode_steps", 40)))
        for k, v in over.items():
            setattr(s, k, v)
        return s

    @classmethod
    def from_config_or_default(cls, path="config.json", **over):
        if os.path.exists(path):
            return cls.from_config(path, **over)
        s = cls()
        for k, v in over.items():
            setattr(s, k, v)
        return s

    def params(self):
        return Params(int(self.discrete), int(self.landing_ops),
                      int(self.tactics == "aggressive"), int(self.side == "blue"),
                      int(self.trained_red), int(self.movement_threshold),
                      int(self.ew_threshold), int(self.landing_zone[0]),
                      int(self.landing_zone[1]), float(self.red_aggression),
                      int(self.episode_steps), int(self.auto_reset), int(self.los_mode),
                      int(self.move_mode))

    def asdict(self):
        return asdict(self)
