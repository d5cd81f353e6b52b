"""Reference-compatible Game facade over the HIP step (one environment).

Drop-in for `from game import Game` in the reference's ppo.py:6, ddqn.py:6 and
main.py:14 (valauri/Littoral-Naval-Warfare-MARL game.py:106-626). It keeps the
attributes and call signatures callers use (game.py:107-158, 298-525, 528-613;
ship.get_obs()/target_list, combatant.py:90-233) while every step, observation
and reset runs through liblnw.so on the GPU (BatchedGame with E=1).

Differences from the reference, by design:
  * in-step random draws come from Philox keyed by a seed drawn from Python's
    `random` at reset (the reference calls `random` directly); reset-time draws
    (ducting beta(1,3) from numpy's global RNG, landing-ship spawns from
    `random.randint`) use the same global generators as the reference;
  * observations are float32 values returned in float64 arrays; rewards and
    the cog distance are the float64 values (lnw_set_reward_dtype);
  * the analytics side channels (engagements, launch_sites, heatmap / coldmap,
    blue_ew / red_ew, coa_path) are filled from the device logs after every
    step and get_obs;
  * visualize_grid / visualize_heatmap (game.py:628-890) draw with matplotlib
    when it imports (Agg backend without a display) and keep the reference's
    side effects (imagen counter, engagements cleared, the reset before the
    heatmap); without matplotlib they only apply those side effects.
"""
import csv
import os
import random

import numpy as np
import torch

from . import _abi
from .batched import BatchedGame, default_grid
from .config import Scenario

_TYPES = {"small": 0, "large": 1, "ls": 2, "medium": 3}
_NAMES = {0: "small", 1: "large", 2: "ls", 3: "medium"}
_DEFAULT_BLUE = {2: [(6, 61), (10, 81)], 3: [(6, 61), (10, 81), (8, 70)],
                 4: [(6, 61), (10, 81), (8, 70), (11, 58)]}   # game.py:551-556
_LZ = (14, 82)                                                  # game.py:590


def _coa_path_on(sc):
    return getattr(sc, "coa_path", True)


def _pyplot():
    """matplotlib.pyplot with a non-interactive backend when there is no
    display; None when matplotlib is not installed."""
    try:
        import matplotlib
        if not os.environ.get("DISPLAY"):
            matplotlib.use("Agg")
        import matplotlib.pyplot as plt
        return plt
    except ImportError:
        return None


def _circle(centre, radius):
    from matplotlib.patches import Circle
    return Circle(centre, radius, alpha=0.2, edgecolor=None)


class ShipSpec:
    """A ship to hand to Game.reset(blue_ships=..., red_ships=...) (the
    reference passes Combatant/LandingShip objects; anything with `ship_type`
    and `position` works)."""

    def __init__(self, side, ship_type, position):
        self.side, self.ship_type, self.position = side, ship_type, tuple(position)


class ShipProxy:
    """A live ship slot: the attributes callers read, backed by device state."""

    def __init__(self, game, index, side, ship_type):
        self._g = game
        self._i = index
        self.side = side
        self.ship_type = ship_type
        self.speed = 2 if ship_type in ("ls", "medium") else 3   # combatant.py:64
        self.line_of_sight = 4
        self.radar_coverage = 20
        self.missile_range = 60
        self.mast_height = 15 if ship_type == "small" else 30
        self.rcs = 0.7 if ship_type == "small" else (0.9 if ship_type == "ls" else 1)
        self.environment = game
        self.n_actions = game.action_space
        self.n_obs = game.observation_space
        self.landing_zone = _LZ if ship_type == "ls" else None
        # game.py:665 reads `landing_spot` (LandingShip stores the same cell as
        # landing_zone, landingship.py:68; the reference's drawing of a red
        # LandingShip would raise AttributeError there)
        self.landing_spot = self.landing_zone
        self.replenishment_points = (game.blue_replenishment_points if side == "blue"
                                     else game.red_replenishment_points)

    def _st(self, key):
        return self._g._state()[key][self._i]

    @property
    def position(self):
        st = self._g._state()
        return (int(st["x"][self._i]), int(st["y"][self._i]))

    @property
    def radar_transmission(self):
        return int(self._st("radar"))

    @property
    def missiles(self):
        return int(self._st("missiles"))

    @property
    def steps_done(self):
        return int(self._st("steps_done"))

    @property
    def distance_to_landing_zone(self):
        return float(self._st("dist_lz"))

    @property
    def target_list(self):
        return list(self._g._tlists()[self._i])

    def get_obs(self):
        """ship.get_obs() (combatant.py:90-233): refreshes this ship's target
        list (RNG draws included) and returns its observation vector."""
        return self._g._observe_one(self._i)

    def __repr__(self):
        return f"<{self.side} {self.ship_type} @ {self.position}>"


class Game:
    """game.py:106 Game, stepped by liblnw.so."""

    def __init__(self, config_path="config.json", device=0):
        self.scenario = Scenario.from_config_or_default(config_path)
        sc = self.scenario
        self.device = device
        self.grid_size = 100
        self.grid = np.zeros((self.grid_size, self.grid_size))
        self.blue_ships = []
        self.red_ships = []
        self.blue_replenishment_points = [(6, 76), (13, 86)]
        self.red_replenishment_points = [(98, 40)]
        self.num_blue = sc.n_blue
        self.num_red = sc.n_red
        self.beta = np.random.beta(1, 3)
        self.ducting_factor = 1 + self.beta
        self.imagen = 0
        self.red_ew, self.blue_ew, self.engagements = [], [], []
        self.blue, self.red = [], []
        self.steps_done = 0
        self.action_space = 4
        self.observation_space = 60 if not sc.discrete else 50
        self.blue_movement = 3
        self.red_movement = 3
        self.red_observation_space = 60
        self.red1_actions, self.red2_actions, self.red3_actions = [], [], []
        self.red_victory = 0
        self.blue_victory = 0
        self.blue_engagements = 0
        self.red_engagements = 0
        self.red_landing_ships = 0 if not sc.landing_ops else sc.n_red_landingship
        self.heatmap = np.zeros((100, 100))
        self.coldmap = np.zeros((100, 100))
        self.coa_path = {"blue": [], "red": [], "ls": []}
        self.launch_sites = {"blue": [], "red": []}
        self.neutralized_units = {"blue": [], "red": []}
        self.n_blue_left = 0
        self.n_red_left = 0
        self._g = None
        self._key = None
        self._cache = None
        self._tl_cache = None
        self._all = []

    # ------------------------------------------------------------------ reset
    def define_red_actions(self, lst, file):
        """game.py:174-182"""
        path = os.path.join(os.getcwd(), file)
        if not os.path.exists(path):
            return
        with open(path, "r") as f:
            for row in csv.reader(f):
                lst.append([float(c) for c in row])

    def define_grid_from_image(self, image_path, grid_size):
        """game.py:616-626 (PIL LANCZOS resize + grayscale); falls back to the
        packaged grid produced by exactly that pipeline."""
        if os.path.exists(image_path):
            from PIL import Image
            img = Image.open(image_path).resize((grid_size, grid_size), Image.LANCZOS).convert("L")
            self.grid = np.asarray(img)
        else:
            self.grid = default_grid(grid_size)

    def reset(self, n_blue, n_red, grid=None, blue_ships=None, red_ships=None):
        sc = self.scenario
        self.steps_done = 0
        self.imagen = 0
        self.ducting_factor = 1 + np.random.beta(1, 3)          # game.py:531
        self.blue_victory = 0
        self.red_victory = 0
        if n_red == 2:
            self.define_red_actions(self.red1_actions, "red_steps.csv")
            self.define_red_actions(self.red2_actions, "red_steps2.csv")
        elif n_red == 3:
            self.define_red_actions(self.red1_actions, "red_steps.csv")
            self.define_red_actions(self.red2_actions, "red_steps2.csv")
            self.define_red_actions(self.red3_actions, "red_steps3.csv")
        if grid is None:
            self.define_grid_from_image("balt_mod_400x400_2.png", 100)
        else:
            self.grid = grid
        if blue_ships is None:
            if n_blue not in _DEFAULT_BLUE:
                raise UnboundLocalError("local variable 'blue_pos' referenced before assignment")
            blue = [("small", p) for p in _DEFAULT_BLUE[n_blue]]
        else:
            blue = [(s.ship_type, tuple(s.position)) for s in blue_ships]
        if red_ships is None:
            rpos = [(98, 48), (98, 52)]
            if n_red == 3 and sc.n_red_landingship == 0:
                rpos.append((98, 56))
            red = [("large", p) for p in rpos]
        else:
            red = [(s.ship_type, tuple(s.position)) for s in red_ships]
        for _ in range(sc.n_red_landingship):                     # game.py:587-591
            xs, ys = random.randint(98, 99), random.randint(48, 56)
            red.append(("ls", (xs, ys)))
        self.num_blue, self.num_red = len(blue), len(red)
        types = [_TYPES[t] for t, _ in blue + red]
        grid_arr = np.ascontiguousarray(np.asarray(self.grid), np.uint8)
        key = (tuple(types), len(blue), grid_arr.shape, grid_arr.tobytes().__hash__())
        if self._g is None or key != self._key:
            if self._g is not None:
                self._g.close()
            self._g = BatchedGame(1, [_NAMES[t] for t in types[:len(blue)]],
                                  [_NAMES[t] for t in types[len(blue):]], scenario=sc,
                                  device=self.device, grid=grid_arr, reward_dtype=torch.float64)
            self._g.enable_analytics(eng_cap=4096, ew_cap=4096, maps=False)
            self._key = key
        g = self._g
        g.set_rng(random.getrandbits(63))
        g.reset(positions=[p for _, p in blue + red])
        g.set(_abi.F_DUCT, torch.tensor([self.ducting_factor], dtype=torch.float64))
        self._all = [ShipProxy(self, a, "blue" if a < len(blue) else "red", t)
                     for a, (t, _) in enumerate(blue + red)]
        self.blue_ships = self._all[:len(blue)]
        self.red_ships = self._all[len(blue):]
        ms_b = max(s.speed for s in self.blue_ships)
        ms_r = max(s.speed for s in self.red_ships)
        self.blue_movement = ms_b * 2 + 1
        self.red_movement = ms_r * 2 + 1
        # game.py:609-610: 4 n + (2 * fastest speed + 1)^2 + 3 (the 7x7 window
        # unless the side is all medium ships: the rows the kernel writes)
        self.observation_space = self._g.Db
        self.red_observation_space = self._g.Dr
        for s in self._all:
            s.n_obs = self.observation_space
        self.n_blue_left = len(self.blue_ships)
        self.n_red_left = len(self.red_ships)
        self._invalidate()

    # ------------------------------------------------------------------- step
    def _invalidate(self):
        self._cache = None
        self._tl_cache = None

    def _state(self):
        if self._cache is None:
            st = self._g.agents()
            self._cache = {k: v[0] for k, v in st.items()}
        return self._cache

    def _tlists(self):
        if self._tl_cache is None:
            self._tl_cache = self._g.tlists(0)
        return self._tl_cache

    def _pull_analytics(self):
        """Append the step's / observe's analytics records to the reference's
        side channels: engagements, launch_sites, heatmap / coldmap (the side
        being trained, combatant.py:640-657) and blue_ew / red_ew (:146-150)."""
        eng, ew = self._g.drain_analytics()
        trained = 0 if self.scenario.side == "blue" else 1
        for _, _, side, sx, sy, tx, ty, msl in eng.tolist():
            self.engagements.append(((sx, sy), (tx, ty), msl))
            if msl > 0:
                if side == trained:
                    self.heatmap[sx, sy] += 1
                    self.coldmap[tx, ty] += 1
                self.launch_sites["blue" if side == 0 else "red"].append((sx, sy))
        for _, _, side, ox, oy, fx, fy in ew.tolist():
            (self.blue_ew if side == 0 else self.red_ew).append(((ox, oy), (fx, fy)))

    def _observe_one(self, a):
        ob, orr = self._g.observe(a)
        self._pull_analytics()
        self._invalidate()
        nb = self._g.nb
        row = ob[0, a] if a < nb else orr[0, a - nb]
        return row.double().cpu().numpy()

    def step(self, action):
        """game.py:298-525 -> (obs (1, n, D) float64, rewards list, done, cog|None)."""
        g = self._g
        A = g.A
        rows = [action[a] for a in range(A)]
        live0 = [s is not None for s in self.blue_ships + self.red_ships]
        if self.scenario.discrete:
            # an integer ndarray keeps integer semantics (the salvo rewrite of
            # game.py:379 truncates); list rows (ddqn.py:396) hold Python numbers
            # and take the rewritten float as is: float64 buffer
            int_array = isinstance(action, np.ndarray) and action.dtype.kind in "iu"
            buf = np.zeros((1, A, 4), np.int32 if int_array else np.float64)
            for a, r in enumerate(rows):
                v = np.asarray(r).reshape(-1)[:4]
                buf[0, a, :len(v)] = [int(x) for x in v]
            t = torch.from_numpy(buf).cuda(self.device)
            out = g.step(t)
            kinds = None
        else:
            buf = np.zeros((1, A, 4), np.float64)
            kinds = np.zeros((1, A), np.uint8)
            for a, r in enumerate(rows):
                arr = np.asarray(r, dtype=np.float64).reshape(-1)[:4]
                buf[0, a, :len(arr)] = arr
                if isinstance(r, np.ndarray) and r.dtype == np.float32:
                    kinds[0, a] = _abi.LNW_KIND_F32
                elif isinstance(r, np.ndarray):
                    kinds[0, a] = _abi.LNW_KIND_F64
                else:
                    kinds[0, a] = _abi.LNW_KIND_PYFLOAT
            t = torch.from_numpy(buf).cuda(self.device)
            out = g.step(t, torch.from_numpy(kinds))
        torch.cuda.synchronize(self.device)
        self._pull_analytics()
        after = t.cpu().numpy()[0]
        if not self.scenario.trained_red:                          # game.py:379 mutation
            for a in range(g.nb, A):
                if after[a, 1] != buf[0, a, 1]:
                    try:
                        rows[a][1] = after[a, 1].item()
                    except TypeError:
                        pass
        side_blue = self.scenario.side == "blue"
        obs = (out["obs_blue"] if side_blue else out["obs_red"]).double().cpu().numpy()
        rew = (out["rew_blue"] if side_blue else out["rew_red"]).double().cpu().numpy()[0]
        done = int(out["done"].cpu().numpy()[0])
        cog = float(out["cog"].cpu().numpy()[0])
        self._invalidate()
        st = self._state()
        alive = st["alive"]
        self.blue_ships = [s if alive[i] else None for i, s in enumerate(self._all[:g.nb])]
        self.red_ships = [s if alive[g.nb + i] else None for i, s in enumerate(self._all[g.nb:])]
        es = g.env_state()
        self.n_blue_left = int(es["n_blue_left"][0])
        self.n_red_left = int(es["n_red_left"][0])
        self.blue_victory = int(es["blue_victory"][0])
        self.red_victory = int(es["red_victory"][0])
        self.blue_engagements = int(es["blue_engagements"][0])
        self.red_engagements = int(es["red_engagements"][0])
        self.steps_done = int(es["steps_done"][0])
        if _coa_path_on(self.scenario) and (done == 0 or
                                           self.steps_done == self.scenario.episode_steps - 1):
            # game.py:489-498: positions after the step of every ship that was
            # not None when it began (ships sunk this step included)
            for a, shp in enumerate(self._all):
                if live0[a]:
                    key = "blue" if a < g.nb else ("ls" if shp.ship_type == "ls" else "red")
                    self.coa_path[key].append(shp.position)
        return obs, [float(r) for r in rew], done, (None if np.isnan(cog) else cog)

    def get_grid(self):
        return self.grid

    # ---------------------------------------------------------- visualisation
    def visualize_grid(self, show=False, path=None, animation=False):
        """game.py:628-748: terrain, ships, radar circles, replenishment points,
        EW fixes and engagements of the current state. Side effects kept: the
        engagement list is cleared and `imagen` counts the frames. The image
        goes to `path/imagen<k>.png` when a path is given."""
        plt = _pyplot()
        if plt is not None:
            fig, ax = plt.subplots()
            ax.set_aspect("equal")
            ax.imshow(np.asarray(self.grid), cmap="gray", origin="upper",
                      extent=[-0.5, 100 - 0.5, -0.5, 100 - 0.5])
            # game.py:643-666: combatants as circles sized by type (small 4,
            # medium 6, large 8); a red LandingShip as a square with its
            # landing spot as a star (the reference draws no blue LandingShip)
            marks = {"small": 4, "medium": 6, "large": 8}
            for col, ships in (("b", self.blue_ships), ("r", self.red_ships)):
                for shp in ships:
                    if shp is None:
                        continue
                    x, y = shp.position
                    if shp.ship_type in marks:
                        ax.plot(y, 100 - x - 1, col + "o", markersize=marks[shp.ship_type])
                    elif shp.ship_type == "ls" and col == "r":
                        ax.plot(y, 100 - x - 1, "rs", markersize=6)
                        lx, ly = shp.landing_spot
                        ax.plot(ly, 100 - lx - 1, "r*", markersize=6)
                for shp in ships:
                    if shp is None:
                        continue
                    x, y = shp.position
                    if shp.radar_transmission == 1:
                        r = ((np.sqrt((4 / 3) * 6370 * 2) * (np.sqrt(shp.mast_height / 1000)
                                                             + np.sqrt(30 / 1000))) / 5
                             * self.ducting_factor)
                        ax.add_patch(_circle((y, 100 - x - 1), r))
            for col, pts in (("bv", self.blue_replenishment_points),
                             ("rv", self.red_replenishment_points)):
                for px, py in pts:
                    ax.plot(py, 100 - px - 1, col, markersize=5)
            for col, lst in (("b-", self.blue_ew), ("r-", self.red_ew)):
                for (ox, oy), (fx, fy) in lst:
                    ax.plot([oy, fy], [100 - ox - 1, 100 - fx - 1], col)
            for (lx, ly), (tx, ty), msl in self.engagements:
                ax.plot(ty, 100 - tx - 1, "X", color="orange")
                ax.plot([ly, ty], [100 - lx - 1, 100 - tx - 1], "-",
                        color="yellow" if msl == 0 else "orange")
            ax.set_xlim(-0.5, 100.5)
            ax.set_ylim(-0.5, 100.5)
            ax.set_title("Game Grid")
            if show:
                plt.show()
            if path is not None:
                fig.savefig(os.path.join(path, f"imagen{self.imagen}.png"))
            plt.close(fig)
        self.engagements.clear()
        self.imagen += 1

    def visualize_heatmap(self, heatmap, coldmap, path=None):
        """game.py:750-890: resets the game (as the reference does first), then
        draws the terrain with the missile-launch heatmap and the launch-site /
        end-position cluster centres (KMeans, when scikit-learn imports)."""
        self.reset(self.num_blue, self.num_red)
        plt = _pyplot()
        if plt is None:
            return
        fig = plt.figure()
        plt.imshow(np.asarray(self.grid), cmap="gray", origin="upper",
                   extent=[-0.5, 100 - 0.5, -0.5, 100 - 0.5])
        if np.max(heatmap) > 0:
            plt.imshow(heatmap, cmap="hot", alpha=0.25, origin="upper",
                       extent=[-0.5, 100 - 0.5, -0.5, 100 - 0.5])
        try:
            from sklearn.cluster import KMeans
        except ImportError:
            KMeans = None
        for key in ("blue", "red", "ls"):
            pts = self.launch_sites.get(key, []) if key != "ls" else []
            n = self.num_blue if key == "blue" else (self.num_red if key == "red" else 1)
            if len(pts) < n:
                pts = self.coa_path[key]
            if KMeans is None or len(pts) < max(n, 1):
                continue
            centres = KMeans(n_clusters=max(n, 1), random_state=0,
                             n_init="auto").fit(np.asarray(pts)).cluster_centers_
            for cx, cy in centres:
                plt.plot(cy, 100 - cx - 1, "yo" if key != "ls" else "rs", markersize=25,
                         alpha=0.2)
        if np.max(heatmap) > 0:
            plt.colorbar()
        if path is not None:
            fig.savefig(os.path.join(path, "heatmap.png"))
        plt.show()
        plt.close(fig)

    def close(self):
        if self._g is not None:
            self._g.close()
            self._g = None
