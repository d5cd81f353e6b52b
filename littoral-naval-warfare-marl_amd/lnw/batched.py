"""BatchedGame: E independent reference games stepped together on one MI355X.

Host side of the drop-in boundary: PyTorch-ROCm tensors for the caller-owned
buffers (actions, observations, rewards) and the C-ABI (include/lnw.h) for
everything else. One instance = one lnw handle = one device (one process per
GPU for multi-GPU; shard envs by global id, see lnw.shard).

Reference correspondence (valauri/Littoral-Naval-Warfare-MARL):
  reset()    Game.reset            game.py:528-613
  step()     Game.step             game.py:298-525
  observe()  Combatant.get_obs     combatant.py:90-233 (side effects included)
"""
import ctypes as C
import os

import numpy as np
import torch

from . import _abi
from ._abi import (F_ALIVE, F_DIST_LZ, F_DUCT, F_ENV, F_ERR, F_MISSILES, F_MKIND, F_POS,
                   F_RADAR, F_RNG, F_STEPS, F_TL, F_TL_CNT, F_TYPE, LNW_ACT_F32, LNW_ACT_F64,
                   LNW_ACT_I32, LNW_LARGE, LNW_LS, LNW_MEDIUM, LNW_RNG_PHILOX, LNW_RNG_TAPE, LNW_SMALL,
                   Spawn,
                   check)
from .config import Scenario

DATA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data")
TYPE_CODES = {"small": LNW_SMALL, "large": LNW_LARGE, "ls": LNW_LS, "medium": LNW_MEDIUM}


def side_obs_dim(types):
    """Observation row length of a side (game.py:595-610): 4 per ship plus the
    movement window of its fastest ship, (2 * speed + 1)^2 cells, plus 3. Only
    a side of medium ships (speed 2) has 5x5 windows."""
    codes = [TYPE_CODES.get(t, t) for t in types]
    return 4 * len(codes) + (25 if codes and all(c == LNW_MEDIUM for c in codes) else 49) + 3

# field -> (torch dtype of the raw bytes, shape builder)
_FIELDS = {
    F_POS: (torch.int32, lambda g: (g.A, g.E)),
    F_RADAR: (torch.int32, lambda g: (g.A, g.E)),
    F_MISSILES: (torch.uint8, lambda g: (g.A, g.E)),
    F_MKIND: (torch.uint8, lambda g: (g.A, g.E)),
    F_ALIVE: (torch.uint8, lambda g: (g.A, g.E)),
    F_TYPE: (torch.uint8, lambda g: (g.A, g.E)),
    F_STEPS: (torch.int32, lambda g: (g.A, g.E)),
    F_DIST_LZ: (torch.float64, lambda g: (g.A, g.E)),
    F_TL_CNT: (torch.int16, lambda g: (g.A, g.E)),
    F_TL: (torch.int16, lambda g: (g.A, g.T, g.E)),
    F_DUCT: (torch.float64, lambda g: (g.E,)),
    F_ENV: (torch.int32, lambda g: (8, g.E)),
    F_RNG: (torch.int64, lambda g: (g.E,)),
    F_ERR: (torch.int32, lambda g: (g.E,)),
}
ENV_KEYS = ["n_blue_left", "n_red_left", "steps_done", "blue_victory", "red_victory",
            "blue_engagements", "red_engagements", "episode"]


def default_grid(G=100):
    """The reference's terrain: balt_mod_400x400_2.png -> LANCZOS resize -> L
    (game.py:616-626), committed as data at G=100 and G=200."""
    return np.load(os.path.join(DATA, f"baltic_grid{G}.npy"))


def _ptr(t):
    return C.c_void_p(t.data_ptr()) if t is not None else None


class BatchedGame:
    def __init__(self, n_envs, blue_types, red_types, scenario=None, device=0, env_id_base=0,
                 grid=None, seed=0, reward_dtype=torch.float32):
        self.L = _abi.load()
        self.sc = scenario or Scenario()
        self.E = int(n_envs)
        self.blue_types = [TYPE_CODES.get(t, t) for t in blue_types]
        self.red_types = [TYPE_CODES.get(t, t) for t in red_types]
        self.nb, self.nr = len(self.blue_types), len(self.red_types)
        self.A = self.nb + self.nr
        self.Db, self.Dr = side_obs_dim(self.blue_types), side_obs_dim(self.red_types)
        self.device = torch.device("cuda", device)
        self.env_id_base = int(env_id_base)
        self._params = self.sc.params()
        h = C.c_void_p()
        check(self.L.lnw_create(C.byref(self._params), self.E, self.nb, self.nr, device,
                                self.env_id_base, C.byref(h)))
        self.h = h
        self.T = self.L.lnw_tlist_cap(self.h)
        self.grid = np.ascontiguousarray(default_grid(100) if grid is None else grid, np.uint8)
        self.G = self.grid.shape[0]
        check(self.L.lnw_load_terrain(self.h, self.grid.ctypes.data_as(C.c_void_p), self.G))
        self.epw = self.L.lnw_set_epw(self.h, 0)
        self._tape = None
        self.set_rng(seed)
        dev = self.device
        self.obs_blue = torch.zeros((self.E, self.nb, self.Db), dtype=torch.float32, device=dev)
        self.obs_red = torch.zeros((self.E, self.nr, self.Dr), dtype=torch.float32, device=dev)
        # rewards and cog: float32, or float64 (the reference's Python floats,
        # game.py:522-525) through lnw_set_reward_dtype
        if reward_dtype not in (torch.float32, torch.float64):
            raise TypeError("reward_dtype must be torch.float32 or torch.float64")
        rdt = reward_dtype
        check(self.L.lnw_set_reward_dtype(self.h, int(rdt == torch.float64)))
        self.rew_blue = torch.zeros((self.E, self.nb), dtype=rdt, device=dev)
        self.rew_red = torch.zeros((self.E, self.nr), dtype=rdt, device=dev)
        self.done = torch.ones((self.E,), dtype=torch.int32, device=dev)
        self.cog = torch.zeros((self.E,), dtype=rdt, device=dev)
        self._spawn = None
        self._ana = None
        # step() hot path: output pointers and the accepted action layout, cached
        self._outp = tuple(_ptr(t) for t in (self.obs_blue, self.obs_red, self.rew_blue,
                                             self.rew_red, self.done, self.cog))
        self._outd = dict(obs_blue=self.obs_blue, obs_red=self.obs_red, rew_blue=self.rew_blue,
                          rew_red=self.rew_red, done=self.done, cog=self.cog)
        self._ashape = torch.Size((self.E, self.A, 4))
        self._dtypes = {torch.float32: LNW_ACT_F32, torch.float64: LNW_ACT_F64,
                        torch.int32: LNW_ACT_I32}

    # ---------------------------------------------------------------- rng
    def set_epw(self, epw=0):
        """Environments per workgroup of the step launch (lnw_set_epw): 0 = automatic
        (64 unless E is too small to fill the GPU), 1..64 forces it. Returns the
        value in force. Results do not depend on it."""
        rc = self.L.lnw_set_epw(self.h, int(epw))
        if rc < 0:
            check(rc)
        self.epw = rc
        return rc

    def set_variant(self, contact):
        """Step-kernel code variant (lnw_set_variant): contact=True for workloads
        whose fleets are in sensor range most steps (melee spawns, MAPPO rollouts
        against a closing red); False (default) for mostly quiet ones. Results do
        not depend on it."""
        check(self.L.lnw_set_variant(self.h, int(bool(contact))))
        self.contact = bool(contact)

    def set_rng(self, seed):
        """Production RNG: Philox4x32-10 keyed by (seed, global env id)."""
        self._tape = None
        check(self.L.lnw_set_rng(self.h, LNW_RNG_PHILOX, int(seed) & (2**64 - 1), None, None))

    def set_tape(self, tape, offsets):
        """Parity RNG: env e consumes tape[offsets[e]:offsets[e+1]] in call order."""
        tape = torch.as_tensor(tape, dtype=torch.float64).to(self.device).contiguous()
        offs = torch.as_tensor(offsets, dtype=torch.int64).to(self.device).contiguous()
        assert offs.numel() == self.E + 1
        self._tape = (tape, offs)
        check(self.L.lnw_set_rng(self.h, LNW_RNG_TAPE, 0, _ptr(tape), _ptr(offs)))

    def _stream(self):
        return C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    # -------------------------------------------------------------- reset
    def reset(self, positions=None, rand_ls=None, env_mask=None, pos_per_env=None, box=None):
        """Game.reset for the masked envs (all by default). positions: A (x, y)
        spawn cells (blue then red); rand_ls: A flags drawing the LandingShip
        spawn (game.py:587-591); pos_per_env: [E, A, 2] int32 tensor; box:
        ((x0, y0), (x1, y1)) random-water-cell spawn box."""
        sp = Spawn()
        types = self.blue_types + self.red_types
        for a, t in enumerate(types):
            sp.types[a] = int(t)
        if positions is not None:
            for a, (x, y) in enumerate(positions):
                sp.pos[a][0], sp.pos[a][1] = int(x), int(y)
        if rand_ls is not None:
            for a, f in enumerate(rand_ls):
                sp.rand_ls[a] = int(bool(f))
        if box is not None:
            (x0, y0), (x1, y1) = box
            sp.box_lo[0], sp.box_lo[1], sp.box_hi[0], sp.box_hi[1] = x0, y0, x1, y1
        self._spawn = sp
        mask = None
        if env_mask is not None:
            mask = torch.as_tensor(env_mask, dtype=torch.uint8, device=self.device).contiguous()
        pe = None
        if pos_per_env is not None:
            pe = torch.as_tensor(pos_per_env, dtype=torch.int32, device=self.device).contiguous()
            self._pos_per_env = pe
        check(self.L.lnw_reset(self.h, _ptr(mask), C.byref(sp), _ptr(pe), self._stream()))
        if mask is not None or pe is not None:
            torch.cuda.current_stream(self.device).synchronize()

    # --------------------------------------------------------------- step
    def step(self, actions, row_kind=None, obs=True):
        """Game.step for all envs. actions: [E, A, 4] float32 / float64 tensor
        (continuous) or int32 (discrete). Mutated in place where the reference
        mutates its action rows (game.py:379). Returns the output tensors.
        obs=False: no observation rows are written (obs_blue / obs_red keep
        their contents; a caller that observes afresh, as ppo.py does)."""
        a = actions
        if a.shape != self._ashape or not a.is_cuda or not a.is_contiguous():
            raise ValueError(f"actions must be a contiguous cuda tensor of shape {tuple(self._ashape)}")
        dt = self._dtypes.get(a.dtype)
        if dt is None:
            raise TypeError(f"unsupported action dtype {a.dtype}")
        rk = None
        if row_kind is not None:
            rk = _ptr(torch.as_tensor(row_kind, dtype=torch.uint8, device=self.device).contiguous())
        ob, orr, rb, rr, dn, cg = self._outp
        if not obs:
            ob = orr = None
        check(self.L.lnw_step(self.h, a.data_ptr(), dt, rk, ob, orr, rb, rr, dn, cg,
                              torch.cuda.current_stream(self.device).cuda_stream))
        return self._outd

    def step_seq(self, actions, row_kind=None, obs=True, keep="last"):
        """K Game.step calls on an action sequence known ahead of time
        (lnw_step_seq): actions [K, E, A, 4] (contiguous cuda, the step()
        dtypes), row_kind [K, E, A] or None. The results are those of K step()
        calls; the rows of a step are mutated where step() mutates them.
        keep="last": every step writes the game's output tensors (so they end
        holding step K-1's outputs, as after K step() calls); keep="all":
        returns new tensors with every step's outputs, [K, ...]."""
        a = actions
        if a.dim() != 4 or a.shape[1:] != self._ashape or not a.is_cuda or not a.is_contiguous():
            raise ValueError(f"actions must be a contiguous cuda tensor of shape (K, {tuple(self._ashape)})")
        dt = self._dtypes.get(a.dtype)
        if dt is None:
            raise TypeError(f"unsupported action dtype {a.dtype}")
        K = a.shape[0]
        rk = None
        sq = _abi.Seq(K, self.E * self.A * 4, 0, 0, 0, 0, 0, 0, 0)
        if row_kind is not None:
            rkt = torch.as_tensor(row_kind, dtype=torch.uint8, device=self.device).contiguous()
            assert rkt.shape == (K, self.E, self.A)
            rk, sq.kind_step = _ptr(rkt), self.E * self.A
        if keep == "last":
            out = self._outd
        elif keep == "all":
            # uninitialised: every step writes every element of its output set (a
            # sunk ship's row as zeros); no observation tensors when obs=False
            out = {k: torch.empty((K,) + tuple(v.shape), dtype=v.dtype, device=self.device)
                   for k, v in self._outd.items() if obs or not k.startswith("obs_")}
            sq.obs_blue_step, sq.obs_red_step = self.E * self.nb * self.Db, self.E * self.nr * self.Dr
            sq.rew_blue_step, sq.rew_red_step = self.E * self.nb, self.E * self.nr
            sq.done_step = sq.cog_step = self.E
        else:
            raise ValueError("keep must be 'last' or 'all'")
        p = {k: _ptr(v) for k, v in out.items()}
        ob, orr = (p["obs_blue"], p["obs_red"]) if obs else (None, None)
        if not obs:
            sq.obs_blue_step = sq.obs_red_step = 0
        check(self.L.lnw_step_seq(self.h, C.byref(sq), a.data_ptr(), dt, rk, ob, orr, p["rew_blue"],
                                  p["rew_red"], p["done"], p["cog"],
                                  torch.cuda.current_stream(self.device).cuda_stream))
        return out

    # ---------------------------------------------------------- analytics
    def enable_analytics(self, eng_cap=1 << 20, ew_cap=1 << 20, maps=True):
        """Bind device buffers for the reference's analytics side channels
        (heatmap / coldmap / launch sites / engagements / blue_ew / red_ew,
        game.py:119-154) accumulated over all envs and steps (lnw_set_analytics).
        maps=False binds the two logs only (the maps follow from the records)."""
        dev = self.device
        z = lambda *s: torch.zeros(s, dtype=torch.int32, device=dev)  # noqa: E731
        self._ana = dict(heatmap=z(100, 100) if maps else None,
                         coldmap=z(100, 100) if maps else None,
                         launch=z(2, 100, 100) if maps else None,
                         eng_log=z(max(1, eng_cap), 4), eng_count=z(1),
                         ew_log=z(max(1, ew_cap), 4), ew_count=z(1))
        t = self._ana
        p = lambda k: t[k].data_ptr() if t[k] is not None else None  # noqa: E731
        self._ana_struct = _abi.Analytics(p("heatmap"), p("coldmap"), p("launch"),
                                          p("eng_log"), p("eng_count"), int(eng_cap),
                                          p("ew_log"), p("ew_count"), int(ew_cap))
        check(self.L.lnw_set_analytics(self.h, C.byref(self._ana_struct)))

    def drain_analytics(self):
        """Decoded records written since the last drain (numpy int64: see
        analytics()), then both logs restart empty."""
        an = self.analytics()
        eng, ew = an["engagements"].cpu().numpy(), an["ew_fixes"].cpu().numpy()
        self._ana["eng_count"].zero_()
        self._ana["ew_count"].zero_()
        return eng, ew

    def disable_analytics(self):
        check(self.L.lnw_set_analytics(self.h, None))
        self._ana = None

    def analytics(self):
        """Decoded analytics: maps (device tensors) and the engagement / EW
        records as int64 [n, 7] tensors (env, step, side, x1, y1, x2, y2) with
        the missile count as an 8th engagement column; totals include records
        past the capacity."""
        t = self._ana
        if t is None:
            raise RuntimeError("analytics not enabled")

        def recs(log, count, fix):
            n = int(count.item())
            r = log[: min(n, log.shape[0])].to(torch.int64) & 0xFFFFFFFF
            w1, w2, w3 = r[:, 1], r[:, 2], r[:, 3]
            cols = [r[:, 0], w1 & 0xFFFF, (w1 >> 16) & 0xFF, w2 & 0xFFFF, w2 >> 16]
            if fix:  # int16 fix coordinates
                cols += [((w3 & 0xFFFF) ^ 0x8000) - 0x8000, ((w3 >> 16) ^ 0x8000) - 0x8000]
            else:
                cols += [w3 & 0xFFFF, w3 >> 16, w1 >> 24]
            return torch.stack(cols, 1), n

        eng, n_eng = recs(t["eng_log"], t["eng_count"], False)
        ew, n_ew = recs(t["ew_log"], t["ew_count"], True)
        return dict(heatmap=t["heatmap"], coldmap=t["coldmap"], launch=t["launch"],
                    engagements=eng, engagements_total=n_eng, ew_fixes=ew, ew_total=n_ew)

    def count_work(self, on=True):
        """Bind (on) or unbind the device work counters (lnw_set_counters):
        rays ray-marched, Bresenham cells visited, A* searches run, EW bearings
        evaluated in wave-pooled rounds (contact variant)."""
        if on:
            self._ctr = torch.zeros(4, dtype=torch.int64, device=self.device)
            check(self.L.lnw_set_counters(self.h, _ptr(self._ctr)))
        else:
            check(self.L.lnw_set_counters(self.h, None))

    def work_counts(self):
        c = self._ctr.cpu().tolist()
        return dict(rays_marched=c[0], cells_marched=c[1], astar_searches=c[2],
                    pooled_bearings=c[3])

    def observe(self, agent=-1):
        """ship.get_obs() for every live ship (agent=-1, blue then red), one side
        (-2 blue, -3 red) or one agent index, in every env."""
        check(self.L.lnw_observe(self.h, int(agent), _ptr(self.obs_blue), _ptr(self.obs_red),
                                 self._stream()))
        return self.obs_blue, self.obs_red

    def observe_into(self, agent, blue_ptr, blue_env_stride=0, red_ptr=None, red_env_stride=0):
        """observe() with the rows written to caller memory (device pointers;
        env e's rows at ptr + e * stride floats, 0 = packed) or nowhere (None:
        the side's get_obs side effects still happen) — lnw_observe_ex."""
        check(self.L.lnw_observe_ex(self.h, int(agent), blue_ptr, int(blue_env_stride), red_ptr,
                                    int(red_env_stride), self._stream()))

    # -------------------------------------------------------------- state
    def _field(self, f):
        p = C.c_void_p()
        n = C.c_int64()
        check(self.L.lnw_state_field(self.h, f, C.byref(p), C.byref(n)))
        return p, n.value

    def get(self, f):
        dt, shp = _FIELDS[f]
        p, n = self._field(f)
        out = torch.empty(shp(self), dtype=dt, device=self.device)
        assert out.numel() * out.element_size() == n
        check(self.L.lnw_copy(_ptr(out), p, n, self._stream()))
        return out

    def set(self, f, value):
        dt, shp = _FIELDS[f]
        p, n = self._field(f)
        v = torch.as_tensor(value).to(device=self.device, dtype=dt).reshape(shp(self)).contiguous()
        check(self.L.lnw_copy(p, _ptr(v), n, self._stream()))
        torch.cuda.current_stream(self.device).synchronize()

    def agents(self):
        """Per-agent state as numpy arrays shaped [E, A] (host copy)."""
        pos = self.get(F_POS).cpu().numpy().astype(np.int64)
        out = dict(x=(pos & 0x7fff).T, y=((pos >> 16) & 0x7fff).T,
                   radar=self.get(F_RADAR).cpu().numpy().T,
                   missiles=self.get(F_MISSILES).cpu().numpy().T,
                   mkind=self.get(F_MKIND).cpu().numpy().T,
                   alive=self.get(F_ALIVE).cpu().numpy().T,
                   type=self.get(F_TYPE).cpu().numpy().T,
                   steps_done=self.get(F_STEPS).cpu().numpy().T,
                   dist_lz=self.get(F_DIST_LZ).cpu().numpy().T,
                   tl_cnt=self.get(F_TL_CNT).cpu().numpy().T.astype(np.int64))
        return out

    def env_state(self):
        e = self.get(F_ENV).cpu().numpy()
        d = {k: e[i] for i, k in enumerate(ENV_KEYS)}
        d["ducting"] = self.get(F_DUCT).cpu().numpy()
        d["rng"] = self.get(F_RNG).cpu().numpy()
        d["err"] = self.get(F_ERR).cpu().numpy()
        return d

    def tlists(self, env):
        """Target lists of one env: list (per agent) of (x, y) tuples."""
        cnt = self.get(F_TL_CNT).cpu().numpy().astype(np.int64)[:, env]
        tl = self.get(F_TL).cpu().numpy().astype(np.int64)[:, :, env] & 0xffff
        return [[(int(v & 0xff), int(v >> 8)) for v in tl[a, :cnt[a]]] for a in range(self.A)]

    def step_kernel(self):
        """Which step kernel the last step() launched (lnw_step_kernel:
        _abi.KERNEL_*): build-side launch shape, for tests and diagnostics."""
        return self.L.lnw_step_kernel(self.h)

    def get_state(self, device="cpu"):
        """Whole-state snapshot (lnw_get_state) as a uint8 tensor on `device`:
        every state field, the auto-reset's spawn spec and the RNG mode/seed.
        Waits for the current stream."""
        n = self.L.lnw_state_bytes(self.h)
        if n < 0:
            check(n)
        dev = torch.device(device)
        buf = torch.zeros(n, dtype=torch.uint8, device=dev, pin_memory=False)
        check(self.L.lnw_get_state(self.h, _ptr(buf), n, self._stream()))
        return buf

    def set_state(self, snapshot):
        """Restore a get_state() snapshot (lnw_set_state) taken from a handle of
        the same shape and terrain; stepping then continues exactly as the
        saved handle would have. A tape-mode snapshot needs the same tape bound
        (set_tape) first."""
        buf = torch.as_tensor(snapshot, dtype=torch.uint8).contiguous()
        # the observation buffers are sized by this game's ship types: a
        # snapshot of another fleet (a medium side has shorter rows) is refused
        # here, before the library would select kernels for its row length
        # (header: magic, version, then E, nb, nr as int32 at bytes 12..23; a
        # snapshot of another shape is left to the library to refuse)
        hdr = buf[:24].cpu().view(torch.int32).tolist() if buf.numel() >= 24 else []
        off = 256
        for f in range(_abi.LNW_NFIELDS):
            off += (self._field(f)[1] + 255) & ~255
        if hdr[3:6] == [self.E, self.nb, self.nr] and buf.numel() >= off + 4 * self.A:
            types = buf[off:off + 4 * self.A].cpu().view(torch.int32).tolist()
            if types != [int(t) for t in self.blue_types + self.red_types]:
                raise ValueError(f"snapshot fleet {types} differs from this game's "
                                 f"{self.blue_types + self.red_types}")
        check(self.L.lnw_set_state(self.h, _ptr(buf), buf.numel(), self._stream()))

    def close(self):
        if getattr(self, "h", None) is not None and self.h.value:
            self.L.lnw_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
