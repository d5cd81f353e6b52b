"""Replay golden episode fixtures through the HIP path (BatchedGame) in tape mode.

Each episode of a fixture becomes one environment of a single batched handle, so
all of a scenario's episodes step together on the GPU. Test infrastructure.
"""
import numpy as np
import torch

from _oracle import K_F32, K_F64, K_PYFLOAT, episode_meta, fixture_kinds

import lnw
from lnw.batched import BatchedGame
from lnw.config import Scenario


def scenario_from_meta(meta, **over):
    F = meta["flags"]
    return Scenario(discrete=F["DISCRETE"], landing_ops=F["LANDING_OPS"], tactics=F["TACTICS"],
                    side=F["SIDE"], trained_red=F["TRAINED_RED"],
                    red_aggression=F["RED_AGGRESSION"], **over)


def replay_gpu(fx, grids, los_mode=0, move_mode=0, contact=False):
    """Yields (step index s, list of (env, fixture row)) plus the game and the
    output dict after each batched step. Before each step, if the fixture was
    recorded with caller-side observes, yields ('observe', ...) first."""
    meta = episode_meta(fx)
    eps = meta["episodes"]
    E = len(eps)
    nb, nr = eps[0]["nb"], eps[0]["nr"]
    types = eps[0]["types"]
    sc = scenario_from_meta(meta, los_mode=los_mode, move_mode=move_mode)
    grid = grids[meta["grid_id"]]
    names = {0: "small", 1: "large", 2: "ls", 3: "medium"}
    # float64 rewards / cog: the reference's Python floats, compared with rtol=0
    g = BatchedGame(E, [names[t] for t in types[:nb]], [names[t] for t in types[nb:]],
                    scenario=sc, grid=grid, reward_dtype=torch.float64)
    g.set_variant(contact)
    # tape slices, one per env
    tapes = [fx["tape"][em["tape_start"]:em["tape_end"]] for em in eps]
    offs = np.concatenate([[0], np.cumsum([len(t) for t in tapes])]).astype(np.int64)
    g.set_tape(np.concatenate(tapes) if len(tapes) else np.zeros(0), offs)
    pos = np.array([em["spawn"] for em in eps], np.int32)
    rand_ls = np.zeros(nb + nr, np.int32)
    nls = meta["flags"]["N_RED_LANDINGSHIP"]
    if nls > 0:
        rand_ls[nb + nr - nls:] = 1
    g.reset(positions=pos[0], rand_ls=rand_ls, pos_per_env=torch.from_numpy(pos))
    yield ("reset", None, g, None)
    S = max(em["n_steps"] for em in eps)
    A = nb + nr
    discrete = meta["flags"]["DISCRETE"]
    is_f32 = meta["dtype"] == "f32"
    for s in range(S):
        rows = [(e, em["first_step"] + s) for e, em in enumerate(eps) if s < em["n_steps"]]
        if meta["observe"]:
            ob, orr = g.observe(-1)
            yield ("observe", (s, rows), g, (ob.cpu().numpy(), orr.cpu().numpy()))
        list_rows = discrete and meta.get("list_rows", False)
        if discrete and not list_rows:
            act = np.zeros((E, A, 4), np.int32)
        elif is_f32:
            act = np.zeros((E, A, 4), np.float32)
        else:
            act = np.zeros((E, A, 4), np.float64)
        kinds = np.full((E, A), K_F64, np.uint8)
        for e, i in rows:
            act[e] = fx["actions"][i].astype(act.dtype)
            kinds[e] = fixture_kinds(fx, meta, i)
        at = torch.from_numpy(act).cuda()
        rk = None
        if (not discrete and not is_f32) or list_rows:
            rk = torch.from_numpy(kinds).cuda()
        out = g.step(at, rk)
        torch.cuda.synchronize()
        res = {k: v.cpu().numpy().copy() for k, v in out.items()}
        res["actions_after"] = at.cpu().numpy()
        yield ("step", (s, rows), g, res)
