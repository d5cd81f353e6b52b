"""The N>1 path on CPU: two ranks over gloo (127.0.0.1). Checks the env
sharding, the max-over-ranks timing reduction bench.py reports, and that a
global env's trajectory (oracle, Philox keyed by global env id) is the same
whichever rank and shard size steps it."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _digest(gids, steps=12):
    import _oracle
    from lnw.batched import default_grid
    grid = default_grid(100)
    out = {}
    for gid in gids:
        o = _oracle.OracleEnv(grid, 4, 4, landing_ops=False)
        o.set_philox(42, gid)
        o.reset([0] * 4 + [1] * 4, [(40, 45), (44, 47), (38, 52), (42, 50),
                                    (50, 55), (52, 50), (47, 58), (53, 61)])
        rng = np.random.default_rng(gid)
        h = []
        for _ in range(steps):
            r = o.step(rng.random((8, 4)).astype(np.float32).astype(np.float64),
                       np.full(8, _oracle.K_F32, np.int32))
            h.append(float(r["rew_blue"].sum() + r["rew_red"].sum()))
            h.append(float(r["obs_blue"].sum()))
        out[gid] = h
    return out


def _worker(rank, world, port, total, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world),
                      RANK=str(rank), LOCAL_RANK=str(rank))
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [here, os.path.join(os.path.dirname(here), "littoral-naval-warfare-marl_amd")]
    from lnw import dist
    ws, r, _ = dist.init("gloo")
    lo, hi = dist.env_range(total, ws, r)
    t = dist.reduce_max([float(r + 1), 10.0 - r])
    n = dist.reduce_sum([float(hi - lo)])
    dig = _digest(range(lo, hi))
    dist.barrier()
    q.put((r, lo, hi, t, n, dig))
    dist.finalize()


@pytest.mark.parametrize("world", [2])
def test_two_rank_gloo(world):
    total = 6
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, total, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)])
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    spans = [(lo, hi) for _, lo, hi, *_ in res]
    assert spans == [(0, 3), (3, 6)]
    for _, _, _, t, n, _ in res:
        assert t == [float(world), 10.0] and n == [float(total)]
    merged = {}
    for *_, dig in res:
        merged.update(dig)
    single = _digest(range(total))
    assert merged == single
