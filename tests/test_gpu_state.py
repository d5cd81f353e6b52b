"""Whole-state snapshots (lnw_get_state / lnw_set_state): a
snapshot taken mid-episode and restored — into the same handle later, or into a
fresh handle with a different seed — continues with exactly the trajectory of
the uninterrupted run (observations, rewards, done, cog, written-back actions
and the final state, bit for bit), through firing, sinkings, EW fixes and the
in-kernel auto-reset on per-env spawn cells. Shape and terrain mismatches are
refused. Needs an MI355X."""
import numpy as np
import pytest
import torch

from _oracle import load_fixture

pytestmark = pytest.mark.gpu

CASES = {
    # templated 4v4 kernel, contact spawns, f32 actions, trained red
    "4v4": dict(blue=["small"] * 4, red=["large"] * 4, G=0, landing_ops=False, trained_red=True,
                box_b=(30, 45, 40, 60), box_r=(55, 70, 45, 65), E=256, dtype=torch.float32),
    # group kernel: config 4's shape on 200x200, landing ops, untrained red, f64
    "8v10ls": dict(blue=["small"] * 8, red=["large"] * 8 + ["ls"] * 2, G=1, landing_ops=True,
                   trained_red=False, box_b=(30, 45, 90, 120), box_r=(45, 60, 95, 125), E=128,
                   dtype=torch.float64),
    # a medium side (5x5 windows, 4n+28-float rows, runtime-size kernels):
    # restored into a fresh handle that was never reset, the library must take
    # the side's row length and kernels from the snapshot
    "3v3medium": dict(blue=["medium"] * 3, red=["large"] * 3, G=0, landing_ops=False,
                      trained_red=True, box_b=(30, 45, 40, 60), box_r=(50, 65, 45, 65), E=192,
                      dtype=torch.float32),
}


def _box_positions(grid, E, nb, nr, seed, box_b, box_r):
    rng = np.random.default_rng(seed)
    water = lambda x0, x1, y0, y1: [(x, y) for x in range(x0, x1) for y in range(y0, y1)  # noqa: E731
                                    if grid[x, y] <= 74]
    wb, wr = water(*box_b), water(*box_r)
    return np.array([[wb[i] for i in rng.integers(0, len(wb), nb)] +
                     [wr[i] for i in rng.integers(0, len(wr), nr)] for _ in range(E)], np.int32)


def _game(cs, grid, seed):
    from lnw.batched import BatchedGame
    from lnw.config import Scenario
    sc = Scenario(landing_ops=cs["landing_ops"], auto_reset=True, episode_steps=12,
                  trained_red=cs["trained_red"])
    return BatchedGame(cs["E"], cs["blue"], cs["red"], scenario=sc, grid=grid, seed=seed)


def _run(g, acts):
    traj = []
    for a in acts:
        a = a.clone()
        out = g.step(a)
        traj.append({k: v.cpu().numpy().copy() for k, v in out.items()})
        traj[-1]["actions"] = a.cpu().numpy()
    torch.cuda.synchronize()
    return traj


def _same(t1, t2):
    for s, (x, y) in enumerate(zip(t1, t2)):
        for k in x:
            assert np.array_equal(x[k], y[k], equal_nan=True), (s, k)


@pytest.mark.parametrize("name", sorted(CASES))
def test_snapshot_restore_continues_identically(name):
    cs = CASES[name]
    grid = load_fixture("grids.npz")["grid200" if cs["G"] else "grid100"]
    E = cs["E"]
    nb, nr = len(cs["blue"]), len(cs["red"])
    A = nb + nr
    pos = _box_positions(grid, E, nb, nr, 3, cs["box_b"], cs["box_r"])
    rng = np.random.default_rng(9)
    acts = [torch.from_numpy(rng.random((E, A, 4))).to(cs["dtype"]).cuda() for _ in range(30)]
    g = _game(cs, grid, seed=5)
    rand_ls = [0] * (A - 2) + [1, 1] if cs["landing_ops"] else None
    g.reset(positions=pos[0], rand_ls=rand_ls, pos_per_env=torch.from_numpy(pos))
    _run(g, acts[:10])                      # mid-episode
    snap = g.get_state()                    # host snapshot
    snap_dev = g.get_state(device="cuda")   # device snapshot
    assert torch.equal(snap, snap_dev.cpu())
    ref = _run(g, acts[10:30])              # the uninterrupted run (crosses auto-resets)
    end = g.get_state()
    assert int(g.env_state()["episode"].sum()) > 0
    # a fresh handle with another seed: the snapshot brings the seed along
    g2 = _game(cs, grid, seed=777)
    g2.set_state(snap_dev)
    _same(ref, _run(g2, acts[10:30]))
    assert torch.equal(g2.get_state(), end)
    # the same handle, rewound
    g.set_state(snap)
    _same(ref, _run(g, acts[10:30]))
    assert torch.equal(g.get_state(), end)
    g.close()
    g2.close()


def test_snapshot_refuses_other_shapes_and_terrain():
    from lnw import _abi
    grids = load_fixture("grids.npz")
    cs = CASES["4v4"]
    g = _game(cs, grids["grid100"], seed=1)
    g.reset(positions=[(6, 61), (10, 81), (8, 70), (11, 58), (98, 48), (98, 52), (98, 56), (96, 52)])
    snap = g.get_state()
    other = _game(dict(cs, E=128), grids["grid100"], seed=1)
    with pytest.raises(_abi.LnwError, match="shape"):
        other.set_state(snap)
    terrain = grids["grid100"].copy()
    terrain[0, 0] ^= 1
    moved = _game(cs, terrain, seed=1)
    with pytest.raises(_abi.LnwError, match="terrain"):
        moved.set_state(snap)
    bad = snap.clone()
    bad[0] ^= 0xFF
    with pytest.raises(_abi.LnwError, match="magic"):
        g.set_state(bad)
    # another fleet of the same shape: its rows would not fit this game's buffers
    med = _game(dict(cs, blue=["medium"] * 4), grids["grid100"], seed=1)
    with pytest.raises(ValueError, match="fleet"):
        med.set_state(snap)
    # a snapshot whose side mixes medium and speed-3 ships is refused by the
    # library before anything is overwritten
    off = 256
    for f in range(_abi.LNW_NFIELDS):
        off += (g._field(f)[1] + 255) & ~255
    mixed = snap.clone()
    mixed[off:off + 4] = torch.tensor([_abi.LNW_MEDIUM], dtype=torch.int32).view(torch.uint8)
    before = g.get_state()
    with pytest.raises(_abi.LnwError, match="medium"):
        _abi.check(g.L.lnw_set_state(g.h, mixed.data_ptr(), mixed.numel(), None))
    assert torch.equal(g.get_state(), before)
    for x in (g, other, moved, med):
        x.close()
