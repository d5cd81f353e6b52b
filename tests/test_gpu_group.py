"""The group kernel (csrc/lnw_group.inc: runtime team sizes, 16 lanes per env)
against the one-lane-per-env kernel step_kernel<0, 0> (LNW_NO_GROUP) on the
same envs: identical observations, rewards, done, cog, written-back actions,
state, target lists and analytics records, over episodes that fire, sink
ships, take EW bearings and auto-reset. Both are checked against the oracle
elsewhere (golden 8v10 replays, test_gpu_fullsize config 4)."""
import numpy as np
import pytest
import torch

from _oracle import load_fixture

pytestmark = pytest.mark.gpu


def _box_positions(grid, E, nb, nr, seed, box_b, box_r):
    rng = np.random.default_rng(seed)
    water = lambda x0, x1, y0, y1: [(x, y) for x in range(x0, x1) for y in range(y0, y1)
                                    if grid[x, y] <= 74]
    wb, wr = water(*box_b), water(*box_r)
    return np.array([[wb[i] for i in rng.integers(0, len(wb), nb)] +
                     [wr[i] for i in rng.integers(0, len(wr), nr)] for _ in range(E)], np.int32)


CASES = {
    # config 4's shape: 8 small vs 8 large + 2 landing ships on 200x200, landing ops
    "8v10ls_g200": dict(blue=["small"] * 8, red=["large"] * 8 + ["ls"] * 2, G=1, landing_ops=True,
                        box_b=(30, 45, 90, 120), box_r=(45, 60, 95, 125), E=200, dtype="f32"),
    "5v3_g100": dict(blue=["small"] * 5, red=["large"] * 3, G=0, landing_ops=False,
                     box_b=(30, 45, 40, 60), box_r=(50, 65, 45, 65), E=333, dtype="f64"),
    "12v12_g100": dict(blue=["small"] * 12, red=["large"] * 12, G=0, landing_ops=False,
                       box_b=(30, 45, 40, 60), box_r=(45, 60, 45, 65), E=96, dtype="f32"),
    "3v6ls_untrained": dict(blue=["small"] * 3, red=["large"] * 5 + ["ls"], G=0, landing_ops=True,
                            box_b=(30, 45, 40, 60), box_r=(45, 60, 45, 65), E=150, dtype="f64",
                            trained_red=False),
}


@pytest.mark.parametrize("name", sorted(CASES))
def test_group_kernel_equals_lane_kernel(name, monkeypatch):
    from lnw import _abi
    from lnw.batched import BatchedGame
    from lnw.config import Scenario
    cs = CASES[name]
    g = load_fixture("grids.npz")
    grid = g["grid200"] if cs["G"] else g["grid100"]
    E = cs["E"]
    nb, nr = len(cs["blue"]), len(cs["red"])
    A = nb + nr
    sc = Scenario(landing_ops=cs["landing_ops"], auto_reset=True, episode_steps=25,
                  trained_red=cs.get("trained_red", True))
    pos = _box_positions(grid, E, nb, nr, 5, cs["box_b"], cs["box_r"])
    games = []
    for no_group in (False, True):
        if no_group:
            monkeypatch.setenv("LNW_NO_GROUP", "1")  # read once, by lnw_create
        gm = BatchedGame(E, cs["blue"], cs["red"], scenario=sc, grid=grid, seed=11,
                         reward_dtype=torch.float64)
        monkeypatch.delenv("LNW_NO_GROUP", raising=False)
        gm.enable_analytics(eng_cap=1 << 20, ew_cap=1 << 20)
        gm.reset(positions=pos[0], pos_per_env=torch.from_numpy(pos))
        games.append(gm)
    rng = np.random.default_rng(3)
    dt = torch.float32 if cs["dtype"] == "f32" else torch.float64
    for s in range(30):
        act = torch.from_numpy(rng.random((E, A, 4))).to(dt).cuda()
        acts = [act.clone() for _ in games]
        outs = [{k: v.cpu().numpy().copy() for k, v in gm.step(a).items()} for gm, a in zip(games, acts)]
        for k in outs[0]:
            assert np.array_equal(outs[0][k], outs[1][k], equal_nan=True), (s, k)
        assert torch.equal(acts[0], acts[1]), (s, "actions written back")
    sts = [gm.env_state() for gm in games]
    for k in sts[0]:
        assert np.array_equal(sts[0][k], sts[1][k], equal_nan=True), k
    assert sts[0]["episode"].sum() > 0
    for f in range(_abi.F_ERR + 1):
        a, b = (gm.get(f).cpu().numpy() for gm in games)
        if f == _abi.F_TL:  # contents past each list's count are scratch
            cnt = games[0].get(_abi.F_TL_CNT).cpu().numpy().astype(np.int64)
            keep = np.arange(a.shape[1])[None, :, None] < cnt[:, None, :]
            a, b = np.where(keep, a, 0), np.where(keep, b, 0)
        assert np.array_equal(a, b, equal_nan=True), f
    an = [gm.analytics() for gm in games]
    assert an[0]["engagements_total"] == an[1]["engagements_total"] > 0
    assert an[0]["ew_total"] == an[1]["ew_total"]
    assert an[0]["ew_total"] <= 1 << 20  # every record stored (append order differs)
    for key in ("engagements", "ew_fixes"):
        x, y = (sorted(map(tuple, a[key].cpu().numpy().tolist())) for a in an)
        assert x == y, key
    for key in ("heatmap", "coldmap", "launch"):
        assert torch.equal(an[0][key], an[1][key]), key
    for gm in games:
        gm.close()


def test_group_kernel_counts_pooled_bearings(monkeypatch):
    """lnw_set_counters with the group kernel: counter [3] counts the EW
    bearings evaluated pooled over an env's 16 lanes (every bearing of an
    opponent that gets a fix), which config 4's bench line reports; the
    one-lane kernel pools nothing. Results are unchanged with counters bound."""
    from lnw import _abi
    from lnw.batched import BatchedGame
    from lnw.config import Scenario
    cs = CASES["8v10ls_g200"]
    grid = load_fixture("grids.npz")["grid200"]
    E = cs["E"]
    nb, nr = len(cs["blue"]), len(cs["red"])
    sc = Scenario(landing_ops=True, auto_reset=True, episode_steps=25)
    pos = _box_positions(grid, E, nb, nr, 5, cs["box_b"], cs["box_r"])
    rng = np.random.default_rng(4)
    acts = [torch.from_numpy(rng.random((E, nb + nr, 4)).astype(np.float32)).cuda() for _ in range(12)]
    runs = {}
    for label, count, no_group in (("group", True, False), ("plain", False, False), ("lane", True, True)):
        if no_group:
            monkeypatch.setenv("LNW_NO_GROUP", "1")
        gm = BatchedGame(E, cs["blue"], cs["red"], scenario=sc, grid=grid, seed=11)
        monkeypatch.delenv("LNW_NO_GROUP", raising=False)
        gm.reset(positions=pos[0], pos_per_env=torch.from_numpy(pos))
        if count:
            gm.count_work(True)
        traj = []
        for a in acts:
            traj.append({k: v.cpu().numpy().copy() for k, v in gm.step(a.clone()).items()})
            assert gm.step_kernel() == (_abi.KERNEL_GENERIC if no_group else _abi.KERNEL_GROUP)
        torch.cuda.synchronize()
        runs[label] = (traj, gm.work_counts() if count else None)
        gm.close()
    for s in range(len(acts)):
        for k in runs["group"][0][s]:
            assert np.array_equal(runs["group"][0][s][k], runs["plain"][0][s][k], equal_nan=True), (s, k)
    assert runs["group"][1]["pooled_bearings"] > 0, runs["group"][1]
    assert runs["lane"][1]["pooled_bearings"] == 0, runs["lane"][1]
