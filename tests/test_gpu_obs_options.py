"""Observation-output options of the step and observe entry points (the MAPPO
rollout's fast path, lnw/rollout.py):

* lnw_step with both observation pointers NULL writes no rows and changes
  nothing else: rewards, done, cog, the written-back action rows and the whole
  state equal a step that writes its rows, on every kernel (units, templated
  quiet / contact variants, the group kernel);
* lnw_observe_ex writes the rows of env e at ptr + e * stride, or none for a
  side passed as NULL, with the same get_obs side effects (target lists, RNG
  draws: the state after it equals lnw_observe's).

Two handles start from one whole-state snapshot (lnw_get_state / set_state).
Needs an MI355X."""
import numpy as np
import pytest
import torch

from _oracle import load_fixture
from test_gpu_state import _box_positions

pytestmark = pytest.mark.gpu

REF = [(6, 61), (10, 81), (8, 70), (11, 58), (98, 48), (98, 52), (98, 56), (96, 52)]

CASES = {
    # units kernel (E % 256 == 0, quiet reference spawns)
    "units_quiet": dict(blue=["small"] * 4, red=["large"] * 4, G=0, E=512, box=None, contact=False),
    # templated default variant, envs in contact, small workgroups
    "team_melee": dict(blue=["small"] * 4, red=["large"] * 4, G=0, E=200, box=((40, 48, 44, 56), (48, 56, 48, 60)),
                       contact=False),
    # contact variant
    "contact_melee": dict(blue=["small"] * 4, red=["large"] * 4, G=0, E=256,
                          box=((40, 48, 44, 56), (48, 56, 48, 60)), contact=True),
    # group kernel (runtime team sizes)
    "group_8v10": dict(blue=["small"] * 8, red=["large"] * 8 + ["ls"] * 2, G=1, E=64,
                       box=((30, 45, 90, 120), (45, 60, 95, 125)), contact=False),
}


def _game(cs, grid, seed=5):
    from lnw.batched import BatchedGame
    from lnw.config import Scenario
    sc = Scenario(landing_ops=False, auto_reset=True, episode_steps=9, trained_red=False)
    g = BatchedGame(cs["E"], cs["blue"], cs["red"], scenario=sc, grid=grid, seed=seed)
    if cs["contact"]:
        g.set_variant(True)
    return g


def _start(cs, grid):
    g = _game(cs, grid)
    nb, nr = len(cs["blue"]), len(cs["red"])
    if cs["box"] is None:
        g.reset(positions=REF)
    else:
        pos = _box_positions(grid, cs["E"], nb, nr, 3, cs["box"][0], cs["box"][1])
        g.reset(positions=pos[0], pos_per_env=torch.from_numpy(pos))
    return g


@pytest.mark.parametrize("name", sorted(CASES))
def test_step_without_observation_rows(name):
    cs = CASES[name]
    grid = load_fixture("grids.npz")["grid200" if cs["G"] else "grid100"]
    E, A = cs["E"], len(cs["blue"]) + len(cs["red"])
    g1 = _start(cs, grid)
    snap = g1.get_state(device="cuda")
    g2 = _game(cs, grid, seed=11)
    g2.set_state(snap)
    rng = np.random.default_rng(4)
    kernels = set()
    for s in range(20):  # crosses the 9-step auto-reset twice
        a = torch.from_numpy(rng.random((E, A, 4))).float().cuda()
        a1, a2 = a.clone(), a.clone()
        o1 = {k: v.clone() for k, v in g1.step(a1).items()}
        kernels.add(g1.step_kernel())
        before = g2.obs_blue.clone()
        o2 = g2.step(a2, obs=False)
        assert torch.equal(g2.obs_blue, before)  # no row written
        for k in o1:
            if k.startswith("obs"):
                continue
            assert torch.equal(torch.nan_to_num(o1[k], nan=7.0), torch.nan_to_num(o2[k], nan=7.0)), (s, k)
        assert torch.equal(a1, a2), s
    assert torch.equal(g1.get_state(), g2.get_state())
    print(name, "kernels", sorted(kernels))
    g1.close()
    g2.close()


def test_step_refuses_one_null_observation_pointer():
    from lnw import _abi
    cs = CASES["team_melee"]
    g = _start(cs, load_fixture("grids.npz")["grid100"])
    a = torch.rand((cs["E"], 8, 4), device="cuda")
    with pytest.raises(_abi.LnwError, match="both or neither"):
        _abi.check(g.L.lnw_step(g.h, a.data_ptr(), _abi.LNW_ACT_F32, None, g.obs_blue.data_ptr(), None,
                                None, None, None, None, torch.cuda.current_stream().cuda_stream))
    g.close()


@pytest.mark.parametrize("name", ["contact_melee", "team_melee", "group_8v10"])
def test_observe_ex_strided_rows_and_null_side(name):
    cs = CASES[name]
    grid = load_fixture("grids.npz")["grid200" if cs["G"] else "grid100"]
    E, A = cs["E"], len(cs["blue"]) + len(cs["red"])
    g1 = _start(cs, grid)
    rng = np.random.default_rng(8)
    for _ in range(4):  # into contact: target lists, bearings, draws
        g1.step(torch.from_numpy(rng.random((E, A, 4))).float().cuda())
    snap = g1.get_state(device="cuda")
    g2 = _game(cs, grid, seed=12)
    g2.set_state(snap)
    ob, orr = (x.clone() for x in g1.observe(-1))
    T, t = 5, 3  # a [E][T][nb][Db] rollout buffer, step t
    nb, Db = g2.nb, g2.Db
    buf = torch.full((E, T, nb, Db), -1.0, device="cuda")
    g2.observe_into(-1, buf.data_ptr() + t * nb * Db * 4, T * nb * Db, None, 0)
    torch.cuda.synchronize()
    assert torch.equal(buf[:, t], ob)
    others = torch.cat([buf[:, :t], buf[:, t + 1:]], 1)
    assert bool((others == -1.0).all())  # nothing outside step t's rows
    assert torch.equal(g1.get_state(), g2.get_state())  # red's get_obs ran too
    # both sides strided
    rb = torch.zeros((E, 2, g2.nr, g2.Dr), device="cuda")
    g1.observe(-1)
    g2.observe_into(-1, buf.data_ptr(), T * nb * Db, rb.data_ptr() + g2.nr * g2.Dr * 4, 2 * g2.nr * g2.Dr)
    torch.cuda.synchronize()
    assert torch.equal(buf[:, 0], g1.obs_blue) and torch.equal(rb[:, 1], g1.obs_red)
    assert torch.equal(g1.get_state(), g2.get_state())
    from lnw import _abi
    with pytest.raises(_abi.LnwError, match="stride"):
        g2.observe_into(-1, buf.data_ptr(), nb * Db - 4, None, 0)
    g1.close()
    g2.close()


@pytest.mark.parametrize("with_live", [True, False])
def test_policy_act_strided_input_equals_packed(with_live):
    """lnw_policy_act reading its rows from a [E][T][n][D] rollout buffer at
    step t (obs_in_env_stride) gives the outputs of the packed [E][n][D] rows
    bit for bit, call after call, and in place (obs_out == obs) leaves live
    envs' rows alone and zeroes the ended ones. E = 32 768 (config 5's size):
    512-thread blocks, one per CU, two waves per SIMD — the shape at which a
    wave's head running beside its SIMD partner's MLP came back wrong in lanes
    48-63 ("The policy kernel's nondeterminism"), which
    head_and_mlp's schedule (every head, a barrier, every MLP) and the host's
    one-block-per-CU LDS request rule out; 12 calls compared bit for bit."""
    import ctypes as C
    from lnw import _abi
    from lnw.rollout import BatchedActor
    L = _abi.load()
    torch.manual_seed(7)
    a = BatchedActor.for_obs(68).cuda()
    E, n, D, T, t = 32768, 4, 68, 40, 5
    obs = torch.rand((E, n, D), device="cuda")
    obs[:, :, :49] = torch.randint(0, 256, (E, n, 49), device="cuda") / 255.0
    buf = torch.rand((E, T, n, D), device="cuda")
    buf[:, t] = obs
    act = torch.rand((E, n, 4), device="cuda")
    alive = torch.ones((2 * n, E), dtype=torch.uint8, device="cuda")
    live = torch.ones(E, dtype=torch.uint8, device="cuda")
    live[::5] = 0
    params = a.packed_policy()
    call = torch.zeros(1, dtype=torch.int64, device="cuda")
    res = []
    for rep, strided in enumerate([False] + [True] * 11):
        lp = torch.zeros((E, n, 4), device="cuda")
        ac = torch.zeros((E, n, 4), device="cuda")
        full = torch.zeros((E, 2 * n, 4), dtype=torch.float64, device="cuda")
        pa = _abi.PolicyArgs()
        src = buf.data_ptr() + t * n * D * 4 if strided else obs.data_ptr()
        pa.obs, pa.E, pa.n, pa.D, pa.own0, pa.A = src, E, n, D, 0, 2 * n
        pa.obs_in_env_stride = T * n * D if strided else 0
        # sampled (keyed) actions, as the rollout draws them; the log-probabilities
        # and the f64 action array come out of the whole kernel
        pa.params, pa.noise, pa.seed, pa.call_dev, pa.T, pa.t = params.data_ptr(), 0.05, 99, call.data_ptr(), T, t
        pa.alive, pa.act_out, pa.logp_out, pa.act_env_stride = alive.data_ptr(), ac.data_ptr(), lp.data_ptr(), n * 4
        pa.full = full.data_ptr()
        if with_live:
            pa.live = live.data_ptr()
        if strided:
            pa.obs_out, pa.obs_env_stride = src, T * n * D
        _abi.check(L.lnw_policy_act(C.byref(pa), None))
        torch.cuda.synchronize()
        res.append((ac, lp, full))
    # (with live flags the first in-place call zeroes the ended envs' rows, so
    # later calls read zeros there: their f64 action rows are compared on live
    # envs; act / log-prob rows of ended envs are zero either way)
    rowmask = (live.bool() if with_live else torch.ones(E, dtype=torch.bool, device="cuda"))
    for k in range(1, len(res)):
        for x, y in zip(res[0], res[k]):
            m = rowmask[:, None].expand(E, x.shape[1]).reshape(-1)
            bad = ((x != y).reshape(E * x.shape[1], -1).any(1) & m).nonzero().flatten()
            assert bad.numel() == 0, f"call {k}: rows {bad[:6].tolist()} differ"
    if with_live:
        keep = live.bool()
        assert torch.equal(buf[keep, t], obs[keep]) and not buf[~keep, t].any()
    else:
        assert torch.equal(buf[:, t], obs)
    others = [s for s in range(T) if s != t]
    assert not (buf[:, others] == 0).all()
