"""lnw_step_seq (BatchedGame.step_seq): K steps of an action sequence known
ahead of time in one call (K launches on the caller's stream). Its results
must be those of K lnw_step calls: every step's observations, rewards, done
and cog, the action rows as each step left them (an untrained red's salvo
write-back, game.py:375-379) and the whole state afterwards, bit for bit. The
workloads cross the 40-step horizon's in-kernel auto-reset and mix quiet and
fighting envs. Needs an MI355X."""
import numpy as np
import pytest
import torch

import _oracle

pytestmark = pytest.mark.gpu

REF_SPAWNS = [(6, 61), (10, 81), (8, 70), (11, 58), (98, 48), (98, 52), (98, 56), (96, 52)]


def _melee(grid, n, seed, nb=4, nr=4):
    rng = np.random.default_rng(seed)
    wb = np.argwhere(grid[30:45, 40:60] <= 74) + np.array([30, 40])
    wr = np.argwhere(grid[55:70, 45:65] <= 74) + np.array([55, 45])
    return np.concatenate([wb[rng.integers(0, len(wb), (n, nb))], wr[rng.integers(0, len(wr), (n, nr))]],
                          1).astype(np.int32)


CASES = {
    # units kernel (E % 256 == 0, 64 envs per workgroup): quiet units beside fighting ones
    "units": dict(E=512, epw=64, block=64, nb=4, trained_red=True, kernel="units"),
    "units_untrained": dict(E=512, epw=64, block=64, nb=4, trained_red=False, kernel="units"),
    # config 3's per-GPU shard at N = 8: 16 envs per workgroup (quiet direct mode)
    "shard8192": dict(E=8192, epw=0, block=16, nb=4, trained_red=True, kernel="team"),
    # a partial last workgroup and 32 envs per workgroup
    "partial": dict(E=1000, epw=32, block=32, nb=4, trained_red=False, kernel="team"),
    # the 3v3 templated kernel
    "team3v3": dict(E=640, epw=0, block=64, nb=3, trained_red=True, kernel="team"),
}


def _setup(cs, grid, seed):
    from lnw.batched import BatchedGame
    from lnw.config import Scenario
    E, nb = cs["E"], cs["nb"]
    spawns = REF_SPAWNS[:nb] + REF_SPAWNS[4:4 + nb]
    pos = np.array([spawns] * E, np.int32)
    blk = cs["block"]
    loud = np.array([e for e in range(E) if (e // blk) % 2 == 1])  # every other workgroup fights
    pos[loud] = _melee(grid, len(loud), seed=E + nb, nb=nb, nr=nb)
    sc = Scenario(landing_ops=False, auto_reset=True, episode_steps=40, trained_red=cs["trained_red"])
    g = BatchedGame(E, ["small"] * nb, ["large"] * nb, scenario=sc, grid=grid, seed=seed)
    if cs["epw"]:
        g.set_epw(cs["epw"])
    g.reset(positions=spawns, pos_per_env=torch.from_numpy(pos))
    return g


def _same(x, y):
    """Bit for bit (cog is NaN for a side without ships left)."""
    if x.dtype == torch.float32:
        x, y = x.view(torch.int32), y.view(torch.int32)
    elif x.dtype == torch.float64:
        x, y = x.view(torch.int64), y.view(torch.int64)
    return torch.equal(x, y)


@pytest.mark.parametrize("name", sorted(CASES))
def test_step_seq_equals_steps(name):
    from lnw import _abi
    cs = CASES[name]
    grid = _oracle.load_fixture("grids.npz")["grid100"]
    E, nb, K = cs["E"], cs["nb"], 45
    A = 2 * nb
    acts = torch.from_numpy(np.random.default_rng(21).random((K, E, A, 4), dtype=np.float32)).cuda()
    g1 = _setup(cs, grid, seed=55)
    ref, after = [], []
    for k in range(K):
        a = acts[k].clone()
        out = g1.step(a)
        ref.append({n: v.clone() for n, v in out.items()})
        after.append(a)
    if cs["kernel"] == "units":
        assert g1.step_kernel() == _abi.KERNEL_UNITS
    g2 = _setup(cs, grid, seed=55)
    seq_acts = acts.clone()
    got = g2.step_seq(seq_acts, keep="all")
    torch.cuda.synchronize()
    for k in range(K):
        for n, v in ref[k].items():
            assert _same(got[n][k], v), (name, k, n)
        assert _same(seq_acts[k], after[k]), (name, k, "actions after the step")
    assert torch.equal(g1.get_state(), g2.get_state())
    if not cs["trained_red"]:
        assert not torch.equal(seq_acts, acts)  # salvos were written back
    d = torch.stack([r["done"] for r in ref])
    assert bool((d == 0).any())  # fights ended in victories
    # keep="last": the game's own buffers end holding the last step's outputs
    g3 = _setup(cs, grid, seed=55)
    out = g3.step_seq(acts.clone(), keep="last")
    torch.cuda.synchronize()
    for n, v in ref[-1].items():
        assert _same(out[n], v), (name, n, "keep=last")
    assert torch.equal(g1.get_state(), g3.get_state())
    for g in (g1, g2, g3):
        g.close()


def test_step_seq_vs_oracle_shard():
    """A sequence at config 3's per-GPU shard (8 192 envs, quiet direct mode,
    mixed quiet / fighting workgroups) against the CPU oracle directly: 45
    steps in one call, per (step, env) observation hashes, done, rewards and
    cog (orc_fullsize_range)."""
    from lnw.batched import BatchedGame
    from lnw.config import Scenario
    grid = _oracle.load_fixture("grids.npz")["grid100"]
    E, S, seed = 8192, 45, 313
    pos = np.array([REF_SPAWNS] * E, np.int32)
    loud = np.arange(E).reshape(-1, 32)[:, 16:].reshape(-1)
    pos[loud] = _melee(grid, len(loud), seed=7)
    sc = Scenario(landing_ops=False, auto_reset=True, episode_steps=40)
    g = BatchedGame(E, ["small"] * 4, ["large"] * 4, scenario=sc, grid=grid, seed=seed)
    g.reset(positions=REF_SPAWNS, pos_per_env=torch.from_numpy(pos))
    acts = np.random.default_rng(9).random((S, E, 8, 4), dtype=np.float32)
    out = g.step_seq(torch.from_numpy(acts).cuda(), keep="all")
    mult = (np.random.default_rng(4).integers(0, 1 << 30, 2 * 4 * 68, dtype=np.int64) * 2 + 1)
    mt = torch.from_numpy(mult).cuda()
    w = torch.cat([out["obs_blue"].reshape(S, E, -1), out["obs_red"].reshape(S, E, -1)], 2)
    w = w.contiguous().view(torch.int32).to(torch.int64) & 0xFFFFFFFF
    gh = (w * mt).sum(2).cpu().numpy().view(np.uint64)
    gr = torch.cat([out["rew_blue"], out["rew_red"]], 2).cpu().numpy()
    gd, gc = out["done"].cpu().numpy(), out["cog"].cpu().numpy()
    assert int((g.env_state()["err"] != 0).sum()) == 0
    g.close()
    oh, orw, od, oc = _oracle.fullsize(grid, 4, 4, [0] * 4 + [1] * 4, pos, acts, mult, seed, 40, pos_per_env=True)
    bad = np.argwhere(gh != oh)
    assert bad.size == 0, f"{len(bad)} (step, env) hashes differ, first {bad[:6].tolist()}"
    assert np.array_equal(gd, od)
    assert np.allclose(gr, orw, rtol=0, atol=1e-5)
    assert np.allclose(gc, oc, rtol=0, atol=1e-5, equal_nan=True)
    assert (gd == 0).any()


def test_step_seq_obs_false_keep_all():
    """keep="all" with obs=False: no observation tensors are allocated, and the
    other outputs equal K step(obs=False) calls."""
    from lnw.batched import BatchedGame
    from lnw.config import Scenario
    grid = _oracle.load_fixture("grids.npz")["grid100"]
    E, K = 256, 6
    acts = torch.from_numpy(np.random.default_rng(3).random((K, E, 8, 4), dtype=np.float32)).cuda()
    outs = []
    for mode in ("steps", "seq"):
        g = BatchedGame(E, ["small"] * 4, ["large"] * 4, scenario=Scenario(landing_ops=False), grid=grid, seed=9)
        g.reset(positions=REF_SPAWNS, pos_per_env=torch.from_numpy(_melee(grid, E, seed=4)))
        if mode == "steps":
            outs.append([{k: v.clone() for k, v in g.step(acts[k].clone(), obs=False).items()
                          if not k.startswith("obs_")} for k in range(K)])
        else:
            got = g.step_seq(acts.clone(), obs=False, keep="all")
            assert not any(k.startswith("obs_") for k in got)
            outs.append([{n: v[k] for n, v in got.items()} for k in range(K)])
        g.close()
    for a, b in zip(*outs):
        for n in a:
            assert _same(a[n], b[n]), n
