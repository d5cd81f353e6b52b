#!/usr/bin/env python3
"""Benchmark: env-steps/sec of the batched 4v4 littoral env step on MI355X.

Driver contract: `python bench.py --gpus N --steps K --warmup W` (N>1 under
torch.distributed.run, one process per GPU). Prints ONE JSON line on rank 0.

Workload (BASELINE.json metric, config 3): 65 536 parallel 4v4 environments
on the whole node — rank r of N steps the global envs lnw.shard.env_range
gives it (65 536 / N each, RNG keyed by global env id), on the 100x100 Baltic
grid, reference spawns (blue game.py:556; red (98,48),(98,52),(98,56),(96,52)),
40-step episodes with in-kernel auto-reset, U[0,1)^4 float32 actions from
Philox (seed 42), tactics aggressive, side blue, trained red. Total work is
fixed as N grows (strong scaling); `--envs E` instead fixes E envs per GPU
(weak scaling). A "step" = one Game.step over every env of the GPU; inputs
(actions for all timed steps) are resident in HBM before the timed region.
At N=1 the line also carries `secondary` measurements: config 3's per-GPU
shard (8 192 envs) and config 2 (4 096), melee spawns, the unpruned LOS
march / A* mode, config 4 and config 5, each with its kernel time and the
fraction of the HBM roofline its algorithmic bytes reach.
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "littoral-naval-warfare-marl_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

REF_BLUE = [(6, 61), (10, 81), (8, 70), (11, 58)]
REF_RED = [(98, 48), (98, 52), (98, 56), (96, 52)]
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


# 8 small blue vs 8 large + 2 LandingShip red, landing
# ops, the 200x200 grid, spawns on water cells of a box inside x in [0, 99]
CONFIG4 = dict(blue=["small"] * 8, red=["large"] * 8 + ["ls"] * 2, G=200, landing_ops=True,
               box=((20, 60), (80, 140)), rand_ls=[0] * 16 + [1, 1], envs=8192)


def algorithmic_bytes(nb, nr, quiet=False):
    """Minimum HBM bytes one env-step must move:
    actions in (f32), observations + rewards + done + cog out, and the SoA state
    read once (26 B/agent + 52 B/env) and written back: all of it, or for a
    quiet step (no pair in sensor range: reference spawns on the LOS-table path)
    only what such a step changes — cell, radar and step counter per agent
    (12 B) and the env's step counter (4 B)."""
    A = nb + nr
    act = A * 4 * 4
    obs = (nb * (4 * nb + 52) + nr * (4 * nr + 52)) * 4
    out = A * 4 + 4 + 4
    state = A * 26 + 52
    return act + obs + out + state + (A * 12 + 4 if quiet else state)


REF_LOS_CELLS = 10996  # Bresenham cells per 4v4 env-step, reference spawns


def survey_bytes(nb, nr):
    """SURVEY.md §8(d)'s estimate of the same quantity, with a generic 64 B of
    state per agent and 32 B per env (3 432 B at 4v4); reported beside the
    build's own minimum for reference."""
    A = nb + nr
    return A * 16 + (nb * (4 * nb + 52) + nr * (4 * nr + 52)) * 4 + A * 4 + 8 + 2 * A * 64 + 2 * 32


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--global-envs", type=int, default=65536,
                   help="environments over all ranks (BASELINE config 3: 65 536), split by "
                        "lnw.shard.env_range")
    p.add_argument("--envs", type=int, default=None,
                   help="environments per GPU instead (weak scaling)")
    p.add_argument("--spawns", choices=["reference", "melee"], default="reference")
    p.add_argument("--workload", choices=["config3", "config4"], default="config3",
                   help="config3 = the headline 4v4 line; config4 = 8v10+LS on 200x200 "
                        "(diagnostics, e.g. with LNW_PROF=1)")
    p.add_argument("--los-mode", type=int, default=0, help="0 LOS table, 1 ray march")
    p.add_argument("--move-mode", type=int, default=0, help="0 move table, 1 direct A*")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=12.0)
    p.add_argument("--cpu-threads", type=int, default=min(16, os.cpu_count() or 1),
                   help="threads for the CPU baseline (the GPU box's share is 16 cores)")
    p.add_argument("--episode-steps", type=int, default=40,
                   help="episode horizon (config.json: 40); diagnostics only")
    p.add_argument("--no-secondary", action="store_true",
                   help="skip the secondary lines (configs 2, 3-shard, 4, 5, melee, march)")
    p.add_argument("--secondary-steps", type=int, default=100)
    p.add_argument("--dry-run", action="store_true",
                   help="launcher plumbing only (runs without a GPU): the ranks start, join the "
                        "process group and run the barrier / max-over-ranks timing around an "
                        "empty region; the line's value is null")
    return p.parse_args()


def free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n):
    """`bench.py --gpus N` without a launcher (WORLD_SIZE unset): start the N
    rank processes through torch.distributed.run as a child process, before
    this process has touched the GPU (nothing here initialises HIP, so no
    exec-after-GPU-init), with the same arguments. Rank 0 prints the JSON line
    to the inherited stdout; returns the launcher's exit code."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__)]
    cmd += sys.argv[1:]
    log(f"bench.py: --gpus {n} without a launcher; starting {n} ranks: {' '.join(cmd[1:])}")
    return subprocess.call(cmd, cwd=ROOT)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


EPISODE_STEPS = 40  # config.json hyperparameters.episode_steps


def make_game(E, env_base, spawns, los_mode, move_mode, cfg=None):
    from lnw.batched import BatchedGame, default_grid
    from lnw.config import Scenario
    if cfg is None:
        sc = Scenario(landing_ops=False, tactics="aggressive", side="blue", trained_red=True,
                      auto_reset=True, episode_steps=EPISODE_STEPS, los_mode=los_mode,
                      move_mode=move_mode)
        g = BatchedGame(E, ["small"] * 4, ["large"] * 4, scenario=sc,
                        device=torch.cuda.current_device(), env_id_base=env_base, seed=1234)
        # melee: fleets in contact every step -> the contact variant of the
        # step kernel (lnw_set_variant; identical results)
        g.set_variant(spawns == "melee")
        box = ((40, 40), (57, 65)) if spawns == "melee" else None
        g.reset(positions=REF_BLUE + REF_RED, box=box)
        return g
    sc = Scenario(landing_ops=cfg["landing_ops"], tactics="aggressive", side="blue",
                  trained_red=True, auto_reset=True, episode_steps=40, los_mode=los_mode,
                  move_mode=move_mode)
    g = BatchedGame(E, cfg["blue"], cfg["red"], scenario=sc, device=torch.cuda.current_device(),
                    env_id_base=env_base, seed=1234, grid=default_grid(cfg["G"]))
    n = len(cfg["blue"]) + len(cfg["red"])
    g.reset(positions=[(0, 0)] * n, rand_ls=cfg["rand_ls"], box=cfg["box"])
    return g


def run_workload(E, env_base, spawns, los_mode, move_mode, steps, warmup, cfg=None, digest=False,
                 count_work=True):
    """Create the envs [env_base, env_base + E) of one rank, fill the actions of
    every step (Philox keyed by global env id and step, so a global env's
    inputs do not depend on the sharding), run `warmup` untimed steps, then
    time `steps` launches between barriers. Returns a dict: wall seconds, mean
    kernel ms from HIP events on the launch stream, envs with error bits,
    episodes completed, with `count_work` the device work counters (rays /
    cells marched, A* searches, pooled bearings) per env-step over exactly the
    timed window (a second, untimed pass that replays the same warmup and timed
    steps from the same initial state with the counters bound: the step is
    deterministic, so it walks the same trajectory), and with `digest` the
    per-env final state."""
    from lnw import _abi
    L = _abi.load()
    g = make_game(E, env_base, spawns, los_mode, move_mode, cfg)
    A = g.A
    # inputs resident before the timed region: actions for every step; the
    # value of (global env, agent, component) at step s sits at Philox counter
    # offset s * 2^40 + (env * A + agent) * 4 + component
    acts = torch.empty((warmup + steps, E, A, 4), dtype=torch.float32, device="cuda")
    per = E * A * 4
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    for s in range(warmup + steps):
        off = (s << 40) + env_base * A * 4
        _abi.check(L.lnw_fill_uniform_f32(ctypes.c_void_p(acts[s].data_ptr()), per, 42, off, stream))
    torch.cuda.synchronize()
    for s in range(warmup):
        g.step(acts[s])
    torch.cuda.synchronize()
    # HIP events on the stream the step kernel is launched on (torch's current
    # stream), bracketing the K back-to-back launches of the timed region
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    from lnw import dist
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record()
    for s in range(steps):
        g.step(acts[warmup + s])
    ev1.record()
    torch.cuda.synchronize()
    dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    kms = ev0.elapsed_time(ev1) / steps
    st = g.env_state()
    err = int((st["err"] != 0).sum())
    episodes = int(st["episode"].sum())
    work = None
    if count_work and not digest:
        # untimed replay of the same window with the work counters bound
        # (atomics): a fresh game from the same seed and spawns, the warmup
        # steps, then the timed steps counted
        final = {k: st[k].copy() for k in ("rng", "episode", "steps_done")}
        g.close()
        g = make_game(E, env_base, spawns, los_mode, move_mode, cfg)
        for s in range(warmup):
            g.step(acts[s])
        g.count_work(True)
        for s in range(steps):
            g.step(acts[warmup + s])
        torch.cuda.synchronize()
        work = {k: v / (E * steps) for k, v in g.work_counts().items()}
        g.count_work(False)
        st2 = g.env_state()
        same = all(np.array_equal(final[k], st2[k]) for k in final)
        work["window"] = (f"the {steps} timed steps (after {warmup} warmup steps), replayed "
                          f"untimed with counters bound; same trajectory: {same}")
    dig = None
    if digest:
        ag = g.agents()
        dig = np.stack([ag["x"], ag["y"], ag["radar"], ag["missiles"], ag["alive"],
                        ag["steps_done"]], 2).astype(np.int64).reshape(E, -1)
        dig = np.concatenate([dig, np.stack([st[k] for k in ("n_blue_left", "n_red_left",
                                                             "steps_done", "episode")], 1),
                              st["rng"].astype(np.int64)[:, None]], 1)
    g.close()
    del acts
    return dict(elapsed=elapsed, kernel_ms=kms, err=err, episodes=episodes, digest=dig,
                work_per_env_step=work)


def measured_traffic(args, E):
    """HBM bytes per launch from rocprofv3 PMC counters (2 x FETCH_SIZE +
    WRITE_SIZE, MI355X_MICROARCH.md's gfx950 correction), as recorded in
    profiles/traffic.json by tools/gpu/prof.sh together with the SHA-256 of
    the sources and flags of the liblnw.so it measured (lnw.build.source_digest).
    Reported only if this run's library is built from those same sources (and
    is the in-tree build); otherwise null."""
    from lnw import _abi
    from lnw.build import DEPS, OUT, source_digest
    tf = os.path.join(ROOT, "profiles", "traffic.json")
    try:
        tj = json.load(open(tf))
        lib = os.path.realpath(os.environ.get("LNW_LIB", _abi.LIB_PATH))
        if lib != os.path.realpath(OUT) or any(os.path.getmtime(d) > os.path.getmtime(OUT) for d in DEPS):
            return None  # another library, or an in-tree build older than its sources
        if tj.get("src_sha256") != source_digest():
            return None
        wl = "config4" if args.workload == "config4" else args.spawns
        return tj.get("launch_bytes", {}).get(f"{wl}_e{E}_los{args.los_mode}_mv{args.move_mode}")
    except (OSError, ValueError):
        return None


def ray_march(n=1 << 22, reps=10):
    """The LOS ray-march kernel alone (lnw_los_batch, combatant.py:436-456) on
    n random rays with offsets in [-37, 37]^2 (the sensor ranges): rays/s and
    reference-equivalent Bresenham cells/s (max(|dx|,|dy|) + 1 per ray)."""
    from lnw import _abi
    from lnw.batched import default_grid
    L = _abi.load()
    rng = np.random.default_rng(3)
    x1 = rng.integers(0, 100, n)
    y1 = rng.integers(0, 100, n)
    x2 = np.clip(x1 + rng.integers(-37, 38, n), 0, 99)
    y2 = np.clip(y1 + rng.integers(-37, 38, n), 0, 99)
    cells = float(np.sum(np.maximum(np.abs(x2 - x1), np.abs(y2 - y1)) + 1))
    pairs = torch.from_numpy(np.stack([x1, y1, x2, y2], 1).astype(np.int16)).cuda()
    grid = torch.from_numpy(default_grid(100)).cuda()
    out = torch.empty(n, dtype=torch.uint8, device="cuda")
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)

    def launch():
        _abi.check(L.lnw_los_batch(ctypes.c_void_p(grid.data_ptr()), 100,
                                   ctypes.c_void_p(pairs.data_ptr()), n, 74, 70,
                                   ctypes.c_void_p(out.data_ptr()), stream))
    launch()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        launch()
    e1.record()
    torch.cuda.synchronize()
    sec = e0.elapsed_time(e1) / reps * 1e-3
    return dict(rays_per_sec=n / sec, cells_per_sec=cells / sec, ms_per_launch=sec * 1e3,
                rays=n, mean_cells_per_ray=cells / n)


def config5_bytes(nb=4, nr=4):
    """Algorithmic HBM bytes per env-step of config 5's four launches (a 4v4
    rollout step, blue actor, scripted red; ppo.py:497-605's data flow), each
    read or written once:
      observe      state read (26 B/agent + 52 B/env), blue rows out (4 nb + 52
                   floats each), target-list counts and the RNG counter back;
      policy       blue rows in, alive / live flags; the f64 action array of the
                   step (every agent), the rollout's f32 actions and log-probs,
                   row kinds and the f32 flag out;
      step         the action array and kinds in, the state read and written back
                   (contact), f64 rewards, done and cog out;
      post         blue rows (the critic's input), rewards, done and live in; the
                   value, rewards, running and live flags out."""
    A = nb + nr
    state = A * 26 + 52
    rows = nb * (4 * nb + 52) * 4
    out = dict(observe=state + rows + A * 2 + 8,
               policy=rows + A + 1 + A * 4 * 8 + 2 * nb * 4 * 4 + A + 1,
               step=A * 4 * 8 + A + 2 * state + A * 8 + 4 + 8,
               post=rows + nb * 8 + 4 + 1 + 4 + nb * 8 + 1 + 1)
    out["total"] = sum(out.values())
    return out


def mappo_rollout(total=32768, T=40, reps=3):
    """40-step MAPPO rollouts of `total` envs over the
    ranks (rank r holds lnw.shard.env_range's share, env_id_base = its first
    global env), the batched actor (network.py MLP) acting for every blue ship
    and the critic scoring every step, interleaved with the step kernel
    (lnw.rollout.Rollout, scripted red). Each rank times its rollouts between
    barriers; the slowest rank's time (max over ranks) sets the whole-job
    env-steps/s, policy forwards included."""
    from lnw import dist
    from lnw.batched import BatchedGame
    from lnw.config import Scenario
    from lnw.rollout import BatchedActor, BatchedCritic, Rollout
    world, rank, _ = dist.world()
    lo, hi = dist.env_range(total, world, rank)
    E = hi - lo
    sc = Scenario(landing_ops=False, tactics="aggressive", side="blue", trained_red=False,
                  auto_reset=True, episode_steps=40)
    g = BatchedGame(E, ["small"] * 4, ["large"] * 4, scenario=sc,
                    device=torch.cuda.current_device(), seed=77, env_id_base=lo)
    torch.manual_seed(0)
    actor = BatchedActor.for_obs(g.Db).cuda()
    critic = BatchedCritic(g.Db * g.nb).cuda()
    gen = torch.Generator(device="cuda").manual_seed(5 + rank)
    g.set_variant(True)  # scripted red closes in: contact most steps
    r = Rollout(g, actor, critic, steps=T, noise=0.05, seed=5)  # fused HIP policy kernels, keyed by global row
    g.reset(positions=REF_BLUE + REF_RED)
    r.run(generator=gen)
    torch.cuda.synchronize()

    def timed(fn):
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            g.reset(positions=REF_BLUE + REF_RED)
            fn()
        torch.cuda.synchronize()
        dist.barrier()
        return dist.reduce_max([(time.perf_counter() - t0) / reps])[0]

    dt = timed(lambda: r.run(generator=gen))
    # the same rollout replayed from a HIP graph (Rollout.capture): no host work
    # between the four launches of a step
    g.reset(positions=REF_BLUE + REF_RED)
    r.capture(generator=gen)
    torch.cuda.synchronize()
    dtg = timed(r.replay)
    g.close()
    # roofline of the whole step (its four launches back to back from the graph):
    # algorithmic bytes per env-step x this rank's envs / the step's wall time
    B = config5_bytes()
    step_s = dtg / T
    ach = B["total"] * E / step_s / 1e9
    roof = dict(bound="hbm", achieved=ach, peak=HBM_PEAK_GBS, unit="GB/s", frac=ach / HBM_PEAK_GBS,
                algorithmic_bytes_per_env_step=B, us_per_step=step_s * 1e6,
                note="all four launches of a step together (observe, policy, step, post); per-kernel "
                     "split and PMC traffic in profiles/r06_config5_rocprof.md")
    return dict(env_steps_per_sec=total * T / dtg, ms_per_rollout=dtg * 1e3, roofline=roof,
                eager_env_steps_per_sec=total * T / dt, eager_ms_per_rollout=dt * 1e3,
                envs=total, envs_per_gpu=E, n_gpus=world, steps=T,
                policy="fused HIP policy step (lnw_policy_act: conv head + MLP + keyed sample + "
                       "log-prob + action array; lnw_rollout_post: critic + rewards), fp32; per step "
                       "observe, policy, step, post = 4 launches; HIP-graph replay (eager loop "
                       "alongside); max over ranks")


def cpu_baseline(seconds, threads):
    """The CPU oracle (oracle/lnw_oracle.c, a C restatement of the reference
    step) timed on the host over a bounded sample of the same workload: one
    thread, then `threads` threads over disjoint env ranges (ctypes drops the
    GIL). The threaded rate is the reported baseline."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import _oracle
    from concurrent.futures import ThreadPoolExecutor
    L = _oracle.lib()
    L.orc_bench_range.restype = ctypes.c_int64
    L.orc_bench_range.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                  ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                  ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_uint64]
    from lnw.batched import default_grid
    grid = np.ascontiguousarray(default_grid(100), np.uint8)
    P = _oracle.OrcParams(0, 0, 1, 1, 1, 0.4, 74, 70, 14, 82)
    types = np.array([0] * 4 + [1] * 4, np.int32)
    pos = np.array(REF_BLUE + REF_RED, np.int32).reshape(-1)

    def run(env0, n_envs):
        return L.orc_bench_range(ctypes.byref(P), grid.ctypes.data_as(ctypes.c_void_p), 100, 4, 4,
                                 types.ctypes.data_as(ctypes.c_void_p),
                                 pos.ctypes.data_as(ctypes.c_void_p), env0, n_envs, 40, 40, 42)

    t = time.perf_counter()
    run(0, 16)
    dt = time.perf_counter() - t
    per_env = max(dt / 16, 1e-5)
    half = seconds / 2
    env1 = max(16, int(half / per_env))
    t = time.perf_counter()
    n1 = run(0, env1)
    dt1 = time.perf_counter() - t
    envs_t = max(16, int(half / per_env)) * threads
    chunk = (envs_t + threads - 1) // threads
    t = time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:
        nt = sum(ex.map(lambda i: run(i * chunk, chunk), range(threads)))
    dtt = time.perf_counter() - t
    return dict(value=nt / dtt, unit="env-steps/sec", cores=threads, kind="port",
                sample=f"{threads * chunk} envs x 40 steps on {threads} threads ({dtt:.1f} s); "
                       f"1 thread: {env1} envs x 40 steps ({dt1:.1f} s); 4v4, reference spawns, "
                       "U[0,1) f32 actions, auto-reset; CPU oracle restatement",
                single_thread_value=n1 / dt1)


def line_entry(E, res, steps, nb=4, nr=4, desc="", quiet=False):
    """One secondary measurement: env-steps/s over the wall clock, the step
    kernel's mean time and its algorithmic bytes against the HBM roofline,
    and the device-counted ray-march / A* work per env-step."""
    B = algorithmic_bytes(nb, nr, quiet)
    el, km = res["elapsed"], res["kernel_ms"]
    ach = B * E / (km * 1e-3) / 1e9
    return dict(workload=desc, envs=E, env_steps_per_sec=E * steps / el, ms_per_step=el / steps * 1e3,
                kernel_ms=km, err_envs=res["err"], work_per_env_step=res["work_per_env_step"],
                roofline=dict(bound="hbm", achieved=ach, peak=HBM_PEAK_GBS, unit="GB/s",
                              frac=ach / HBM_PEAK_GBS, algorithmic_bytes_per_env_step=B))


def secondary_lines(args):
    """N=1 only: the other BASELINE configs and kernel modes, each timed like
    the headline (warmup, then K launches between barriers)."""
    K, W = args.secondary_steps, min(args.warmup, 20)
    out = {}
    for name, E, sp, lm, mm, desc in (
            ("config3_shard_32768", 32768, "reference", 0, 0,
             "config 3's per-GPU shard at N=2: 32 768 4v4 envs, reference spawns"),
            ("config3_shard_16384", 16384, "reference", 0, 0,
             "config 3's per-GPU shard at N=4: 16 384 4v4 envs, reference spawns"),
            ("config3_shard_8192", 8192, "reference", 0, 0,
             "config 3's per-GPU shard at N=8: 8 192 4v4 envs, reference spawns"),
            ("config2_4096", 4096, "reference", 0, 0, "config 2: 4 096 4v4 envs, reference spawns"),
            ("melee_65536", 65536, "melee", 0, 0,
             "65 536 4v4 envs, melee spawns (contact every step), contact kernel variant"),
            ("reference_march_astar", 65536, "reference", 1, 1,
             "65 536 4v4 envs, reference spawns, direct A* for every move (no move table) and "
             "LOS by ray march instead of the LOS table (los_mode 1); range pruning precedes "
             "every LOS query, and at these spawns no pair is in sensor range, so no ray is "
             "marched: this line measures direct A*"),
            ("reference_los_work", 65536, "reference", 2, 0,
             "65 536 4v4 envs, reference spawns, plus the reference's LOS work: every own x "
             "opponent Bresenham ray of every get_obs marched in full (los_mode 2)")):
        out[name] = line_entry(E, run_workload(E, 0, sp, lm, mm, K, W), K, desc=desc,
                               quiet=sp == "reference" and lm == 0)
        log(name, out[name])
    E4 = CONFIG4["envs"]
    out["config4_8v10ls_g200"] = line_entry(
        E4, run_workload(E4, 0, "config4", 0, 0, K, W, CONFIG4), K, len(CONFIG4["blue"]),
        len(CONFIG4["red"]),
        desc="config 4: 8 192 envs, 8 small blue vs 8 large + 2 landing ships, 200x200, landing ops")
    log("config4", out["config4_8v10ls_g200"])
    out["ray_march"] = ray_march()
    log("ray_march", out["ray_march"])
    out["config5_mappo_rollout"] = mappo_rollout()
    log("config5", out["config5_mappo_rollout"])
    return out


def dry_run(args, world, rank):
    """--dry-run: the launcher and process-group plumbing of an N-rank run
    without the step (no GPU needed): barrier, an empty timed region, the
    max-over-ranks reduction, and the line's rank and backend fields."""
    from lnw import dist
    dist.barrier()
    t0 = time.perf_counter()
    dist.barrier()
    elapsed = dist.reduce_max([time.perf_counter() - t0])[0]
    if rank == 0:
        print(json.dumps({"metric": "env-steps/sec (dry run: launcher plumbing only)", "value": None,
                          "unit": "env-steps/sec", "n_gpus": world, "steps": 0, "warmup": 0,
                          "ms_per_step": None, "higher_is_better": True, "dry_run": True,
                          "barrier_s": elapsed,
                          "config": {"dist_backend": dist.backend(), "dist_world_size": dist.size(),
                                     "launcher": os.environ.get("LNW_BENCH_LAUNCHER", "external")}}),
              flush=True)
    dist.finalize()


def main():
    args = parse()
    global EPISODE_STEPS
    EPISODE_STEPS = args.episode_steps
    from lnw import dist
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # the driver's contract names `--gpus N`: without a launcher, become one
        n_dev = torch.cuda.device_count()  # (does not initialise HIP on this image)
        if not args.dry_run and "LNW_FORCE_DEVICE" not in os.environ and n_dev < args.gpus:
            log(f"bench.py: --gpus {args.gpus} but {n_dev} GPU(s) visible")
            sys.exit(2)
        os.environ["LNW_BENCH_LAUNCHER"] = "self"
        sys.exit(launch_ranks(args.gpus))
    world, rank, local = dist.world()
    if world != args.gpus:
        log(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: the rank count must match")
        sys.exit(2)
    if args.dry_run:
        dist.init(os.environ.get("LNW_DIST_BACKEND", "gloo"))
        return dry_run(args, world, rank)
    # LNW_FORCE_DEVICE / LNW_DIST_BACKEND: the multi-rank test runs two ranks on
    # one GPU over gloo (tests/test_gpu_bench_ranks.py); the driver sets neither
    torch.cuda.set_device(int(os.environ.get("LNW_FORCE_DEVICE", local)))
    dist.init(os.environ.get("LNW_DIST_BACKEND", "nccl"))
    cfg = CONFIG4 if args.workload == "config4" else None
    if args.envs is not None:  # weak scaling: E per GPU
        E, env_base, total = args.envs, rank * args.envs, args.envs * world
        scaling = "weak"
    else:
        total = CONFIG4["envs"] if (cfg is not None and args.global_envs == 65536) else args.global_envs
        lo, hi = dist.env_range(total, world, rank)
        E, env_base = hi - lo, lo
        scaling = "strong"
    res = run_workload(E, env_base, args.spawns, args.los_mode, args.move_mode, args.steps,
                       args.warmup, cfg)
    elapsed, kms_mean, err, episodes = res["elapsed"], res["kernel_ms"], res["err"], res["episodes"]
    elapsed, kms_mean = dist.reduce_max([elapsed, kms_mean])
    err, episodes = (int(v) for v in dist.reduce_sum([err, episodes]))
    value = total * args.steps / elapsed
    nb, nr = (len(cfg["blue"]), len(cfg["red"])) if cfg else (4, 4)
    B = algorithmic_bytes(nb, nr, quiet=cfg is None and args.spawns == "reference" and args.los_mode == 0)
    achieved = B * E / (kms_mean * 1e-3) / 1e9
    traffic = measured_traffic(args, E)
    secondary = {}
    if world == 1 and not args.no_secondary and cfg is None:
        secondary = secondary_lines(args)
    elif world > 1 and not args.no_secondary and cfg is None:
        # config 5 is quoted on 8 GPUs: its 32 768 envs split over the ranks
        secondary = {"config5_mappo_rollout": mappo_rollout()}
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args.cpu_seconds, args.cpu_threads)
    if rank == 0:
        line = {
            "metric": (f"env-steps/sec (whole node), {total} parallel 4v4 envs on 100x100 grid"
                       if cfg is None else f"env-steps/sec, config 4 ({total} envs, diagnostic line)"),
            "value": value,
            "unit": "env-steps/sec",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": "f64+i32",
            "data": "synthetic",
            "config": {
                "workload": (f"{total} parallel 4v4 envs over {world} GPU(s) ({E} on rank 0), "
                             f"100x100 Baltic grid, {args.spawns} spawns, 40-step episodes with "
                             "auto-reset, U[0,1)^4 f32 actions") if cfg is None else
                            (f"{total} parallel 8v8+2LS envs (config 4) over {world} GPU(s), "
                             "200x200 grid, box spawns, landing ops, 40-step episodes with "
                             "auto-reset, U[0,1)^4 f32 actions"),
                "global_envs": total, "envs_per_gpu": E,
                "agents": "4v4" if cfg is None else f"{nb}v{nr}",
                "grid": 100 if cfg is None else cfg["G"],
                "spawns": args.spawns if cfg is None else "box",
                "kernel_variant": "contact" if (cfg is None and args.spawns == "melee") else "default",
                "los_mode": args.los_mode,
                "move_mode": args.move_mode, "parallelism": f"env-shard x{world}",
                "dist_backend": dist.backend(),
                "dist_world_size": dist.size(),
                "launcher": os.environ.get("LNW_BENCH_LAUNCHER", "external" if world > 1 else None),
            },
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "algorithmic_bytes_per_env_step": B,
                         "survey_bytes_per_env_step": survey_bytes(nb, nr),
                         "frac_at_survey_bytes": survey_bytes(nb, nr) * E / (kms_mean * 1e-3) / 1e9
                                                 / HBM_PEAK_GBS,
                         "kernel_ms_mean": kms_mean},
            "cpu_baseline": cpu,
            "err_envs": err,
            "episodes_completed": episodes,
        }
        if cfg is None and args.spawns == "reference" and args.los_mode == 0:
            # SURVEY §8(d) secondary work metric: the reference marches a Bresenham
            # ray for every own x opponent pair of every get_obs, 10 996 cells per
            # 4v4 env-step at these spawns (measured there)
            w = res["work_per_env_step"] or {}
            line["los_work"] = {"reference_equivalent_cells_per_env_step": REF_LOS_CELLS,
                                "reference_equivalent_cells_per_sec": REF_LOS_CELLS * value,
                                "marched_cells_per_env_step": w.get("cells_marched"),
                                "marched_rays_per_env_step": w.get("rays_marched"),
                                "astar_searches_per_env_step": w.get("astar_searches"),
                                "counted_over": "rank 0, device counters (lnw_set_counters): "
                                                + str(w.get("window"))}
        if secondary:
            line["secondary"] = secondary
        print(json.dumps(line), flush=True)
    dist.finalize()


if __name__ == "__main__":
    main()
