"""The N>1 path of bench.py on one GPU: two rank processes (gloo, both on
cuda:0) each step their lnw.shard.env_range half of the global envs through
bench.run_workload (env_id_base = the shard's first global env, actions keyed
by global env id), with bench.main's reduce_max / barrier; their final
per-env states must equal a single-rank run over all envs. Then bench.main
itself runs with two ranks (torch.distributed.run) and must report the whole
job's throughput over the global env count."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _ranks(tmp_path, world, total, steps, spawns):
    port = _port()
    procs = []
    for r in range(world):
        env = dict(os.environ, WORLD_SIZE=str(world), RANK=str(r), LOCAL_RANK=str(r),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "_bench_rank.py"),
                                       str(tmp_path / f"w{world}_r{r}.npz"), str(total), str(steps),
                                       spawns], env=env))
    for p in procs:
        assert p.wait(timeout=240) == 0
    return [np.load(tmp_path / f"w{world}_r{r}.npz") for r in range(world)]


@pytest.mark.parametrize("spawns", ["reference", "melee"])
def test_two_ranks_equal_one(tmp_path, spawns):
    total, steps = 4096, 45  # crosses the 40-step auto-reset
    one = _ranks(tmp_path, 1, total, steps, spawns)[0]
    two = _ranks(tmp_path, 2, total, steps, spawns)
    assert [(int(d["lo"]), int(d["hi"])) for d in two] == [(0, 2048), (2048, 4096)]
    got = np.concatenate([d["digest"] for d in two])
    assert np.array_equal(got, one["digest"])
    assert int(one["err"]) == 0 and sum(int(d["err"]) for d in two) == 0
    assert sum(int(d["episodes"]) for d in two) == int(one["episodes"]) > 0


def test_bench_main_two_ranks():
    env = dict(os.environ, LNW_FORCE_DEVICE="0", LNW_DIST_BACKEND="gloo")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_port()}", os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "20", "--warmup", "5", "--global-envs", "8192",
           "--no-cpu-baseline"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["scaling"] == "strong"
    assert line["config"]["global_envs"] == 8192 and line["config"]["envs_per_gpu"] == 4096
    assert line["value"] == pytest.approx(8192 * 20 / (line["ms_per_step"] * 20 / 1e3), rel=1e-9)
    assert line["err_envs"] == 0 and line["config"]["dist_backend"] == "gloo"
    # at N > 1 the line carries config 5 split over the ranks
    c5 = line["secondary"]["config5_mappo_rollout"]
    assert list(line["secondary"]) == ["config5_mappo_rollout"]
    assert c5["envs"] == 32768 and c5["envs_per_gpu"] == 16384 and c5["n_gpus"] == 2
    assert c5["env_steps_per_sec"] == pytest.approx(32768 * 40 / (c5["ms_per_rollout"] / 1e3))


def test_bench_gpus_two_self_launched():
    """`python bench.py --gpus 2` with no launcher: bench.py starts its two
    ranks itself (torch.distributed.run as a child) and the line reports them."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "TORCHELASTIC_RUN_ID", "LNW_BENCH_LAUNCHER")}
    env.update(LNW_FORCE_DEVICE="0", LNW_DIST_BACKEND="gloo")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "20", "--warmup", "5",
           "--global-envs", "8192", "--no-cpu-baseline", "--no-secondary"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["config"]["dist_world_size"] == 2
    assert line["config"]["launcher"] == "self" and line["config"]["dist_backend"] == "gloo"
    assert line["config"]["envs_per_gpu"] == 4096 and line["err_envs"] == 0 and line["value"] > 0


def test_bench_main_rccl_one_rank():
    """bench.py under torch.distributed.run with one rank: the process group
    is RCCL ("nccl" backend) and the max-over-ranks all_reduce and barriers
    the driver's N > 1 runs use go through it."""
    env = dict(os.environ)
    env.pop("LNW_DIST_BACKEND", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr=127.0.0.1", f"--master-port={_port()}", os.path.join(ROOT, "bench.py"),
           "--gpus", "1", "--steps", "20", "--warmup", "5", "--global-envs", "8192",
           "--no-cpu-baseline", "--no-secondary"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert line["config"]["dist_backend"] == "nccl" and line["config"]["dist_world_size"] == 1
    assert line["n_gpus"] == 1 and line["err_envs"] == 0 and line["value"] > 0
