"""bench.py's rank launching on the CPU (no GPU): `--gpus N` without a
launcher starts its own N ranks through torch.distributed.run (the driver's
contract names `bench.py --gpus N`), and a rank count that disagrees with
WORLD_SIZE is refused. `--dry-run` runs the launcher and process-group
plumbing (gloo, barrier, max-over-ranks) without the step; the real two-rank
step through the same self-launch is tests/test_gpu_bench_ranks.py."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LAUNCH_VARS = ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "TORCHELASTIC_RUN_ID",
               "LNW_BENCH_LAUNCHER")


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in LAUNCH_VARS}
    env.update(kw)
    return env


def test_gpus_two_without_launcher_starts_two_ranks():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run"],
                       env=_env(), capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 alone prints
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["dry_run"] is True and line["value"] is None
    assert line["config"]["dist_backend"] == "gloo"
    assert line["config"]["dist_world_size"] == 2
    assert line["config"]["launcher"] == "self"
    assert "starting 2 ranks" in r.stderr


def test_world_size_must_match_gpus():
    env = _env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "3", "--dry-run"],
                       env=env, capture_output=True, text=True, timeout=120, cwd=ROOT)
    assert r.returncode == 2
    assert "rank count must match" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def test_gpus_more_than_visible_refused():
    """Without LNW_FORCE_DEVICE, asking for more ranks than visible GPUs fails
    before any rank starts (this container has none)."""
    env = _env()
    env.pop("LNW_FORCE_DEVICE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"],
                       env=env, capture_output=True, text=True, timeout=120, cwd=ROOT)
    assert r.returncode == 2 and "GPU(s) visible" in r.stderr
