"""Probe: one config-5 MAPPO rollout (32768 envs x 40 steps, batched actor +
critic + step kernel) for rocprofv3 kernel traces."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "littoral-naval-warfare-marl_amd"))
import bench  # noqa: E402

print(bench.mappo_rollout(E=int(os.environ.get("E", 32768)), T=40, reps=1))
