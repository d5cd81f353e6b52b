"""Config 5 rollout alone (bench.mappo_rollout), for rocprofv3 kernel stats:
rocprofv3 --kernel-trace --stats -d DIR -- python3 tools/rollout_probe.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "littoral-naval-warfare-marl_amd")]
import bench  # noqa: E402

print(json.dumps(bench.mappo_rollout(reps=2)))
