#!/usr/bin/env python3
"""Config 5 under a profiler: bench.mappo_rollout on one GPU
-- 32 768 envs, 40-step MAPPO rollouts of the batched actor + critic
interleaved with the step kernel, eager and replayed from a HIP graph -- so a
`rocprofv3 --kernel-trace --stats` of this script gives the per-kernel split of
a rollout step (tools/gpu/prof_r03.sh, profiles/r03_config5_rocprof.md)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "littoral-naval-warfare-marl_amd")]


def main():
    import torch
    import bench
    torch.cuda.set_device(0)
    res = bench.mappo_rollout(total=int(sys.argv[1]) if len(sys.argv) > 1 else 32768)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
