"""One rank of the multi-rank bench test (tests/test_gpu_bench_ranks.py):
bench.run_workload over this rank's env_range share of the global envs, the
max-over-ranks reduction and barrier bench.main uses, then the per-env state
digest saved for the parent. Run as a child process (WORLD_SIZE / RANK /
MASTER_* in the environment, gloo, every rank on cuda:0)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "littoral-naval-warfare-marl_amd")]


def main():
    out, total, steps, spawns = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    import torch
    import bench
    from lnw import dist
    ws, rank, _ = dist.init("gloo")
    torch.cuda.set_device(0)
    lo, hi = dist.env_range(total, ws, rank)
    res = bench.run_workload(hi - lo, lo, spawns, 0, 0, steps, 5, digest=True)
    el, km, err, eps, dig = (res[k] for k in ("elapsed", "kernel_ms", "err", "episodes", "digest"))
    el_max, km_max = dist.reduce_max([el, km])
    assert el_max >= el and km_max >= km
    n = dist.reduce_sum([hi - lo])[0]
    assert n == total
    dist.barrier()
    np.savez(out, lo=lo, hi=hi, digest=dig, err=err, episodes=eps, elapsed=el_max)
    dist.finalize()


if __name__ == "__main__":
    main()
