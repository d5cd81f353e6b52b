"""One rank of the sharded-rollout test (tests/test_gpu_rollout.py::
test_rollout_shards_equal_one_rank): lnw.rollout.Rollout over this rank's
env_range share of the global envs (env_id_base = its first global env),
keyed sampling (keyed_normal), two rollouts back to back; saves the rollout
buffers for the parent. Child process: WORLD_SIZE / RANK / MASTER_* in the
environment, gloo, every rank on cuda:0."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "littoral-naval-warfare-marl_amd")]

BLUE = [(6, 61), (10, 81), (8, 70), (11, 58)]
RED = [(98, 48), (98, 52), (98, 56), (96, 52)]


def main():
    out, total, red = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    import torch
    from lnw import dist
    from lnw.batched import BatchedGame
    from lnw.config import Scenario
    from lnw.rollout import BatchedActor, BatchedCritic, Rollout
    ws, rank, _ = dist.init("gloo")
    torch.cuda.set_device(0)
    lo, hi = dist.env_range(total, ws, rank)
    sc = Scenario(landing_ops=False, tactics="aggressive", side="blue",
                  trained_red=red != "script", auto_reset=True, episode_steps=40)
    g = BatchedGame(hi - lo, ["small"] * 4, ["large"] * 4, scenario=sc, device=0, seed=77,
                    env_id_base=lo, reward_dtype=torch.float64)
    g.set_variant(True)
    torch.manual_seed(0)
    actor = BatchedActor.for_obs(g.Db).cuda()
    critic = BatchedCritic(g.Db * g.nb).cuda()
    red_actor = BatchedActor.for_obs(g.Dr).cuda() if red == "actor" else None
    r = Rollout(g, actor, critic, steps=40, red=red, red_actor=red_actor, noise=0.05,
                keyed_seed=11)
    # melee-box spawns: contact, fire and sinkings inside the 40 steps
    g.reset(positions=BLUE + RED, box=((40, 40), (57, 65)))
    res = {}
    for k in range(2):
        o = r.run()
        for key, v in o.items():
            res[f"{key}{k}"] = v.cpu().numpy()
    torch.cuda.synchronize()
    dist.barrier()
    np.savez(out, lo=lo, hi=hi, **res)
    g.close()
    dist.finalize()


if __name__ == "__main__":
    main()
