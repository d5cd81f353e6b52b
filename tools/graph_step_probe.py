#!/usr/bin/env python3
"""Probe: the headline workload (65 536 4v4 envs, reference spawns, fresh
U[0,1) actions per step) stepped K times eagerly vs replayed from a HIP graph
of the same K step launches (torch.cuda.graph around BatchedGame.step): does the
graph shorten the gap between back-to-back step kernels?

usage: python tools/graph_step_probe.py [--steps 200]
"""
import argparse
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "littoral-naval-warfare-marl_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    args = ap.parse_args()
    from lnw import _abi
    from lnw.batched import BatchedGame
    from lnw.config import Scenario
    import bench
    L = _abi.load()
    E, K = 65536, args.steps
    sc = Scenario(landing_ops=False, tactics="aggressive", side="blue", trained_red=True,
                  auto_reset=True, episode_steps=40)
    g = BatchedGame(E, ["small"] * 4, ["large"] * 4, scenario=sc, device=0, seed=1234)
    g.reset(positions=bench.REF_BLUE + bench.REF_RED)
    acts = torch.empty((3 * K, E, 8, 4), dtype=torch.float32, device="cuda")
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    for s in range(3 * K):
        _abi.check(L.lnw_fill_uniform_f32(ctypes.c_void_p(acts[s].data_ptr()), E * 32, 42, s * E * 32, st))
    torch.cuda.synchronize()
    for s in range(20):
        g.step(acts[s])
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    for s in range(K):
        g.step(acts[K + s])
    e1.record()
    torch.cuda.synchronize()
    print(f"eager: wall {1e6 * (time.perf_counter() - t0) / K:.1f} us/step, "
          f"events {1e3 * e0.elapsed_time(e1) / K:.1f} us/step", flush=True)
    graph = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        with torch.cuda.graph(graph, stream=side):
            for s in range(K):
                g.step(acts[2 * K + s])
    torch.cuda.synchronize()
    for rep in range(2):
        t0 = time.perf_counter()
        e0.record()
        graph.replay()
        e1.record()
        torch.cuda.synchronize()
        print(f"graph replay {rep}: wall {1e6 * (time.perf_counter() - t0) / K:.1f} us/step, "
              f"events {1e3 * e0.elapsed_time(e1) / K:.1f} us/step", flush=True)
    st_ = g.env_state()
    print("err envs", int((st_["err"] != 0).sum()))
    g.close()


if __name__ == "__main__":
    main()
