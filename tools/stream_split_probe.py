#!/usr/bin/env python3
"""Probe: the headline workload (65 536 4v4 envs, reference spawns) stepped as
S env shards on S HIP streams (one lnw handle each), so one shard's latency
head (state/action reads, move lookups) can overlap another shard's observation
stream. Prints ms per full step for S = 1, 2, 4 with and without a start offset.

usage: python tools/stream_split_probe.py [--steps 200]
"""
import argparse
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
    ap.add_argument("--envs", type=int, default=65536)
    args = ap.parse_args()
    import ctypes
    from lnw import _abi
    from lnw.batched import BatchedGame
    from lnw.config import Scenario
    import bench
    L = _abi.load()
    E = args.envs
    NA = args.steps + 20  # fresh actions every step, as bench.py (repeating a few
    # action sets drifts the fleets into contact and off the quiet path)
    for S, default in ((1, True), (1, False), (2, False), (4, False)):
        for offset in ((False,) if S == 1 else (False, True)):
            sc = Scenario(landing_ops=False, tactics="aggressive", side="blue", trained_red=True,
                          auto_reset=True, episode_steps=40)
            Es = E // S
            streams = [torch.cuda.current_stream() if default else torch.cuda.Stream() for _ in range(S)]
            games, acts = [], []
            for s in range(S):
                with torch.cuda.stream(streams[s]):
                    g = BatchedGame(Es, ["small"] * 4, ["large"] * 4, scenario=sc,
                                    device=torch.cuda.current_device(), env_id_base=s * Es, seed=1234)
                    # 64 envs per workgroup (full waves: the quiet path) so each
                    # shard's grid takes only its share of the resident slots
                    assert L.lnw_set_epw(g.h, 64) == 64
                    g.reset(positions=bench.REF_BLUE + bench.REF_RED)
                    a = torch.empty((NA, Es, 8, 4), dtype=torch.float32, device="cuda")
                    for k in range(NA):
                        _abi.check(L.lnw_fill_uniform_f32(ctypes.c_void_p(a[k].data_ptr()), Es * 32, 42,
                                                          (k * E + s * Es) * 32,
                                                          ctypes.c_void_p(streams[s].cuda_stream)))
                    games.append(g)
                    acts.append(a)
            torch.cuda.synchronize()

            # raw C-ABI calls with pre-converted arguments (no per-call torch
            # stream context, whose cost alone would exceed a step)
            calls = []
            for s in range(S):
                g = games[s]
                ob, orr, rb, rr, dn, cg = g._outp
                calls.append([(g.h, acts[s][k].data_ptr(), 0, None, ob, orr, rb, rr, dn, cg,
                               streams[s].cuda_stream) for k in range(NA)])
            f = L.lnw_step

            def run(n, stagger, k0=0):
                for k in range(k0, k0 + n):
                    for s in range(S):
                        if stagger and k == k0 and s > 0:
                            with torch.cuda.stream(streams[s]):
                                torch.cuda._sleep(int(20000 * s / S))  # ~ a fraction of a step
                        f(*calls[s][k % NA])
            run(20, offset)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            run(args.steps, offset, 20)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / args.steps
            print(f"shards={S} default_stream={default} offset={offset}: {dt * 1e6:.1f} us/step, {E / dt / 1e9:.3f} G env-steps/s",
                  flush=True)
            for g in games:
                g.close()


if __name__ == "__main__":
    main()
