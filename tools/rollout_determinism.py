#!/usr/bin/env python3
"""Diagnostics: the fused rollout run repeatedly from one env state (same
rollout index) -- direct path twice, then the non-direct path (per-step
callback) -- and where the buffers first differ.
usage: python tools/rollout_determinism.py [E] [T] [contact 0/1]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "littoral-naval-warfare-marl_amd")]


def main():
    import torch
    from lnw.batched import BatchedGame
    from lnw.config import Scenario
    from lnw.rollout import BatchedActor, BatchedCritic, Rollout
    E = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
    T = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    contact = bool(int(sys.argv[3])) if len(sys.argv) > 3 else True
    blue, red = [(6, 61), (10, 81), (8, 70), (11, 58)], [(98, 48), (98, 52), (98, 56), (96, 52)]
    sc = Scenario(landing_ops=False, auto_reset=False, trained_red=False)
    g = BatchedGame(E, ["small"] * 4, ["large"] * 4, scenario=sc, seed=5)
    g.set_variant(contact)
    g.reset(positions=blue + red, box=((40, 40), (57, 65)))
    torch.manual_seed(2)
    actor = BatchedActor.for_obs(g.Db).cuda()
    critic = BatchedCritic(g.Db * g.nb).cuda()
    r = Rollout(g, actor, critic, steps=T, noise=0.05, seed=99)
    snap = g.get_state(device="cuda")
    outs = []
    plain = g.observe_into

    def synced(*args, **kw):  # the same call, then a full device synchronisation
        plain(*args, **kw)
        torch.cuda.synchronize()
    modes = sys.argv[4].split(",") if len(sys.argv) > 4 else ["direct", "direct", "callback", "direct"]
    for mode in [m for m in modes if m != "graph"]:
        g.set_state(snap)
        r.call_index(7)
        cb = (lambda t, out: None) if mode == "callback" else None
        g.observe_into = synced if mode == "sync" else plain
        import lnw.rollout as lr
        lr.STRIDED_POLICY_INPUT = mode == "strided"
        o = {k: v.clone() for k, v in r.run(on_step=cb).items() if v is not None}
        torch.cuda.synchronize()
        outs.append((mode, o, g.get_state()))
    if "graph" in modes or len(sys.argv) > 5:
        r.capture()
        for k in range(int(sys.argv[5]) if len(sys.argv) > 5 else 2):
            g.set_state(snap)
            r.call_index(7)
            o = {k2: v.clone() for k2, v in r.replay().items() if v is not None}
            torch.cuda.synchronize()
            outs.append(("graph", o, g.get_state()))
    base = outs[0]
    for mode, o, st in outs[1:]:
        bad = []
        for k, v in base[1].items():
            if not torch.equal(torch.nan_to_num(v, nan=7.0), torch.nan_to_num(o[k], nan=7.0)):
                d = (torch.nan_to_num(v, nan=7.0) != torch.nan_to_num(o[k], nan=7.0))
                idx = d.nonzero()
                first_t = int(idx[:, 1].min()) if v.dim() > 1 else -1
                bad.append(f"{k}: {int(d.sum())} differ, first step {first_t}, e.g. {idx[0].tolist()}")
        print(mode, "vs direct:", "identical" if not bad else bad, "| final state equal:", torch.equal(st, base[2]),
              flush=True)


if __name__ == "__main__":
    main()
