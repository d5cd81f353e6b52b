#!/usr/bin/env python3
"""A/B timing of lnw_step_seq's kernels against lnw_step launches at the
headline shape (reference spawns): per-step milliseconds from HIP events for
K separate steps (sync) and for K-step sequences through the one-launch
sequence kernels (seq: LNW_SEQ_FUSED, read at lnw_create, so each
configuration builds its own game).
usage: python tools/seq_timing.py [E] [K] [config,...]   config = sync | seq"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "littoral-naval-warfare-marl_amd")]


def main():
    import ctypes
    import torch
    import bench
    from lnw import _abi
    E = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    cfgs = sys.argv[3].split(",") if len(sys.argv) > 3 else ["sync", "seq"]
    L = _abi.load()
    acts = torch.empty((3 * K, E, 8, 4), dtype=torch.float32, device="cuda")
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    for s in range(3 * K):
        _abi.check(L.lnw_fill_uniform_f32(ctypes.c_void_p(acts[s].data_ptr()), E * 32, 42, s << 40, st))
    for cfg in cfgs:
        os.environ.pop("LNW_SEQ_FUSED", None)
        if cfg == "seq":
            os.environ["LNW_SEQ_FUSED"] = "1"
        g = bench.make_game(E, 0, "reference", 0, 0)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        res = []
        for rep in range(3):
            a = acts[rep * K:(rep + 1) * K]
            torch.cuda.synchronize()
            ev[0].record()
            if cfg == "sync":
                for s in range(K):
                    g.step(a[s])
            else:
                g.step_seq(a, keep="last")
            ev[1].record()
            torch.cuda.synchronize()
            res.append(ev[0].elapsed_time(ev[1]) / K * 1e3)
        print(f"{cfg:10s} E={E} K={K}: us/step per rep " + " ".join(f"{x:.2f}" for x in res),
              "kernel", g.step_kernel(), flush=True)
        g.close()


if __name__ == "__main__":
    main()
