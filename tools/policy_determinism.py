#!/usr/bin/env python3
"""Diagnostics: lnw_policy_act called repeatedly on the same rows (packed, and
strided in place like the rollout's direct path) -- are the outputs
bit-identical from call to call?
usage: python tools/policy_determinism.py [E] [reps] [variants,...]
POLICY_LIB=path: an lnw_actor.hip-only build (tools/probe). Differing rows are
reported with their 64-row waves."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "littoral-naval-warfare-marl_amd")]


def main():
    import torch
    from lnw import _abi
    from lnw.rollout import BatchedActor
    path = os.environ.get("POLICY_LIB")
    if path:  # an lnw_actor.hip-only build (tools/probe)
        L = C.CDLL(path)
        L.lnw_policy_act.argtypes = [C.POINTER(_abi.PolicyArgs), C.c_void_p]
        print("lib", path, flush=True)
    else:
        L = _abi.load()
    E = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    n, D, T, t = 4, 68, 40, 5
    rows = E * n
    torch.manual_seed(0)
    actor = BatchedActor.for_obs(D).cuda()
    ap = actor.packed_policy()
    obs = torch.rand((E, n, D), device="cuda")
    obs[:, :, :49] = torch.randint(0, 256, (E, n, 49), device="cuda") / 255.0
    buf = torch.zeros((E, T, n, D), device="cuda")
    alive = torch.ones((2 * n, E), dtype=torch.uint8, device="cuda")
    live = torch.ones(E, dtype=torch.bool, device="cuda")
    call = torch.zeros(1, dtype=torch.int64, device="cuda")
    out2 = torch.zeros((E, T, n, D), device="cuda")
    variants = sys.argv[3].split(",") if len(sys.argv) > 3 else ["packed", "strided", "strided_sync",
                                                                   "strided_copy", "packed_inplace",
                                                                   "strided_nolive", "strided_noout"]
    if "critic" in variants:  # lnw_rollout_post's critic (MFMA f32), strided rollout-buffer rows
        from lnw.rollout import BatchedCritic
        variants = [v for v in variants if v != "critic"]
        cp = BatchedCritic(n * D).cuda().packed(n, D)
        val = torch.zeros((E, T), device="cuda")
        ref = None
        nd = 0
        for k in range(reps):
            buf[:, t] = obs
            val.zero_()
            pp = _abi.RolloutPostArgs()
            pp.obs, pp.obs_env_stride, pp.E, pp.n, pp.D = buf.data_ptr() + t * n * D * 4, T * n * D, E, n, D
            pp.critic, pp.val, pp.val_env_stride = cp.data_ptr(), val.data_ptr() + t * 4, T
            assert L.lnw_rollout_post(C.byref(pp), None) == 0
            torch.cuda.synchronize()
            cur = val[:, t].clone()
            if ref is None:
                ref = cur
                continue
            if not torch.equal(cur, ref):
                d = (cur != ref).nonzero()[:, 0]
                nd += 1
                if nd <= 6:
                    print("critic rep", k, len(d), "envs differ, max |d|", float((cur - ref).abs().max()),
                          "envs", d[:6].tolist(), "lanes", sorted(set((d % 64).tolist()))[:8], flush=True)
        print("critic mismatching reps:", nd, "of", reps - 1, flush=True)
    for var in variants:
        strided = var.startswith("strided")
        ref = None
        nd = 0
        waves, lanes = set(), set()
        for k in range(reps):
            buf[:, t] = obs
            if var == "strided_sync":
                torch.cuda.synchronize()
            acts = torch.zeros((E, T, n, 4), device="cuda")
            logp = torch.zeros((E, T, n, 4), device="cuda")
            full = torch.zeros((E, 2 * n, 4), dtype=torch.float64, device="cuda")
            pa = _abi.PolicyArgs()
            src = buf.data_ptr() + t * n * D * 4 if strided else obs.data_ptr()
            pa.obs, pa.E, pa.n, pa.D, pa.own0, pa.A = src, E, n, D, 0, 2 * n
            pa.obs_in_env_stride = T * n * D if strided else 0
            pa.params, pa.noise, pa.seed, pa.call_dev, pa.T, pa.t = ap.data_ptr(), 0.05, 99, call.data_ptr(), T, t
            pa.alive, pa.live = alive.data_ptr(), live.data_ptr()
            pa.obs_out, pa.obs_env_stride = buf.data_ptr() + t * n * D * 4, T * n * D
            if var == "strided_copy":
                pa.obs_out = out2.data_ptr() + t * n * D * 4
            if var == "packed_inplace":
                pa.obs_out, pa.obs_env_stride = obs.data_ptr(), n * D
            if var == "strided_nolive":
                pa.live = None
            if var == "strided_noout":
                pa.obs_out = None
            pa.act_out, pa.logp_out, pa.act_env_stride = acts.data_ptr() + t * n * 16, logp.data_ptr() + t * n * 16, T * n * 4
            pa.full = full.data_ptr()
            assert L.lnw_policy_act(C.byref(pa), None) == 0
            torch.cuda.synchronize()
            cur = [acts[:, t].clone(), logp[:, t].clone(), full.clone()]
            names = ["act", "logp", "full"]
            if ref is None:
                ref = cur
                continue
            for name, x, y in zip(names, cur, ref):
                if not torch.equal(x, y):
                    d = (x != y).nonzero()
                    nd += 1
                    rr = d[:, 0] * n + d[:, 1]   # (env, ship) -> row
                    waves |= set((rr // 64).tolist())
                    lanes |= set((rr % 64).tolist())
                    if nd <= 6:
                        print(var, "rep", k, name, int((x != y).sum()), "differ, max |d|",
                              float((x - y).abs().max()), "rows", sorted(set(rr.tolist()))[:6],
                              "waves", sorted(set((rr // 64).tolist()))[:6], flush=True)
        if hasattr(L, "lnw_probe_counts"):  # probe 12: rows whose second head differed, per stage
            cnt = (C.c_uint * 640)()
            L.lnw_probe_counts(cnt)
            names = (["fc1 bf16 split terms, row tiles 0-2", "fc1 bf16 split terms, row tile 3",
                      "fc1 before tanh, row tiles 0-2", "fc1 before tanh, row tile 3",
                      "h1 after tanh, row tiles 0-2", "h1 after tanh, row tile 3", "-", "-", "-", "-"]
                     if "disturb16" in (path or "") else
                     [f"layer {lay} ({'heads' if lay == 'h4' else 'tanh'}) in row tiles {t} vs the rerun"
                      for lay in ("h1", "h2", "h3", "h4") for t in ("0-2", "3")]
                     if "disturb15" in (path or "") else
                     ["tile read back after the second head's write (beside the partner's MLP)",
                      "tile row just before the wave's own MLP",
                      "fc1 operands as the MLP loaded them from the tile",
                      "per-row outputs vs a rerun of the MLP (MLPs beside MLPs)",
                      "head outputs before the lane gather vs the rerun"]
                     if ("disturb13" in (path or "") or "disturb14" in (path or "")) else
                     ["window loads", "pooled conv1 maps (LDS)", "conv head out", "LayerNorm tail loads",
                      "LayerNorm out"])
            for st, name in enumerate(names):
                if name == "-":
                    continue
                c = list(cnt[st * 64:(st + 1) * 64])
                if sum(c):
                    ln = [l for l in range(64) if c[l]]
                    print(var, "probe stage", name, ":", sum(c), "rows, lanes", ln[0], "..", ln[-1], flush=True)
                else:
                    print(var, "probe stage", name, ": 0 rows", flush=True)
        print(var, "mismatching (rep, output) pairs:", nd, "of", len(ref) * (reps - 1),
              "waves involved:", len(waves), sorted(waves)[:10],
              "lanes:", (min(lanes), max(lanes)) if lanes else None, flush=True)


if __name__ == "__main__":
    main()
