#!/usr/bin/env python3
"""Timing probe of the fused rollout kernels alone (csrc/lnw_actor.hip):
lnw_policy_act and lnw_rollout_post over config 5's 32 768 4v4 envs (131 072
actor rows) on random observation rows, HIP-event timed on the launch stream.
usage: python tools/policy_probe.py [lib.so ...]   (default: the in-tree
liblnw.so; tools/probe/*.so are lnw_actor.hip builds with LNW_PROBE_* defines)."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "littoral-naval-warfare-marl_amd")]


def main():
    import torch
    from lnw import _abi
    from lnw.rollout import BatchedActor, BatchedCritic
    libs = sys.argv[1:] or [_abi.LIB_PATH]
    torch.manual_seed(0)
    E, n, D, T = 32768, 4, 68, 40
    actor = BatchedActor.for_obs(D).cuda()
    critic = BatchedCritic(D * n).cuda()
    ap, cp = actor.packed_policy(), critic.packed(n, D)
    obs = torch.rand((E, n, D), device="cuda")
    obs[:, :, :49] = torch.randint(0, 256, (E, n, 49), device="cuda") / 255.0
    alive = torch.ones((2 * n, E), dtype=torch.uint8, device="cuda")
    live = torch.ones(E, dtype=torch.bool, device="cuda")
    full = torch.zeros((E, 2 * n, 4), dtype=torch.float64, device="cuda")
    kinds = torch.zeros((E, 2 * n), dtype=torch.uint8, device="cuda")
    obuf = torch.zeros((E, T, n, D), device="cuda")
    abuf = torch.zeros((E, T, n, 4), device="cuda")
    lbuf = torch.zeros((E, T, n, 4), device="cuda")
    val = torch.zeros((E, T), device="cuda")
    rew = torch.zeros((E, n), dtype=torch.float64, device="cuda")
    rbuf = torch.zeros((E, T, n), dtype=torch.float64, device="cuda")
    done = torch.ones(E, dtype=torch.int32, device="cuda")
    run = torch.zeros((E, T), dtype=torch.bool, device="cuda")
    call = torch.zeros(1, dtype=torch.int64, device="cuda")
    table = torch.zeros((3, 40, 4), dtype=torch.float64, device="cuda")
    for path in libs:
        L = C.CDLL(path)
        L.lnw_policy_act.argtypes = [C.POINTER(_abi.PolicyArgs), C.c_void_p]
        L.lnw_rollout_post.argtypes = [C.POINTER(_abi.RolloutPostArgs), C.c_void_p]
        pa = _abi.PolicyArgs()
        pa.obs, pa.E, pa.n, pa.D, pa.own0, pa.A = obs.data_ptr(), E, n, D, 0, 2 * n
        pa.params, pa.noise, pa.seed, pa.call_dev, pa.T, pa.t = ap.data_ptr(), 0.05, 5, call.data_ptr(), T, 3
        pa.alive, pa.live, pa.obs_out, pa.obs_env_stride = alive.data_ptr(), live.data_ptr(), obuf.data_ptr(), T * n * D
        pa.act_out, pa.logp_out, pa.act_env_stride = abuf.data_ptr(), lbuf.data_ptr(), T * n * 4
        pa.full, pa.script, pa.script_n, pa.script_steps = full.data_ptr(), table.data_ptr(), 3, 40
        pa.script_own0, pa.script_cnt, pa.kinds = n, n, kinds.data_ptr()
        pp = _abi.RolloutPostArgs()
        pp.obs, pp.obs_env_stride, pp.E, pp.n, pp.D = obuf.data_ptr(), T * n * D, E, n, D
        pp.critic, pp.val, pp.val_env_stride = cp.data_ptr(), val.data_ptr(), T
        pp.rew, pp.rew_f64, pp.n_rew, pp.rew_out, pp.rew_env_stride = rew.data_ptr(), 1, n, rbuf.data_ptr(), T * n
        pp.done, pp.live, pp.running, pp.running_env_stride, pp.stop_at_done = (
            done.data_ptr(), live.data_ptr(), run.data_ptr(), T, 1)
        st = torch.cuda.current_stream().cuda_stream
        res = {}
        for name, fn, args in (("policy_act", L.lnw_policy_act, pa), ("rollout_post", L.lnw_rollout_post, pp)):
            for _ in range(5):
                assert fn(C.byref(args), st) == 0
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(50):
                fn(C.byref(args), st)
            e1.record()
            torch.cuda.synchronize()
            res[name] = round(e0.elapsed_time(e1) / 50 * 1e3, 1)
        print(os.path.basename(path), res, flush=True)


if __name__ == "__main__":
    main()
