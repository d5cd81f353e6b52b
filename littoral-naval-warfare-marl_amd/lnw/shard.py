"""Env sharding across GPUs (one process per GPU): rank r owns the contiguous
global env range [lo, hi). The RNG is keyed by global env id
(lnw_create's env_id_base), so a trajectory does not depend on the GPU count."""


def env_range(total_envs, world_size, rank):
    base, extra = divmod(int(total_envs), int(world_size))
    lo = rank * base + min(rank, extra)
    hi = lo + base + (1 if rank < extra else 0)
    return lo, hi
