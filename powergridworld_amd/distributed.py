"""One process per GPU, env-sharded data parallelism.

Envs are independent: the agents -> bus load -> power flow -> voltage penalty
coupling stays inside one env.  So each rank steps its own contiguous shard of
the global batch and the step path has no collective.  The only collectives
are after the fact: max-over-ranks of a wall time, and an optional all-gather
of per-env episode statistics (<= N x 8 B per rank; over xGMI with the "nccl"
backend, which is RCCL on ROCm).
"""
import os
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass(frozen=True)
class Shard:
    rank: int
    world: int
    start: int      # first global env index owned by this rank
    count: int      # envs owned by this rank

    @property
    def stop(self):
        return self.start + self.count


def shard_bounds(total_envs: int, rank: int, world: int) -> Shard:
    """Contiguous split of `total_envs`; the first `total_envs % world` ranks get one more."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank %d / world %d" % (rank, world))
    base, extra = divmod(int(total_envs), world)
    start = rank * base + min(rank, extra)
    return Shard(rank, world, start, base + (1 if rank < extra else 0))


def rank_seed(base_seed: int, rank: int, stream: int = 0) -> int:
    """Distinct, reproducible seed per (rank, stream) (e.g. stream = agent index)."""
    return int(base_seed) + 1000 * int(rank) + int(stream)


def env_rank():
    """(rank, local_rank, world) from the torchrun environment (1 process if unset)."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")),
            int(os.environ.get("WORLD_SIZE", "1")))


def init(backend: str, device=None):
    """init_process_group from the torchrun environment (MASTER_ADDR defaults to
    127.0.0.1); a no-op for world size 1.  Returns (rank, local_rank, world)."""
    rank, local, world = env_rank()
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        kw = {"device_id": device} if (backend == "nccl" and device is not None) else {}
        dist.init_process_group(backend, **kw)
    return rank, local, world


def max_over_ranks(value: float, device=None) -> float:
    """The job's time is its slowest rank's."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(value)
    if dist.get_backend() == "gloo":
        device = "cpu"
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_episode_stats(stats: torch.Tensor) -> torch.Tensor:
    """All-gather per-env statistics [n_local, ...] into [sum n_local, ...] in
    global env order (shards are contiguous and rank-ordered).  Called once per
    episode, never on the step path."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return stats
    if dist.get_backend() == "gloo" and stats.device.type != "cpu":
        # gloo collectives run on host tensors: stage through the CPU
        return gather_episode_stats(stats.cpu()).to(stats.device)
    world = dist.get_world_size()
    n = torch.tensor([stats.shape[0]], dtype=torch.int64, device=stats.device)
    counts = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(counts, n)
    counts = [int(c.item()) for c in counts]
    width = max(counts)
    pad = torch.zeros((width,) + tuple(stats.shape[1:]), dtype=stats.dtype, device=stats.device)
    pad[:stats.shape[0]] = stats
    parts = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(parts, pad)
    return torch.cat([p[:c] for p, c in zip(parts, counts)])
