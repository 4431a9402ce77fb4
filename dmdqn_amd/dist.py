"""Multi-GPU plumbing: one process per GPU, torch.distributed over RCCL ("nccl").

The hot path shards embarrassingly: each rank owns env replicas
[rank*E, (rank+1)*E) with their own agents, replay rings and streams, seeded by
global env id, and runs with NO data-path collectives.  Collectives appear only
(a) outside timed regions (barrier, max-over-ranks timing) and (b) in the
shared-parameter DQN configuration (C5), where the flat f32 gradient is
all-reduced and averaged (`allreduce_mean_`).
"""
import os

import numpy as np
import torch
import torch.distributed as dist


def world():
    """(rank, world_size, local_rank) from the torch.distributed.run environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init(backend=None, device=None):
    rank, ws, local = world()
    if ws > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        kw = {"device_id": device} if (backend == "nccl" and device is not None) else {}
        dist.init_process_group(backend, **kw)
    return rank, ws, local


def shard(rank, envs_per_rank, base_seed=0):
    """Global env ids and seeds of this rank's replicas (weak scaling)."""
    offset = rank * envs_per_rank
    ids = np.arange(offset, offset + envs_per_rank, dtype=np.int64)
    return offset, ids + base_seed


def barrier():
    if dist.is_initialized():
        dist.barrier()


def max_over_ranks(x: float, device="cpu"):
    """Slowest rank's value (the job's wall time)."""
    if not dist.is_initialized():
        return float(x)
    if dist.get_backend() == "gloo":
        device = "cpu"
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def allreduce_mean_(t: torch.Tensor):
    """In-place sum over ranks then scale by 1/world (shared-parameter DQN, C5).
    One fused flat buffer per learn step: the 114 KB gradient is latency-bound
    on xGMI, so it goes as a single collective."""
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        t.mul_(1.0 / dist.get_world_size())
    return t
