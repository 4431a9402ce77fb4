"""Multi-GPU plumbing: one process per GPU, torch.distributed over RCCL ("nccl").

The hot path shards embarrassingly: each rank owns env replicas
[rank*E, (rank+1)*E) with their own agents, replay rings and streams, seeded by
global env id, and runs with NO data-path collectives.  Collectives appear only
(a) outside timed regions (barrier, max-over-ranks timing) and (b) in the
shared-parameter DQN configuration (C5), where the flat f32 gradient is
all-reduced and averaged (`allreduce_mean_`).

Every collective call here is bounded: init_process_group gets a timeout (the
rendezvous and the backend's own operations), and barrier / max_over_ranks
wait on their work with a timeout.  A failure raises DistError naming the rank
and the call, so a first-time RCCL problem ends the run with a cause instead of
hanging to an outer limit.  DMDQN_DIST_TIMEOUT_S overrides the default.
"""
import datetime
import os

import numpy as np
import torch
import torch.distributed as dist


def world():
    """(rank, world_size, local_rank) from the torch.distributed.run environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


DEFAULT_TIMEOUT_S = float(os.environ.get("DMDQN_DIST_TIMEOUT_S", "180"))


class DistError(RuntimeError):
    """A collective failed or timed out (the message names rank and call)."""


def _td(timeout_s):
    return datetime.timedelta(seconds=DEFAULT_TIMEOUT_S if timeout_s is None else timeout_s)


def _fail(call, exc):
    raise DistError(f"rank {world()[0]} of {world()[1]}: {call} failed: "
                    f"{type(exc).__name__}: {exc}") from exc


def init(backend=None, device=None, timeout_s=None, force=False):
    """init_process_group from the torch.distributed.run environment, with a
    timeout (rendezvous and the backend's operations); raises DistError.
    force: also for a world of one (tests: the RCCL path on a one-GPU box)."""
    rank, ws, local = world()
    if (ws > 1 or force) and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        kw = {"device_id": device} if (backend == "nccl" and device is not None) else {}
        try:
            dist.init_process_group(backend, timeout=_td(timeout_s), **kw)
        except Exception as e:  # noqa: BLE001 -- any failure is reported with its cause
            _fail(f"init_process_group({backend}, MASTER_ADDR="
                  f"{os.environ.get('MASTER_ADDR')}, MASTER_PORT={os.environ.get('MASTER_PORT')})", e)
    return rank, ws, local


def _wait(work, call, timeout_s):
    try:
        work.wait(timeout=_td(timeout_s))
    except Exception as e:  # noqa: BLE001
        _fail(call, e)


def shard(rank, envs_per_rank, base_seed=0):
    """Global env ids and seeds of this rank's replicas (weak scaling)."""
    offset = rank * envs_per_rank
    ids = np.arange(offset, offset + envs_per_rank, dtype=np.int64)
    return offset, ids + base_seed


def barrier(timeout_s=None):
    """All ranks meet, within the timeout (DistError otherwise)."""
    if dist.is_initialized():
        try:
            work = dist.barrier(async_op=True)
        except Exception as e:  # noqa: BLE001
            _fail("barrier", e)
        _wait(work, "barrier", timeout_s)


def max_over_ranks(x: float, device="cpu", timeout_s=None):
    """Slowest rank's value (the job's wall time)."""
    if not dist.is_initialized():
        return float(x)
    if dist.get_backend() == "gloo":
        device = "cpu"
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    try:
        work = dist.all_reduce(t, op=dist.ReduceOp.MAX, async_op=True)
    except Exception as e:  # noqa: BLE001
        _fail("all_reduce(MAX) of the timed region", e)
    _wait(work, "all_reduce(MAX) of the timed region", timeout_s)
    return float(t.item())


def allreduce_mean_(t: torch.Tensor):
    """In-place sum over ranks then scale by 1/world (shared-parameter DQN, C5).
    One fused flat buffer per learn step: the 114 KB gradient is latency-bound
    on xGMI, so it goes as a single collective."""
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        t.mul_(1.0 / dist.get_world_size())
    return t
