"""Multi-GPU plumbing: one process per GPU, torch.distributed over RCCL ("nccl").

The hot path shards embarrassingly: each rank owns env replicas
[rank*E, (rank+1)*E) with their own agents, replay rings and streams, seeded by
global env id, and runs with NO data-path collectives.  Collectives appear only
(a) outside timed regions (barrier, max-over-ranks timing) and (b) in the
shared-parameter DQN configuration (C5), where the flat f32 gradient is
all-reduced (`BoundedAllReduce`; the Adam kernel applies the 1/world mean).

Every collective call here is bounded: init_process_group gets a timeout (the
rendezvous and the backend's own operations), and barrier / max_over_ranks /
gather_device_ids wait on their work with a timeout; the per-learn gradient
all-reduce is bounded with a lag (BoundedAllReduce).  A failure raises DistError naming the rank
and the call, so a first-time RCCL problem ends the run with a cause instead of
hanging to an outer limit.  DMDQN_DIST_TIMEOUT_S overrides the default.
"""
import datetime
import os
import time

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
    timeout_s also becomes the default of every later bounded call.
    force: also for a world of one (tests: the RCCL path on a one-GPU box)."""
    global DEFAULT_TIMEOUT_S
    if timeout_s is not None:  # every later bounded call of this process uses it
        DEFAULT_TIMEOUT_S = float(timeout_s)
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


class BoundedAllReduce:
    """all_reduce(SUM) of one flat buffer per call -- the C5 shared-net
    gradient (agent.BatchedDQN._learn_shared; the 1/world mean is applied by
    the Adam kernel's gscale) -- bounded like every other collective here.

    RCCL ("nccl"): issued with async_op, and work.wait() without a timeout
    orders the caller's stream after it, so the host keeps running ahead of
    the GPU.  The host blocks only when more than `lag` reductions are still
    incomplete, and then for at most timeout_s on the oldest one: a peer that
    stalls or never issues its reduction raises DistError naming this rank and
    the call instead of hanging to the watchdog.
    gloo (CPU tensors; several ranks on one device in the tests): the work is
    waited on at once with the timeout."""

    def __init__(self, lag=4, timeout_s=None,
                 call="all_reduce(SUM) of the shared-net gradient"):
        self.lag, self.timeout_s, self.call = int(lag), timeout_s, call
        self._pending = []  # (work, issue time) of the incomplete RCCL reductions

    def __call__(self, t: torch.Tensor):
        if not dist.is_initialized() or dist.get_world_size() == 1:
            return t
        gloo = dist.get_backend() == "gloo"
        try:
            work = dist.all_reduce(t, op=dist.ReduceOp.SUM, async_op=True)
        except Exception as e:  # noqa: BLE001
            _fail(self.call, e)
        if gloo:
            _wait(work, self.call, self.timeout_s)
            return t
        try:
            work.wait()  # stream order only (no host block without a timeout)
        except Exception as e:  # noqa: BLE001
            _fail(self.call, e)
        self._pending = [(w, t0) for w, t0 in self._pending if not w.is_completed()]
        self._pending.append((work, time.monotonic()))
        if len(self._pending) > self.lag:
            self._await_oldest()
        return t

    def _await_oldest(self):
        w, t0 = self._pending.pop(0)
        limit = _td(self.timeout_s).total_seconds()
        while not w.is_completed():
            if time.monotonic() - t0 > limit:
                _fail(self.call, TimeoutError(
                    f"not complete {limit:.0f} s after it was issued ({self.lag} later "
                    "reductions queued behind it): a peer rank stalled or skipped it"))
            time.sleep(50e-6)

    def drain(self):
        """Wait (bounded) for every outstanding reduction."""
        while self._pending:
            self._await_oldest()


def gather_device_ids(device, timeout_s=None):
    """Every rank's (rank, device name, PCI domain:bus:device, UUID) --
    bench.py prints them so a multi-GPU record shows N distinct GPUs.  One
    bounded all_gather of fixed-size byte rows."""
    import torch as _t
    if _t.device(device).type == "cuda":
        p = _t.cuda.get_device_properties(device)
        me = (f"{world()[0]}|{p.name}|{getattr(p, 'pci_domain_id', 0):04x}:"
              f"{getattr(p, 'pci_bus_id', 0):02x}:{getattr(p, 'pci_device_id', 0):02x}|"
              f"{getattr(p, 'uuid', '')}")
    else:  # the CPU rehearsals (gloo)
        me = f"{world()[0]}|cpu|-|-"
    if not dist.is_initialized():
        return [me]
    row = 256
    dev = "cpu" if dist.get_backend() == "gloo" else device
    buf = _t.zeros(row, dtype=_t.uint8)
    b = me.encode()[:row]
    buf[:len(b)] = _t.tensor(list(b), dtype=_t.uint8)
    buf = buf.to(dev)
    outs = [_t.zeros(row, dtype=_t.uint8, device=dev) for _ in range(dist.get_world_size())]
    try:
        work = dist.all_gather(outs, buf, async_op=True)
    except Exception as e:  # noqa: BLE001
        _fail("all_gather of the device ids", e)
    _wait(work, "all_gather of the device ids", timeout_s)
    return [bytes(o.cpu().tolist()).rstrip(b"\0").decode(errors="replace") for o in outs]
