"""world_size-2 gloo tests of the multi-process plumbing (CPU only)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, ws, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(ws), LOCAL_RANK=str(rank))
    from dmdqn_amd import dist as D
    r, w, _ = D.init(backend="gloo")
    off, seeds = D.shard(r, 8, base_seed=1000)
    m = D.max_over_ranks(1.5 + r)
    g = torch.full((5,), float(r + 1))
    D.BoundedAllReduce()(g)
    ids = D.gather_device_ids("cpu")
    D.barrier()
    q.put((r, off, seeds.tolist(), m, g.tolist(), ids))
    dist.destroy_process_group()


@pytest.mark.parametrize("ws", [2])
def test_shard_timing_and_allreduce(ws):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, ws, port, q)) for r in range(ws)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(ws))
    for p in ps:
        p.join(timeout=60)
    seeds = [s for r in res for s in r[2]]
    assert len(set(seeds)) == 8 * ws                       # disjoint replicas
    assert [r[1] for r in res] == [0, 8]                   # env offsets
    assert all(r[3] == 1.5 + ws - 1 for r in res)          # max over ranks
    assert all(np.allclose(r[4], ws * (1 + ws) / 2.0) for r in res)  # sum of 1..ws
    assert all(r[5] == [f"{k}|cpu|-|-" for k in range(ws)] for r in res)  # every rank's id


def test_single_process_defaults():
    from dmdqn_amd import dist as D
    assert D.max_over_ranks(3.0) == 3.0
    t = torch.ones(3)
    assert torch.equal(D.BoundedAllReduce()(t), torch.ones(3))
    off, seeds = D.shard(3, 4, 10)
    assert off == 12 and list(seeds) == [22, 23, 24, 25]


def _shared_worker(rank, ws, port, q):
    """C5 orchestration across ranks with the kernels stubbed (CPU): the
    gradient each rank hands to Adam is the SUM over ranks of the per-rank
    (already 1/NA-scaled) gradients, with gscale = 1/world."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(ws), LOCAL_RANK=str(rank))
    from types import SimpleNamespace

    import dmdqn_amd.agent as AG
    from dmdqn_amd import dist as D
    D.init(backend="gloo")
    P = 8
    seen = {}

    def learn_shared_grad(*args, **kw):
        fake.grad.copy_(torch.arange(P, dtype=torch.float32) * (rank + 1))
        seen["scale"] = args[-1]

    def adam(params, m, v, target, target_h, params_h, grad, gscale, alpha, c1, c2, eps, sync):
        seen["grad"] = grad.tolist()
        seen["gscale"] = gscale
        seen["sync"] = sync

    ring = SimpleNamespace(s=None, n=None, a=None, d=None, r=None, start=0)
    fake = SimpleNamespace(NA=4, n_slabs=2, P=P, device="cpu", ring=ring, idx=None,
                           cfg=AG.AgentConfig(), loss=None, rn_out=None,
                           slab=torch.zeros((2, P)), grad=torch.zeros(P),
                           params=torch.zeros(P), adam_m=torch.zeros(P), adam_v=torch.zeros(P),
                           target=torch.zeros(P), target_h=None, params_h=None, shared_work=None,
                           shared_paths={"adam_slabs": 0, "allreduce": 0},
                           _ops=SimpleNamespace(learn_shared_grad=learn_shared_grad, adam=adam))
    AG.BatchedDQN._learn_shared(fake, 1e-3, 0.1, 1e-3, 1e-7, True, None)
    seen["paths"] = dict(fake.shared_paths)
    q.put((rank, seen))
    dist.destroy_process_group()


def test_shared_param_gradient_allreduce_two_ranks():
    ws = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_shared_worker, args=(r, ws, port, q)) for r in range(ws)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(ws))
    for p in ps:
        p.join(timeout=60)
    expect = (np.arange(8) * (1 + 2)).tolist()        # rank 0 (x1) + rank 1 (x2)
    for _, seen in res:
        assert np.isclose(seen["scale"], 1 / 4)        # 1 / local agents
        assert np.allclose(seen["grad"], expect)       # identical on every rank
        assert np.isclose(seen["gscale"], 1 / ws)      # mean over ranks in Adam
        assert seen["paths"] == {"adam_slabs": 0, "allreduce": 1}  # reduce, all-reduce, Adam
        assert seen["sync"] == 1


def _lonely_rank(port, q):
    """Rank 0 of a world of 2 whose rank 1 never starts."""
    import time
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0",
                      WORLD_SIZE="2", LOCAL_RANK="0")
    from dmdqn_amd import dist as D
    t0 = time.time()
    try:
        D.init(backend="gloo", timeout_s=4)
        q.put(("joined", time.time() - t0))
    except D.DistError as e:
        q.put((str(e), time.time() - t0))


def _stalled_peer(rank, port, q):
    """Both ranks join; rank 1 then never reaches the barrier."""
    import time
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE="2", LOCAL_RANK=str(rank))
    from dmdqn_amd import dist as D
    D.init(backend="gloo", timeout_s=4)
    if rank == 1:
        time.sleep(30)
        return
    t0 = time.time()
    try:
        D.barrier(timeout_s=4)
        q.put(("passed", time.time() - t0))
    except D.DistError as e:
        q.put((str(e), time.time() - t0))


def test_missing_rank_fails_fast_with_its_cause():
    """A rank that never joins: init_process_group raises DistError naming
    the rank and the call within its timeout (the driver's multi-GPU run
    then exits non-zero instead of hanging to the driver's limit)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_lonely_rank, args=(_free_port(), q))
    p.start()
    msg, dt = q.get(timeout=90)
    p.join(timeout=30)
    assert msg.startswith("rank 0 of 2: init_process_group(gloo"), msg
    assert dt < 60, dt


def test_stalled_barrier_fails_fast_with_its_cause():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_stalled_peer, args=(r, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    msg, dt = q.get(timeout=90)
    for p in ps:  # rank 1 is still asleep
        p.kill()
        p.join(timeout=30)
    assert msg.startswith("rank 0 of 2: barrier failed"), msg
    assert dt < 30, dt


def _skipping_peer(rank, port, q):
    """C5 learn orchestration (kernels stubbed) where rank 1 skips its
    gradient all-reduce and then stalls: rank 0's bounded all-reduce must
    raise DistError naming the rank and the call within the timeout
    (DMDQN_DIST_TIMEOUT_S, read at import)."""
    import time
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE="2", LOCAL_RANK=str(rank), DMDQN_DIST_TIMEOUT_S="4")
    from types import SimpleNamespace

    import dmdqn_amd.agent as AG
    from dmdqn_amd import dist as D
    D.init(backend="gloo")
    if rank == 1:
        time.sleep(30)
        return
    P = 8
    ring = SimpleNamespace(s=None, n=None, a=None, d=None, r=None, start=0)
    fake = SimpleNamespace(NA=4, n_slabs=2, P=P, device="cpu", ring=ring, idx=None,
                           cfg=AG.AgentConfig(), loss=None, rn_out=None,
                           slab=torch.zeros((2, P)), grad=torch.zeros(P),
                           params=torch.zeros(P), adam_m=torch.zeros(P), adam_v=torch.zeros(P),
                           target=torch.zeros(P), target_h=None, params_h=None, shared_work=None,
                           shared_paths={"adam_slabs": 0, "allreduce": 0},
                           _ops=SimpleNamespace(learn_shared_grad=lambda *a, **k: None,
                                                adam=lambda *a, **k: None))
    t0 = time.time()
    try:
        AG.BatchedDQN._learn_shared(fake, 1e-3, 0.1, 1e-3, 1e-7, False, None)
        q.put(("passed", time.time() - t0))
    except D.DistError as e:
        q.put((str(e), time.time() - t0))


def test_skipped_gradient_allreduce_fails_fast_naming_the_rank():
    """the C5 gradient all-reduce is bounded -- a peer that
    skips it makes the learn raise within the timeout instead of hanging."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_skipping_peer, args=(r, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    msg, dt = q.get(timeout=90)
    for p in ps:  # rank 1 is still asleep
        p.kill()
        p.join(timeout=30)
    assert msg.startswith("rank 0 of 2: all_reduce(SUM) of the shared-net gradient failed"), msg
    assert dt < 30, dt


class _FakeWork:
    def __init__(self, done_after):
        self.t = __import__("time").monotonic() + done_after

    def wait(self, timeout=None):
        return True

    def is_completed(self):
        return __import__("time").monotonic() >= self.t


def test_bounded_allreduce_lag_and_timeout(monkeypatch):
    """The RCCL branch of BoundedAllReduce without a device: the host blocks
    only once more than `lag` reductions are incomplete, and raises DistError
    (rank, call) once the oldest is older than the timeout."""
    from dmdqn_amd import dist as D
    works = []

    def fake_all_reduce(t, op=None, async_op=False):
        w = _FakeWork(done_after=works_delay[0])
        works.append(w)
        return w

    works_delay = [0.0]
    monkeypatch.setattr(D.dist, "is_initialized", lambda: True)
    monkeypatch.setattr(D.dist, "get_world_size", lambda: 2)
    monkeypatch.setattr(D.dist, "get_backend", lambda: "nccl")
    monkeypatch.setattr(D.dist, "all_reduce", fake_all_reduce)
    ar = D.BoundedAllReduce(lag=2, timeout_s=0.5)
    t = torch.zeros(3)
    for _ in range(5):  # complete at once: nothing stays pending
        ar(t)
    assert len(ar._pending) <= 1
    works_delay[0] = 3600.0  # never completes within the test
    ar(t)
    ar(t)
    import time
    t0 = time.monotonic()
    with pytest.raises(D.DistError, match="all_reduce\\(SUM\\) of the shared-net gradient failed"):
        ar(t)  # the third incomplete one: blocks on the oldest, then times out
    assert 0.3 < time.monotonic() - t0 < 5


def test_skipped_final_allreduce_raises_at_synchronize(monkeypatch):
    """the last `lag` reductions of a run are still pending when it
    ends.  Trainer.synchronize() / checkpoint.save() / bench's timed region
    drain them first (agent.drain_collectives), bounded: a final reduction a
    peer skipped raises DistError instead of hanging the device-wide sync."""
    from dmdqn_amd import dist as D
    from dmdqn_amd.agent import BatchedDQN
    monkeypatch.setattr(D.dist, "is_initialized", lambda: True)
    monkeypatch.setattr(D.dist, "get_world_size", lambda: 2)
    monkeypatch.setattr(D.dist, "get_backend", lambda: "nccl")
    monkeypatch.setattr(D.dist, "all_reduce",
                        lambda t, op=None, async_op=False: _FakeWork(done_after=3600.0))
    ag = BatchedDQN.__new__(BatchedDQN)  # only the collective state matters here
    ag._allreduce = D.BoundedAllReduce(lag=4, timeout_s=0.4)
    ag._allreduce(torch.zeros(3))  # the final reduction: its peer never joins
    assert len(ag._allreduce._pending) == 1  # within the lag: the host ran on
    import time
    t0 = time.monotonic()
    with pytest.raises(D.DistError, match="a peer rank stalled or skipped it"):
        ag.drain_collectives()
    assert time.monotonic() - t0 < 5
    ag2 = BatchedDQN.__new__(BatchedDQN)
    ag2.drain_collectives()  # no collectives: a no-op
