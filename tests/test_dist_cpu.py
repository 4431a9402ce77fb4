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
    D.allreduce_mean_(g)
    D.barrier()
    q.put((r, off, seeds.tolist(), m, g.tolist()))
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
    assert all(np.allclose(r[4], (1 + ws) / 2.0) for r in res)  # mean of 1..ws


def test_single_process_defaults():
    from dmdqn_amd import dist as D
    assert D.max_over_ranks(3.0) == 3.0
    t = torch.ones(3)
    assert torch.equal(D.allreduce_mean_(t), torch.ones(3))
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
                           _ops=SimpleNamespace(learn_shared_grad=learn_shared_grad, adam=adam))
    AG.BatchedDQN._learn_shared(fake, 1e-3, 0.1, 1e-3, 1e-7, True, None)
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
        assert seen["sync"] == 1
