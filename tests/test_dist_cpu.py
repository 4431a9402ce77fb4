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
