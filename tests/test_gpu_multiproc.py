"""Multi-process rehearsal of the C4 / C5 paths with the real kernels on ONE
GPU: two fresh processes (spawned, one rank each, both on cuda:0, gloo --
RCCL needs one device per rank) against a single process over the union of
their replicas ("averaged gradient equals the single-GPU gradient
over the union batch").

  C4  env-sharded independent DQN, no collectives: every rank's replicas,
      agents, replay indices and weights are bit-identical to the same global
      replicas of the single-process run.
  C5  shared-parameter DQN: per-rank gradient sums all-reduced over ranks;
      the shared weights after 8 learns equal the single-process run over the
      union of agents within 2e-6 (fp16 operands, f32 gradient sums whose
      order differs: per rank then across ranks)."""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

STEPS = 135  # 8 learns
E_RANK = 4


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(rank, ws, shared):
    from dmdqn_amd.agent import AgentConfig
    from dmdqn_amd.env import EnvConfig
    from dmdqn_amd.trainer import Trainer
    E = E_RANK if ws > 1 else E_RANK * 2
    cfg = AgentConfig(precision="fp16", seed=7, shared_params=shared, replay_buffer_size=500)
    tr = Trainer(EnvConfig(rows=2, cols=2, num_envs=E, seed=100, env_offset=rank * E), cfg)
    idx = []
    for _ in range(STEPS):
        tr.step()
        idx.append(tr.agent.idx.cpu().numpy().copy())
    torch.cuda.synchronize()
    return {"obs": tr.obs.cpu().numpy(), "params": tr.agent.params.cpu().numpy(),
            "target": tr.agent.target.cpu().numpy(), "loss": tr.agent.loss.cpu().numpy(),
            "idx": np.stack(idx[-3:]), "seeds": tr.env.seeds.copy()}


def _worker(rank, ws, port, shared, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(ws), LOCAL_RANK=str(rank))
    import torch.distributed as dist
    from dmdqn_amd import dist as D
    D.init(backend="gloo")
    torch.cuda.set_device(0)
    try:
        q.put((rank, _run(rank, ws, shared)))
    finally:
        dist.barrier()
        dist.destroy_process_group()


def _two_ranks(shared):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, shared, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(2))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def test_c4_env_shards_equal_single_process():
    res = _two_ranks(shared=False)
    one = _run(0, 1, False)
    A = 4
    for r in range(2):
        sl = slice(r * E_RANK, (r + 1) * E_RANK)
        asl = slice(r * E_RANK * A, (r + 1) * E_RANK * A)
        np.testing.assert_array_equal(res[r]["seeds"], one["seeds"][sl])
        np.testing.assert_array_equal(res[r]["obs"], one["obs"][sl])
        np.testing.assert_array_equal(res[r]["idx"], one["idx"][:, asl])
        np.testing.assert_array_equal(res[r]["params"], one["params"][asl])
        np.testing.assert_array_equal(res[r]["target"], one["target"][asl])
        np.testing.assert_array_equal(res[r]["loss"], one["loss"][asl])


def test_c5_shared_allreduce_equals_union_batch():
    res = _two_ranks(shared=True)
    one = _run(0, 1, True)
    A = 4
    # identical update on every rank
    np.testing.assert_array_equal(res[0]["params"], res[1]["params"])
    for r in range(2):
        sl = slice(r * E_RANK, (r + 1) * E_RANK)
        asl = slice(r * E_RANK * A, (r + 1) * E_RANK * A)
        np.testing.assert_array_equal(res[r]["obs"], one["obs"][sl])
        np.testing.assert_array_equal(res[r]["idx"], one["idx"][:, asl])
    d = np.abs(res[0]["params"] - one["params"]).max()
    print(f"C5 2-rank vs union: max |dw| {d:.3g}")
    np.testing.assert_allclose(res[0]["params"], one["params"], rtol=0, atol=2e-6)
