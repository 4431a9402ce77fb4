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


def _run(rank, ws, shared, overlap="none"):
    from dmdqn_amd.agent import AgentConfig
    from dmdqn_amd.env import EnvConfig
    from dmdqn_amd.trainer import Trainer
    E = E_RANK if ws > 1 else E_RANK * 2
    cfg = AgentConfig(precision="fp16", seed=7, shared_params=shared, replay_buffer_size=500)
    tr = Trainer(EnvConfig(rows=2, cols=2, num_envs=E, seed=100, env_offset=rank * E), cfg,
                 overlap=overlap)
    idx = []
    for _ in range(STEPS):
        tr.step()
        idx.append(tr.agent.idx.cpu().numpy().copy())
    torch.cuda.synchronize()
    return {"obs": tr.obs.cpu().numpy(), "params": tr.agent.params.cpu().numpy(),
            "target": tr.agent.target.cpu().numpy(), "loss": tr.agent.loss.cpu().numpy(),
            "idx": np.stack(idx[-3:]), "seeds": tr.env.seeds.copy()}


def _worker(rank, ws, port, shared, q, overlap="none"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(ws), LOCAL_RANK=str(rank))
    import torch.distributed as dist
    from dmdqn_amd import dist as D
    D.init(backend="gloo")
    torch.cuda.set_device(0)
    try:
        q.put((rank, _run(rank, ws, shared, overlap)))
    finally:
        dist.barrier()
        dist.destroy_process_group()


def _two_ranks(shared, overlap="none"):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, shared, q, overlap)) for r in range(2)]
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


@pytest.mark.parametrize("shared,ranks,grid", [(False, 2, (2, 2, 64)), (True, 2, (8, 8, 64)),
                                               (False, 4, (2, 2, 64)), (False, 2, (4, 4, 320))])
def test_bench_multi_rank_launch(shared, ranks, grid):
    """The launch the driver's multi-GPU bench uses (torch.distributed.run,
    one rank per GPU, max-over-ranks timing), rehearsed with 2 and 4 ranks on
    this one GPU (DMDQN_DEVICE_OVERRIDE=0, gloo: RCCL needs a device per rank):
    rank 0 prints one JSON line with n_gpus = ranks, the whole-job value over
    every rank's replicas, "weak" scaling; the shared run goes through the C5
    gradient all-reduce every learn.  The schedules --overlap auto picks: the
    env step beside the learn (2x2), the draws beside the learn (8x8 shared),
    the env step beside the learn on an unmasked side stream (4x4 x 320:
    5,120 agents per rank, C4's per-GPU schedule)."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    R, C, E = grid
    args = ["--rows", str(R), "--cols", str(C)] + (["--shared"] if shared else [])
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node",
           str(ranks), "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(root, "bench.py"), "--gpus", str(ranks), "--envs", str(E), "--steps", "5",
           "--warmup", "2", "--prefill-steps", "130", "--no-cpu-baseline",
           "--dist-backend", "gloo"] + args
    env = dict(os.environ, DMDQN_DEVICE_OVERRIDE="0", MASTER_ADDR="127.0.0.1")
    r = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    out = json.loads(lines[0])
    A = R * C
    assert out["n_gpus"] == ranks and out["scaling"] == "weak"
    if R * C * E > 4096 and not shared:
        assert out["config"]["schedule"].startswith("the fused env step + replay draws of step t+1")
        assert "CUs" not in out["config"]["schedule"]
    assert out["config"]["global_envs"] == ranks * E
    assert out["steps"] == 5 and out["value"] > 0
    # value = agent-env steps of every rank / max-over-ranks wall time
    np.testing.assert_allclose(out["value"], 5 * ranks * E * A / (out["ms_per_step"] * 5 / 1e3),
                               rtol=2e-3)
    if shared:
        assert "all-reduce" in out["config"]["parallelism"]


def test_c5_allreduce_beside_next_step_bit_identical():
    """C5 with the "full" schedule at 2 ranks: the next step's act / sim /
    observe / sample run on the side stream while this step's shared learn,
    its gradient all-reduce and Adam run on the main stream -- the
    all-reduce overlaps the next step's env work.  Weights, losses, replay
    indices and observations are bit-identical to the sequential order."""
    seq = _two_ranks(shared=True)
    ovl = _two_ranks(shared=True, overlap="full")
    for r in range(2):
        for k in ("params", "target", "loss", "idx", "obs"):
            np.testing.assert_array_equal(ovl[r][k], seq[r][k], err_msg=f"rank {r} {k}")


_NCCL_ONE_RANK = r"""
import os, sys, json, torch
sys.path.insert(0, sys.argv[1])
import torch.distributed as dist
from dmdqn_amd import dist as D
from dmdqn_amd.agent import AgentConfig, BatchedDQN
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
D.init(backend="nccl", device=dev, timeout_s=60, force=True)
assert dist.get_backend() == "nccl" and dist.get_world_size() == 1
D.barrier(30)
m = D.max_over_ranks(1.25, device=dev, timeout_s=30)
ag = BatchedDQN(2, 4, AgentConfig(precision="fp16", shared_params=True, replay_buffer_size=200))
g = torch.Generator(device="cuda").manual_seed(0)
for t in range(130):
    s = torch.randint(-1, 24, (2, 4, 89), device=dev, generator=g).float()
    a = torch.randint(0, 4, (2, 4), device=dev, generator=g, dtype=torch.int32)
    r = -torch.rand((2, 4), device=dev, generator=g, dtype=torch.float64) * 100
    ag.remember(s, a, r, s, False)
ag.learn()
g0 = ag.grad.clone()
dist.all_reduce(ag.grad, op=dist.ReduceOp.SUM)  # RCCL, one rank: the identity
torch.cuda.synchronize()
print(json.dumps({"max": m, "same": bool(torch.equal(g0, ag.grad)),
                  "finite": bool(torch.isfinite(g0).all())}))
dist.destroy_process_group()
"""


def test_rccl_one_rank_group_on_this_gpu():
    """The nccl (= RCCL) branch of dmdqn_amd.dist on the real device: a
    one-rank process group with device_id and timeouts, the timed barrier,
    the max-over-ranks all-reduce and an all-reduce of a C5 gradient on the
    learn's buffer (the identity for one rank).  The driver's multi-GPU run
    takes this code path first; a failure here names the call."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0",
               WORLD_SIZE="1", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, "-c", _NCCL_ONE_RANK, root], cwd=root, env=env,
                       capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert out == {"max": 1.25, "same": True, "finite": True}


# ------------------------------------------------- the C5 bench schedule at 2 ranks
C5_E_RANK = 16      # 8x8 x 16 envs per rank: 1,024 agents
C5_STEPS = 420      # replay 300: the rings wrap at step 300
C5_CAP = 300
C5_STATS_EVERY = 7
C5_EARLY_LEARNS = 8  # the union comparison's point (as test_c5_shared_allreduce_equals_union_batch)


def _digest(h, t):
    h.update(t.contiguous().view(torch.uint8).cpu().numpy().tobytes())


def _run_c5_schedule(rank, ws, overlap):
    """One rank of C5 under `overlap` ("learn" = what bench.auto_schedule picks
    for the shared net), on bench.make_streams' dedicated learn stream.  Small
    state comes back whole, large state (observations every step, rings,
    random streams) as sha1 digests."""
    import hashlib

    import bench
    from dmdqn_amd.agent import AgentConfig
    from dmdqn_amd.env import EnvConfig
    from dmdqn_amd.trainer import Trainer
    E = C5_E_RANK if ws > 1 else 2 * C5_E_RANK  # one process: the union of 2 ranks
    dev = torch.device("cuda", 0)
    work, side = bench.make_streams(dev, None)
    cfg = AgentConfig(precision="fp16", seed=2, shared_params=True, replay_buffer_size=C5_CAP)
    out = {}
    with torch.cuda.stream(work):
        tr = Trainer(EnvConfig(rows=8, cols=8, num_envs=E, seed=2, env_offset=rank * E), cfg,
                     device=dev, overlap=overlap, side_stream=side)
        losses, stats, h_obs = [], [], hashlib.sha1()
        for t in range(C5_STEPS):
            st = tr.step(collect_stats=t % C5_STATS_EVERY == 0)
            assert st.loss_launched == (t + 1 >= 128)
            if tr.last_loss is not None:
                losses.append(tr.last_loss.cpu().numpy().copy())
                if len(losses) == 1:  # the first learn's reduced gradient (same weights everywhere)
                    out["grad1"] = tr.agent.grad.cpu().numpy().copy()
                if t % C5_STATS_EVERY == 0:
                    stats.append(tr.agent.qstats.cpu().numpy().copy())
                if len(losses) == C5_EARLY_LEARNS:
                    out["params_early"] = tr.agent.params.cpu().numpy().copy()
            _digest(h_obs, tr.obs)
        tr.synchronize()  # drains the bounded all-reduces first
        ag = tr.agent
        assert ag.ring.start != 0 and len(ag.ring) == C5_CAP
        out.update(losses=np.stack(losses), stats=np.stack(stats), obs_sha1=h_obs.hexdigest(),
                   paths=dict(ag.shared_paths), sampler_lds=tr._sampler_lds,
                   **{k: getattr(ag, k).cpu().numpy().copy()
                      for k in ("params", "target", "adam_m", "adam_v")},
                   target_h=ag.target_h.float().cpu().numpy())
        for k in ("np_state", "py_state"):
            h = hashlib.sha1()
            _digest(h, getattr(ag, k))
            out[k + "_sha1"] = h.hexdigest()
        for k in ("s", "n", "a", "r", "d"):
            h = hashlib.sha1()
            _digest(h, getattr(ag.ring, k))
            out["ring_" + k + "_sha1"] = h.hexdigest()
    return out


def _c5_worker(rank, ws, port, q, overlap):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(ws), LOCAL_RANK=str(rank))
    import torch.distributed as dist
    from dmdqn_amd import dist as D
    D.init(backend="gloo", timeout_s=120)
    torch.cuda.set_device(0)
    try:
        q.put((rank, _run_c5_schedule(rank, ws, overlap)))
    finally:
        dist.barrier()
        dist.destroy_process_group()


def _c5_two_ranks(overlap):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_c5_worker, args=(r, 2, port, q, overlap)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=400) for _ in range(2))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def test_c5_bench_schedule_two_ranks_bit_identical_to_one_stream():
    """the schedule bench.py --overlap auto picks for C5
    ("learn": the next step's replay draws on a side stream beside the learn,
    the sampler's LDS cut to what the S' pass leaves of a CU) at 2 ranks, where
    the shared learn is k_shared_next + k_shared_grad -> k_reduce_slabs ->
    all-reduce over ranks -> k_adam(1/world) instead of one rank's fused
    k_reduce_adam.  8x8 x 16 envs per rank, replay 300 (wrapped at step 300),
    420 steps, Q statistics every 7th step: per rank, losses, Q statistics,
    observations, the network, Adam slots, the f16 target shadow, random
    streams and rings are bit-identical to the same 2 ranks on one stream
    (overlap "none"), and the network is identical on both ranks.
    Against one process over the union of the replicas ("averaged
    gradient equals the single-GPU gradient over the union batch"): the first
    learn's gradient (same weights on both sides) -- the all-reduced sum over
    2 ranks, halved by Adam's gscale -- equals the union's within 1e-5 of its
    largest element (f32 sums in another order: per rank, then across ranks).
    The weights after 8 learns agree within 2e-6 except where Adam's
    normalisation m / (sqrt(v) + eps) turns an order-of-summation difference
    in a near-zero gradient into a visible step: there the bound is Adam's own
    step size, lr per learn (measured: 7 of 28,548 weights, 1.9e-5)."""
    import bench
    sched, cus, side_learn = bench.auto_schedule(8, 8, C5_E_RANK, True, False, False, None)
    assert (sched, cus, side_learn) == ("learn", None, 0)
    got = _c5_two_ranks(sched)
    ref = _c5_two_ranks("none")
    n_learn = C5_STEPS - 127
    for r in range(2):
        assert got[r]["paths"] == {"adam_slabs": 0, "allreduce": n_learn}, got[r]["paths"]
        assert ref[r]["paths"] == {"adam_slabs": 0, "allreduce": n_learn}, ref[r]["paths"]
        assert got[r]["sampler_lds"] > 0 and ref[r]["sampler_lds"] == 0
        assert got[r].keys() == ref[r].keys()
        for k in ref[r]:
            if k in ("paths", "sampler_lds"):
                continue
            a, b = ref[r][k], got[r][k]
            if isinstance(a, np.ndarray):
                np.testing.assert_array_equal(b, a, err_msg=f"rank {r} {k}")
            else:
                assert a == b, f"rank {r} {k}"
    for k in ("params", "target", "adam_m", "adam_v", "target_h", "params_early"):
        np.testing.assert_array_equal(got[0][k], got[1][k], err_msg=k)
    one = _run_c5_schedule(0, 1, "none")
    assert one["paths"] == {"adam_slabs": n_learn, "allreduce": 0}
    g2, g1 = got[0]["grad1"] * 0.5, one["grad1"]  # the 2-rank sum x Adam's gscale 1/world
    gmax = float(np.abs(g1).max())
    dg = float(np.abs(g2 - g1).max())
    d = np.abs(got[0]["params_early"] - one["params_early"])
    d_end = np.abs(got[0]["params"] - one["params"]).max()
    print(f"C5 2-rank 'learn' vs union: first gradient max |dg| {dg:.3g} (max |g| {gmax:.3g}); "
          f"max |dw| {d.max():.3g} after {C5_EARLY_LEARNS} learns ({int((d > 2e-6).sum())} "
          f"above 2e-6), {d_end:.3g} after {n_learn}")
    assert dg <= 1e-5 * gmax
    lr = 1e-3  # AgentConfig.learning_rate: Adam moves a weight at most ~lr per learn
    assert (d > 2e-6).sum() <= 1e-3 * d.size and d.max() <= C5_EARLY_LEARNS * lr
