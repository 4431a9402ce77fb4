"""BASELINE configurations at their real size on one GPU, checked against the
oracle on sampled replicas and agents (BASELINE.json configs).

  C1  1x1 grid, 1 agent, the drop-in src/scripts/train.py loop (one episode)
  C2  2x2 grid x 256 replicas, bf16, replay 10000
  C3  4x4 grid x 1024 replicas, fp16 (mixed_float16), replay 10000: 16,384
      learn workgroups, 21 GB per ring array (byte offsets past 2^31), 1100
      steps so the sampler runs CPython's set branch (n > 1045)
  C3' the same past 10,000 steps: wrapped rings, the steady state bench.py
      times
  C5  8x8 grid x 256 replicas, one shared network (the 8x8 sim takes the
      register path), replay 10000

Per step, for sampled replicas (first, middle, last): actions, rewards and
observations bit-exact vs oracle.OracleLoop (same seeds); once the replay is
active, every sampled agent's 128 replay indices bit-exact vs CPython's
random.sample.  At the checked learns, for 8 agents across those replicas: the
device z-scored rewards bit-exact, the loss vs oracle.learn_mixed (Keras 3's
mixed-precision learn, pinned to the reference's own DQNAgent in
tests/test_learn_mixed_golden_cpu.py; test_gpu_learn TOL16) and vs the fp32
oracle (rtol 2e-2), and the gradient >= 99 % within the checker's
tolerance; every agent's loss finite.
C4 (8 GPUs, env-sharded) is the C3 shard per GPU (tests/test_gpu_multiproc.py
covers the sharding with real kernels)."""
import json
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import oracle as O  # noqa: E402
from dmdqn_amd.agent import AgentConfig, initial_weights, kernel_to_keras  # noqa: E402
from dmdqn_amd.env import EnvConfig  # noqa: E402
from dmdqn_amd.trainer import Trainer  # noqa: E402

from test_gpu_learn import ROUND, TOL16, _host_batch, _mixed_emulation  # noqa: E402

DEV = "cuda"


def _rows(t, idx):
    return t[torch.as_tensor(idx, device=t.device)].cpu().numpy()


def _check_shared_grad(tr, raw, pre, agents0, n_sub=64):
    """The C5 learn just run, from the pre-learn state raw = (params, target,
    adam_m, adam_v) in the device layout (pre: the same in Keras order):
      * Adam exact: params / m / v = the Keras-3 update (k_adam, f32, no fma)
        of the pre-learn state with the all-agent gradient ag.grad;
      * the gradient: the shared passes re-run through the C ABI on the n_sub
        agents from agents0 (their rings, indices and loss rows; pointers offset
        into the full arrays, start != 0 on a wrapped ring) from the pre-learn
        weights -- >= 99 % of entries within 2e-3 max|g| + 1e-2 |g| of the mean
        of those agents' oracle.learn_mixed gradients (the tolerance of
        test_gpu_shared.py) and the per-agent losses the full launch wrote."""
    import ctypes as C
    from dmdqn_amd._lib import call, ptr, stream_of
    ag, ring = tr.agent, tr.agent.ring
    p0, t0, m0, v0 = (x.cpu().numpy()[0] for x in raw)
    g = ag.grad.cpu().numpy()
    assert np.isfinite(g).all()
    alpha, c1, c2, eps = O.keras_adam_consts(ag.learn_step_counter, ag.cfg.learning_rate)
    m1 = m0 + (g - m0) * c1
    v1 = v0 + (g * g - v0) * c2
    p1 = p0 - (m1 * alpha) / (np.sqrt(v1) + eps)
    np.testing.assert_array_equal(ag.adam_m.cpu().numpy()[0], m1)
    np.testing.assert_array_equal(ag.adam_v.cpu().numpy()[0], v1)
    np.testing.assert_array_equal(ag.params.cpu().numpy()[0], p1)
    # the gradient of n_sub agents, from the pre-learn weights
    params = raw[0].clone()
    target = raw[1].clone()
    ph = torch.zeros_like(ag.params_h)
    ph[:, :ag.P].copy_(params.to(ph.dtype))
    th = torch.zeros_like(ag.target_h)
    th[:, :ag.P].copy_(target.to(th.dtype))
    loss = torch.zeros(n_sub, dtype=torch.float32, device=DEV)
    slab = torch.empty((ag.n_slabs, ag.P), dtype=torch.float32, device=DEV)
    g_sub = torch.empty(ag.P, dtype=torch.float32, device=DEV)
    work = torch.empty(n_sub * 128 * 5, dtype=torch.uint8, device=DEV)
    a = ag.c_learn_args()
    j0, cap = agents0, ring.slots  # the physical row stride
    a.NA = n_sub
    for f, t, per in (("ring_s", ring.s, cap * 128), ("ring_n", ring.n, cap * 128),
                      ("ring_a", ring.a, cap), ("ring_d", ring.d, cap), ("ring_r", ring.r, cap * 8),
                      ("idx", ag.idx, 128 * 4)):
        setattr(a, f, t.data_ptr() + j0 * per)
    a.params, a.target, a.params_h, a.target_h = (t.data_ptr() for t in (params, target, ph, th))
    a.loss = loss.data_ptr()
    a.rn_out = a.qstats = a.stamps = None
    call("dmdqn_learn_shared_grad", C.byref(a), ptr(slab), ag.n_slabs, ptr(g_sub),
         C.c_float(1.0 / n_sub), ptr(work), stream_of())
    torch.cuda.synchronize()
    np.testing.assert_array_equal(loss.cpu().numpy(), ag.loss[j0:j0 + n_sub].cpu().numpy())
    g_g = kernel_to_keras(g_sub.cpu().numpy()[None], 128)[0]
    zero = np.zeros_like(pre[0][0])
    idx = ag.idx.cpu().numpy()
    ges = []
    for j in range(j0, j0 + n_sub):
        S, Aa, Rn, S2, D = _host_batch(ag, j, idx[j])
        l_e, g_e, _, _, _ = _mixed_emulation(pre[0][0], pre[1][0], zero, zero.copy(), S, Aa, Rn,
                                             S2, D, 1, round_grad=False)
        np.testing.assert_allclose(loss[j - j0].item(), l_e, rtol=2e-3, err_msg=f"agent {j}")
        ges.append(g_e)
    g_e = np.mean(np.stack(ges), axis=0)
    close = np.abs(g_g - g_e) <= 2e-3 * np.abs(g_e).max() + 1e-2 * np.abs(g_e)
    assert close.mean() > 0.99, f"{np.sum(~close)} shared-gradient entries off"


def _check_learn(tr, agents, pre, precision, shared, t32=None, stats=False):
    """One learn of tr's last step for `agents`, from the pre-step state `pre`.
    t32: the loss tolerance vs the fp32 oracle: an rtol, or "q-scaled"
    (default): TOL16's rtol or, where larger, the change in the mean squared
    TD error that an error of delta = 4 16-bit ulps of max|Q| in q - y can
    make, 2 sqrt(L) delta + delta^2 -- Keras's mixed learn rounds Q and y to
    f16 / bf16 (the device matches that learn to TOL16 above), so once |Q| is
    a few times |q - y| a fixed rtol on L measures the 16-bit format, not the
    kernel (round 3: C2 bf16 5.2 % in its first 13 learns, C3 fp16 5.8 % after
    10,000 steps)."""
    ag = tr.agent
    rnd = ROUND[precision]
    tl, ta, tr_, _, t32_ = TOL16[precision]
    t32 = "q-scaled" if t32 is None else t32
    q_scaled = t32 == "q-scaled"
    ulp = 2.0 ** -11 if precision == "fp16" else 2.0 ** -8
    loss = ag.loss.cpu().numpy()
    assert np.isfinite(loss).all(), "every agent's loss is finite"
    idx = ag.idx.cpu().numpy()
    qs = ag.qstats.cpu().numpy() if stats else None
    rn = ag.rn_out.cpu().numpy()
    t = ag.learn_step_counter
    p_now = kernel_to_keras(ag.params[0:1].cpu().numpy(), 128)[0] if shared else None
    for k, j in enumerate(agents):
        S, Aa, Rn, S2, D = _host_batch(ag, j, idx[j])
        np.testing.assert_array_equal(rn[j], Rn)  # device z-score == numpy's
        p0, t0, m0, v0 = (x[0 if shared else k] for x in pre)
        l_e, g_e, _, _, _ = _mixed_emulation(p0, t0, m0, v0, S, Aa, Rn, S2, D, t, rnd=rnd)
        np.testing.assert_allclose(loss[j], l_e, rtol=tl, err_msg=f"agent {j} vs emulation")
        if stats:
            # dqn_agent.py:361-363: sum Q, sum Q^2 and the action counts of
            # the batch's online Q(S) -- the 16-bit forward of the pre-learn net
            q = O.qnet_forward_mixed(p0, S, precision).astype(np.float64)
            np.testing.assert_allclose(qs[j, 0], q.sum(), rtol=1e-3, atol=1e-3 * np.abs(q).sum(),
                                       err_msg=f"agent {j}: sum Q")
            np.testing.assert_allclose(qs[j, 1], (q * q).sum(), rtol=2e-3,
                                       err_msg=f"agent {j}: sum Q^2")
            np.testing.assert_array_equal(qs[j, 2:6], np.bincount(Aa, minlength=4),
                                          err_msg=f"agent {j}: action counts")
        p1, m1, v1 = p0.copy(), m0.copy(), v0.copy()
        l32 = O.learn(p1, t0, m1, v1, S, Aa, Rn, S2, D, t)
        if q_scaled:
            qmax = float(np.abs(O.qnet_forward(p0, S)).max())
            delta = 4 * ulp * qmax
            bound = max(t32_ * l32, 2 * np.sqrt(l32) * delta + delta * delta)
            assert abs(loss[j] - l32) <= bound, (
                f"agent {j}: loss {loss[j]} vs fp32 {l32}, max|Q| {qmax}, bound {bound}")
        else:
            np.testing.assert_allclose(loss[j], l32, rtol=t32, err_msg=f"agent {j} vs fp32 oracle")
        if not shared:
            m_g = kernel_to_keras(ag.adam_m[j:j + 1].cpu().numpy(), 128)[0]
            g_g = m0 + (m_g - m0) / np.float32(0.1)  # m1 = m0 + (g - m0) c1
            gs = np.abs(g_e).max()
            close = np.abs(g_g - g_e) <= 2 * ta * gs + tr_ * np.abs(g_e)
            assert close.mean() > 0.99, f"agent {j}: {np.sum(~close)} gradient entries off"
    if shared:
        assert np.isfinite(p_now).all() and not np.array_equal(p_now, pre[0][0])


# steps past the deque's maxlen in the steady-state tests: beyond the ring's
# spare slots (kernels.ReplayRing.SPARE, 16), so the PHYSICAL ring wraps too
# (the learns' slot arithmetic takes its wrap branch) -- as in bench.py's timed
# region (10,000 prefill + 210 steps)
PAST = 70


def _run_config(rows, cols, envs, precision, steps, learn_checks, shared=False, sparse_until=0,
                t32=None, shared_grad_checks=(), trainer_kw=None, stats_checks=()):
    """sparse_until: before this step, compare with the oracle only every 97th
    step (the oracle loops still run every step).  t32: _check_learn's.
    shared_grad_checks: learns (as in learn_checks) at which _check_shared_grad
    also runs, on the agents of the middle replica.  trainer_kw: extra Trainer
    arguments (a schedule, its streams).  stats_checks: steps whose learn runs
    with collect_stats, its per-agent Q statistics checked against the oracle
    forward of the pre-learn weights for the picked agents."""
    cfg = AgentConfig(precision=precision, seed=0, shared_params=shared)
    tr = Trainer(EnvConfig(rows=rows, cols=cols, num_envs=envs, seed=0), cfg, **(trainer_kw or {}))
    A, ag = tr.env.A, tr.agent
    sampled = [0, envs // 2, envs - 1]
    loops = [O.OracleLoop(rows, cols, int(tr.env.seeds[e]), learn=False) for e in sampled]
    arows = [e * A + j for e in sampled for j in range(A)]
    pick = [sampled[0] * A, sampled[0] * A + A - 1, sampled[1] * A + A // 3,
            sampled[1] * A + A - 1, sampled[2] * A, sampled[2] * A + A // 2,
            sampled[2] * A + A - 2, sampled[2] * A + A - 1]
    ag.rn_out = torch.zeros((ag.NA, 128), dtype=torch.float32, device=DEV)
    checked = 0
    for step in range(steps):
        pre = raw = None
        if step + 1 in learn_checks:
            src = [0] if shared else pick
            pre = [kernel_to_keras(_rows(getattr(ag, k), src), 128)
                   for k in ["params", "target", "adam_m", "adam_v"]]
            if step + 1 in shared_grad_checks:
                raw = [getattr(ag, k).clone() for k in ["params", "target", "adam_m", "adam_v"]]
        tr.step(collect_stats=step + 1 in stats_checks)
        outs = [lp.step() for lp in loops]
        if step < sparse_until and step % 97 and pre is None:
            continue
        acts, obs, rew = (_rows(x, sampled) for x in (ag.actions, tr.obs, tr.last_reward))
        for i, out in enumerate(outs):
            np.testing.assert_array_equal(acts[i], out["actions"], err_msg=f"step {step} env {i}")
            np.testing.assert_array_equal(rew[i], out["reward"], err_msg=f"step {step} env {i}")
            np.testing.assert_array_equal(obs[i], loops[i].obs, err_msg=f"step {step} env {i}")
        if outs[0]["idx"] is not None:
            idx = _rows(ag.idx, arows).reshape(len(sampled), A, 128)
            for i, out in enumerate(outs):
                np.testing.assert_array_equal(idx[i], out["idx"], err_msg=f"step {step} env {i}")
        if pre is not None:
            _check_learn(tr, pick, pre, precision, shared, t32,
                         stats=step + 1 in stats_checks)
            if raw is not None:
                _check_shared_grad(tr, raw, pre, sampled[1] * A)
            checked += 1
    assert checked == len(learn_checks)
    return tr


def test_c3_4x4x1024_fp16_full_size():
    tr = _run_config(4, 4, 1024, "fp16", 1100, {128, 1100})
    assert len(tr.agent.ring) == 1100 and tr.agent.ring.s.numel() > 2 ** 31
    assert tr.episode == 4  # episode boundaries at 240, 480, 720, 960
    del tr
    torch.cuda.empty_cache()


def test_c3_steady_state_wrapped_rings():
    """The regime bench.py times: C3 (4x4 x 1024, fp16, replay
    10,000) driven past 10,000 steps, so every ring is full and wrapped (deque
    position 0 = the oldest transition at ring slot start != 0,
    dqn_agent.py:29, 59-85) and the sampler runs CPython's set branch at
    n = 10,000.  Sampled replicas {0, 511, 1023} vs OracleLoop every 97th step
    and at every step after the wrap: actions, rewards, observations and replay
    indices bit-exact; at the learns of steps PAST - 3 and PAST - 1 after the wrap, for 8 agents,
    the device z-score bit-exact and the loss vs the Keras mixed-precision
    checker (pinned to the reference's own learn; rtol 2e-3, as at step 128)
    and, as a sanity bound, the fp32 oracle "q-scaled" (_check_learn).  Under
    the schedule bench.py times at C3 (bench.auto_schedule: the replay draws on
    a side stream beside the env step, trainer "sample")."""
    cap = 10000
    work, kw = _bench_c3_schedule()
    try:
        with torch.cuda.stream(work):
            tr = _run_config(4, 4, 1024, "fp16", cap + PAST, {cap + PAST - 3, cap + PAST - 1},
                             sparse_until=cap,
                             trainer_kw=kw)
            assert tr.overlap == "env" and tr.side_learn == 0
            ring = tr.agent.ring
            assert len(ring) == cap and ring.total == cap + PAST and ring.start == PAST
            del tr
    finally:
        torch.cuda.synchronize()
    torch.cuda.empty_cache()


def _bench_c3_schedule():
    """The schedule bench.py --overlap auto times at C3 (round 6): the fused
    env step of t+1 and its draws on an unmasked side stream beside learn t."""
    import bench
    sched, cus, side_learn = bench.auto_schedule(4, 4, 1024, False, False, False, None)
    assert (sched, cus, side_learn) == ("env", None, 0)
    work, side = bench.make_streams(torch.device(DEV), cus)
    assert side is None  # the Trainer makes its side stream
    return work, dict(overlap=sched)


def test_c2_steady_state_wrapped_rings():
    """C2 (2x2 x 256, bf16 = Keras' mixed_bfloat16, replay 10,000) in the
    regime bench.py times: driven past 10,000 steps, every ring full and
    wrapped (start != 0) on int8 rows, the sampler in CPython's set branch at
    n = 10,000.  Sampled replicas {0, 128, 255} vs OracleLoop every 97th step
    and at every step after the wrap (actions, rewards, observations, replay
    indices bit-exact); at the learns of steps PAST - 3 and PAST - 1 after the wrap the device
    z-score bit-exact and the loss vs oracle.learn_mixed (bf16, TOL16) for 8
    agents (dqn_agent.py:29, 59-85)."""
    cap = 10000
    tr = _run_config(2, 2, 256, "bf16", cap + PAST, {cap + PAST - 3, cap + PAST - 1},
                     sparse_until=cap)
    ring = tr.agent.ring
    assert len(ring) == cap and ring.total == cap + PAST and ring.start == PAST
    del tr
    torch.cuda.empty_cache()


def test_c5_steady_state_wrapped_rings():
    """C5 (8x8 x 256, ONE shared fp16 network, replay 10,000), the regime
    bench.py's C5 line times: past 10,000 steps, wrapped rings (start != 0,
    the wrap arithmetic of k_shared_next / k_shared_grad4) and the set-branch
    sampler.  Sampled replicas vs OracleLoop as C2 / C3; at the learns of
    steps PAST - 3 and PAST - 1 after the wrap the device z-score bit-exact and 8 agents' losses vs
    oracle.learn_mixed; at both, Adam exact on the all-agent gradient and the
    gradient of the middle replica's 64 agents vs the mean of their
    oracle.learn_mixed gradients (_check_shared_grad)."""
    cap = 10000
    checks = {cap + PAST - 3, cap + PAST - 1}
    tr = _run_config(8, 8, 256, "fp16", cap + PAST, checks, shared=True, sparse_until=cap,
                     shared_grad_checks=checks)
    ring = tr.agent.ring
    assert len(ring) == cap and ring.total == cap + PAST and ring.start == PAST
    del tr
    torch.cuda.empty_cache()


def test_c2_2x2x256_bf16_full_size():
    tr = _run_config(2, 2, 256, "bf16", 140, {128, 140})
    del tr
    torch.cuda.empty_cache()


def test_c5_8x8x256_shared_full_size():
    tr = _run_config(8, 8, 256, "fp16", 130, {128, 130}, shared=True)
    del tr
    torch.cuda.empty_cache()


def test_c1_train_py_1x1_episode(tmp_path):
    """The drop-in src/scripts/train.py loop (DQNAgent per junction, process-
    global streams) for one 240-step episode on a 1x1 grid vs OracleLoop with
    learning on: per-step rewards exact, per-step loss rtol 1e-4 (fp32)."""
    from src.agents import dqn_agent as DA
    from src.scripts import train as T
    seed = 3
    mpath = os.path.join(str(tmp_path), "m.jsonl")
    agents = T.train_agents(episodes=1, rows=1, cols=1, seed=seed, metrics=mpath)
    recs = [json.loads(x) for x in open(mpath)]
    assert len(recs) == 240
    s0 = DA.init_seed(0, "J_0_0")
    w0 = initial_weights(s0, [s0], 1, 128)  # BatchedDQN(1, 1) inside DQNAgent: env seed = seed
    ol = O.OracleLoop(1, 1, seed, cap=10000, tuf=500, weights=w0)
    for rec in recs:
        out = ol.step()
        assert rec["total_reward"] == float(out["reward"].sum())
        if out["loss"] is None:
            assert rec["total_loss"] == 0
        else:
            np.testing.assert_allclose(rec["total_loss"], float(out["loss"].sum()), rtol=1e-4)
    assert ol.learn_steps == 240 - 127
    got = np.concatenate([w.reshape(-1) for w in agents["J_0_0"]._core.get_weights(0)])
    np.testing.assert_allclose(got, ol.params[0], atol=5e-5)


def test_c3_overlap_schedules_bit_identical_at_size():
    """The optional stream schedules (trainer.py: "sample", "full") at C3 size
    (4x4 x 1024, fp16; replay 500 to bound memory): 140 steps, losses and
    every agent's weights bit-identical to the one-stream order."""
    res = {}
    for sched in ("none", "full", "sample"):
        tr = Trainer(EnvConfig(rows=4, cols=4, num_envs=1024, seed=2),
                     AgentConfig(precision="fp16", replay_buffer_size=500, seed=2),
                     overlap=sched)
        losses = []
        for _ in range(140):
            tr.step()
            if tr.last_loss is not None:
                losses.append(tr.last_loss.clone())
        torch.cuda.synchronize()
        res[sched] = (torch.stack(losses).cpu(), tr.agent.params.cpu(), tr.obs.cpu())
        del tr
        torch.cuda.empty_cache()
    for sched in ("full", "sample"):
        for a, b in zip(res["none"], res[sched]):
            assert torch.equal(a, b), sched


def test_c2_env_beside_learn_bit_identical_at_size():
    """overlap "env" (the fused env step of t+1 beside learn t; the store in
    the ring's spare slot) at C2 size (2x2 x 256, bf16), the ring wrapped
    (replay 300, 420 steps): losses, weights, rings and observations
    bit-identical to the one-stream order (train.py:207-292's order)."""
    res = {}
    for sched in ("none", "env"):
        tr = Trainer(EnvConfig(rows=2, cols=2, num_envs=256, seed=2),
                     AgentConfig(precision="bf16", replay_buffer_size=300, seed=2),
                     overlap=sched)
        losses = []
        for _ in range(420):
            tr.step()
            if tr.last_loss is not None:
                losses.append(tr.last_loss.clone())
        torch.cuda.synchronize()
        assert tr.agent.ring.start != 0
        res[sched] = (torch.stack(losses).cpu(), tr.agent.params.cpu(), tr.obs.cpu(),
                      tr.agent.ring.s.cpu(), tr.agent.ring.n.cpu())
        del tr
        torch.cuda.empty_cache()
    for a, b in zip(res["none"], res["env"]):
        assert torch.equal(a, b)


def _bench_c2_schedule():
    """The schedule bench.py --overlap auto times at C2 (bench.auto_schedule,
    bench.make_streams): the fused env step of t+1 and the draws beside learn
    t on a 64-CU masked side stream, the last 64 agents learned on it."""
    import bench
    sched, cus, side_learn = bench.auto_schedule(2, 2, 256, False, False, False, None)
    assert (sched, cus, side_learn) == ("env", 64, 64)
    work, side = bench.make_streams(torch.device(DEV), cus)
    return work, dict(overlap=sched, side_stream=side, side_learn=side_learn)


def test_c2_bench_schedule_steady_state_wrapped_rings():
    """C2 (2x2 x 256, bf16, replay 10,000) under the
    exact schedule bench.py times -- env step beside the learn on 64 masked
    CUs, agents 960..1023 learned on the side stream -- driven past 10,000
    steps (wrapped rings, the store in the spare slot, the set-branch
    sampler).  Sampled replicas {0, 128, 255} vs OracleLoop every 97th step
    and at every step after the wrap: actions, observations, rewards, replay
    indices bit-exact.  At the learns of steps PAST - 3 and PAST - 1 after the wrap, agents of both
    launches (0, 3, 513, 515 on the learn stream; 1020..1023 on the side
    stream) are checked: device z-score bit-exact, loss vs
    oracle.learn_mixed (bf16, TOL16), gradient, and (learn 5) the Q
    statistics of collect_stats (train.py:274-292, dqn_agent.py:29, 59-85)."""
    cap = 10000
    work, kw = _bench_c2_schedule()
    try:
        with torch.cuda.stream(work):
            tr = _run_config(2, 2, 256, "bf16", cap + PAST, {cap + PAST - 3, cap + PAST - 1},
                             sparse_until=cap,
                             trainer_kw=kw, stats_checks={cap + PAST - 1})
            assert tr.side_learn == 64 and tr.overlap == "env"
            ring = tr.agent.ring
            assert len(ring) == cap and ring.total == cap + PAST and ring.start == PAST
            del tr
    finally:
        torch.cuda.synchronize()
    torch.cuda.empty_cache()


def _run_schedule(kw, steps=420, cap=300, stats_every=7, grid=(2, 2, 256), precision="bf16",
                  shared=False, marks=None, spare=16):
    R, C, E = grid
    tr = Trainer(EnvConfig(rows=R, cols=C, num_envs=E, seed=2),
                 AgentConfig(precision=precision, replay_buffer_size=cap, seed=2,
                             shared_params=shared, ring_spare=spare), **kw)
    losses, stats, obs = [], [], []
    for t in range(steps):
        st = tr.step(collect_stats=t % stats_every == 0)
        if tr.last_loss is not None:
            losses.append(tr.last_loss.clone())
            if t % stats_every == 0:
                stats.append(tr.agent.qstats.clone())
        obs.append(tr.obs.clone())
        assert st.loss_launched == (t + 1 >= 128)
    torch.cuda.synchronize()
    assert tr.agent.ring.start != 0
    if marks is not None:
        marks.append((tr.n_marks, tr.agent.learn_launches))
    ag = tr.agent
    out = dict(losses=torch.stack(losses).cpu(), stats=torch.stack(stats).cpu(),
               obs=torch.stack(obs).cpu(),
               **{k: getattr(ag, k).cpu() for k in ("params", "target", "adam_m", "adam_v",
                                                    "target_h", "np_state", "py_state")},
               **{"ring_" + k: getattr(ag.ring, k).cpu() for k in ("s", "n", "a", "r", "d")})
    del tr
    torch.cuda.empty_cache()
    return out


@pytest.mark.parametrize("fenced,spare", [(False, 16), (True, 16), (False, 64), (False, 2),
                                          (False, 1)])
def test_c2_bench_schedule_bit_identical_to_one_stream(fenced, spare):
    """C2 size, replay 300 (wrapped by step 300), 420
    steps: the bench's C2 schedule (masked streams, side learn of 64 agents,
    ordering-only learn events; fenced=True: default events, bench
    --fenced-events) gives losses, Q statistics (collect_stats every 7th
    step), observations, weights, Adam slots, target shadows,
    random streams and rings bit-identical to the one-stream order -- with
    the ring's default 16 spare slots (the side stream up to 16 env steps
    ahead, every 16th learn marked), with 64 and two, and with one (round
    5's ring, every learn marked)."""
    ref = _run_schedule({}, spare=spare)
    work, kw = _bench_c2_schedule()
    kw["war_events"] = not fenced
    marks = []
    try:
        with torch.cuda.stream(work):
            got = _run_schedule(kw, marks=marks, spare=spare)
    finally:
        torch.cuda.synchronize()
    # s spare ring slots: ordering-only events mark every s-th learn for the
    # side stream (the first learn always); default events mark every one
    n_marks, n_learns = marks[0]
    if fenced or spare == 1:
        assert n_marks == n_learns, (n_marks, n_learns)
    else:
        assert abs(n_marks - n_learns / spare) <= 1.5, (n_marks, n_learns)
    assert ref.keys() == got.keys()
    for k in ref:
        assert torch.equal(ref[k], got[k]), k


def test_c5_bench_schedule_bit_identical_to_one_stream():
    """The schedule bench.py --overlap auto times at C5 (8x8 x 256, shared
    fp16): the next step's replay draws on a side stream beside the learn, the
    sampler's LDS cut to what the S' pass leaves of a CU (trainer "learn").
    Replay 300 (wrapped by step 300), 420 steps: losses, Q statistics,
    observations, the network, Adam slots, target shadows, random streams and
    rings bit-identical to the one-stream order."""
    import bench
    sched, cus, side_learn = bench.auto_schedule(8, 8, 256, True, False, False, None)
    assert sched == "learn" and cus is None and side_learn == 0
    cfg = dict(grid=(8, 8, 256), precision="fp16", shared=True)
    ref = _run_schedule({}, **cfg)
    got = _run_schedule({"overlap": sched}, **cfg)
    assert ref.keys() == got.keys()
    for k in ref:
        assert torch.equal(ref[k], got[k]), k


def test_c3_bench_schedule_bit_identical_to_one_stream():
    """The C3 schedule of bench.py (4x4 x 1024, fp16; the env step of t+1 and
    its draws beside learn t, ring stores in the two spare slots) vs the
    one-stream order in the sampler's set branch with the rings
    wrapped: replay 1,100 (n >= 1,046 from step 1,046 on), 1,200 steps (past the
    ring's 1,164 physical slots).
    Losses of every learn, Q statistics (collect_stats every 50th step), the
    last observations, weights, Adam slots, target shadows, random streams and
    rings bit-identical (compared on the device)."""
    def run(kw):
        tr = Trainer(EnvConfig(rows=4, cols=4, num_envs=1024, seed=2),
                     AgentConfig(precision="fp16", replay_buffer_size=1100, seed=2), **kw)
        losses, stats = [], []
        for t in range(1200):
            tr.step(collect_stats=t % 50 == 0)
            if tr.last_loss is not None:
                losses.append(tr.last_loss.clone())
                if t % 50 == 0:
                    stats.append(tr.agent.qstats.clone())
        torch.cuda.synchronize()
        ag = tr.agent
        assert len(ag.ring) == 1100 and ag.ring.start == 100 and ag.ring.total > ag.ring.slots
        out = dict(losses=torch.stack(losses), stats=torch.stack(stats), obs=tr.obs.clone(),
                   **{k: getattr(ag, k).clone() for k in ("params", "target", "adam_m", "adam_v",
                                                          "target_h", "np_state", "py_state")},
                   **{"ring_" + k: getattr(ag.ring, k).clone() for k in ("s", "n", "a", "r", "d")})
        del tr, ag
        torch.cuda.empty_cache()
        return out

    ref = run({})
    work, kw = _bench_c3_schedule()
    try:
        with torch.cuda.stream(work):
            got = run(kw)
    finally:
        torch.cuda.synchronize()
    assert ref.keys() == got.keys()
    for k in ref:
        assert torch.equal(ref[k], got[k]), k
    del ref, got
    torch.cuda.empty_cache()
