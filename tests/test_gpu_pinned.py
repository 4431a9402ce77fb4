"""GPU parity pinned to the reference's own DQNAgent code, over many chained
learns without re-syncing, plus the loss option, the device z-score, replay
range errors and the reference's `done` rule.

* tests/golden/learn.npz is the reference's DQNAgent (dqn_agent.py:97-434) run
  under a torch-backed TF shim (tests/golden/make_learn_golden.py).  The drop-in
  src/agents/dqn_agent.py on the GPU replays the same loop from the same seeds
  and initial weights: 393 MSE / 233 Huber learns, never re-synced.
* Trainer (batched) vs oracle.OracleLoop (the C restatement of train.py's loop
  body) over 330 steps = 203 learns per agent, never re-synced.

Tolerances (stated): actions, replay indices, halting counts and observations
bit-exact; fp32 per-learn loss rtol 1e-4 vs the reference fixture and 1e-3 vs
the oracle loop; fp32 weights |dw| <= 5e-5 after the last learn.
fp16 (mixed_float16, the reference's policy) and bf16 vs the reference's own
learn under that policy (tests/golden/learn_mixed.npz): see
test_dropin_h16_matches_reference_mixed_per_learn for the stated bounds."""
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import oracle as O  # noqa: E402
from dmdqn_amd import _lib  # noqa: E402
from dmdqn_amd.agent import AgentConfig, BatchedDQN, keras_to_kernel, kernel_to_keras  # noqa: E402
from dmdqn_amd.env import EnvConfig, TrafficEnv  # noqa: E402
from dmdqn_amd.trainer import Trainer  # noqa: E402

import mixed_fixture as MF  # noqa: E402
from test_gpu_learn import TOL16, _fill, _host_batch  # noqa: E402

DEV = "cuda"
HERE = os.path.dirname(os.path.abspath(__file__))
G = np.load(os.path.join(HERE, "golden", "learn.npz"))


def _keras_list(flat, H=128):
    shapes = [(89, H), (H,), (H, H), (H,), (H, 4), (4,)]
    out, o = [], 0
    for sh in shapes:
        n = int(np.prod(sh))
        out.append(flat[o:o + n].reshape(sh))
        o += n
    return out


def _run_dropin(tag, precision):
    from src.agents import dqn_agent as DA
    steps, greedy_from, buf, tuf, seed, _ = (int(x) for x in G[f"{tag}_cfg"])
    obs = G[f"{tag}_obs"].astype(np.float32)
    rew, done = G[f"{tag}_rew"], G[f"{tag}_done"]
    cfg = {"learning_rate": 0.001, "gamma": 0.99, "epsilon_start": 1.0, "epsilon_min": 0.01,
           "epsilon_decay_steps": 200000, "replay_buffer_size": buf, "batch_size": 128,
           "target_update_frequency": tuf, "nn_layers": [128, 128], "precision": precision,
           "loss": tag}
    DA.seed(seed)  # random.seed(seed); np.random.seed(seed)
    ag = DA.DQNAgent(89, 4, "J_0_0", cfg)
    ag._core.set_weights(0, _keras_list(G[f"{tag}_w0"]))
    actions = np.zeros(steps, np.int32)
    losses = np.full(steps, np.nan)
    for t in range(steps):
        if t == greedy_from:
            ag.global_step_count = 40000
        actions[t] = ag.select_action(obs[t][None])
        ag.remember(obs[t][None], int(actions[t]), float(rew[t]), obs[t + 1][None], bool(done[t]))
        loss = ag.learn()
        if loss is not None:
            losses[t] = loss
    assert ag.learn_step_counter == int(G[f"{tag}_learn_steps"][0])
    online = np.concatenate([w.reshape(-1) for w in ag._core.get_weights(0)])
    target = kernel_to_keras(ag._core.target[0].cpu().numpy(), 128)
    return actions, losses, online, target


@pytest.mark.parametrize("tag", ["mse", "huber"])
def test_dropin_fp32_matches_reference_dqnagent(tag):
    """The drop-in DQNAgent (fp32 MFMA learn kernel) vs the reference's own
    DQNAgent: every action (numpy stream, greedy branch on the trained net)
    bit-exact; every loss rtol 1e-4; final online / target weights 5e-5."""
    actions, losses, online, target = _run_dropin(tag, "fp32")
    np.testing.assert_array_equal(actions, G[f"{tag}_actions"])
    ref = G[f"{tag}_losses"]
    assert np.array_equal(np.isnan(losses), np.isnan(ref))
    ok = ~np.isnan(ref)
    rel = np.abs(losses[ok] - ref[ok]) / np.abs(ref[ok])
    print(f"{tag} fp32: loss rel err max {rel.max():.3g} median {np.median(rel):.3g}; "
          f"|dw| max {np.abs(online - G[f'{tag}_final_online']).max():.3g}")
    np.testing.assert_allclose(losses[ok], ref[ok], rtol=1e-4)
    np.testing.assert_allclose(online, G[f"{tag}_final_online"], atol=5e-5)
    np.testing.assert_allclose(target, G[f"{tag}_final_target"], atol=5e-5)


# ---------------------------------------------------------------------------
# the 16-bit learn pinned to the reference's own DQNAgent under Keras 3's
# mixed precision policy (train.py:61): tests/golden/learn_mixed.npz
GM = MF.load()


def _run_dropin_mixed(tag, resync):
    """The drop-in DQNAgent (16-bit kernel) over the fixture's loop.  resync:
    before every learn inside the fixture's windows, load the reference's
    exact state (w, Adam m, v, target) into the agent; returns per-learn
    records (k, fragile, loss, ref loss, m' / w' equal shares and worst
    deviations) and the un-synced loss curve."""
    from src.agents import dqn_agent as DA
    precision, loss_kind = MF.RUNS[tag]
    c = MF.cfg(GM, tag)
    obs = GM[f"{tag}_obs"].astype(np.float32)
    rew, done = GM[f"{tag}_rew"], GM[f"{tag}_done"]
    cfg = {"learning_rate": 0.001, "gamma": 0.99, "epsilon_start": 1.0, "epsilon_min": 0.01,
           "epsilon_decay_steps": 200000, "replay_buffer_size": c["buf"], "batch_size": 128,
           "target_update_frequency": c["tuf"], "nn_layers": [128, 128], "precision": precision,
           "loss": "huber" if loss_kind else "mse"}
    DA.seed(c["seed"])
    ag = DA.DQNAgent(89, 4, "J_0_0", cfg)
    core = ag._core
    core.set_weights(0, _keras_list(GM[f"{tag}_w0"]))
    states = MF.window_states(GM, tag)[0] if resync else {}
    lref = GM[f"{tag}_losses"]
    lref = lref[~np.isnan(lref)]
    ties = GM[f"{tag}_tie_ulps"]
    put = lambda t, x: t[0].copy_(torch.from_numpy(keras_to_kernel(x, 128)))  # noqa: E731
    recs, curve = [], []
    for t in range(c["steps"]):
        a = ag.select_action(obs[t][None])
        assert a == GM[f"{tag}_actions"][t], f"step {t}"  # numpy stream, epsilon 1 (A-1)
        ag.remember(obs[t][None], a, float(rew[t]), obs[t + 1][None], bool(done[t]))
        k = core.learn_step_counter + 1 if len(core.ring) >= 128 else 0
        st = states.get(k)
        if st is not None:
            w, m, v, tg, g = st
            for name, x in (("params", w), ("adam_m", m), ("adam_v", v), ("target", tg)):
                put(getattr(core, name), x)
            core._refresh_target_h()
        loss = ag.learn()
        if loss is None:
            continue
        curve.append(loss)
        if st is not None:
            alpha, c1, c2, eps = O.keras_adam_consts(k)
            m_ref = m + (g - m) * c1
            v_ref = v + (g * g - v) * c2
            w_ref = w - (m_ref * alpha) / (np.sqrt(v_ref) + eps)
            m_g = core.keras_params("adam_m")[0]
            w_g = core.keras_params("params")[0]
            e = np.floor(np.log2(np.maximum(np.abs(g), 2.0 ** -14)))
            ulp = 2.0 ** (e - (10 if precision == "fp16" else 7))
            gap = np.abs(m_g - m_ref) / c1  # |g_gpu - g_ref|, up to m's own rounding
            recs.append(dict(k=k, fragile=bool(ties[k - 1] <= 1), loss=loss, ref=lref[k - 1],
                             m_eq=float(np.mean(m_g == m_ref)), w_eq=float(np.mean(w_g == w_ref)),
                             g_near=float(np.mean(gap <= ulp + 1e-3 * np.abs(g).max()
                                                  + 1e-6 * np.abs(m_ref) / c1)),
                             dw=float(np.abs(w_g - w_ref).max())))
    assert ag.learn_step_counter == int(GM[f"{tag}_learn_steps"][0])
    return recs, np.array(curve), lref


@pytest.mark.parametrize("tag", list(MF.RUNS))
def test_dropin_h16_matches_reference_mixed_per_learn(tag):
    """The 16-bit learn kernel (fp16 = the reference's mixed_float16, bf16 =
    mixed_bfloat16) vs the reference's own DQNAgent run under that policy, at
    every learn of the fixture's windows, each from the reference's exact
    state: mse_f16 learns 1-64 (target sync at 50) and 181-212 (replay
    wrapped) and 333; huber_f16 / mse_bf16 learns 1-16 and 203.
    Stated tolerances:
      * actions bit-exact (numpy stream);
      * loss rtol 2e-4; 2e-3 where the batch holds a Double-DQN near-tie (two
        16-bit online Q(S') of a row within one ulp: the argmax may then take
        the other action under another f32 summation order) -- measured
        3.0e-5 / 3.4e-4 (mse_f16), 6.4e-6 (huber_f16), 1.2e-7 (mse_bf16);
      * the gradient Adam received (from m'): >= 99 % of the entries within one
        16-bit ulp + 1e-3 of the largest entry of the reference's;
      * Adam bit-exact given the same gradient: >= 50 % of m' and w' entries
        bit-equal to Keras-3 Adam on the reference's gradient, and every
        weight within 5e-3 (one Adam step) of it."""
    recs, _, _ = _run_dropin_mixed(tag, resync=True)
    n_win = sum(int(n) for _, n in GM[f"{tag}_windows"])
    assert len(recs) == n_win
    rel = np.array([abs(r["loss"] - r["ref"]) / abs(r["ref"]) for r in recs])
    frag = np.array([r["fragile"] for r in recs])
    print(f"{tag}: {len(recs)} re-synced learns; loss rel err max {rel[~frag].max():.3g} "
          f"(near-tie learns {frag.sum()}, max {rel[frag].max() if frag.any() else 0:.3g}); "
          f"gradient near min {min(r['g_near'] for r in recs):.5f}; m' equal min "
          f"{min(r['m_eq'] for r in recs):.4f}, w' equal min {min(r['w_eq'] for r in recs):.4f}, "
          f"|dw| max {max(r['dw'] for r in recs):.3g}")
    for r, e in zip(recs, rel):
        assert e <= (2e-3 if r["fragile"] else 2e-4), (r["k"], e)
        assert r["g_near"] >= 0.99, r
        assert r["m_eq"] >= 0.5 and r["w_eq"] >= 0.5 and r["dw"] <= 5e-3, r


@pytest.mark.parametrize("tag", list(MF.RUNS))
def test_dropin_h16_unsynced_tracks_reference_mixed(tag):
    """The same loop never re-synced: every action bit-exact; the loss within
    2e-3 of the reference's over the first 8 learns; the two loss curves
    correlate > 0.98 over the whole run.  Two correct 16-bit runs part ways
    after a few dozen learns (a summation-order flip of one 16-bit rounding
    moves a tiny gradient entry, and Adam's first steps are ~lr * sign(g)):
    oracle.learn_mixed vs the fixture measures the same (mse_f16: 1e-3 by
    learn 25), so only the early learns are held to the per-learn bound."""
    _, curve, lref = _run_dropin_mixed(tag, resync=False)
    assert len(curve) == len(lref)
    rel = np.abs(curve - lref) / np.abs(lref)
    corr = float(np.corrcoef(curve, lref)[0, 1])
    print(f"{tag} un-synced: first-8 max {rel[:8].max():.3g}, median {np.median(rel):.3g}, "
          f"corr {corr:.4f}")
    assert rel[:8].max() <= 2e-3 and corr > 0.98


def test_trainer_many_learns_match_oracle_loop():
    """Trainer (2x2 grid x 2 replicas, fp32) vs oracle.OracleLoop for replica 1
    over 330 steps: the ring wraps (cap 250), 203 learns per agent, 4 target
    syncs, an episode boundary at step 240.  Actions, observations and replay
    indices are bit-exact at every step.  Two oracle loops run beside it:

    * free (never re-synced): each agent's loss rtol 1e-4 until its first
      Double-DQN near-tie -- a batch with two online Q(S') within 1e-5
      (relative), where the argmax (dqn_agent.py:342) may go either way under
      another fp32 summation order -- or learn 100, whichever comes first;
      >= 200 agent-learns in total.  In this env the two fp32 trajectories part
      after ~100-150 learns even without a tie (measured on the CPU between the
      C oracle and a torch restatement: first 1e-5 difference at learns 53 / 136
      / 151 / never), as the reference fixture's do after ~420
      (test_learn_golden_cpu.py); the drop-in test above covers 393 un-synced
      learns against the reference itself.
    * forced (its weights, target and Adam slots copied from the GPU before
      every step): every one of the 812 agent-learns rtol 1e-4 and the
      updated weights (stated below) -- each learn of the long run, syncs, wrap and episode
      boundary included, is checked from the state the GPU actually had."""
    E, steps = 2, 330
    cfg = AgentConfig(precision="fp32", replay_buffer_size=250, target_update_frequency=50,
                      seed=21)
    tr = Trainer(EnvConfig(rows=2, cols=2, num_envs=E, seed=40), cfg)
    A, ag = tr.env.A, tr.agent
    rows = slice(A, 2 * A)
    w0 = ag.keras_params("params")[rows]
    free = O.OracleLoop(2, 2, int(tr.env.seeds[1]), cap=250, tuf=50, weights=w0, track_ties=True)
    forced = O.OracleLoop(2, 2, int(tr.env.seeds[1]), cap=250, tuf=50, weights=w0)
    lg, lf, lo, n_off = [], [], [], []
    for t in range(steps):
        for k in ["params", "target", "adam_m", "adam_v"]:
            setattr(forced, k, kernel_to_keras(getattr(ag, k)[rows].cpu().numpy(), 128))
        forced.learn_steps = ag.learn_step_counter
        tr.step()
        out, outf = free.step(), forced.step()
        np.testing.assert_array_equal(ag.actions[1].cpu().numpy(), out["actions"])
        np.testing.assert_array_equal(tr.obs[1].cpu().numpy(), free.obs)
        if out["idx"] is not None:
            np.testing.assert_array_equal(ag.idx[rows].cpu().numpy(), out["idx"])
            lg.append(tr.last_loss[rows].cpu().numpy())
            lo.append(out["loss"])
            lf.append(outf["loss"])
            # >= 99.5 % of the updated weights within 1e-6 + 1e-5 |w|, all within
            # one Adam step (5e-3).  What is left outside: ReLU-boundary flips --
            # a pre-activation within rounding of 0 lands on opposite sides, and
            # that unit's gradient column for that row switches between 0 and
            # its value (~50-100 entries of an agent's 28,548; a few per run) --
            # and Adam's m / (sqrt(v) + eps) amplifying last-bit differences of
            # rarely driven parameters (test_gpu_learn.py)
            pg = ag.keras_params("params")[rows]
            close = np.abs(pg - forced.params) <= 1e-6 + 1e-5 * np.abs(forced.params)
            assert close.mean() >= 0.995, f"forced step {t}: {np.sum(~close)} off"
            np.testing.assert_allclose(pg, forced.params, atol=5e-3, err_msg=f"forced step {t}")
            n_off.append(int(np.sum(~close)))
    lg, lo, lf = np.array(lg), np.array(lo), np.array(lf)
    assert lg.shape == (203, A)
    np.testing.assert_allclose(lg, lf, rtol=1e-4)
    tied = np.array(free.tie_gaps) < 1e-5
    horizon = [min(100, int(np.argmax(tied[:, j])) if tied[:, j].any() else len(lg))
               for j in range(A)]
    rel = np.abs(lg - lo) / np.abs(lo)
    print(f"trainer vs oracle loop: un-synced horizons {horizon}, loss rel err inside max "
          f"{max(rel[:h, j].max() for j, h in enumerate(horizon) if h):.3g}; forced max "
          f"{(np.abs(lg - lf) / np.abs(lf)).max():.3g}, learns with weights outside 1e-5: "
          f"{sum(x > 0 for x in n_off)} (max {max(n_off)} entries)")
    assert sum(horizon) >= 200
    for j, h in enumerate(horizon):
        np.testing.assert_allclose(lg[:h, j], lo[:h, j], rtol=1e-4, err_msg=f"agent {j}")


# ---------------------------------------------------------------------------
# Huber loss (loss_kind 1) in every precision, and the device z-score
def test_learn_fp32_huber_matches_oracle():
    E, A = 2, 3
    ag = BatchedDQN(E, A, AgentConfig(replay_buffer_size=300, seed=4, loss="huber"))
    rng = np.random.RandomState(8)
    _fill(ag, 260, rng)
    p_h = ag.keras_params("params").copy()
    t_h = ag.keras_params("target").copy()
    m_h, v_h = np.zeros_like(p_h), np.zeros_like(p_h)
    for step in range(1, 4):
        loss = ag.learn().cpu().numpy()
        idx = ag.idx.cpu().numpy()
        for j in range(ag.NA):
            S, Aa, Rn, S2, D = _host_batch(ag, j, idx[j])
            lj = O.learn(p_h[j], t_h[j], m_h[j], v_h[j], S, Aa, Rn, S2, D, step, loss_kind=1)
            np.testing.assert_allclose(loss[j], lj, rtol=1e-5)
        np.testing.assert_allclose(ag.keras_params("params"), p_h, rtol=0, atol=1e-5)
        p_h = ag.keras_params("params").copy()
        m_h = ag.keras_params("adam_m").copy()
        v_h = ag.keras_params("adam_v").copy()


@pytest.mark.parametrize("precision", ["fp16", "bf16"])
def test_learn_h16_huber_loss_and_gradient(precision):
    """16-bit Huber learn vs the fp32 Huber oracle: loss within the MSE paths'
    stated rtol vs fp32 (2e-2), update direction correlated > 0.97, and the
    per-row dL/dq is the clipped one (gradient of W3's bias = sum of dL/dq per
    action, compared with the oracle's Huber gradient)."""
    E, A = 2, 4
    ag = BatchedDQN(E, A, AgentConfig(replay_buffer_size=300, seed=6, precision=precision,
                                      loss="huber"))
    rng = np.random.RandomState(3)
    _fill(ag, 200, rng)
    p0 = ag.keras_params("params").copy()
    t0 = ag.keras_params("target").copy()
    loss = ag.learn().cpu().numpy()
    idx = ag.idx.cpu().numpy()
    g_g = ag.keras_params("adam_m") / np.float32(0.1)
    p_g = ag.keras_params("params")
    t32 = TOL16[precision][4]
    for j in range(ag.NA):
        S, Aa, Rn, S2, D = _host_batch(ag, j, idx[j])
        p1, m1, v1 = p0[j].copy(), np.zeros_like(p0[j]), np.zeros_like(p0[j])
        l32, g32 = O.learn(p1, t0[j], m1, v1, S, Aa, Rn, S2, D, 1, want_grad=True, loss_kind=1)
        np.testing.assert_allclose(loss[j], l32, rtol=t32)
        gb3 = g_g[j][-4:]
        np.testing.assert_allclose(gb3, g32[-4:], rtol=3e-2, atol=3e-3 * np.abs(g32[-4:]).max())
        assert np.corrcoef(p_g[j] - p0[j], p1 - p0[j])[0, 1] > 0.97


@pytest.mark.parametrize("precision", ["fp32", "fp16", "bf16"])
def test_device_zscore_bit_exact(precision):
    """The z-scored rewards each learn kernel used (rn_out) equal numpy's
    (rewards - mean) / (std + 1e-8) of dqn_agent.py:66-69 bit for bit."""
    ag = BatchedDQN(2, 3, AgentConfig(replay_buffer_size=400, seed=2, precision=precision))
    rng = np.random.RandomState(4)
    _fill(ag, 300, rng)
    ag.rn_out = torch.zeros((ag.NA, 128), dtype=torch.float32, device=DEV)
    for _ in range(2):
        ag.learn()
        idx = ag.idx.cpu().numpy()
        rn = ag.rn_out.cpu().numpy()
        for j in range(ag.NA):
            slots = ag.ring.slots_of(idx[j])
            r = ag.ring.r[j].cpu().numpy()[slots]
            np.testing.assert_array_equal(rn[j], O.zscore(r))
            # and numpy itself (the reference's expression)
            np.testing.assert_array_equal(rn[j], ((r - np.mean(r)) / (np.std(r) + 1e-8)).astype(np.float32))


def test_dropin_replaybuffer_sample_zscore_bit_exact():
    from src.agents import dqn_agent as DA
    G2 = np.load(os.path.join(HERE, "golden", "replay_sample.npz"))
    n, seed = 1046, 1
    DA.seed(seed)
    buf = DA.ReplayBuffer(10000)
    loc, glob = G2[f"n{n}_loc"], G2[f"n{n}_glob"]
    for i in range(n):
        s = np.zeros((1, 89), np.float32)
        r = 0.3 * (-1.0 * float(loc[i])) + 0.7 * (-1.0 * float(glob[i]))
        buf.add((s, i % 4, r, s, (i % 240) == 239))
    for rep in range(3):
        _, _, rw, _, _ = buf.sample(128)
        np.testing.assert_array_equal(rw.cpu().numpy(), G2[f"n{n}_s{seed}_rew"][rep])


# ---------------------------------------------------------------------------
# replay range errors on the product path
def test_remember_non_integer_observation_raises():
    """A non-int8 observation raises within 2 POLL_LAG - 1 stores after it
    (kernels.ReplayRing.poll: one event per POLL_LAG polls; it can raise
    sooner when the GPU is ahead, never later), and check() raises at once."""
    from dmdqn_amd.kernels import POLL_LAG
    ag = BatchedDQN(1, 2, AgentConfig(replay_buffer_size=50))
    good = torch.zeros((1, 2, 89), dtype=torch.float32, device=DEV)
    bad = good.clone()
    bad[0, 1, 5] = 0.5
    a = torch.zeros((1, 2), dtype=torch.int32, device=DEV)
    r = torch.zeros((1, 2), dtype=torch.float64, device=DEV)
    for _ in range(POLL_LAG + 2):  # a clean ring never raises
        ag.remember(good, a, r, good, False)
    ag.ring.check()
    ag.remember(bad, a, r, good, False)
    with pytest.raises(_lib.DmdqnError, match="not an integer"):
        for _ in range(2 * POLL_LAG - 1):
            ag.remember(good, a, r, good, False)
    with pytest.raises(_lib.DmdqnError, match="not an integer"):
        ag.ring.check()


def test_dropin_remember_raises_immediately():
    """With the opt-in int8 rows (the drop-in default is float rows,
    tests/test_gpu_float_rows.py)."""
    from src.agents import dqn_agent as DA
    ag = DA.DQNAgent(89, 4, "J_0_0", {"replay_buffer_size": 50, "replay_rows": "int8"})
    s = np.zeros((1, 89), np.float32)
    ag.remember(s, 1, -3.0, s, False)
    s2 = s.copy()
    s2[0, 3] = 300.0  # out of int8 range
    with pytest.raises(_lib.DmdqnError):
        ag.remember(s2, 1, -3.0, s, False)


def test_trainer_raises_on_non_integer_observation():
    """... within 2 POLL_LAG steps of the bad store (kernels.ReplayRing.poll)."""
    from dmdqn_amd.kernels import POLL_LAG
    tr = Trainer(EnvConfig(rows=2, cols=2, num_envs=2, seed=1), AgentConfig(replay_buffer_size=50))
    tr.step()
    tr.obs = tr.obs + 0.25  # a caller feeding its own features
    with pytest.raises(_lib.DmdqnError):
        for _ in range(2 * POLL_LAG):
            tr.step()


# ---------------------------------------------------------------------------
# done = t >= MAX_SIM_TIME or no vehicle running / pending (train.py:233-236)
def test_done_when_demand_drains_before_max_time():
    cfg = EnvConfig(rows=2, cols=2, num_envs=1, seed=9, end_ms=60_000)
    env = TrafficEnv(cfg)
    assert env.drains_early
    ref = O.OracleEnv(2, 2, int(env.seeds[0]), end_ms=60_000)
    env.reset()
    nps = O.np_stream(3)
    t, done, steps = 0, False, 0
    while not done:
        acts = O.act(nps, 4, 1.0)
        _, _, done, info = env.step(torch.from_numpy(acts.reshape(1, 4)).to(DEV))
        _, _, _, d_ref = ref.step(acts, 3, t, 10, cfg.max_sim_time)
        t += 10
        steps += 1
        assert done == d_ref, f"step {steps}"
    assert t < cfg.max_sim_time  # ended by the empty network, not the clock
    # the Trainer stores the last transition with done = 1 and starts a new
    # episode at the step the reference loop (OracleLoop, same seeds) ends
    tr = Trainer(EnvConfig(rows=2, cols=2, num_envs=1, seed=9, end_ms=60_000),
                 AgentConfig(replay_buffer_size=500))
    ol = O.OracleLoop(2, 2, int(tr.env.seeds[0]), learn=False,
                      env=O.OracleEnv(2, 2, int(tr.env.seeds[0]), end_ms=60_000))
    n = 0
    while tr.episode == 0:
        tr.step()
        out = ol.step()
        n += 1
        assert out["done"] == (tr.episode == 1), f"step {n}"
        assert n < 240
    d = tr.agent.ring.d[:, :n].cpu().numpy()
    assert (d[:, -1] == 1).all() and (d[:, :-1] == 0).all()


def test_replicas_restart_on_their_own_done():
    """Three replicas whose demand drains at different steps (end_ms 60 s),
    each vs its own OracleLoop (train.py:188-207 for one env: traci.load when
    THAT env is done, replay kept): every step's actions, rewards, the
    observation the next act sees (the restart state after a done), the
    per-replica done flags stored with the transitions and the replay indices
    are bit-exact; each replica runs several episodes of its own length."""
    E, steps = 3, 130
    tr = Trainer(EnvConfig(rows=2, cols=2, num_envs=E, seed=9, end_ms=60_000),
                 AgentConfig(replay_buffer_size=500))
    assert tr.env.drains_early
    A = tr.env.A
    loops = [O.OracleLoop(2, 2, int(s), learn=False,
                          env=O.OracleEnv(2, 2, int(s), end_ms=60_000)) for s in tr.env.seeds]
    ends = [[] for _ in range(E)]
    for t in range(steps):
        tr.step()
        outs = [lp.step() for lp in loops]
        acts, rew = tr.agent.actions.cpu().numpy(), tr.last_reward.cpu().numpy()
        obs = tr.obs.cpu().numpy()
        d = tr.agent.ring.d[:, t].cpu().numpy().reshape(E, A)
        for e, out in enumerate(outs):
            np.testing.assert_array_equal(acts[e], out["actions"], err_msg=f"step {t} env {e}")
            np.testing.assert_array_equal(rew[e], out["reward"], err_msg=f"step {t} env {e}")
            np.testing.assert_array_equal(obs[e], loops[e].obs, err_msg=f"step {t} env {e}")
            assert (d[e] == int(out["done"])).all(), f"step {t} env {e}"
            if out["done"]:
                ends[e].append(t)
            if out["idx"] is not None:
                np.testing.assert_array_equal(tr.agent.idx[e * A:(e + 1) * A].cpu().numpy(),
                                              out["idx"], err_msg=f"step {t} env {e}")
    lens = [np.diff([-1] + x) for x in ends]
    print("episode lengths per replica:", [list(x) for x in lens])
    assert all(len(x) >= 2 for x in ends)
    assert len({tuple(x[:2]) for x in lens}) > 1, "replicas should drain at different steps"
    assert tr.episode == min(len(x) for x in ends)
