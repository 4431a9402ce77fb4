"""GPU parity of the fused learn kernel (dmdqn_learn) vs the C oracle restatement
of DQNAgent.learn (Keras semantics), through the C ABI.

Tolerances (stated): fp32 path -- loss rtol 1e-5; weights after each Adam
step: >= 99.99 % within 1e-6 + 1e-5|w| and ALL within 1e-5 absolute (1 % of one
Adam step at lr 1e-3; Adam's update m/(sqrt(v)+eps) amplifies the last-bit
summation-order differences of gradients whose magnitude is near eps);
Adam m / v rtol 1e-4 scaled by the largest gradient.  Replay indices and the
z-scored rewards feeding the kernel are bit-exact (tested separately)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import oracle as O  # noqa: E402
from dmdqn_amd import kernels as K  # noqa: E402
from dmdqn_amd.agent import (AgentConfig, BatchedDQN, PRECISIONS, keras_to_kernel,  # noqa: E402
                             kernel_to_keras)

DEV = "cuda"


def _fill(agent, T, rng):
    E, A = agent.E, agent.A
    for t in range(T):
        s = torch.from_numpy(rng.randint(-1, 24, size=(E, A, 89)).astype(np.float32)).to(DEV)
        n = torch.from_numpy(rng.randint(-1, 24, size=(E, A, 89)).astype(np.float32)).to(DEV)
        a = torch.from_numpy(rng.randint(0, 4, size=(E, A)).astype(np.int32)).to(DEV)
        loc = rng.randint(0, 40, size=(E, A))
        glob = rng.randint(0, 400, size=(E, 1))
        r = 0.3 * (-1.0 * loc) + 0.7 * (-1.0 * glob)
        agent.remember(s, a, torch.from_numpy(r).to(DEV), n, (t % 60) == 59)
    agent.ring.check()


def _host_batch(agent, ag, idx):
    ring = agent.ring
    slots = ring.slots_of(idx)
    S = ring.s[ag].cpu().numpy()[slots, :89].astype(np.float32)
    S2 = ring.n[ag].cpu().numpy()[slots, :89].astype(np.float32)
    A = ring.a[ag].cpu().numpy()[slots].astype(np.int32)
    r = ring.r[ag].cpu().numpy()[slots]
    D = ring.d[ag].cpu().numpy()[slots].astype(np.float32)
    return S, A, O.zscore(r), S2, D


@pytest.mark.parametrize("hidden", [128, 64])
def test_learn_fp32_matches_oracle(hidden):
    E, A = 2, 5
    cfg = AgentConfig(replay_buffer_size=300, nn_layers=[hidden, hidden], target_update_frequency=3,
                      seed=3)
    ag = BatchedDQN(E, A, cfg)
    rng = np.random.RandomState(0)
    _fill(ag, 330, rng)  # wraps the ring (start != 0)
    assert ag.ring.start == 30
    p_h = ag.keras_params("params").copy()
    t_h = ag.keras_params("target").copy()
    m_h = np.zeros_like(p_h)
    v_h = np.zeros_like(p_h)
    for step in range(1, 5):
        loss = ag.learn()
        assert loss is not None
        idx = ag.idx.cpu().numpy()
        losses = []
        for j in range(ag.NA):
            S, Aa, Rn, S2, D = _host_batch(ag, j, idx[j])
            losses.append(O.learn(p_h[j], t_h[j], m_h[j], v_h[j], S, Aa, Rn, S2, D, step,
                                  H1=hidden, H2=hidden))
        if step % 3 == 0:
            t_h = p_h.copy()
        p_g = ag.keras_params("params")
        np.testing.assert_allclose(loss.cpu().numpy(), np.array(losses), rtol=1e-5)
        close = np.abs(p_g - p_h) <= 1e-6 + 1e-5 * np.abs(p_h)
        assert close.mean() >= 0.9999, f"params step {step}: {close.size - close.sum()} off"
        np.testing.assert_allclose(p_g, p_h, rtol=0, atol=1e-5, err_msg=f"params step {step}")
        gs = np.sqrt(np.abs(v_h).max() / 1e-3)
        np.testing.assert_allclose(ag.keras_params("adam_m"), m_h, rtol=1e-4, atol=1e-6 * gs)
        np.testing.assert_allclose(ag.keras_params("adam_v"), v_h, rtol=1e-4, atol=1e-8 * gs * gs)
        np.testing.assert_allclose(ag.keras_params("target"), t_h, rtol=0, atol=1e-5)
        # keep the oracle on the GPU trajectory so errors do not compound
        p_h = p_g.copy()
        m_h = ag.keras_params("adam_m").copy()
        v_h = ag.keras_params("adam_v").copy()
        t_h = ag.keras_params("target").copy()


def test_learn_gate_and_q_argmax():
    ag = BatchedDQN(1, 3, AgentConfig(replay_buffer_size=500))
    rng = np.random.RandomState(1)
    _fill(ag, 127, rng)
    assert ag.learn() is None  # dqn_agent.py:333-335
    _fill(ag, 1, rng)
    assert ag.learn() is not None
    obs = torch.from_numpy(rng.randint(-1, 24, size=(1, 3, 89)).astype(np.float32)).to(DEV)
    from dmdqn_amd._lib import call, ptr, stream_of
    qd = torch.empty((3, 4), dtype=torch.float32, device=DEV)
    call("dmdqn_q_argmax", ptr(ag.params), 3, ag.P, ag.H, 0, ptr(obs), ptr(ag.greedy), ptr(qd),
         stream_of())
    pk = ag.keras_params("params")
    q_ref = np.stack([O.qnet_forward(pk[j], obs[0, j:j + 1].cpu().numpy())[0] for j in range(3)])
    np.testing.assert_allclose(qd.cpu().numpy(), q_ref, rtol=1e-5, atol=1e-5)
    np.testing.assert_array_equal(ag.greedy.cpu().numpy().reshape(-1), q_ref.argmax(1))


@pytest.mark.parametrize("precision", ["fp16", "bf16"])
def test_q_argmax_mixed_policy(precision):
    """The greedy forward under mixed_float16 / mixed_bfloat16 (precision 1 / 2)
    vs oracle.qnet_forward_mixed: 16-bit Q values equal except where an f32
    summation-order difference flips one 16-bit rounding (one ulp), and the
    argmax (first max on ties) equal on every row without a top-2 gap of at
    most one ulp.  200 agents of random weights."""
    NA = 200
    ag = BatchedDQN(1, NA, AgentConfig(replay_buffer_size=200, precision=precision, seed=3))
    rng = np.random.RandomState(5)
    obs = torch.from_numpy(rng.randint(-1, 24, size=(1, NA, 89)).astype(np.float32)).to(DEV)
    from dmdqn_amd._lib import call, ptr, stream_of
    qd = torch.empty((NA, 4), dtype=torch.float32, device=DEV)
    call("dmdqn_q_argmax", ptr(ag.params), NA, ag.P, ag.H, PRECISIONS[precision], ptr(obs),
         ptr(ag.greedy), ptr(qd), stream_of())
    pk = ag.keras_params("params")
    q_ref = np.stack([O.qnet_forward_mixed(pk[j], obs[0, j:j + 1].cpu().numpy(), precision)[0]
                      for j in range(NA)])
    q = qd.cpu().numpy()
    rnd = ROUND[precision]
    assert np.array_equal(rnd(q), q), "16-bit Q values"
    ulp = np.abs(q_ref) * (2.0 ** -10 if precision == "fp16" else 2.0 ** -7)
    assert (np.abs(q - q_ref) <= ulp + 1e-6).all()
    assert np.mean(q == q_ref) >= 0.97
    top = np.sort(q_ref, 1)
    safe = (top[:, -1] - top[:, -2]) > ulp.max(1)
    np.testing.assert_array_equal(ag.greedy.cpu().numpy().reshape(-1)[safe], q_ref.argmax(1)[safe])


# ---------------------------------------------------------------------------
# fp16 (mixed_float16) and bf16 (mixed_bfloat16) paths
def _f16r(x):
    return np.asarray(x, np.float32).astype(np.float16).astype(np.float32)


def _bf16r(x):
    """f32 -> bf16 -> f32, round to nearest even (v_cvt_pk_bf16_f32; finite inputs)."""
    u = np.ascontiguousarray(x, dtype=np.float32).view(np.uint32).astype(np.uint64)
    u = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16
    return u.astype(np.uint32).view(np.float32)


ROUND = {"fp16": _f16r, "bf16": _bf16r}


def _mixed_emulation(p, tgt, m, v, S, Aa, Rn, S2, D, t, H=128, gamma=0.99, lr=1e-3,
                     w3_dz2=None, rnd=_f16r, loss_kind=0, round_grad=True):
    """One learn under Keras 3's mixed policy: oracle.learn_mixed (the checker
    pinned to the reference's own DQNAgent run under mixed_float16 /
    mixed_bfloat16, tests/test_learn_mixed_golden_cpu.py) on copies of the
    state.  Returns (loss, 16-bit gradient, w', m', v').  w3_dz2 overrides the
    W3 [H][4] that backprop uses for dZ2 (test hook: the correct value is the
    pre-update W3)."""
    precision = "fp16" if rnd is _f16r else "bf16"
    p2, m2, v2 = (np.array(x, np.float32, copy=True) for x in (p, m, v))
    loss, g = O.learn_mixed(p2, tgt, m2, v2, S, Aa, Rn, S2, D, t, precision=precision,
                            gamma=gamma, lr=lr, H=H, loss_kind=loss_kind, round_grad=round_grad,
                            want_grad=True, w3_bwd=w3_dz2)
    return loss, g, p2, m2, v2


# per precision: (loss rtol vs the emulation, gradient abs tol x max|g|, gradient
# rel tol, share of bias / W3 entries within it, loss rtol vs the fp32 oracle).
# bf16 keeps 8 mantissa bits to f16's 11, so a rounding-boundary flip moves a
# value 8x further.
TOL16 = {"fp16": (2e-3, 2e-3, 1e-2, 0.97, 2e-2),
         "bf16": (1.6e-2, 1.6e-2, 8e-2, 0.95, 2e-2)}


@pytest.mark.parametrize("precision", ["fp16", "bf16"])
def test_learn_h16_matches_mixed_emulation_and_fp32_oracle(precision):
    E, A = 2, 4
    cfg = AgentConfig(replay_buffer_size=300, target_update_frequency=2, seed=5, precision=precision)
    rnd = ROUND[precision]
    tl, ta, tr, tshare, t32 = TOL16[precision]
    ag = BatchedDQN(E, A, cfg)
    rng = np.random.RandomState(2)
    _fill(ag, 200, rng)
    p0 = ag.keras_params("params").copy()
    t0 = ag.keras_params("target").copy()
    loss = ag.learn().cpu().numpy()
    idx = ag.idx.cpu().numpy()
    m_g = ag.keras_params("adam_m")
    p_g = ag.keras_params("params")
    for j in range(ag.NA):
        S, Aa, Rn, S2, D = _host_batch(ag, j, idx[j])
        zero = np.zeros_like(p0[j])
        l_e, g_e, p_e, m_e, v_e = _mixed_emulation(p0[j], t0[j], zero, zero.copy(), S, Aa, Rn, S2, D, 1,
                                                   rnd=rnd)
        # tight: same rounding points.  What remains is accumulation order: an
        # f16 ulp here and there, and ReLU-boundary flips (a pre-activation within
        # rounding of 0 lands on opposite sides), each of which moves one column
        # of dW1 or one row of dW2 -- a few dozen entries per agent.
        np.testing.assert_allclose(loss[j], l_e, rtol=tl)
        g_g = m_g[j] / np.float32(0.1)
        assert np.isfinite(g_g).all()
        gs = np.abs(g_e).max()
        close = np.abs(g_g - g_e) <= ta * gs + tr * np.abs(g_e)
        assert close.mean() > 0.99, f"agent {j}: {np.sum(~close)} gradient entries off"
        H = 128
        o_b1, o_b2, o_w3 = 89 * H, 89 * H + H + H * H, 89 * H + H + H * H + H
        for lo, hi in [(o_b1, o_b1 + H), (o_b2, o_b2 + H), (o_w3, o_w3 + 4 * H + 4)]:
            assert close[lo:hi].mean() > tshare, (lo, hi)
        # stated tolerance vs the fp32 oracle (rtol 2e-2 on the loss)
        p1, m1, v1 = p0[j].copy(), zero.copy(), zero.copy()
        l32 = O.learn(p1, t0[j], m1, v1, S, Aa, Rn, S2, D, 1)
        np.testing.assert_allclose(loss[j], l32, rtol=t32)
        # backprop must use the PRE-update W3 (Adam on W3 runs first in the
        # kernel): the gradients of W1/b1/W2/b2 sit far closer to that emulation
        # than to one using the post-update W3 (a ~1% relative shift)
        o_w3e = o_w3 + 4 * H
        w3_new = p_e[o_w3:o_w3e].reshape(H, 4)
        _, g_bad, _, _, _ = _mixed_emulation(p0[j], t0[j], zero, zero.copy(), S, Aa, Rn, S2, D, 1,
                                             w3_dz2=w3_new, rnd=rnd)
        big = np.abs(g_e[:o_w3]) > 0.1 * np.abs(g_e[:o_w3]).max()
        err_ok = np.median(np.abs(g_g[:o_w3] - g_e[:o_w3])[big] / np.abs(g_e[:o_w3])[big])
        err_bad = np.median(np.abs(g_g[:o_w3] - g_bad[:o_w3])[big] / np.abs(g_bad[:o_w3])[big])
        assert err_ok < 0.3 * err_bad, (err_ok, err_bad)
        dw_g, dw_o = p_g[j] - p0[j], p1 - p0[j]
        assert np.corrcoef(dw_g, dw_o)[0, 1] > 0.97
    # second learn triggers the target sync (frequency 2)
    ag.learn()
    np.testing.assert_array_equal(ag.target.cpu().numpy(), ag.params.cpu().numpy())
    # ... and its 16-bit shadow (the target forward's operand) is the RNE rounding
    th = ag.target_h[:, :ag.P].float().cpu().numpy()
    np.testing.assert_array_equal(th, rnd(ag.target.cpu().numpy()))

