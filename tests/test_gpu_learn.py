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
from dmdqn_amd.agent import AgentConfig, BatchedDQN, keras_to_kernel, kernel_to_keras  # noqa: E402

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
    slots = (ring.start + idx) % ring.cap
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
    call("dmdqn_q_argmax", ptr(ag.params), 3, ag.P, ag.H, ptr(obs), ptr(ag.greedy), ptr(qd),
         stream_of())
    pk = ag.keras_params("params")
    q_ref = np.stack([O.qnet_forward(pk[j], obs[0, j:j + 1].cpu().numpy())[0] for j in range(3)])
    np.testing.assert_allclose(qd.cpu().numpy(), q_ref, rtol=1e-5, atol=1e-5)
    np.testing.assert_array_equal(ag.greedy.cpu().numpy().reshape(-1), q_ref.argmax(1))


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
                     w3_dz2=None, rnd=_f16r):
    """numpy restatement of the kernel's rounding points: 16-bit operands (rnd:
    f16 or bf16), f32 accumulation, 16-bit activations / Q / activation-gradients,
    f32 Adam.  w3_dz2 overrides the W3 [H][4] that backprop uses for dZ2 (test
    hook: the correct value is the pre-update W3)."""
    f32 = np.float32

    def split(w):
        sizes = [89 * H, H, H * H, H, H * 4, 4]
        out, o = [], 0
        for s in sizes:
            out.append(w[o:o + s])
            o += s
        W1, b1, W2, b2, W3, b3 = out
        return (rnd(W1.reshape(89, H)), b1, rnd(W2.reshape(H, H)), b2, rnd(W3.reshape(H, 4)), b3)

    def fwd(ws, X):
        W1, b1, W2, b2, W3, b3 = ws
        h1 = rnd(np.maximum(X @ W1 + b1, 0))
        h2 = rnd(np.maximum(h1 @ W2 + b2, 0))
        q = rnd(h2 @ W3 + b3)
        return h1, h2, q

    wo, wt = split(p), split(tgt)
    _, _, q2 = fwd(wo, S2)
    _, _, qt = fwd(wt, S2)
    a_star = q2.argmax(1)
    y = Rn + f32(gamma) * (1.0 - D) * qt[np.arange(128), a_star]
    h1, h2, q = fwd(wo, S)
    pred = q[np.arange(128), Aa]
    dq = (2.0 * (pred - y) / 128).astype(f32)
    loss = np.mean((y - pred) ** 2)
    dq16 = rnd(dq)
    DQ = np.zeros((128, 4), f32)
    DQ[np.arange(128), Aa] = dq16
    W1, b1, W2, b2, W3, b3 = wo
    gW3 = h2.T @ DQ
    gb3 = DQ.sum(0)
    W3b = W3 if w3_dz2 is None else rnd(w3_dz2)
    dz2 = rnd(np.where(h2 > 0, (dq16[:, None] * W3b[:, Aa].T), 0))
    gb2 = dz2.sum(0)
    gW2 = h1.T @ dz2
    dz1 = rnd(np.where(h1 > 0, dz2 @ W2.T, 0))
    gb1 = dz1.sum(0)
    gW1 = S.T @ dz1
    g = np.concatenate([gW1.ravel(), gb1, gW2.ravel(), gb2, gW3.ravel(), gb3]).astype(f32)
    alpha, c1, c2, eps = O.keras_adam_consts(t, lr)
    m2 = m + (g - m) * c1
    v2 = v + (g * g - v) * c2
    p2 = p - (m2 * alpha) / (np.sqrt(v2) + eps)
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

