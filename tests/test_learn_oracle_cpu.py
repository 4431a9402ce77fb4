"""The C learn-step oracle (Keras semantics) vs an independent torch-autograd
fp32 restatement on the CPU.  Tolerance: rtol 1e-4 / atol 1e-6 (summation order)."""
import numpy as np
import pytest
import torch

import oracle as O

H = 128


def _split(p, H1=H, H2=H, NA=4):
    sizes = [89 * H1, H1, H1 * H2, H2, H2 * NA, NA]
    shapes = [(89, H1), (H1,), (H1, H2), (H2,), (H2, NA), (NA,)]
    out, o = [], 0
    for s, sh in zip(sizes, shapes):
        out.append(p[o:o + s].reshape(sh))
        o += s
    return out


def _fwd(ws, x):
    W1, b1, W2, b2, W3, b3 = ws
    h1 = torch.relu(x @ W1 + b1)
    h2 = torch.relu(h1 @ W2 + b2)
    return h2 @ W3 + b3


def torch_learn(p, tgt, m, v, S, A, Rn, S2, Dn, t, gamma=0.99, lr=1e-3):
    ws = [torch.tensor(w, requires_grad=True) for w in _split(p)]
    wt = [torch.tensor(w) for w in _split(tgt)]
    S, S2 = torch.tensor(S), torch.tensor(S2)
    with torch.no_grad():
        a_star = torch.argmax(_fwd(ws, S2), dim=1)
        tq = _fwd(wt, S2).gather(1, a_star[:, None])[:, 0]
        y = torch.tensor(Rn) + np.float32(gamma) * (1.0 - torch.tensor(Dn)) * tq
    q = _fwd(ws, S).gather(1, torch.tensor(A, dtype=torch.long)[:, None])[:, 0]
    loss = torch.mean((y - q) ** 2)
    loss.backward()
    g = torch.cat([w.grad.reshape(-1) for w in ws]).numpy()
    alpha, c1, c2, eps = O.keras_adam_consts(t, lr)
    m2 = m + (g - m) * c1
    v2 = v + (g * g - v) * c2
    p2 = p - (m2 * alpha) / (np.sqrt(v2) + eps)
    return float(loss.detach()), g, p2, m2, v2


def _batch(rng, B=128):
    S = rng.randint(-1, 24, size=(B, 89)).astype(np.float32)
    S2 = rng.randint(-1, 24, size=(B, 89)).astype(np.float32)
    A = rng.randint(0, 4, size=B).astype(np.int32)
    Rn = rng.normal(size=B).astype(np.float32)
    Dn = (rng.rand(B) < 0.1).astype(np.float32)
    return S, A, Rn, S2, Dn


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_learn_oracle_matches_torch(seed):
    rng = np.random.RandomState(seed)
    p = O.keras_init(rng)
    tgt = O.keras_init(rng) if seed == 2 else p.copy()
    m = (rng.normal(size=p.size) * 1e-3).astype(np.float32) if seed else np.zeros_like(p)
    v = (rng.rand(p.size) * 1e-5).astype(np.float32) if seed else np.zeros_like(p)
    S, A, Rn, S2, Dn = _batch(rng)
    t = 1 + 7 * seed
    tl, tg, tp, tm, tv = torch_learn(p, tgt, m, v, S, A, Rn, S2, Dn, t)
    p1, m1, v1 = p.copy(), m.copy(), v.copy()
    loss, g = O.learn(p1, tgt, m1, v1, S, A, Rn, S2, Dn, t, want_grad=True)
    np.testing.assert_allclose(loss, tl, rtol=1e-5)
    gs = np.abs(tg).max()  # summation-order error scales with the largest gradient
    np.testing.assert_allclose(g, tg, rtol=1e-4, atol=1e-6 * gs)
    np.testing.assert_allclose(m1, tm, rtol=1e-4, atol=1e-7 * gs)
    np.testing.assert_allclose(v1, tv, rtol=1e-4, atol=1e-9 * gs * gs)
    np.testing.assert_allclose(p1, tp, rtol=1e-5, atol=1e-6)


def test_forward_matches_torch():
    rng = np.random.RandomState(5)
    p = O.keras_init(rng)
    x = rng.randint(-1, 24, size=(64, 89)).astype(np.float32)
    q = O.qnet_forward(p, x)
    qt = _fwd([torch.tensor(w) for w in _split(p)], torch.tensor(x)).numpy()
    np.testing.assert_allclose(q, qt, rtol=1e-5, atol=1e-5)


def test_keras_adam_constants():
    alpha, c1, c2, eps = O.keras_adam_consts(1)
    # t=1: alpha = lr*sqrt(1-b2)/(1-b1) = 1e-3*sqrt(1e-3)/0.1
    np.testing.assert_allclose(alpha, 1e-3 * np.sqrt(1e-3) / 0.1, rtol=1e-4)
    assert c1 == np.float32(0.1) and c2 == np.float32(0.001) and eps == np.float32(1e-7)


def test_cpu_baseline_loop_runs_multithreaded():
    """oracle_loop.c (bench's CPU baseline): the full loop body over replicas
    with OpenMP; learn is active in every timed step (fill 127)."""
    import oracle as O
    el, n = O.train_loop(2, 2, 3, 127, 2, 0, 3)
    assert el > 0 and n == 3 * 2 * 4
