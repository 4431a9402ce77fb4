"""The 16-bit learn checker (oracle.learn_mixed: DQNAgent.learn under Keras 3's
mixed precision policy, in numpy) pinned to the reference's own DQNAgent run
under that policy (tests/golden/learn_mixed.npz, see tests/mixed_fixture.py).

Stated tolerances, at every learn inside the fixture's windows, from the
reference's exact state before that learn:
  * loss rtol 1e-4, or 2e-3 at a learn whose batch has a Double-DQN near-tie
    (two online Q(S') of a row within one 16-bit ulp, tie_ulps <= 1): the
    argmax of dqn_agent.py:342 may then pick the other action for that row
    under another f32 summation order, moving the loss by ~1e-4..1e-3;
  * gradient: >= 75 % of the entries bit-equal to the reference's 16-bit
    gradient and >= 99.9 % within one 16-bit ulp of it plus 1e-3 of the
    largest entry -- what is left is f32 summation order (torch CPU in the
    fixture, numpy here) flipping a 16-bit rounding or a ReLU boundary.
The state replay itself is exact: Keras-3 Adam on the stored gradients gives
the stored weights after each window bit for bit."""
import numpy as np
import pytest

import oracle as O
import mixed_fixture as MF

G = MF.load()


def _ulp16(x, precision):
    e = np.floor(np.log2(np.maximum(np.abs(x), 2.0 ** -14)))
    return 2.0 ** (e - (10 if precision == "fp16" else 7))


@pytest.mark.parametrize("tag", list(MF.RUNS))
def test_state_replay_exact(tag):
    states, post = MF.window_states(G, tag)
    for i, (a, n) in enumerate(G[f"{tag}_windows"]):
        k = int(a + n - 1)
        np.testing.assert_array_equal(post[k], G[f"{tag}_win_post_w"][i])


@pytest.mark.parametrize("tag", list(MF.RUNS))
def test_learn_mixed_matches_reference_per_learn(tag):
    precision, loss_kind = MF.RUNS[tag]
    states, _ = MF.window_states(G, tag)
    losses = G[f"{tag}_losses"]
    lref = losses[~np.isnan(losses)]
    n_checked, worst_eq = 0, 1.0
    for k, t, S, A, Rn, S2, D, _ in MF.batches(G, tag):
        if k not in states:
            continue
        w, m, v, tg, g_ref = states[k]
        l, g = O.learn_mixed(w, tg, m, v, S, A, Rn, S2, D, k, precision=precision,
                             loss_kind=loss_kind, want_grad=True)
        fragile = G[f"{tag}_tie_ulps"][k - 1] <= 1
        np.testing.assert_allclose(l, lref[k - 1], rtol=2e-3 if fragile else 1e-4,
                                   err_msg=f"learn {k}")
        eq = float(np.mean(g == g_ref))
        near = np.abs(g - g_ref) <= _ulp16(g_ref, precision) + 1e-3 * np.abs(g_ref).max()
        assert eq >= 0.75 and near.mean() >= 0.999, f"learn {k}: {eq:.4f} equal, {near.mean():.5f} near"
        worst_eq = min(worst_eq, eq)
        n_checked += 1
    assert n_checked == sum(int(n) for _, n in G[f"{tag}_windows"])
    print(f"{tag}: {n_checked} learns, worst bit-equal gradient share {worst_eq:.4f}")


def test_fixture_covers_the_asked_regimes():
    """>= 300 learns with the deque wrapped and target syncs for mse_f16; the
    windows reach into the wrapped regime."""
    c = MF.cfg(G, "mse_f16")
    assert int(G["mse_f16_learn_steps"][0]) >= 300
    assert c["steps"] > c["buf"] and int(G["mse_f16_learn_steps"][0]) // c["tuf"] >= 6
    wrap_learn = c["buf"] - 127 + 1  # first learn after the deque holds buf and drops one
    assert any(a + n - 1 >= wrap_learn for a, n in G["mse_f16_windows"])
