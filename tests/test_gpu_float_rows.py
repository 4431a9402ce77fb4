"""Float32 replay rows (AgentConfig.replay_rows = "f32"; the per-agent drop-in
DQNAgent's default): any observation value is stored as the reference's
ReplayBuffer stores it (dqn_agent.py:39-56) and learned from.

  * integer observations: the float-row learn is bit-identical to the int8-row
    learn in every precision (the same operands reach the MFMAs);
  * non-integer observations, fp32: each learn vs the fp32 oracle (oracle.learn,
    pinned to the reference's own learn by tests/golden/learn.npz) from the same
    state: loss rtol 1e-5, >= 99.99 % of the parameters within 1e-6 + 1e-5 |p|
    and every one within Adam's step (2e-3);
  * non-integer observations, fp16 / bf16: vs the Keras mixed-precision checker
    (oracle.learn_mixed: the input cast to 16 bits as the policy casts it);
  * the drop-in surface keeps 0.25 and 300.0 exactly; "int8" rows still refuse them."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import oracle as O  # noqa: E402
from dmdqn_amd import _lib  # noqa: E402
from dmdqn_amd.agent import AgentConfig, BatchedDQN  # noqa: E402

from test_gpu_learn import ROUND, TOL16, _host_batch, _mixed_emulation  # noqa: E402

DEV = "cuda"


def _fill(agent, T, rng, floats):
    E, A = agent.E, agent.A
    for t in range(T):
        if floats:
            s = rng.standard_normal((E, A, 89)).astype(np.float32) * 5
            n = rng.standard_normal((E, A, 89)).astype(np.float32) * 5
        else:
            s = rng.randint(-1, 24, size=(E, A, 89)).astype(np.float32)
            n = rng.randint(-1, 24, size=(E, A, 89)).astype(np.float32)
        a = torch.from_numpy(rng.randint(0, 4, size=(E, A)).astype(np.int32)).to(DEV)
        r = torch.from_numpy(-rng.rand(E, A) * 50).to(DEV)
        agent.remember(torch.from_numpy(s).to(DEV), a, r, torch.from_numpy(n).to(DEV),
                       (t % 60) == 59)
    agent.ring.check()


@pytest.mark.parametrize("precision,hidden", [("fp32", 128), ("fp32", 64), ("fp16", 128),
                                              ("bf16", 128)])
def test_float_rows_bit_identical_to_int8_rows_on_integers(precision, hidden):
    res = {}
    for rows in ("int8", "f32"):
        cfg = AgentConfig(precision=precision, nn_layers=[hidden, hidden], replay_buffer_size=200,
                          target_update_frequency=3, seed=4, replay_rows=rows)
        ag = BatchedDQN(2, 3, cfg)
        assert ag.ring.row_format == rows
        rng = np.random.RandomState(5)
        _fill(ag, 230, rng, floats=False)  # wraps the rings
        losses = [ag.learn().clone() for _ in range(4)]
        torch.cuda.synchronize()
        res[rows] = [torch.stack(losses), ag.params.clone(), ag.adam_v.clone(), ag.target.clone()]
    for a, b in zip(res["int8"], res["f32"]):
        assert torch.equal(a.view(torch.int32), b.view(torch.int32))


@pytest.mark.parametrize("hidden", [128, 64])
def test_float_rows_fp32_learn_matches_oracle(hidden):
    cfg = AgentConfig(replay_buffer_size=300, nn_layers=[hidden, hidden], target_update_frequency=3,
                      seed=3, replay_rows="f32")
    ag = BatchedDQN(2, 3, cfg)
    rng = np.random.RandomState(0)
    _fill(ag, 330, rng, floats=True)
    S0 = ag.ring.s.cpu().numpy()
    assert np.any(S0 != np.round(S0)), "the rows hold non-integers"
    p_h = ag.keras_params("params").copy()
    t_h = ag.keras_params("target").copy()
    m_h = np.zeros_like(p_h)
    v_h = np.zeros_like(p_h)
    for step in range(1, 5):
        loss = ag.learn()
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
        # near-zero gradient entries can take Adam's full step (~lr) either way
        # when the summation order flips their sign: a share bound plus the
        # step bound, as for the integer rows' >= 99.99 % (test_gpu_learn.py)
        close = np.abs(p_g - p_h) <= 1e-6 + 1e-5 * np.abs(p_h)
        assert close.mean() >= 0.9999, f"params step {step}: {close.size - close.sum()} off"
        np.testing.assert_allclose(p_g, p_h, rtol=0, atol=2e-3, err_msg=f"params step {step}")
        p_h, m_h = p_g.copy(), ag.keras_params("adam_m").copy()
        v_h, t_h = ag.keras_params("adam_v").copy(), ag.keras_params("target").copy()


@pytest.mark.parametrize("precision", ["fp16", "bf16"])
def test_float_rows_mixed_learn_matches_checker(precision):
    cfg = AgentConfig(replay_buffer_size=300, target_update_frequency=2, seed=5,
                      precision=precision, replay_rows="f32")
    ag = BatchedDQN(2, 2, cfg)
    rng = np.random.RandomState(2)
    _fill(ag, 200, rng, floats=True)
    tl = TOL16[precision][0]
    for _ in range(3):
        p0 = ag.keras_params("params").copy()
        t0 = ag.keras_params("target").copy()
        m0, v0 = ag.keras_params("adam_m").copy(), ag.keras_params("adam_v").copy()
        loss = ag.learn().cpu().numpy()
        idx = ag.idx.cpu().numpy()
        t = ag.learn_step_counter
        for j in range(ag.NA):
            S, Aa, Rn, S2, D = _host_batch(ag, j, idx[j])
            l_e = _mixed_emulation(p0[j], t0[j], m0[j], v0[j], S, Aa, Rn, S2, D, t,
                                   rnd=ROUND[precision])[0]
            np.testing.assert_allclose(loss[j], l_e, rtol=tl, err_msg=f"agent {j} learn {t}")


def test_dropin_keeps_float_observations():
    from src.agents import dqn_agent as DA
    ag = DA.DQNAgent(89, 4, "J_0_0", {"replay_buffer_size": 50})
    assert ag.replay_buffer.ring.row_format == "f32"
    s = np.zeros((1, 89), np.float32)
    s2 = s.copy()
    s2[0, 3] = 300.0
    s2[0, 7] = 0.25
    for _ in range(3):
        ag.remember(s2, 1, -3.0, s, False)
    rows = ag.replay_buffer.ring.s[0, :3, :89].cpu().numpy()
    np.testing.assert_array_equal(rows, np.repeat(s2, 3, axis=0))
    # the opt-in int8 rows refuse them at once
    ai = DA.DQNAgent(89, 4, "J_0_1", {"replay_buffer_size": 50, "replay_rows": "int8"})
    ai.remember(s, 1, -3.0, s, False)
    with pytest.raises(_lib.DmdqnError):
        ai.remember(s2, 1, -3.0, s, False)
