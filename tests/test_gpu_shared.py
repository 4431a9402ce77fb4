"""GPU parity of the shared-parameter DQN (configuration C5; not in
the reference): ONE network for all agents, trained on the mean of the
per-agent Double-DQN MSE losses.

Checked through the C ABI (dmdqn_learn_shared_grad, dmdqn_adam,
dmdqn_q_argmax_shared):
  * the summed-and-scaled gradient equals the mean over agents of the
    per-agent gradients of the mixed-precision emulation (the same restatement
    and tolerance as the independent fp16 test: >= 99 % of entries within
    2e-3 * max|g| + 1e-2 |g|), and the per-agent losses match it (rtol 2e-3);
  * the Adam step applied to that gradient is the Keras-3 update (rtol 1e-6);
  * the target sync copies the shared network (and its f16 shadow);
  * greedy actions with the shared network equal per-agent argmax on
    replicated weights.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import oracle as O  # noqa: E402
from dmdqn_amd.agent import AgentConfig, BatchedDQN, kernel_to_keras  # noqa: E402
from test_gpu_learn import _fill, _host_batch, _mixed_emulation  # noqa: E402

DEV = "cuda"


def _shared(E, A, freq=500, seed=7, cap=300):
    cfg = AgentConfig(replay_buffer_size=cap, target_update_frequency=freq, seed=seed,
                      precision="fp16", shared_params=True)
    return BatchedDQN(E, A, cfg)


@pytest.mark.parametrize("cap,fill", [(300, 200), (300, 330), (1100, 1160)])
def test_shared_gradient_is_mean_of_agent_gradients(cap, fill):
    """(300, 200): a partly filled ring (start 0, the sampler's pool branch);
    (300, 330): a wrapped ring, deque position 0 at slot 30 (the ring-slot
    arithmetic of both shared passes, learn_shared.hip ring_slot / xrows_issue);
    (1100, 1160): wrapped at n = 1100 > 1045, the sampler's set branch -- the
    regime every steady-state C5 step runs in (dqn_agent.py:29, 59-85)."""
    ag = _shared(3, 4, cap=cap)
    assert ag.params.shape[0] == 1 and ag.NA == 12
    rng = np.random.RandomState(4)
    _fill(ag, fill, rng)
    assert ag.ring.start == max(0, fill - cap) and len(ag.ring) == min(fill, cap)
    p0 = ag.keras_params("params")[0].copy()
    t0 = ag.keras_params("target")[0].copy()
    loss = ag.learn().cpu().numpy()
    idx = ag.idx.cpu().numpy()
    g_g = kernel_to_keras(ag.grad.cpu().numpy()[None], ag.H)[0]
    zero = np.zeros_like(p0)
    ges, les = [], []
    for j in range(ag.NA):
        S, Aa, Rn, S2, D = _host_batch(ag, j, idx[j])
        l_e, g_e, _, _, _ = _mixed_emulation(p0, t0, zero, zero.copy(), S, Aa, Rn, S2, D, 1,
                                             round_grad=False)
        ges.append(g_e)
        les.append(l_e)
    np.testing.assert_allclose(loss, np.array(les), rtol=2e-3)
    g_e = np.mean(np.stack(ges), axis=0)
    assert np.isfinite(g_g).all()
    close = np.abs(g_g - g_e) <= 2e-3 * np.abs(g_e).max() + 1e-2 * np.abs(g_e)
    assert close.mean() > 0.99, f"{np.sum(~close)} gradient entries off"
    # Keras-3 Adam (t = 1, m = v = 0) applied to exactly the kernel's gradient
    alpha, c1, c2, eps = O.keras_adam_consts(1, 1e-3)
    m = np.float32(c1) * g_g
    v = np.float32(c2) * g_g * g_g
    p1 = p0 - (m * np.float32(alpha)) / (np.sqrt(v) + np.float32(eps))
    np.testing.assert_allclose(ag.keras_params("params")[0], p1, rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(ag.keras_params("adam_m")[0], m, rtol=1e-6, atol=1e-12)


def test_shared_target_sync_and_shadow():
    ag = _shared(2, 2, freq=2)
    _fill(ag, 140, np.random.RandomState(5))
    ag.learn()
    assert not torch.equal(ag.target, ag.params)
    ag.learn()  # learn_step_counter 2: sync
    np.testing.assert_array_equal(ag.target.cpu().numpy(), ag.params.cpu().numpy())
    np.testing.assert_array_equal(ag.target_h[:, :ag.P].cpu().numpy(),
                                  ag.params.to(torch.float16).cpu().numpy())


def test_shared_greedy_act_matches_replicated_argmax():
    ag = _shared(2, 3)
    obs = torch.from_numpy(np.random.RandomState(6).randint(-1, 24, size=(2, 3, 89))
                           .astype(np.float32)).to(DEV)
    from dmdqn_amd._lib import call, ptr, stream_of
    out = torch.empty(6, dtype=torch.int32, device=DEV)
    call("dmdqn_q_argmax_shared", ptr(ag.params), 6, ag.P, ag.H, 0, ptr(obs), ptr(out), None,
         stream_of())
    rep = ag.params.expand(6, ag.P).contiguous()
    ref = torch.empty(6, dtype=torch.int32, device=DEV)
    call("dmdqn_q_argmax", ptr(rep), 6, ag.P, ag.H, 0, ptr(obs), ptr(ref), None, stream_of())
    np.testing.assert_array_equal(out.cpu().numpy(), ref.cpu().numpy())
    pk = ag.keras_params("params")[0]
    q_ref = O.qnet_forward(pk, obs.reshape(6, 89).cpu().numpy())
    np.testing.assert_array_equal(out.cpu().numpy(), q_ref.argmax(1))


def test_shared_many_agents_across_slabs():
    """More agents than persistent workgroups: each slab sums several agents."""
    ag = _shared(64, 16)  # 1024 agents over n_slabs (one per CU) workgroups
    assert ag.NA > ag.n_slabs
    _fill(ag, 130, np.random.RandomState(8))
    p0 = ag.params.clone()
    loss = ag.learn()
    assert torch.isfinite(loss).all() and torch.isfinite(ag.grad).all()
    # the mean over agents of the scaled gradient is invariant to how agents
    # are split over slabs: recompute (pre-Adam weights) with a single slab
    g1 = ag.grad.clone()
    ag.params.copy_(p0)
    ag._refresh_params_h()
    from dmdqn_amd._lib import call, ptr, stream_of
    import ctypes as C
    slab1 = torch.empty((1, ag.P), dtype=torch.float32, device=DEV)
    g_one = torch.empty(ag.P, dtype=torch.float32, device=DEV)
    a = ag.c_learn_args()  # the C ABI directly (the product path uses torch.ops.dmdqn)
    call("dmdqn_learn_shared_grad", C.byref(a), ptr(slab1), 1, ptr(g_one), C.c_float(1.0 / ag.NA),
         ptr(ag.shared_work), stream_of())
    torch.testing.assert_close(g_one, g1, rtol=1e-4, atol=1e-6 * float(g1.abs().max()))


def test_shared_fused_reduce_adam_bit_identical_to_separate_launches():
    """One rank: BatchedDQN's C5 learn reduces the slabs and steps Adam in one
    launch (dmdqn_adam_slabs).  Same inputs through dmdqn_learn_shared_grad
    (grad) + dmdqn_adam: every output bit-identical -- gradient, weights, Adam
    slots, f16 shadow and, on a sync learn, the target and its shadow."""
    from dmdqn_amd.agent import LOSSES
    outs = []
    for fused in (True, False):
        ag = _shared(3, 4, freq=2, cap=300)
        _fill(ag, 260, np.random.RandomState(11))
        for k in range(2):  # learn 2 syncs the target
            if fused:
                ag.learn()
                continue
            assert ag.learn_begin()
            alpha, c1, c2, eps, sync, qstats = ag._last_learn
            ring, cfg = ag.ring, ag.cfg
            ag._ops.learn_shared_grad(ring.s, ring.n, ring.a, ring.d, ring.r, ag.idx, ag.params,
                                      ag.target, ag.target_h, ag.params_h, ag.loss, ring.start,
                                      cfg.gamma, LOSSES[cfg.loss], qstats, ag.rn_out, ag.slab,
                                      ag.grad, 1.0 / ag.NA, work=ag.shared_work)
            ag._ops.adam(ag.params, ag.adam_m, ag.adam_v, ag.target, ag.target_h, ag.params_h,
                         ag.grad, 1.0, alpha, c1, c2, eps, sync)
        torch.cuda.synchronize()
        outs.append({n: getattr(ag, n).cpu().clone() for n in
                     ("grad", "params", "adam_m", "adam_v", "target", "target_h", "params_h",
                      "loss")})
    for n in outs[0]:
        assert torch.equal(outs[0][n], outs[1][n]), n
