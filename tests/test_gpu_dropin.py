"""Drop-in surfaces on the GPU: per-agent DQNAgent draw order vs the oracle
streams, the reference-shaped train loop, and __graft_entry__.smoke()."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import oracle as O  # noqa: E402


def test_dqnagent_draw_order_matches_global_streams():
    from src.agents import dqn_agent
    from src.env.traffic_env import EnvConfig, TrafficEnv
    dqn_agent.seed(1234)
    env = TrafficEnv(EnvConfig(rows=2, cols=2, num_envs=1, seed=3))
    ids = env.get_controlled_intersection_ids()
    cfg = {"nn_layers": [128, 128], "batch_size": 128, "replay_buffer_size": 500}
    agents = {j: dqn_agent.DQNAgent(89, 4, j, cfg) for j in ids}
    nps, pys = O.np_stream(1234), O.py_stream(1234)
    state = env.reset_dict()
    for step in range(130):
        acts = {j: agents[j].select_action(state[j][None]) for j in ids}
        np.testing.assert_array_equal([acts[j] for j in ids], O.act(nps, 4, 1.0))
        nstate, rew, done, _ = env.step_dict(acts)
        for j in ids:
            agents[j].remember(state[j][None], acts[j], rew[j], nstate[j][None], done)
            loss = agents[j].replay()
            if step < 127:
                assert loss == 0
            else:
                n = len(agents[j].replay_buffer)
                exp = O.py_sample(pys, n, 128)
                np.testing.assert_array_equal(agents[j]._core.idx.cpu().numpy()[0], exp)
                assert loss > 0
        state = nstate
    b = agents[ids[0]].replay_buffer.sample(128)
    assert b[0].shape == (128, 89) and b[2].dtype == torch.float32


def test_train_loop_one_episode(tmp_path):
    from src.scripts import train
    m = tmp_path / "m.jsonl"
    agents = train.train_agents(episodes=1, rows=2, cols=2, seed=0, metrics=str(m))
    assert all(a.learn_step_counter == 240 - 127 for a in agents.values())
    lines = m.read_text().strip().splitlines()
    assert len(lines) == 240


def test_graft_smoke():
    import __graft_entry__
    __graft_entry__.smoke()


@pytest.mark.parametrize("precision,rtol", [("fp32", 1e-4), ("fp16", 2e-2), ("bf16", 5e-2)])
def test_learn_metrics_match_host(precision, rtol):
    """qstats (dqn_agent.py:361-363) vs the host: action histogram exact, Q
    moments of the online net on the sampled S within the precision's tolerance."""
    import oracle as O
    from dmdqn_amd.agent import AgentConfig, BatchedDQN
    from test_gpu_learn import _fill, _host_batch
    ag = BatchedDQN(2, 3, AgentConfig(replay_buffer_size=300, seed=2, precision=precision))
    _fill(ag, 150, np.random.RandomState(3))
    p0 = ag.keras_params("params").copy()
    ag.learn(collect_stats=True)
    qs = ag.qstats.cpu().numpy()
    idx = ag.idx.cpu().numpy()
    for j in range(ag.NA):
        S, Aa, _, _, _ = _host_batch(ag, j, idx[j])
        q = O.qnet_forward(p0[j], S)
        np.testing.assert_array_equal(qs[j, 2:], np.bincount(Aa, minlength=4))
        np.testing.assert_allclose(qs[j, 0], q.sum(), rtol=rtol, atol=rtol * np.abs(q).sum())
        np.testing.assert_allclose(qs[j, 1], (q * q).sum(), rtol=5 * rtol)
    m = ag.learn_metrics()
    assert sum(m["action_distribution"]) == ag.NA * 128 and m["epsilon"] == 1.0


def test_train_batched_metrics_and_save(tmp_path):
    import json
    from src.scripts import train
    mfile, sdir = tmp_path / "m.jsonl", tmp_path / "save"
    tr = train.train_batched(1, 2, 2, 8, "fp16", 1, metrics=str(mfile), save_dir=str(sdir),
                             log_every=20)
    recs = [json.loads(x) for x in mfile.read_text().strip().splitlines()]
    assert len(recs) == 12 and recs[0]["step"] == 1
    learned = [r for r in recs if "q_values_mean" in r]
    assert len(learned) == 5                                  # 0-based steps 140, 160, ..., 220
    assert all(sum(r["action_distribution"]) == 8 * 4 * 128 for r in learned)
    assert all(r["global_reward"] <= 0 for r in recs)
    assert (sdir / "checkpoint.pt").exists() and (sdir / "agent_J_1_1.weights.npz").exists()
    assert tr.episode == 1


def test_dropin_learn_writes_the_reference_summaries(tmp_path):
    """DQNAgent.learn records the scalars the reference logs per learn
    (dqn_agent.py:361-370: loss, epsilon, Q mean / std of the batch's online Q
    values, the sampled action histogram), in last_summary and, with
    "summary_dir", as JSON lines under <dir>/<agent_id>/; the Q moments match
    the host forward of the pre-learn weights on the sampled rows."""
    import json
    from src.agents import dqn_agent
    dqn_agent.seed(7)
    cfg = {"nn_layers": [128, 128], "batch_size": 128, "replay_buffer_size": 300,
           "summary_dir": str(tmp_path)}
    ag = dqn_agent.DQNAgent(89, 4, "J1", cfg)
    rs = np.random.RandomState(5)
    for _ in range(140):
        s, n = rs.randint(-1, 20, 89).astype(np.float32), rs.randint(-1, 20, 89).astype(np.float32)
        ag.remember(s, int(rs.randint(4)), float(-rs.rand() * 50), n, False)
    assert ag.learn() is not None
    p0 = ag._core.keras_params("params").copy()
    loss = ag.learn()
    rec = ag.last_summary
    assert rec["step"] == 2 and rec["loss"] == loss and rec["epsilon"] == ag.epsilon
    idx = ag._core.idx.cpu().numpy()[0]
    slots = ag.replay_buffer.ring.slots_of(idx)
    S = ag.replay_buffer.ring.s[0, slots, :89].cpu().numpy()
    A = ag.replay_buffer.ring.a[0, slots].cpu().numpy()
    assert rec["action_distribution"] == np.bincount(A, minlength=4).tolist()
    q = O.qnet_forward(p0[0], S)
    np.testing.assert_allclose(rec["q_values_mean"], q.mean(), rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(rec["q_values_std"], q.std(), rtol=1e-3)
    lines = (tmp_path / "J1" / "summaries.jsonl").read_text().strip().splitlines()
    assert [json.loads(x)["step"] for x in lines] == [1, 2]
