"""GPU: checkpoint / resume is bit-exact, exported weights load into the
DQNAgent surface, and the evaluation harness reproduces the oracle."""
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import oracle as O  # noqa: E402
from dmdqn_amd import checkpoint as CK  # noqa: E402
from dmdqn_amd import evaluate as EV  # noqa: E402
from dmdqn_amd.agent import AgentConfig  # noqa: E402
from dmdqn_amd.env import EnvConfig  # noqa: E402
from dmdqn_amd.trainer import Trainer  # noqa: E402


def _trainer(precision, shared=False):
    return Trainer(EnvConfig(rows=2, cols=2, num_envs=4, seed=5),
                   AgentConfig(replay_buffer_size=300, target_update_frequency=7, seed=3,
                               precision=precision, shared_params=shared))


def _run(tr, n):
    out = []
    for _ in range(n):
        st = tr.step()
        out.append((None if tr.last_loss is None else tr.last_loss.clone(),
                    tr.obs.clone(), tr.last_reward.clone()))
    torch.cuda.synchronize()
    return out


@pytest.mark.parametrize("precision,shared", [("fp32", False), ("fp16", False), ("bf16", False),
                                              ("fp16", True)])
def test_resume_is_bit_exact(tmp_path, precision, shared):
    tr = _trainer(precision, shared)
    _run(tr, 140)                       # learn active, a target sync behind us
    path = os.path.join(str(tmp_path), "ck.pt")
    CK.save(path, tr)
    a = _run(tr, 15)
    p_a = tr.agent.params.clone()
    tr2 = _trainer(precision, shared)
    CK.load(path, tr2)
    b = _run(tr2, 15)
    for (la, oa, ra), (lb, ob, rb) in zip(a, b):
        assert torch.equal(la, lb) and torch.equal(oa, ob) and torch.equal(ra, rb)
    assert torch.equal(p_a, tr2.agent.params)
    assert torch.equal(tr.agent.adam_v, tr2.agent.adam_v)
    assert torch.equal(tr.agent.py_state, tr2.agent.py_state)


def test_export_loads_into_dqnagent(tmp_path):
    tr = _trainer("fp32")
    _run(tr, 130)
    paths = CK.export_keras_weights(tr.agent, str(tmp_path), tr.env.grid.junction_ids, env_index=2)
    from src.agents.dqn_agent import DQNAgent
    ag = DQNAgent(89, 4, "J_1_0", {"nn_layers": [128, 128]})
    assert ag.load_model(paths[2])
    for x, y in zip(ag._core.get_weights(0), tr.agent.get_weights(2 * 4 + 2)):
        np.testing.assert_array_equal(x, y)


def test_random_mode_reproduces_oracle():
    """Random-mode evaluation episodes == the oracle with the same seeds; the
    action stream is test.py:92-93's: np.random.randint(0, 4) alone per agent."""
    rows = EV.run_mode(EnvConfig(rows=2, cols=2), "random", episodes=3, eval_seed_start=77,
                       max_steps=40)
    for r in rows:
        s = r["seed"]
        env, nps = O.OracleEnv(2, 2, s), O.np_stream(s)
        L = O.local_state(np.zeros((4, 12)), np.zeros(4), np.zeros(4), 0)
        tot, q, t = 0.0, 0.0, 0
        for _ in range(40):
            q += float(L[:, :12].sum())
            acts = np.array([O.np_randint(nps, 4) for _ in range(4)], np.int32)
            halt, ph, ts, _ = env.step(acts, 3, t, 10, 2400)
            t += 10
            tot += float(np.sum(O.reward(L)))
            L = O.local_state(halt, ph, ts, 0)
        assert r["steps"] == 40
        assert np.isclose(r["total_reward"], tot, rtol=1e-12)
        assert np.isclose(r["avg_step_queue_sum"], q / (40 * 4), rtol=1e-12)


def test_uniform_act_is_numpy_randint():
    """dmdqn_act_uniform: per env, agents in order, np.random.randint(0, n)
    alone (the numpy stream), for n = 4 and a non-power-of-two n = 3."""
    from dmdqn_amd import kernels as K
    seeds = [5, 6, 7]
    for n in (4, 3):
        st = K.seed_streams(seeds, "np")
        a = K.act(st, 9, n_actions=n, uniform=True)
        b = K.act(st, 9, n_actions=n, uniform=True)
        for e, s in enumerate(seeds):
            rs = np.random.RandomState(s)
            ref = [rs.randint(0, n) for _ in range(18)]
            np.testing.assert_array_equal(np.concatenate([a[e].cpu().numpy(), b[e].cpu().numpy()]),
                                          ref)


def test_evaluation_steps_per_replica_when_demand_drains():
    """Replicas whose demand drains at different times each end their own
    evaluation episode at their own `done` (test.py:75, :115-133): steps,
    total reward and queue average per replica vs the oracle run of that seed."""
    cfg = EnvConfig(rows=2, cols=2, end_ms=40_000)
    rows = EV.run_mode(cfg, "random", episodes=3, eval_seed_start=21, max_steps=200)
    lengths = set()
    for r in rows:
        s = r["seed"]
        env, nps = O.OracleEnv(2, 2, s, end_ms=40_000), O.np_stream(s)
        L = O.local_state(np.zeros((4, 12)), np.zeros(4), np.zeros(4), 0)
        tot, q, t, n, done = 0.0, 0.0, 0, 0, False
        while not done:
            q += float(L[:, :12].sum())
            acts = np.array([O.np_randint(nps, 4) for _ in range(4)], np.int32)
            halt, ph, ts, done = env.step(acts, 3, t, 10, 2400)
            t += 10
            n += 1
            tot += float(np.sum(O.reward(L)))
            L = O.local_state(halt, ph, ts, 0)
        assert r["steps"] == n < 200, (r, n)
        assert np.isclose(r["total_reward"], tot, rtol=1e-12)
        assert np.isclose(r["avg_step_queue_sum"], q / (n * 4), rtol=1e-12)
        lengths.add(n)
    assert len(lengths) > 1, "the seeds should drain at different steps"


def test_fixed_and_dqn_modes_and_cli(tmp_path):
    tr = _trainer("fp32")
    _run(tr, 130)
    ck = os.path.join(str(tmp_path), "ck.pt")
    CK.save(ck, tr, include_replay=False)
    csv = os.path.join(str(tmp_path), "eval.csv")
    from src.scripts.test import main_eval
    rows, summary = main_eval(["--checkpoint", ck, "--scenario", "synthetic", "--grid", "2x2",
                               "--modes", "dqn", "random", "fixed", "--num_eval_episodes", "3",
                               "--max_steps_per_episode", "30", "--output_csv", csv])
    assert len(rows) == 9 and os.path.exists(csv)
    assert set(summary.index) == {"dqn", "random", "fixed"}
    assert (summary["episodes"] == 3).all() and (summary["mean_steps"] == 30).all()
    fixed = [r for r in rows if r["mode"] == "fixed"]
    # deterministic policy + identical demand per seed: queues differ only by seed
    assert all(np.isfinite(r["total_reward"]) for r in rows)
    assert len({r["seed"] for r in fixed}) == 3


def test_resume_refuses_a_different_configuration(tmp_path):
    """checkpoint.load validates every config field that fixes the state's
    layout or meaning: precision, replay size, loss, grid, seeds,
    actuated mode, replay row format ... and refuses a replay-less checkpoint of a filled ring."""
    tr = _trainer("fp16")
    _run(tr, 130)
    path = os.path.join(str(tmp_path), "ck.pt")
    CK.save(path, tr)
    bad = [
        (EnvConfig(rows=2, cols=2, num_envs=4, seed=5), dict(precision="bf16"), "precision"),
        (EnvConfig(rows=2, cols=2, num_envs=4, seed=5), dict(precision="fp32"), "precision"),
        (EnvConfig(rows=2, cols=2, num_envs=4, seed=5), dict(precision="fp16",
                                                               replay_buffer_size=400),
         "replay_buffer_size"),
        (EnvConfig(rows=2, cols=2, num_envs=4, seed=5), dict(precision="fp16", loss="huber"),
         "loss"),
        (EnvConfig(rows=2, cols=2, num_envs=4, seed=6), dict(precision="fp16"), "seed"),
        (EnvConfig(rows=2, cols=2, num_envs=4, seed=5, actuated=True), dict(precision="fp16"),
         "actuated"),
        (EnvConfig(rows=2, cols=2, num_envs=4, seed=5), dict(precision="fp16", replay_rows="f32"),
         "replay_rows"),
    ]
    for env_cfg, agent_kw, field in bad:
        kw = dict(replay_buffer_size=300, target_update_frequency=7, seed=3)
        kw.update(agent_kw)
        tr2 = Trainer(env_cfg, AgentConfig(**kw))
        with pytest.raises(ValueError, match=field):
            CK.load(path, tr2)
    # a checkpoint saved without its replay cannot resume a filled ring
    p2 = os.path.join(str(tmp_path), "noreplay.pt")
    CK.save(p2, tr, include_replay=False)
    with pytest.raises(ValueError, match="without its replay"):
        CK.load(p2, _trainer("fp16"))
    # and the 16-bit target shadow follows the restored target (not the fresh init)
    tr3 = _trainer("fp16")
    CK.load(path, tr3)
    assert torch.equal(tr3.agent.target_h[:, :tr3.agent.P],
                       tr3.agent.target.to(tr3.agent.target_h.dtype))


def test_resume_mismatch_leaves_trainer_untouched(tmp_path):
    """A checkpoint whose LAST tensor does not fit is refused before anything is
    copied: the Trainer keeps its own weights, rings and env."""
    tr = _trainer("fp16")
    _run(tr, 130)
    st = CK.trainer_state(tr)
    st["replay"]["d"] = st["replay"]["d"][:1]  # the last tensor checked
    path = os.path.join(str(tmp_path), "bad.pt")
    torch.save(st, path)
    tr2 = _trainer("fp16")
    _run(tr2, 3)
    before = [t.clone() for t in (tr2.agent.params, tr2.agent.adam_m, tr2.env.t_x,
                                  tr2.agent.ring.s, tr2.agent.np_state)]
    with pytest.raises(ValueError, match="replay.d"):
        CK.load(path, tr2)
    after = (tr2.agent.params, tr2.agent.adam_m, tr2.env.t_x, tr2.agent.ring.s,
             tr2.agent.np_state)
    assert all(torch.equal(a, b) for a, b in zip(before, after))


def test_restore_into_running_side_learn_trainer(tmp_path):
    """under the "env" schedule with side_learn the last
    step's side-stream learn (agents [NA - side_learn, NA)) is waited for
    lazily.  checkpoint.load() into a trainer that is still running it orders
    its copies after that learn (Trainer.quiesce), so the restored weights and
    Adam slots of the side agents are not overwritten by it: the restored run
    continues bit-identically to the run the checkpoint was taken from."""
    def make():
        return Trainer(EnvConfig(rows=2, cols=2, num_envs=8, seed=5),
                       AgentConfig(replay_buffer_size=300, target_update_frequency=7, seed=3,
                                   precision="fp16"), overlap="env", side_learn=8)
    tr = make()
    _run(tr, 140)
    path = os.path.join(str(tmp_path), "ck.pt")
    CK.save(path, tr)
    a = _run(tr, 15)
    tr2 = make()
    for _ in range(150):  # a different history, then restore with its last side learn in flight
        tr2.step()
    CK.load(path, tr2)
    b = _run(tr2, 15)
    for (la, oa, ra), (lb, ob, rb) in zip(a, b):
        assert torch.equal(la, lb) and torch.equal(oa, ob) and torch.equal(ra, rb)
    tr.sync_outputs()
    tr2.sync_outputs()
    torch.cuda.synchronize()
    side = slice(tr.agent.NA - 8, tr.agent.NA)
    for k in ("params", "adam_m", "adam_v", "target"):
        assert torch.equal(getattr(tr.agent, k)[side], getattr(tr2.agent, k)[side]), k
        assert torch.equal(getattr(tr.agent, k), getattr(tr2.agent, k)), k
