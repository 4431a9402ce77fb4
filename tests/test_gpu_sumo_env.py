"""SumoTrafficEnvironment (src/agents/sumo_env.py) on the GPU: the reference's
class surface (src/agents/sumo_env.py:58-67, :420-489, :694-716) over one
replica, checked against the oracle step by step -- observation dicts
{junction_id: f32[89]} and reward dicts bit-exact (train.py's observation and
reward), `done` and info["termination_reason"]: "sumo_halted" when the network
empties (the shipped scenario under the reference's default
max_simulation_time 3600, and a synthetic demand that drains at ~60 s),
"max_time_reached" at the clock."""
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import oracle as O  # noqa: E402
from conftest import ROOT  # noqa: E402
from dmdqn_amd.env import EnvConfig  # noqa: E402
from src.agents.sumo_env import TL_PROGRAM_STATES, SumoTrafficEnvironment  # noqa: E402

NPZ = os.path.join(ROOT, "config", "scenarios", "grid_3x3_p06.npz")


def _ids(R, C):
    return [f"J_{r}_{c}" for r in range(R) for c in range(C)]


def _drive(env, ref, R, C, max_time, step_s, seed=0, max_steps=1000):
    """Random actions through env (the class) and ref (OracleEnv, train.py's
    ACTION_MAP a -> 3a) side by side; returns (steps, last info)."""
    ids = _ids(R, C)
    A = R * C
    obs = env.reset(sumo_seed="random")
    assert list(obs) == ids
    L = O.local_state(np.zeros((A, 12)), np.zeros(A), np.zeros(A), 0)
    want = O.build_obs(R, C, L)
    for j, a in zip(ids, range(A)):
        assert obs[j].dtype == np.float32 and obs[j].shape == (89,)
        np.testing.assert_array_equal(obs[j], want[a])
    rng = np.random.RandomState(seed)
    t = 0
    for step in range(max_steps):
        acts = rng.randint(0, 4, A).astype(np.int32)
        obs, rew, done, info = env.step({j: int(acts[a]) for a, j in enumerate(ids)})
        halt, ph, ts, d_ref = ref.step(acts, 3, t, step_s, max_time)
        t += step_s
        r_ref = O.reward(L)
        L = O.local_state(halt, ph, ts, 0)
        want = O.build_obs(R, C, L)
        assert list(obs) == ids and list(rew) == ids
        for a, j in enumerate(ids):
            np.testing.assert_array_equal(obs[j], want[a], err_msg=f"step {step} {j}")
            assert isinstance(rew[j], float) and rew[j] == r_ref[a], f"step {step} {j}"
        assert done == bool(d_ref), f"step {step}"
        assert info["simulation_time"] == float(t)
        if done:
            return step + 1, info, ref
        assert "termination_reason" not in info
    raise AssertionError("episode did not end")


def test_shipped_scenario_ends_sumo_halted_at_reference_defaults():
    """The shipped scenario (grid_3x3_p06: 4,167 vehicles departing until
    2,499.6 s) with the reference's default max_simulation_time 3600: the
    network empties first -> "sumo_halted" (sumo_env.py:483-484)."""
    env = SumoTrafficEnvironment(NPZ, None, [{"id": j} for j in _ids(3, 3)], step_duration=10,
                                 max_simulation_time=3600)
    assert env.get_controlled_intersection_ids() == _ids(3, 3)
    assert env.get_state_size() == 89 and env.get_action_size("J_1_1") == 4
    from dmdqn_amd.sumo_scenario import scenario_tables
    q, off, vd, _, period = scenario_tables(env.env.scenario, 1)
    ref = O.OracleEnv(3, 3, 0, period_ms=period)
    ref.set_demand(q[0], off[0], vd[0], period)
    steps, info, _ = _drive(env, ref, 3, 3, 3600, 10)
    assert info["termination_reason"] == "sumo_halted" and info["simulation_time"] < 3600
    st = env.env.stats()[0]
    assert st[0] == st[1] == 4167 and st[2] == st[3] == 0  # all arrived (no restart)


def test_synthetic_drain_and_max_time_reasons():
    cfg = EnvConfig(rows=2, cols=2, seed=9, end_ms=60_000)
    env = SumoTrafficEnvironment(None, None, [{"id": j} for j in _ids(2, 2)], step_duration=10,
                                 max_simulation_time=2400, env_config=cfg)
    ref = O.OracleEnv(2, 2, 9, end_ms=60_000)
    steps, info, _ = _drive(env, ref, 2, 2, 2400, 10)
    assert info["termination_reason"] == "sumo_halted" and info["simulation_time"] < 2400
    # demand that outlasts the clock
    env2 = SumoTrafficEnvironment(None, None, [{"id": j} for j in _ids(2, 2)], step_duration=10,
                                  max_simulation_time=50, env_config=EnvConfig(rows=2, cols=2,
                                                                               seed=4))
    ref2 = O.OracleEnv(2, 2, 4)
    steps, info, _ = _drive(env2, ref2, 2, 2, 50, 10, seed=1)
    assert steps == 5 and info["termination_reason"] == "max_time_reached"
    assert info["simulation_time"] == 50.0


def test_int_sumo_seed_reseeds_the_synthetic_demand():
    env = SumoTrafficEnvironment(None, None, [{"id": j} for j in _ids(2, 2)], step_duration=10,
                                 max_simulation_time=100,
                                 env_config=EnvConfig(rows=2, cols=2, seed=1))
    env.reset(sumo_seed=7)
    ref = O.OracleEnv(2, 2, 7)
    steps, info, _ = _drive(env, ref, 2, 2, 100, 10, seed=2)  # reset("random") keeps seed 7
    assert steps == 10 and info["termination_reason"] == "max_time_reached"


def test_action_phases_strings_and_one_second_steps():
    """action_phases as SUMO state strings (the reference's form, :507-513):
    the same phases as train.py's ACTION_MAP give the same trajectory; the
    reference's default step_duration 1.0 runs one substep per step."""
    ids = _ids(2, 2)
    phases = {a: TL_PROGRAM_STATES[3 * a] for a in range(4)}
    env = SumoTrafficEnvironment(None, None, [{"id": j, "action_phases": phases} for j in ids],
                                 max_simulation_time=30,
                                 env_config=EnvConfig(rows=2, cols=2, seed=3))
    assert env.step_duration == 1.0
    ref = O.OracleEnv(2, 2, 3)
    steps, info, _ = _drive(env, ref, 2, 2, 30, 1, seed=5)
    assert steps == 30 and info["termination_reason"] == "max_time_reached"
    with pytest.raises(ValueError):
        env.step({j: 7 for j in ids})  # no phase for action 7


def test_every_junction_must_be_controlled():
    with pytest.raises(ValueError, match="missing"):
        SumoTrafficEnvironment(None, None, [{"id": "J_0_0"}, {"id": "not_a_junction"}],
                               env_config=EnvConfig(rows=2, cols=2))
