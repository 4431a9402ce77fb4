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
from src.agents.sumo_env import (TL_PROGRAM_STATES, TRAIN_PY_ACTION_PHASES,  # noqa: E402
                                  SumoTrafficEnvironment)

NPZ = os.path.join(ROOT, "config", "scenarios", "grid_3x3_p06.npz")


def _ids(R, C):
    return [f"J_{r}_{c}" for r in range(R) for c in range(C)]


def _drive(env, ref, R, C, max_time, step_s, seed=0, max_steps=1000, phase_of=None,
           controlled=None, n_actions=4, seen=None):
    """Random actions 0..n_actions-1 through env (the class) and ref (OracleEnv)
    side by side; returns (steps, last info, ref).  The oracle gets the
    reference class's _apply_actions (sumo_env.py:491-530) restated here:
    phase_of[a] (train.py's ACTION_MAP a -> 3a by default; None = unmapped)
    for the controlled junctions, no setPhase (-1) for an unmapped action, a
    junction already in that phase, or a junction that is not controlled.
    seen: a set that collects every (junction, phase) the program showed."""
    ids = _ids(R, C)
    ctl = ids if controlled is None else controlled
    col = [ids.index(j) for j in ctl]
    phase_of = {a: 3 * a for a in range(4)} if phase_of is None else phase_of
    A = R * C
    obs = env.reset(sumo_seed="random")
    assert list(obs) == ctl
    L = O.local_state(np.zeros((A, 12)), np.zeros(A), np.zeros(A), 0)
    want = O.build_obs(R, C, L)
    for j, a in zip(ctl, col):
        assert obs[j].dtype == np.float32 and obs[j].shape == (89,)
        np.testing.assert_array_equal(obs[j], want[a])
    rng = np.random.RandomState(seed)
    t = 0
    cur = np.zeros(A, np.int32)
    for step in range(max_steps):
        acts = rng.randint(0, n_actions, A).astype(np.int32)
        obs, rew, done, info = env.step({j: int(acts[a]) for j, a in zip(ctl, col)})
        req = np.full(A, -1, np.int32)
        for a in col:
            p = phase_of.get(int(acts[a]))
            if p is not None and p != cur[a]:
                req[a] = p
        halt, ph, ts, d_ref = ref.step(req, 1, t, step_s, max_time)
        cur = np.asarray(ph, np.int32).copy()
        if seen is not None:
            seen.update((a, int(cur[a])) for a in range(A))
        t += step_s
        r_ref = O.reward(L)
        L = O.local_state(halt, ph, ts, 0)
        want = O.build_obs(R, C, L)
        assert list(obs) == ctl and list(rew) == ctl
        for j, a in zip(ctl, col):
            np.testing.assert_array_equal(obs[j], want[a], err_msg=f"step {step} {j}")
            assert isinstance(rew[j], float) and rew[j] == r_ref[a], f"step {step} {j}"
        assert done == bool(d_ref), f"step {step}"
        assert info["simulation_time"] == float(t)
        if done:
            return step + 1, info, ref
        assert "termination_reason" not in info
    raise AssertionError("episode did not end")


def _ctl(ids, phases=TRAIN_PY_ACTION_PHASES):
    return [{"id": j, "action_phases": phases} for j in ids]


def test_shipped_scenario_ends_sumo_halted_at_reference_defaults():
    """The shipped scenario (grid_3x3_p06: 4,167 vehicles departing until
    2,499.6 s) with the reference's default max_simulation_time 3600: the
    network empties first -> "sumo_halted" (sumo_env.py:483-484)."""
    env = SumoTrafficEnvironment(NPZ, None, _ctl(_ids(3, 3)), step_duration=10,
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
    env = SumoTrafficEnvironment(None, None, _ctl(_ids(2, 2)), step_duration=10,
                                 max_simulation_time=2400, env_config=cfg)
    ref = O.OracleEnv(2, 2, 9, end_ms=60_000)
    steps, info, _ = _drive(env, ref, 2, 2, 2400, 10)
    assert info["termination_reason"] == "sumo_halted" and info["simulation_time"] < 2400
    # demand that outlasts the clock
    env2 = SumoTrafficEnvironment(None, None, _ctl(_ids(2, 2)), step_duration=10,
                                  max_simulation_time=50, env_config=EnvConfig(rows=2, cols=2,
                                                                               seed=4))
    ref2 = O.OracleEnv(2, 2, 4)
    steps, info, _ = _drive(env2, ref2, 2, 2, 50, 10, seed=1)
    assert steps == 5 and info["termination_reason"] == "max_time_reached"
    assert info["simulation_time"] == 50.0


def test_int_sumo_seed_reseeds_the_synthetic_demand():
    env = SumoTrafficEnvironment(None, None, _ctl(_ids(2, 2)), step_duration=10,
                                 max_simulation_time=100,
                                 env_config=EnvConfig(rows=2, cols=2, seed=1))
    env.reset(sumo_seed=7)
    ref = O.OracleEnv(2, 2, 7)
    steps, info, _ = _drive(env, ref, 2, 2, 100, 10, seed=2)  # reset("random") keeps seed 7
    assert steps == 10 and info["termination_reason"] == "max_time_reached"


def test_action_phases_indices_and_one_second_steps():
    """action_phases as phase indices (the build's extension) select the same
    phases as the reference's state strings; the reference's default
    step_duration 1.0 runs one substep per step; an action outside the map is
    skipped (no setPhase), not an error (:498-501)."""
    ids = _ids(2, 2)
    env = SumoTrafficEnvironment(None, None, _ctl(ids, {a: 3 * a for a in range(4)}),
                                 max_simulation_time=30,
                                 env_config=EnvConfig(rows=2, cols=2, seed=3))
    assert env.step_duration == 1.0 and env.get_action_size() == 4
    ref = O.OracleEnv(2, 2, 3)
    steps, info, _ = _drive(env, ref, 2, 2, 30, 1, seed=5)
    assert steps == 30 and info["termination_reason"] == "max_time_reached"


def test_unmapped_and_unchanged_actions_let_the_program_run():
    """VERDICT r4 item 7 (sumo_env.py:491-530): with two of four actions
    mapped, and setPhase skipped when the junction is already in the phase,
    the signal program runs on -- its yellow / all-red phases appear, which
    train.py's setPhase-every-step never shows -- bit-exact vs the oracle
    given the same requests, over 400 one-second steps."""
    ids = _ids(2, 2)
    phases = {0: TL_PROGRAM_STATES[0], 1: TL_PROGRAM_STATES[6]}
    env = SumoTrafficEnvironment(None, None, _ctl(ids, phases), max_simulation_time=400,
                                 env_config=EnvConfig(rows=2, cols=2, seed=6))
    assert env.get_action_size("J_0_1") == 2
    steps, info, _ = _drive(env, O.OracleEnv(2, 2, 6), 2, 2, 400, 1, seed=7,
                            phase_of={0: 0, 1: 6})
    assert steps == 400
    # always action 0: phase 0 is requested while it runs (no setPhase), so
    # the program moves on to its yellow phase 1 after 25 s, then the next
    # request sets phase 0 again
    env2 = SumoTrafficEnvironment(None, None, _ctl(ids, phases), max_simulation_time=100,
                                  env_config=EnvConfig(rows=2, cols=2, seed=6))
    seen = set()
    steps, info, _ = _drive(env2, O.OracleEnv(2, 2, 6), 2, 2, 100, 1, seed=7,
                            phase_of={0: 0, 1: 6}, seen=seen, n_actions=1)
    assert steps == 100 and {p for _, p in seen} == {0, 1}, seen


def test_subset_of_junctions_controlled():
    """controlled_intersections naming two of a 2x2 grid's four junctions
    (and one id that is no junction, dropped as :116-123): the dicts hold
    those two; the other two signals run their programs untouched."""
    ids = _ids(2, 2)
    ctl = ["J_1_0", "J_0_1"]
    env = SumoTrafficEnvironment(None, None, _ctl(ctl + ["nope"]), step_duration=5,
                                 max_simulation_time=300,
                                 env_config=EnvConfig(rows=2, cols=2, seed=8))
    assert env.get_controlled_intersection_ids() == ctl
    seen = set()
    steps, info, _ = _drive(env, O.OracleEnv(2, 2, 8), 2, 2, 300, 5, seed=9, controlled=ctl,
                            seen=seen)
    assert steps == 60
    assert {p for a, p in seen if ids[a] not in ctl} >= {0, 1, 2, 3}  # the free-running program


def test_no_action_phases_means_no_actions():
    """Without "action_phases" a junction's map is empty (:113-117):
    get_action_size() is 0 and every action is skipped -- the programs run
    as if nothing were controlled; an unknown phase string is skipped with
    the reference's warning."""
    ids = _ids(2, 2)
    env = SumoTrafficEnvironment(None, None, [{"id": j} for j in ids], step_duration=10,
                                 max_simulation_time=200,
                                 env_config=EnvConfig(rows=2, cols=2, seed=10))
    assert env.get_action_size() == 0 and env.get_action_size("J_1_1") == 0
    steps, info, _ = _drive(env, O.OracleEnv(2, 2, 10), 2, 2, 200, 10, seed=11, phase_of={})
    assert steps == 20
    bad = SumoTrafficEnvironment(None, None, _ctl(ids, {0: "G" * 24}), step_duration=10,
                                 max_simulation_time=50,
                                 env_config=EnvConfig(rows=2, cols=2, seed=10))
    assert bad.get_action_size() == 1
    steps, info, _ = _drive(bad, O.OracleEnv(2, 2, 10), 2, 2, 50, 10, seed=11, phase_of={},
                            n_actions=1)
    assert steps == 5


def test_ids_that_are_not_junctions_are_dropped():
    with pytest.raises(ValueError, match="None of the provided"):
        SumoTrafficEnvironment(None, None, [{"id": "not_a_junction"}],
                               env_config=EnvConfig(rows=2, cols=2))
