"""The SumoTrafficEnvironment surface (src/agents/sumo_env.py, the reference's
src/agents/sumo_env.py:48-716): argument checks that run before any device
allocation, and the phase-string map of _apply_actions (sumo_env.py:507-513).
The GPU behaviour is in tests/test_gpu_sumo_env.py."""
import os

import pytest

from conftest import GOLDEN, ROOT
from src.agents import sumo_env as S

NPZ = os.path.join(ROOT, "config", "scenarios", "grid_3x3_p06.npz")
ALL = [{"id": f"J_{r}_{c}"} for r in range(3) for c in range(3)]


def test_phase_strings_map_to_the_first_matching_phase():
    assert [S._phase_index(p) for p in S.TL_PROGRAM_STATES[:4]] == [0, 1, 2, 3]
    # yellow / all-red strings repeat in the program: the first match wins
    assert S._phase_index("yyyyyyyyyyyyyyyyyyyyyyyy") == 1
    assert S._phase_index("rrrrrrrrrrrrrrrrrrrrrrrr") == 2
    assert S._phase_index(9) == 9
    # a string the program does not have: the reference warns and skips (:519-523)
    assert S._phase_index("GGGGGGGGGGGGGGGGGGGGGGGG") == S.NO_SET_PHASE
    with pytest.raises(ValueError):
        S._phase_index(12)
    assert [S._phase_index(p) for p in S.TRAIN_PY_ACTION_PHASES.values()] == [0, 3, 6, 9]


@pytest.mark.parametrize("kw,exc", [
    ({"net_file_path": "/nonexistent.net.xml"}, FileNotFoundError),
    ({"sumo_cfg_path": "/nonexistent.sumocfg"}, FileNotFoundError),
    ({"controlled_intersections": []}, ValueError),
    ({"padding_value": 0.0}, ValueError),
    ({"max_lanes_per_direction": 4}, ValueError),
    ({"step_duration": 1.5}, ValueError),
    ({"sumo_cfg_path": None}, ValueError),
])
def test_constructor_rejects_bad_arguments(kw, exc):
    args = {"sumo_cfg_path": NPZ, "net_file_path": None, "controlled_intersections": ALL}
    args.update(kw)
    with pytest.raises(exc):
        S.SumoTrafficEnvironment(**args)


def test_reference_defaults_and_signature():
    import inspect
    sig = inspect.signature(S.SumoTrafficEnvironment.__init__)
    names = list(sig.parameters)[1:8]
    assert names == ["sumo_cfg_path", "net_file_path", "controlled_intersections",
                     "max_lanes_per_direction", "step_duration", "max_simulation_time",
                     "padding_value"]
    d = {k: v.default for k, v in sig.parameters.items()}
    assert (d["max_lanes_per_direction"], d["step_duration"], d["max_simulation_time"],
            d["padding_value"]) == (3, 1.0, 3600, -1.0)
    r = inspect.signature(S.SumoTrafficEnvironment.reset).parameters
    assert r["sumo_seed"].default == "random" and r["use_gui"].default is False
    assert os.path.exists(GOLDEN)


def _bare_env(phases, controlled, current):
    """A SumoTrafficEnvironment shell (no device) for the host-side action
    mapping: ids of a 2x2 grid, `controlled` with their action_phases, the
    simulator's current phase per signal."""
    import torch
    from types import SimpleNamespace
    env = S.SumoTrafficEnvironment.__new__(S.SumoTrafficEnvironment)
    ids = [f"J_{r}_{c}" for r in range(2) for c in range(2)]
    env.env = SimpleNamespace(A=4, phase=torch.tensor([current], dtype=torch.int32))
    env.traffic_light_ids = {j: j for j in controlled}
    env.action_to_sumo_phase = {j: phases for j in controlled}
    env._phase_of = {j: {a: S._phase_index(p) for a, p in phases.items() if isinstance(p, int) or p}
                     for j in controlled}
    env._signal = {j: ids.index(j) for j in controlled}
    return env


def test_apply_actions_follows_the_reference_rules(capsys):
    """sumo_env.py:491-530 on the host: an unknown id, an unmapped action and a
    string the program lacks are skipped (the last with the reference's
    warning); setPhase is skipped when the signal is already in the phase;
    signals without an action keep their program (-1 = no setPhase)."""
    P = S.TL_PROGRAM_STATES
    phases = {0: P[0], 1: P[6], 2: "G" * 24, 3: ""}
    env = _bare_env(phases, ["J_0_0", "J_0_1", "J_1_0"], current=[0, 3, 6, 9])
    ph = env._apply_actions({"J_0_0": 0,      # already in phase 0: skipped
                             "J_0_1": 1,      # phase 6
                             "J_1_0": 2,      # string not in the program: warning, skipped
                             "J_1_1": 1,      # not controlled: skipped
                             "nope": 0})
    assert ph.tolist() == [[-1, 6, -1, -1]]
    assert "not found for TL J_1_0" in capsys.readouterr().out
    ph = env._apply_actions({"J_0_0": 3, "J_0_1": 7, "J_1_0": 0})  # "" and unmapped: skipped
    assert ph.tolist() == [[-1, -1, 0, -1]]
    assert env._apply_actions({"J_1_0": 1}).tolist() == [[-1, -1, -1, -1]]  # 6 already runs
    assert S._phase_index(P[6]) == 6 and S.NO_SET_PHASE == -1
