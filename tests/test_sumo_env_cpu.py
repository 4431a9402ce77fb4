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
