"""Evaluation harness and checkpoint helpers that need no GPU."""
import numpy as np

from dmdqn_amd.agent import keras_initial_weights, n_params_keras
from dmdqn_amd.checkpoint import export_keras_weights, load_keras_weights
from dmdqn_amd.evaluate import FIXED_CYCLE, _policy_weights, fixed_cycle_actions


def test_fixed_cycle_matches_reference_state_machine():
    # test.py:93-107: advance when time_in_phase >= duration, then add step_duration
    assert FIXED_CYCLE == ((0, 30.0), (2, 30.0))
    assert fixed_cycle_actions(10, 10) == [0, 0, 0, 2, 2, 2, 0, 0, 0, 2]
    assert fixed_cycle_actions(4, 20) == [0, 0, 2, 2]


def test_policy_weights_replicate_per_junction_nets():
    P = n_params_keras(64)
    w = np.arange(3 * P, dtype=np.float32).reshape(3, P)
    out = _policy_weights(w, 3, 2)
    assert out.shape == (6, P) and (out[3:] == w).all()
    one = _policy_weights(w[:1], 3, 2)
    assert (one == w[0]).all()


class _FakeAgent:
    def __init__(self, H=64, n=4):
        self.w = keras_initial_weights(np.random.RandomState(0), H, n)
        self.H = H

    def get_weights(self, i):
        H, p, out, o = self.H, self.w[i], [], 0
        for sh in [(89, H), (H,), (H, H), (H,), (H, 4), (4,)]:
            k = int(np.prod(sh))
            out.append(p[o:o + k].reshape(sh))
            o += k
        return out


def test_export_keras_weights_naming_and_roundtrip(tmp_path):
    ag = _FakeAgent()
    paths = export_keras_weights(ag, str(tmp_path), ["J_0_0", "J_0_1"], env_index=1)
    assert [p.rsplit("/", 1)[1] for p in paths] == ["agent_J_0_0.weights.npz",
                                                    "agent_J_0_1.weights.npz"]
    back = load_keras_weights(paths[1])
    for a, b in zip(back, ag.get_weights(3)):   # env 1, junction 1 -> agent 3
        np.testing.assert_array_equal(a, b)
