"""Host-side agent logic (no GPU): parameter layout conversion, Keras Adam
constants, epsilon schedule, config keys."""
import numpy as np
import pytest
import yaml

from conftest import ROOT
from dmdqn_amd.agent import (AgentConfig, keras_adam_consts, keras_to_kernel, kernel_to_keras,
                             n_params, n_params_keras, tile_wt, untile_wt)


def test_param_counts():
    assert n_params_keras(128) == 28548  # P = 28,548 for [128,128]
    assert n_params_keras(256) == 89860
    assert n_params(128) == 28548 == n_params_keras(128) and n_params(128) % 4 == 0


def test_layout_roundtrip():
    rng = np.random.RandomState(0)
    for H in (64, 128):
        k = rng.normal(size=(3, n_params_keras(H))).astype(np.float32)
        kk = keras_to_kernel(k, H)
        assert kk.shape == (3, n_params(H))
        np.testing.assert_array_equal(kernel_to_keras(kk, H), k)
        # W1T sits at the device formula's offsets (qnet_layout.hpp qn_w1)
        W1T = np.swapaxes(k[:, :89 * H].reshape(3, 89, H), 1, 2)
        idx = np.array([[_qn_w1(o, i, H) for i in range(89)] for o in range(H)])
        np.testing.assert_array_equal(kk[:, idx], W1T)
        assert sorted(idx.ravel().tolist()) == list(range(89 * H))  # no gaps, no padding


def _qn_w1(o, i, H):  # qnet_layout.hpp qn_w1
    if i < 88:
        return (o >> 4) * 1408 + ((i >> 4) << 8) + (((i >> 3) & 1) << 7) + ((o & 15) << 3) + (i & 7)
    return 88 * H + o


def _qn_wt(o, i, K):  # qnet_layout.hpp qn_wt
    return (((o >> 4) * (K >> 4) + (i >> 4)) << 8) + (((i >> 3) & 1) << 7) + ((o & 15) << 3) + (i & 7)


def test_tiled_weight_layout_matches_device_formula():
    rng = np.random.RandomState(1)
    for N, K in ((128, 96), (128, 128), (64, 96), (64, 64)):
        W = rng.normal(size=(2, N, K)).astype(np.float32)
        t = tile_wt(W)
        idx = np.array([[_qn_wt(o, i, K) for i in range(K)] for o in range(N)])
        np.testing.assert_array_equal(t[:, idx], W)
        np.testing.assert_array_equal(untile_wt(t, N, K), W)
        # one Adam wave-instruction (lane l = lr + 16 lg owns W^T[16t + lr][16w + 4lg .. +3])
        # covers one contiguous 1 KB tile
        offs = sorted(_qn_wt(16 + (l & 15), 16 + 4 * (l >> 4) + e, K) for l in range(64) for e in range(4))
        assert offs == list(range(offs[0], offs[0] + 256))


def test_keras_adam_constants():
    a, c1, c2, eps = keras_adam_consts(1, 1e-3)
    np.testing.assert_allclose(a, 1e-3 * np.sqrt(1 - 0.999) / (1 - 0.9), rtol=1e-4)
    assert np.float32(c1) == np.float32(0.1) and np.float32(eps) == np.float32(1e-7)


def test_config_keys_match_reference_yaml():
    # config/agent_config.yaml keys stay intact
    ref = {"learning_rate", "gamma", "epsilon_start", "epsilon_min", "epsilon_decay_steps",
           "replay_buffer_size", "batch_size", "target_update_frequency", "nn_layers"}
    assert ref <= set(AgentConfig.__dataclass_fields__)
    with open(f"{ROOT}/config/agent_config.yaml") as f:
        y = yaml.safe_load(f)
    assert ref <= set(y)
    cfg = AgentConfig.from_dict(y)
    assert cfg.nn_layers == y["nn_layers"]


@pytest.mark.parametrize("spare", [1, 2, 3, 16, 64])
def test_replay_ring_spare_slot_arithmetic(spare):
    """ReplayRing keeps a deque of maxlen cap in cap + 2 slots: deque position
    p -> slot (start + p) % (cap + 2), the next stores go to the slots no
    position maps to, so the stores of steps t+1 and t+2 never touch the
    window of learn t (trainer overlap "env"), while the store of step t+3 may
    (it waits for learn t, or a later marked one)."""
    from dmdqn_amd.kernels import ReplayRing
    cap = 5
    S = cap + spare
    assert ReplayRing.SPARE == 16  # the default
    r = ReplayRing(2, cap, device="cpu", spare=spare)
    assert r.slots == S and tuple(r.a.shape) == (2, S)
    windows = []
    for t in range(40):
        window = {int(s) for s in r.slots_of(np.arange(len(r)))}
        assert len(window) == len(r) and r.next_slot not in window
        # store t: `window` is what learn t-1 reads (stores 0..t-1), windows[-b]
        # learn t-1-b's; with s spare slots none of learns t-1 .. t-s holds
        # its slot, so store t waits for none of them -- learn t-1-s's window
        # holds it once the ring is full, so store t waits for that learn
        for b in range(1, spare):
            if len(windows) >= b:
                assert r.next_slot not in windows[-b]
        if len(windows) >= spare and len(windows[-spare]) == cap:
            assert r.next_slot in windows[-spare]
        windows.append(window)
        # deque semantics: position 0 is the oldest kept transition
        if t >= cap:
            assert int(r.slots_of(0)) == (t - cap) % S
        r.advance()
    assert len(r) == cap and r.start == (40 - cap) % S


def test_bench_auto_schedule():
    """bench.py --overlap auto: C2 (1,024 independent agents, fused) runs the env
    step beside the learn on 64 CUs (or the --cu-split given), with one agent
    per side CU learned on the side stream (or the --side-learn given), at most
    half the agents (a small grid must not crash the Trainer); C5
    (shared) draws its next batches beside the learn ("learn"); C3 (16,384
    independent agents) runs the env step beside the learn on an unmasked side
    stream without side learns ("env", round 6); the unfused and split-learn
    paths stay on one stream."""
    import bench
    assert bench.auto_schedule(2, 2, 256, False, False, False, None) == ("env", 64, 64)
    assert bench.auto_schedule(2, 2, 256, False, False, False, 48) == ("env", 48, 48)
    assert bench.auto_schedule(2, 2, 256, False, False, False, None, 12) == ("env", 64, 12)
    assert bench.auto_schedule(2, 2, 16, False, False, False, None) == ("env", 64, 32)
    assert bench.auto_schedule(1, 1, 1, False, False, False, None) == ("env", 64, 0)
    assert bench.auto_schedule(4, 4, 1024, False, False, False, None) == ("env", None, 0)
    assert bench.auto_schedule(4, 4, 1024, False, True, False, None) == ("none", None, 0)
    assert bench.auto_schedule(4, 4, 1024, False, False, True, None) == ("none", None, 0)
    assert bench.auto_schedule(8, 8, 256, True, False, False, None) == ("learn", None, 0)
    assert bench.auto_schedule(8, 8, 256, True, True, False, None) == ("learn", None, 0)
    assert bench.auto_schedule(2, 2, 256, False, True, False, None) == ("none", None, 0)
    assert bench.auto_schedule(2, 2, 256, False, False, True, None) == ("none", None, 0)
    for rows, cols, envs in ((2, 2, 16), (1, 1, 3), (2, 2, 256), (1, 2, 7)):
        _, _, m = bench.auto_schedule(rows, cols, envs, False, False, False, None)
        assert 0 <= m < rows * cols * envs
