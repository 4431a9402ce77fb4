"""GPU parity of the HIP microsimulation + observe vs the C oracle (bit-exact),
through the C ABI (TrafficEnv -> dmdqn_sim_step / dmdqn_observe)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import oracle as O  # noqa: E402
from dmdqn_amd import _lib  # noqa: E402
from dmdqn_amd.env import EnvConfig, TrafficEnv  # noqa: E402


def _run(R, C, E, steps, mode="reference", seed=100, check_every=1, full_state_at=(),
         scenario=None, actuated=False, action_fn=None, path_at=None, period_ms=None):
    """Step E replicas through the HIP sim and the oracle side by side.
    action_fn(step, rng) -> [E, A] actions (default: uniform random);
    path_at {step: "reg" | "lds" | "global"} forces the sim path
    (_lib.set_option "sim_path") before that step."""
    import os
    max_cnt = 0
    cfg = EnvConfig(rows=R, cols=C, num_envs=E, seed=seed, signal_features=mode,
                    scenario=scenario, actuated=actuated, period_ms=period_ms)
    env = TrafficEnv(cfg)
    R, C = env.R, env.C
    obs = env.reset()
    refs = [O.OracleEnv(R, C, seed + e, period_ms=period_ms or 0, actuated=actuated)
            for e in range(E)]
    if scenario is not None:
        from dmdqn_amd.sumo_scenario import scenario_tables
        q, off, vd, _, period = scenario_tables(env.scenario, 1)
        for r in refs:
            r.set_demand(q[0], off[0], vd[0], period)
    m = 1 if mode == "intended" else 0
    A = R * C
    prev_local = [O.local_state(np.zeros((A, 12)), np.zeros(A), np.zeros(A), m) for _ in range(E)]
    np.testing.assert_array_equal(obs.cpu().numpy()[0], O.build_obs(R, C, prev_local[0]))
    rng = np.random.RandomState(seed)
    t = 0
    for step in range(steps):
        if path_at and step in path_at:
            _lib.set_option("sim_path", path_at[step])
        acts = (action_fn(step, rng) if action_fn else
                rng.randint(0, 4, size=(E, A))).astype(np.int32)
        obs, rew, done, info = env.step(torch.from_numpy(acts).cuda())
        max_cnt = max(max_cnt, int(env.t_cnt.max()))
        if step % check_every and step not in full_state_at and step != steps - 1:
            for e in range(E):
                halt, ph, ts, _ = refs[e].step(acts[e], 3, t, 10, 2400)
                prev_local[e] = O.local_state(halt, ph, ts, m)
            t += 10
            continue
        halt_g = env.halt.cpu().numpy()
        ph_g, ts_g = env.phase.cpu().numpy(), env.tspent.cpu().numpy()
        obs_g, rew_g = obs.cpu().numpy(), rew.cpu().numpy()
        done_g = info["done_flags"].cpu().numpy()
        for e in range(E):
            halt, ph, ts, dn = refs[e].step(acts[e], 3, t, 10, 2400)
            np.testing.assert_array_equal(halt_g[e], halt, err_msg=f"halt env {e} step {step}")
            np.testing.assert_array_equal(ph_g[e], ph)
            np.testing.assert_array_equal(ts_g[e], ts)
            assert bool(done_g[e]) == dn
            L = O.local_state(halt, ph, ts, m)
            np.testing.assert_array_equal(obs_g[e], O.build_obs(R, C, L))
            np.testing.assert_array_equal(rew_g[e], O.reward(prev_local[e]))
            prev_local[e] = L
        t += 10
        if step in full_state_at or step == steps - 1:
            X = env.t_x.cpu().numpy()
            Vv = env.t_v.cpu().numpy()
            D = env.t_dst.cpu().numpy()
            H = env.t_head.cpu().numpy()
            N = env.t_cnt.cpu().numpy()
            for e in range(E):
                # each lane's vehicles front to back (the register path keeps its
                # rings compacted, head 0; the oracle rotates its head)
                x, v, d, hd, cn = refs[e].lanes()
                np.testing.assert_array_equal(N[e], cn)
                cap = refs[e].cap
                for l in np.nonzero(cn)[0]:
                    mine = [(H[e, l] + i) % cap for i in range(cn[l])]
                    ref = [(hd[l] + i) % cap for i in range(cn[l])]
                    np.testing.assert_array_equal(X[e, l, mine], x[l, ref], err_msg=f"x lane {l}")
                    np.testing.assert_array_equal(Vv[e, l, mine], v[l, ref])
                    np.testing.assert_array_equal(D[e, l, mine], d[l, ref])
            st = env.stats()
            for e in range(E):
                np.testing.assert_array_equal(st[e], refs[e].info()[4:8])
    env.max_cnt_seen = max_cnt
    return env


@pytest.mark.parametrize("grid", [(1, 1), (2, 2), (3, 3), (4, 4), (2, 3)])
def test_sim_matches_oracle(grid):
    R, C = grid
    _run(R, C, E=6, steps=80, full_state_at=(10, 40))


def test_sim_8x8_matches_oracle():
    _run(8, 8, E=3, steps=40, check_every=5, full_state_at=(20,))


def test_sim_intended_mode_full_episode_and_reset():
    env = _run(2, 2, E=4, steps=240, mode="intended", check_every=20)
    assert env.t == 2400
    obs = env.reset()
    assert env.t == 0 and float(obs[:, :, :12].abs().sum()) == 0.0
    assert (env.stats() == 0).all()


def test_dict_api_single_replica():
    env = TrafficEnv(EnvConfig(rows=3, cols=3, num_envs=1, seed=7))
    obs = env.reset_dict()
    assert list(obs) == [f"J_{r}_{c}" for r in range(3) for c in range(3)]
    assert all(o.shape == (89,) and o.dtype == np.float32 for o in obs.values())
    nobs, rew, done, info = env.step_dict({j: 1 for j in obs})
    assert set(rew) == set(obs) and not done and info["simulation_time"] == 10.0
    assert env.get_state_size() == 89 and env.get_action_size() == 4


def test_sim_shipped_3x3_scenario_matches_oracle():
    """The reference's own scenario (grid_3x3.net.xml + grid_3x3_p06.rou.xml,
    4167 routed vehicles, derived by tests/golden/make_scenario.py) through
    the HIP sim: a full 240-step episode, bit-exact vs the oracle."""
    from conftest import GOLDEN
    import os
    env = _run(0, 0, E=3, steps=240, check_every=10, full_state_at=(100, 200),
               scenario=os.path.join(GOLDEN, "grid_3x3_p06_scenario.npz"))
    st = env.stats()  # inserted, arrived, running, pending
    assert (st[:, 0] > 3900).all() and (st[:, 1] > 3500).all()
    assert (st[:, 0] + st[:, 3] == 4167).all()


@pytest.mark.parametrize("grid", [(2, 2), (4, 4)])
def test_sim_actuated_gap_out_matches_oracle(grid):
    """SUMO's actuated phase 0 (A-14, EnvConfig.actuated): bit-exact vs the
    oracle over 120 steps, detector times included; gap-outs do happen."""
    env = _run(*grid, E=4, steps=120, actuated=True, check_every=7, full_state_at=(60,))
    ld = env.t_last_det.cpu().numpy()
    assert (ld > 0).any()


def test_sim_actuated_shipped_scenario():
    from conftest import GOLDEN
    import os
    _run(0, 0, E=2, steps=240, check_every=20, actuated=True,
         scenario=os.path.join(GOLDEN, "grid_3x3_p06_scenario.npz"))


def test_lds_image_long_queues_and_path_switches(lib_option):
    """The LDS image keeps each lane's first 12 positions in LDS and the rest
    in HBM, lanes compacted.  Heavy demand with the signals held (phase 0 only:
    the E-W approaches queue to capacity) drives lanes past 12 vehicles; the
    path changes mid-episode (global rings with a rotated head -> LDS image,
    which compacts them -> register lanes -> LDS image), bit-exact vs the
    oracle throughout."""
    lib_option("sim_path", "global")  # restored after the test (path_at switches it)
    hold = lambda step, rng: np.zeros((3, 16))  # noqa: E731
    env = _run(4, 4, E=3, steps=90, check_every=5, full_state_at=(29, 30, 59, 60),
               action_fn=hold, period_ms=150,
               path_at={0: "global", 30: "lds", 45: "reg", 60: "lds"})
    assert env.max_cnt_seen > 12, env.max_cnt_seen


@pytest.mark.parametrize("path", ["reg", "lds", "global"])
@pytest.mark.parametrize("grid", [(3, 3), (4, 4)])
def test_every_sim_path_matches_oracle(grid, path, lib_option):
    """All three kernel paths (register lanes, LDS image, global memory; the
    launcher picks one by grid size, the sim_path option forces it) are bit-exact,
    actuated mode included."""
    lib_option("sim_path", path)
    _run(*grid, E=3, steps=100, check_every=9, full_state_at=(50,), actuated=(path != "lds"))


def test_advance_matches_oracle():
    """TrafficEnv.advance (the bench's sim probe: K substeps with the signals
    on their program, no setPhase) is the oracle's step with no actions."""
    R, C, E, seed = 2, 3, 4, 21
    env = TrafficEnv(EnvConfig(rows=R, cols=C, num_envs=E, seed=seed))
    env.reset()
    refs = [O.OracleEnv(R, C, seed + e) for e in range(E)]
    rng = np.random.RandomState(seed)
    t = 0
    for step in range(12):
        if step % 3 == 0:  # interleave RL steps (setPhase) with bare advances
            acts = rng.randint(0, 4, size=(E, R * C)).astype(np.int32)
            env.step(torch.from_numpy(acts).cuda())
            outs = [refs[e].step(acts[e], 3, t, 10, 2400) for e in range(E)]
        else:
            env.advance()
            outs = [refs[e].step(None, 3, t, 10, 2400) for e in range(E)]
        t += 10
        halt_g, ph_g, ts_g = env.halt.cpu().numpy(), env.phase.cpu().numpy(), env.tspent.cpu().numpy()
        for e in range(E):
            np.testing.assert_array_equal(halt_g[e], outs[e][0], err_msg=f"halt env {e} step {step}")
            np.testing.assert_array_equal(ph_g[e], outs[e][1])
            np.testing.assert_array_equal(ts_g[e], outs[e][2])
    assert env.t == t
