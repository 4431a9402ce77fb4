"""Host-side scenario generation (product, numpy) vs the oracle's C restatement,
plus conservation/physics invariants of the oracle simulator (CPU only)."""
import numpy as np
import pytest

import oracle as O
from dmdqn_amd.scenario import Grid, demand_tables


@pytest.mark.parametrize("grid", [(1, 1), (2, 2), (3, 3), (4, 4), (8, 8), (2, 3)])
def test_demand_tables_match_oracle(grid):
    R, C = grid
    g = Grid(R, C)
    seeds = [0, 5, 2**40 + 3]
    q, off, vd, N, period = demand_tables(g, seeds)
    assert period == 7200 // (2 * R + 2 * C)
    for e, s in enumerate(seeds):
        env = O.OracleEnv(R, C, s)
        oq, ooff, ovd = env.demand()
        assert env.nveh == N
        np.testing.assert_array_equal(oq, q[e])
        np.testing.assert_array_equal(ooff, off[e])
        np.testing.assert_array_equal(ovd, vd[e])


def test_demand_statistics_like_reference():
    """3x3: 4167 vehicles, ~72% departing on fringe edges (grid_3x3_p06.rou.xml)."""
    g = Grid(3, 3)
    q, off, vd, N, period = demand_tables(g, [1])
    assert N == 4167 and period == 600
    per_edge = np.diff(off[0])
    share = per_edge[g.fringe_in].sum() / N
    assert 0.68 < share < 0.76


def test_lane_ids_match_reference_order():
    from conftest import GOLDEN
    import os
    g = Grid(3, 3)
    ids = g.incoming_lane_ids()
    assert ids[0][0] == "END_N_0_0_to_J_0_0_0" and ids[4][3] == "J_2_1_to_J_1_1_0"
    d = np.load(os.path.join(GOLDEN, "observe_refpad.npz"))
    assert int(d["refpad_3x3_0_lane_order_ok"][0]) == 1


@pytest.mark.parametrize("grid", [(2, 2), (4, 4)])
def test_oracle_sim_invariants(grid):
    R, C = grid
    env = O.OracleEnv(R, C, 11)
    rng = np.random.RandomState(0)
    t = 0
    for step in range(120):
        halt, ph, ts, done = env.step(rng.randint(0, 4, R * C), 3, t, 10, 2400)
        t += 10
        info = env.info()
        inserted, arrived, running = info[4], info[5], info[6]
        assert inserted == arrived + running
        x, v, d, hd, cn = env.lanes()
        assert (cn >= 0).all() and (cn <= env.cap).all()
        assert (v >= 0).all() and (v <= 13.89 + 1e-6).all()
        assert (ts == 10).all() or step == 0
        np.testing.assert_array_equal(ph % 3, 0)
        # vehicles in a lane are ordered and do not overlap
        for l in np.nonzero(cn > 1)[0]:
            idx = [(hd[l] + i) % env.cap for i in range(cn[l])]
            xs = x[l, idx]
            assert (xs[:-1] - xs[1:] >= 5.0 - 1e-4).all(), (l, xs)
        assert (halt >= 0).all()
    assert done is False
