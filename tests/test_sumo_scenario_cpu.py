"""Real-scenario loader (dmdqn_amd/sumo_scenario.py): SUMO
net + route XML -> simulator grid and departure tables.  CPU only."""
import os

import numpy as np
import pytest

import oracle as O
from conftest import GOLDEN
from dmdqn_amd.scenario import Grid
from dmdqn_amd.sumo_scenario import (PHASE_DURATIONS, edge_index, load_scenario,
                                     scenario_tables)

REF_CFG = "/root/reference/src/sumo_files/scenarios/grid_3x3.sumocfg"
FIXTURE = os.path.join(GOLDEN, "grid_3x3_p06_scenario.npz")


def test_fixture_facts():
    sc = load_scenario(FIXTURE)
    assert (sc.rows, sc.cols, sc.nveh, sc.period_ms) == (3, 3, 4167, 600)
    assert (sc.lane_len_inner, sc.lane_len_outer) == (172.8, 86.4)   # grid_3x3.net.xml:652-891
    fringe = set(Grid(3, 3).fringe_in.tolist())
    assert 0.71 < np.isin(sc.origin, list(fringe)).mean() < 0.73     # 72 % fringe
    assert (sc.origin == sc.dest).sum() == 19                        # one-edge routes


@pytest.mark.skipif(not os.path.exists(REF_CFG), reason="reference scenario not present")
def test_loader_on_reference_files_matches_fixture():
    a, b = load_scenario(REF_CFG), load_scenario(FIXTURE)
    np.testing.assert_array_equal(a.origin, b.origin)
    np.testing.assert_array_equal(a.dest, b.dest)
    np.testing.assert_array_equal(a.route, b.route)
    assert (a.rows, a.cols, a.period_ms) == (b.rows, b.cols, b.period_ms)


def test_edge_index_scheme():
    g = Grid(3, 3)
    assert edge_index("END_N_0_0_to_J_0_0", g) == 0                 # from north -> d 0
    assert edge_index("END_W_1_0_to_J_1_0", g) == 3 * 4 + 3         # from west -> d 3
    assert edge_index("J_0_0_to_J_1_0", g) == 3 * 4 + 0             # J_1_0 from north
    assert edge_index("J_1_1_to_J_1_0", g) == 3 * 4 + 2             # J_1_0 from east
    assert edge_index("J_2_1_to_J_1_1", g) == 4 * 4 + 1             # J_1_1 from south
    assert edge_index("J_0_2_to_END_E_0_2", g) == 36 + int(g.exit_id[2, 2])
    for bad in ["J_0_0_to_J_2_0", "J_1_1_to_END_N_1_1", "foo"]:
        with pytest.raises(ValueError):
            edge_index(bad, g)


def _write_mini(tmp, program=PHASE_DURATIONS, depart_step=0.9):
    """A 2x2 net in the reference's naming scheme + 4 routed vehicles."""
    edges = []
    for r in range(2):
        for c in range(2):
            j = f"J_{r}_{c}"
            if r == 0: edges += [f"END_N_{r}_{c}_to_{j}", f"{j}_to_END_N_{r}_{c}"]
            if r == 1: edges += [f"END_S_{r}_{c}_to_{j}", f"{j}_to_END_S_{r}_{c}"]
            if c == 0: edges += [f"END_W_{r}_{c}_to_{j}", f"{j}_to_END_W_{r}_{c}"]
            if c == 1: edges += [f"END_E_{r}_{c}_to_{j}", f"{j}_to_END_E_{r}_{c}"]
            for rr, cc in [(r - 1, c), (r + 1, c), (r, c - 1), (r, c + 1)]:
                if 0 <= rr < 2 and 0 <= cc < 2:
                    edges.append(f"{j}_to_J_{rr}_{cc}")
    lanes = lambda e, L: "".join(f'<lane id="{e}_{k}" index="{k}" length="{L}"/>' for k in range(3))
    xml = ['<net>']
    for e in edges:
        L = 86.4 if "END" in e else 172.8
        xml.append(f'<edge id="{e}">{lanes(e, L)}</edge>')
    xml.append('<edge id=":J_0_0_0"><lane id=":J_0_0_0_0" length="5"/></edge>')
    for r in range(2):
        for c in range(2):
            xml.append(f'<junction id="J_{r}_{c}" type="traffic_light"/>')
            xml.append(f'<tlLogic id="J_{r}_{c}">' + "".join(
                f'<phase duration="{d}" state="G"/>' for d in program) + '</tlLogic>')
    xml.append('</net>')
    open(os.path.join(tmp, "mini.net.xml"), "w").write("\n".join(xml))
    routes = ["END_N_0_0_to_J_0_0 J_0_0_to_J_1_0 J_1_0_to_END_S_1_0",
              "END_E_0_1_to_J_0_1 J_0_1_to_J_0_0",
              "J_1_1_to_J_0_1",
              "END_W_1_0_to_J_1_0 J_1_0_to_J_1_1 J_1_1_to_END_E_1_1"]
    rx = ['<routes>'] + [f'<vehicle id="{i}" depart="{i * depart_step:.2f}"><route edges="{r}"/>'
                         '</vehicle>' for i, r in enumerate(routes)] + ['</routes>']
    open(os.path.join(tmp, "mini.rou.xml"), "w").write("\n".join(rx))
    cfg = ('<configuration><input><net-file value="mini.net.xml"/>'
           '<route-files value="mini.rou.xml"/></input></configuration>')
    p = os.path.join(tmp, "mini.sumocfg")
    open(p, "w").write(cfg)
    return p


def test_loader_on_synthetic_net(tmp_path):
    sc = load_scenario(_write_mini(str(tmp_path)))
    g = Grid(2, 2)
    assert (sc.rows, sc.cols, sc.period_ms, sc.nveh) == (2, 2, 900, 4)
    np.testing.assert_array_equal(sc.origin, [0, 1 * 4 + 2, 1 * 4 + 1, 2 * 4 + 3])
    np.testing.assert_array_equal(sc.dest, [16 + g.exit_id[2, 1], 0 * 4 + 2, 1 * 4 + 1,
                                            16 + g.exit_id[3, 2]])
    q, off, vd, N, p = scenario_tables(sc, 3)
    assert q.shape == (3, 4) and (q == q[0]).all() and p == 900
    assert off[0, -1] == 4 and list(np.diff(off[0])[[0, 5, 6, 11]]) == [1, 1, 1, 1]


def test_loader_rejects_unsupported(tmp_path):
    with pytest.raises(ValueError, match="program"):
        load_scenario(_write_mini(str(tmp_path), program=[30, 3] * 6))
    with pytest.raises(ValueError, match="departures"):
        p = _write_mini(str(tmp_path))
        rou = os.path.join(str(tmp_path), "mini.rou.xml")
        txt = open(rou).read().replace('depart="2.70"', 'depart="3.00"')
        open(rou, "w").write(txt)
        load_scenario(p)


def test_oracle_runs_the_shipped_scenario():
    """The CPU restatement accepts the loaded departures and runs an episode."""
    sc = load_scenario(FIXTURE)
    q, off, vd, N, period = scenario_tables(sc, 1)
    env = O.OracleEnv(3, 3, 100)
    env.set_demand(q[0], off[0], vd[0], period)
    rng = np.random.RandomState(0)
    t = 0
    for _ in range(60):
        env.step(rng.randint(0, 4, 9).astype(np.int32), 3, t, 10, 2400)
        t += 10
    ins, arr, run, pend = env.info()[4:8]
    assert ins + pend == 4167 and ins > 900 and arr > 0


def _traversed(env):
    """vehicle id -> list of simulator edges it entered, in order."""
    seq = {}
    for vid, e in env.trace():
        seq.setdefault(int(vid), []).append(int(e))
    return seq


def test_vehicles_follow_their_scenario_routes():
    """Every vehicle of the shipped scenario drives exactly its duarouter path
    (grid_3x3_p06.rou.xml:23-12524): over a full 240-step episode of the
    oracle simulator (which the HIP sim matches bit for bit, test_gpu_sim), each
    vehicle's entered edges are its route's edges -- all of them for the
    vehicles that arrived, a prefix for those still driving."""
    from dmdqn_amd.sumo_scenario import route_edges
    sc = load_scenario(FIXTURE)
    grid = Grid(3, 3)
    q, off, vd, N, period = scenario_tables(sc, 1)
    env = O.OracleEnv(3, 3, 100)
    env.set_demand(q[0], off[0], vd[0], period)
    env.enable_trace(1 << 16)
    rng = np.random.RandomState(1)
    t = 0
    for _ in range(240):
        env.step(rng.randint(0, 4, 9).astype(np.int32), 3, t, 10, 2400)
        t += 10
    seq = _traversed(env)
    ins, arr, run, pend = env.info()[4:8]
    assert len(seq) == ins > 3900 and arr > 3500
    full = 0
    for vid, got in seq.items():
        want = route_edges(sc.route[vid], sc.origin[vid], grid)
        assert got == want[:len(got)], (vid, got, want)
        full += got == want
    assert full >= arr  # every arrived vehicle drove its whole route
    if os.path.exists(REF_CFG):  # and the words decode to the file's own edge lists
        import xml.etree.ElementTree as ET
        rou = os.path.join(os.path.dirname(REF_CFG), "grid_3x3_p06.rou.xml")
        for i, v in enumerate(ET.parse(rou).getroot().iter("vehicle")):
            edges = [edge_index(e, grid) for e in v.find("route").get("edges").split()]
            assert route_edges(sc.route[i], sc.origin[i], grid) == edges


def test_route_words_roundtrip_and_limits():
    from dmdqn_amd.sumo_scenario import ROUTED, route_edges, route_word
    g = Grid(3, 3)
    path = [edge_index("END_W_1_0_to_J_1_0", g), edge_index("J_1_0_to_J_0_0", g),
            edge_index("J_0_0_to_END_N_0_0", g)]
    w = route_word(path, g)
    assert w & ROUTED and route_edges(w, path[0], g) == path
    assert route_word(path[:1], g) == ROUTED | 1          # one-edge route: sentinel only
    with pytest.raises(ValueError, match="not connected"):
        route_word([path[0], path[2]], g)
    g4 = Grid(1, 9)
    long_path = [edge_index("END_W_0_0_to_J_0_0", g4)] + [
        edge_index(f"J_0_{c}_to_J_0_{c + 1}", g4) for c in range(8)]
    with pytest.raises(ValueError, match="route words hold"):
        route_word(long_path, g4)


def test_synthetic_demand_keeps_on_the_fly_routing():
    """Generated demand carries destinations (< 0x8000), not route words."""
    q, off, vd, N, period = __import__("dmdqn_amd.scenario", fromlist=["x"]).demand_tables(
        Grid(4, 4), [0, 1])
    assert vd.max() < 0x8000
