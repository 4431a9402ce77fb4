"""Real-scenario loader: SUMO net + route files -> the
simulator's static grid and departure tables.

Reads the reference's shipped scenario (src/sumo_files/scenarios/grid_3x3.sumocfg
-> grid_3x3.net.xml + grid_3x3_p06.rou.xml) or any R x C grid built with the same
naming scheme, and maps it onto the HIP simulator:

* junctions ``J_r_c`` (grid_3x3.net.xml:1056-1232) -> agent a = r*C + c;
* edges (grid_3x3.net.xml:652-891), the direction rule of order_lanes.py:48-106:
    ``END_<D>_r_c_to_J_r_c``  approach of J_r_c from side D      -> a*4 + d
    ``J_a_b_to_J_c_d``        approach of J_c_d from n (a<c), s (a>c),
                              w (b<d), e (b>d)                   -> (c*C+d)*4 + side
    ``J_r_c_to_END_<D>_r_c``  exit of J_r_c toward D              -> 4A + exit index
* vehicles (grid_3x3_p06.rou.xml:23-12524): origin = first route edge,
  destination = last route edge, vehicle i departs at i * period (the file's
  departures are exactly i * 0.6 s, checked), and the duarouter path itself:
  the out-direction taken at every junction on the way, packed 2 bits each
  above a sentinel into the vehicle's route word (0x8000 | code, sim.hpp), so
  the simulator drives exactly the file's edges.

Checks that the net matches what the simulator models and raises otherwise:
3 lanes per edge, the 12-phase program of grid_3x3.net.xml:893-906, junction
ids forming a full R x C grid.
"""
import os
import re
import xml.etree.ElementTree as ET
from dataclasses import dataclass

import numpy as np

from .scenario import Grid, neighbor

DIR = {"N": 0, "S": 1, "E": 2, "W": 3}
PHASE_DURATIONS = [25, 6, 2, 20, 6, 2, 25, 6, 2, 20, 6, 2]  # sim.hpp phase_dur

_J = re.compile(r"^J_(\d+)_(\d+)$")
_APPROACH = re.compile(r"^END_([NSEW])_(\d+)_(\d+)_to_J_(\d+)_(\d+)$")
_EXIT = re.compile(r"^J_(\d+)_(\d+)_to_END_([NSEW])_(\d+)_(\d+)$")
_INNER = re.compile(r"^J_(\d+)_(\d+)_to_J_(\d+)_(\d+)$")


@dataclass
class Scenario:
    rows: int
    cols: int
    origin: np.ndarray      # int32 [N] simulator edge id of the first route edge
    dest: np.ndarray        # int32 [N] simulator edge id of the last route edge
    period_ms: int          # vehicle i departs at i * period_ms
    lane_len_inner: float   # J -> J lane length (m)
    lane_len_outer: float   # END -> J / J -> END lane length (m)
    source: str = ""
    route: np.ndarray = None  # uint16 [N] route words (route_word), or None: on-the-fly routing

    @property
    def nveh(self):
        return len(self.origin)

    def save(self, path):
        extra = {} if self.route is None else {"route": self.route}
        np.savez_compressed(path, rows=self.rows, cols=self.cols, origin=self.origin,
                            dest=self.dest, period_ms=self.period_ms,
                            lane_len_inner=self.lane_len_inner,
                            lane_len_outer=self.lane_len_outer, **extra)


def read_sumocfg(path):
    """(net file, [route files]) named by a .sumocfg (grid_3x3.sumocfg:5-17)."""
    root = ET.parse(path).getroot()
    base = os.path.dirname(os.path.abspath(path))
    net = root.find("./input/net-file").get("value")
    routes = root.find("./input/route-files").get("value").split(",")
    return os.path.join(base, net), [os.path.join(base, r.strip()) for r in routes]


def edge_index(edge_id, grid: Grid):
    """Simulator edge id of a SUMO edge id (raises on ids outside the scheme)."""
    C = grid.C
    m = _APPROACH.match(edge_id)
    if m:
        d, r, c, r2, c2 = m.group(1), *map(int, m.groups()[1:])
        if (r, c) != (r2, c2):
            raise ValueError(f"boundary edge {edge_id} does not end at its own junction")
        return (r * C + c) * 4 + DIR[d]
    m = _EXIT.match(edge_id)
    if m:
        r, c, d = int(m.group(1)), int(m.group(2)), m.group(3)
        x = grid.exit_id[r * C + c, DIR[d]]
        if x < 0:
            raise ValueError(f"exit edge {edge_id} leaves toward a neighbour junction")
        return 4 * grid.A + int(x)
    m = _INNER.match(edge_id)
    if m:
        a, b, c, d = map(int, m.groups())
        if abs(a - c) + abs(b - d) != 1:
            raise ValueError(f"edge {edge_id} does not join adjacent junctions")
        side = DIR["N"] if a < c else DIR["S"] if a > c else DIR["W"] if b < d else DIR["E"]
        return (c * C + d) * 4 + side
    raise ValueError(f"edge id {edge_id!r} is not in the J_r_c / END_<D>_r_c scheme")


ROUTED = 0x8000   # sim.hpp kRouted
MAX_TURNS = 7     # 2 bits each above the sentinel in 15 bits


def next_edge(grid: Grid, a, o):
    """Simulator edge reached by leaving junction a toward o (sim.hpp next_edge)."""
    nb = neighbor(grid.R, grid.C, a, o)
    return nb * 4 + (o ^ 1) if nb >= 0 else 4 * grid.A + int(grid.exit_id[a, o])


def route_word(edges, grid: Grid):
    """Route word of a path of simulator edges: the out-direction at each
    junction crossed, 2 bits each from the lowest, above a sentinel 1."""
    turns = []
    for e, e2 in zip(edges[:-1], edges[1:]):
        if e >= 4 * grid.A:
            raise ValueError("a route continues past an exit edge")
        a = e >> 2
        outs = [o for o in range(4) if next_edge(grid, a, o) == e2]
        if not outs:
            raise ValueError(f"edges {e} -> {e2} are not connected at junction {a}")
        turns.append(outs[0])
    if len(turns) > MAX_TURNS:
        raise ValueError(f"route crosses {len(turns)} junctions (route words hold {MAX_TURNS})")
    code = 1 << (2 * len(turns))
    for i, o in enumerate(turns):
        code |= o << (2 * i)
    return ROUTED | code


def route_edges(word, origin, grid: Grid):
    """Inverse of route_word: the simulator edges a route word drives from `origin`."""
    edges, c = [int(origin)], int(word) & 0x7FFF
    while c > 1:
        edges.append(next_edge(grid, edges[-1] >> 2, c & 3))
        c >>= 2
    return edges


def load_net(path):
    """Grid + lane lengths of a SUMO net in the J_r_c scheme; validates lanes per
    edge and the signal program."""
    root = ET.parse(path).getroot()
    js = []
    for j in root.iter("junction"):
        m = _J.match(j.get("id", ""))
        if m:
            js.append((int(m.group(1)), int(m.group(2))))
    if not js:
        raise ValueError(f"{path}: no J_r_c junctions")
    R, C = max(r for r, _ in js) + 1, max(c for _, c in js) + 1
    if len(set(js)) != R * C:
        raise ValueError(f"{path}: junctions do not form a full {R}x{C} grid")
    grid = Grid(R, C)
    inner, outer = [], []
    for e in root.iter("edge"):
        eid = e.get("id", "")
        if eid.startswith(":"):  # internal junction connectors
            continue
        lanes = e.findall("lane")
        if len(lanes) != 3:
            raise ValueError(f"{path}: edge {eid} has {len(lanes)} lanes (the simulator models 3)")
        idx = edge_index(eid, grid)
        L = float(lanes[0].get("length"))
        (outer if (idx >= 4 * grid.A or eid.startswith("END_")) else inner).append(L)
    for tl in root.iter("tlLogic"):
        d = [int(float(p.get("duration"))) for p in tl.findall("phase")]
        if d != PHASE_DURATIONS:
            raise ValueError(f"{path}: tlLogic {tl.get('id')} program {d} != {PHASE_DURATIONS}")
    return grid, float(np.median(inner)) if inner else 0.0, float(np.median(outer))


def load_routes(path, grid: Grid):
    """origin / destination edge and route word per vehicle, and the
    departure period (ms)."""
    root = ET.parse(path).getroot()
    org, dst, dep, words = [], [], [], []
    for i, v in enumerate(root.iter("vehicle")):
        if int(v.get("id")) != i:
            raise ValueError(f"{path}: vehicle ids must be 0..N-1 in order")
        edges = [edge_index(e, grid) for e in v.find("route").get("edges").split()]
        org.append(edges[0])
        dst.append(edges[-1])
        words.append(route_word(edges, grid))
        dep.append(float(v.get("depart")))
    if not org:
        raise ValueError(f"{path}: no vehicles")
    if any(o >= 4 * grid.A for o in org):
        raise ValueError(f"{path}: a route starts on an exit edge")
    dep = np.asarray(dep)
    period_ms = int(round((dep[1] - dep[0]) * 1000)) if len(dep) > 1 else 1000
    if not np.allclose(dep, np.arange(len(dep)) * period_ms / 1000.0, atol=1e-6):
        raise ValueError(f"{path}: departures are not i * {period_ms} ms "
                         "(the simulator's origin queues assume a fixed period)")
    return (np.asarray(org, np.int32), np.asarray(dst, np.int32), period_ms,
            np.asarray(words, np.uint16))


def load_scenario(path):
    """A .sumocfg (net + routes) or a .npz written by Scenario.save."""
    if path.endswith(".npz"):
        with np.load(path) as f:
            return Scenario(int(f["rows"]), int(f["cols"]), f["origin"].astype(np.int32),
                            f["dest"].astype(np.int32), int(f["period_ms"]),
                            float(f["lane_len_inner"]), float(f["lane_len_outer"]), path,
                            f["route"].astype(np.uint16) if "route" in f.files else None)
    net, routes = read_sumocfg(path)
    grid, li, lo = load_net(net)
    o, d, p, w = load_routes(routes[0], grid)
    return Scenario(grid.R, grid.C, o, d, p, li, lo, path, w)


def scenario_tables(sc: Scenario, E):
    """Origin-queue tables (the layout of scenario.demand_tables) with the SAME
    departures in every one of the E replicas."""
    A = sc.rows * sc.cols
    N = sc.nveh
    if N > 65535:
        raise ValueError("too many vehicles for uint16 ids")
    order = np.argsort(sc.origin, kind="stable").astype(np.uint16)
    off = np.zeros(4 * A + 1, np.int32)
    off[1:] = np.cumsum(np.bincount(sc.origin, minlength=4 * A))
    q_ids = np.broadcast_to(order, (E, N)).copy()
    q_off = np.broadcast_to(off, (E, 4 * A + 1)).copy()
    # per vehicle the word the lane rings carry: its explicit route when the
    # scenario has one, else its destination (on-the-fly routing)
    word = sc.route if sc.route is not None else sc.dest.astype(np.uint16)
    vdst = np.broadcast_to(word.astype(np.uint16), (E, N)).copy()
    return q_ids, q_off, vdst, N, sc.period_ms
