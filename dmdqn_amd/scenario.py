"""Synthetic R x C grid scenarios: topology tables and per-env demand.

Mirrors the reference scenario (src/sumo_files/scenarios/grid_3x3.*):
  * geometry: 200 m junction spacing, 3 lanes per edge, 172.8 m J->J lanes and
    86.4 m END->J / J->END lanes, 13.89 m/s (grid_3x3.net.xml:652-891);
  * demand: randomTrips with period 0.6 s for 3x3, fringe-factor 5, departures
    until 2500 s (trips_p06.trips.xml:7-9); the period scales as
    7.2 s / (number of fringe in-edges), i.e. 0.9 / 0.6 / 0.45 / 0.225 s for
    2x2 / 3x3 / 4x4 / 8x8;
  * every episode replays the same demand (traci.load of one route file,
    train.py:190), so the tables are built once per env seed.
Origins are drawn over incoming edges (fringe END->J edges weight 5, J->J
edges weight 1), destinations over J->J edges (weight 1) and J->END exits
(weight 5), origin != destination, with a counter-based splitmix64 stream.
"""
import numpy as np

DIRS = "nsew"
M64 = (1 << 64) - 1


def neighbor(R, C, a, d):
    r, c = divmod(a, C)
    if d == 0:
        return a - C if r > 0 else -1
    if d == 1:
        return a + C if r < R - 1 else -1
    if d == 2:
        return a + 1 if c < C - 1 else -1
    return a - 1 if c > 0 else -1


class Grid:
    """Static topology of an R x C grid (edge / lane numbering of dmdqn.h)."""

    def __init__(self, R, C):
        if not (1 <= R <= 10 and 1 <= C <= 10):
            raise ValueError("grid must be within 1..10 x 1..10 (J_r_c ids use one digit)")
        self.R, self.C = R, C
        self.A = A = R * C
        exit_id = np.full((A, 4), -1, dtype=np.int32)
        ao = []
        for a in range(A):
            for o in range(4):
                if neighbor(R, C, a, o) < 0:
                    exit_id[a, o] = len(ao)
                    ao.append((a, o))
        self.exit_id = exit_id
        self.exit_ao = np.array(ao, dtype=np.int32).reshape(-1, 2)
        self.X = len(ao)
        assert self.X == 2 * R + 2 * C
        self.n_edges = 4 * A + self.X
        self.NL = 3 * self.n_edges
        inc = np.array([neighbor(R, C, e // 4, e % 4) for e in range(4 * A)])
        self.fringe_in = np.nonzero(inc < 0)[0]   # END -> J edges
        self.internal = np.nonzero(inc >= 0)[0]   # J -> J edges
        self.period_ms = 7200 // len(self.fringe_in)
        if 7200 % len(self.fringe_in):
            self.period_ms = int(round(7200 / len(self.fringe_in)))
        self.junction_ids = [f"J_{a // C}_{a % C}" for a in range(A)]

    def neighbors(self):
        return np.array([[neighbor(self.R, self.C, a, d) for d in range(4)]
                         for a in range(self.A)], dtype=np.int32)

    def incoming_lane_ids(self):
        """SUMO lane ids of the 12 observed lanes per junction (n,s,e,w x k)."""
        R, C = self.R, self.C
        out = []
        for a in range(self.A):
            r, c = divmod(a, C)
            j = f"J_{r}_{c}"
            srcs = [f"J_{r-1}_{c}" if r > 0 else f"END_N_{r}_{c}",
                    f"J_{r+1}_{c}" if r < R - 1 else f"END_S_{r}_{c}",
                    f"J_{r}_{c+1}" if c < C - 1 else f"END_E_{r}_{c}",
                    f"J_{r}_{c-1}" if c > 0 else f"END_W_{r}_{c}"]
            out.append([f"{s}_to_{j}_{k}" for s in srcs for k in range(3)])
        return out


def splitmix64(z):
    """Vectorised splitmix64 over uint64 arrays (wrapping arithmetic)."""
    z = (z + np.uint64(0x9E3779B97F4A7C15))
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def demand(grid, seed, end_ms=2_500_000, period_ms=None):
    """(origin_edge[N], dest_edge[N]) for one env; vehicle i departs i*period."""
    g = grid
    period_ms = period_ms or g.period_ms
    N = (end_ms + period_ms - 1) // period_ms
    A = g.A
    o_edges = np.arange(4 * A)
    o_w = np.where(np.isin(o_edges, g.fringe_in), 5, 1).astype(np.uint64)
    d_edges = np.concatenate([g.internal, 4 * A + np.arange(g.X)])
    d_w = np.concatenate([np.ones(len(g.internal)), np.full(g.X, 5)]).astype(np.uint64)
    o_cum, d_cum = np.cumsum(o_w), np.cumsum(d_w)
    with np.errstate(over="ignore"):
        ids = np.arange(N, dtype=np.uint64)
        z = splitmix64(np.uint64(seed) ^ (ids * np.uint64(0xD1B54A32D192ED03)))
        origin = o_edges[np.searchsorted(o_cum, z % o_cum[-1], side="right")]
        z2 = splitmix64(z)
        dest = d_edges[np.searchsorted(d_cum, z2 % d_cum[-1], side="right")]
        bad = dest == origin
        while bad.any():
            z2 = np.where(bad, splitmix64(z2), z2)
            dest = np.where(bad, d_edges[np.searchsorted(d_cum, z2 % d_cum[-1], side="right")], dest)
            bad = dest == origin
    return origin.astype(np.int32), dest.astype(np.int32)


def demand_tables(grid, seeds, end_ms=2_500_000, period_ms=None):
    """Per-env origin queues: q_ids[E][N] (ids sorted by (origin, id)),
    q_off[E][4A+1], vdst[E][N] (uint16)."""
    A = grid.A
    E = len(seeds)
    period_ms = period_ms or grid.period_ms
    N = (end_ms + period_ms - 1) // period_ms
    if N > 65535:
        raise ValueError("too many vehicles per env for uint16 ids")
    q_ids = np.zeros((E, N), dtype=np.uint16)
    q_off = np.zeros((E, 4 * A + 1), dtype=np.int32)
    vdst = np.zeros((E, N), dtype=np.uint16)
    for e, s in enumerate(seeds):
        o, d = demand(grid, int(s), end_ms, period_ms)
        order = np.argsort(o, kind="stable")
        q_ids[e] = order.astype(np.uint16)
        q_off[e, 1:] = np.cumsum(np.bincount(o, minlength=4 * A))
        vdst[e] = d.astype(np.uint16)
    return q_ids, q_off, vdst, N, period_ms
