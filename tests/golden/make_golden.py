"""Generate the golden fixtures that pin the oracle (tests/golden/*.npz).

TEST INFRASTRUCTURE ONLY.  Run in the survey/build container (it needs the
read-only reference checkout at /root/reference); the GPU box never runs it.
The fixtures are data: inputs and the reference's outputs on them.

What is imported from the reference (with stub modules for the absent
third-party packages traci / sumolib / tensorflow / wandb):
  * src/experimental/order_lanes.py   -- lane mapping, get_own_state,
                                          build_state_vector, _get_neighbor_info
  * src/agents/dqn_agent.py           -- ReplayBuffer (add / sample)
  * src/scripts/train.py              -- calculate_local_reward,
                                          calculate_global_reward, SmoothedValue
Plus CPython `random` and numpy's legacy RandomState, which the reference
uses directly (dqn_agent.py:63, dqn_agent.py:263-265).

Usage:  python tests/golden/make_golden.py [--out tests/golden]
"""
import argparse
import importlib
import json
import os
import random
import sys
import types

import numpy as np

REF = "/root/reference"


# --------------------------------------------------------------------------
# stub modules (the reference imports these at module level)
# --------------------------------------------------------------------------
class _TraCIException(Exception):
    pass


class _StubSim:
    """State read by the stub traci: halting counts per lane id and TL state."""

    def __init__(self):
        self.halting = {}
        self.phase = {}
        self.next_switch = {}
        self.phase_duration = {}
        self.time = 0.0


SIM = _StubSim()


def _install_stubs(junction_has_get_type: bool):
    traci = types.ModuleType("traci")
    traci.exceptions = types.SimpleNamespace(
        TraCIException=_TraCIException, FatalTraCIError=_TraCIException)
    traci.lane = types.SimpleNamespace(
        getLastStepHaltingNumber=lambda lid: SIM.halting[lid])
    traci.trafficlight = types.SimpleNamespace(
        getPhase=lambda j: SIM.phase[j],
        getNextSwitch=lambda j: SIM.next_switch[j],
        getPhaseDuration=lambda j: SIM.phase_duration[j])
    junction = types.SimpleNamespace()
    if junction_has_get_type:
        junction.getType = lambda j: "traffic_light"
    traci.junction = junction
    traci.simulation = types.SimpleNamespace(getTime=lambda: SIM.time)
    traci.isconnected = lambda: False
    sys.modules["traci"] = traci

    sumolib = types.ModuleType("sumolib")
    sumolib.net = types.SimpleNamespace(readNet=lambda p: None)
    sys.modules["sumolib"] = sumolib
    sys.modules["sumolib.net"] = sumolib.net

    tf = types.ModuleType("tensorflow")
    tf.float32, tf.int32 = np.float32, np.int32
    tf.convert_to_tensor = lambda x, dtype=None: np.asarray(x, dtype=dtype)
    tf.function = lambda *a, **k: (lambda f: f)
    keras = types.ModuleType("tensorflow.keras")
    keras.initializers = types.SimpleNamespace()
    layers = types.ModuleType("tensorflow.keras.layers")
    layers.Dense = layers.Input = layers.Concatenate = object
    keras.layers = layers
    keras.mixed_precision = types.SimpleNamespace(set_global_policy=lambda p: None)
    tf.keras = keras
    tf.config = types.SimpleNamespace(
        list_physical_devices=lambda kind: [],
        experimental=types.SimpleNamespace(set_memory_growth=lambda g, b: None))
    sys.modules["tensorflow"] = tf
    sys.modules["tensorflow.keras"] = keras
    sys.modules["tensorflow.keras.layers"] = layers

    wandb = types.ModuleType("wandb")
    wandb.Settings = lambda **k: None
    wandb.init = lambda **k: types.SimpleNamespace(log=lambda *a, **k: None,
                                                   finish=lambda: None)
    sys.modules["wandb"] = wandb


def _import_reference(junction_has_get_type: bool):
    _install_stubs(junction_has_get_type)
    if REF not in sys.path:
        sys.path.insert(0, REF)
    for name in ["src.experimental.order_lanes", "src.agents.dqn_agent",
                 "src.scripts.train"]:
        sys.modules.pop(name, None)
    ol = importlib.import_module("src.experimental.order_lanes")
    dq = importlib.import_module("src.agents.dqn_agent")
    tr = importlib.import_module("src.scripts.train")
    return ol, dq, tr


# --------------------------------------------------------------------------
# grid naming (SUMO ids as in grid_3x3.net.xml; docs/environment.md:76-99)
# --------------------------------------------------------------------------
def grid_incoming_lane_ids(R, C):
    """[A][4 dirs n,s,e,w][3 lanes] lane ids of the incoming approaches."""
    out = []
    for r in range(R):
        for c in range(C):
            j = f"J_{r}_{c}"
            srcs = [
                f"J_{r-1}_{c}" if r > 0 else f"END_N_{r}_{c}",
                f"J_{r+1}_{c}" if r < R - 1 else f"END_S_{r}_{c}",
                f"J_{r}_{c+1}" if c < C - 1 else f"END_E_{r}_{c}",
                f"J_{r}_{c-1}" if c > 0 else f"END_W_{r}_{c}",
            ]
            out.append([[f"{s}_to_{j}_{k}" for k in range(3)] for s in srcs])
    return out


def grid_all_lane_ids(R, C, rng):
    """All non-internal lane ids (incoming + exit), shuffled like getIDList."""
    ids = [l for jl in grid_incoming_lane_ids(R, C) for d in jl for l in d]
    for r in range(R):
        for c in range(C):
            j = f"J_{r}_{c}"
            if r == 0:
                ids += [f"{j}_to_END_N_{r}_{c}_{k}" for k in range(3)]
            if r == R - 1:
                ids += [f"{j}_to_END_S_{r}_{c}_{k}" for k in range(3)]
            if c == C - 1:
                ids += [f"{j}_to_END_E_{r}_{c}_{k}" for k in range(3)]
            if c == 0:
                ids += [f"{j}_to_END_W_{r}_{c}_{k}" for k in range(3)]
    rng.shuffle(ids)
    return ids


# --------------------------------------------------------------------------
def gen_observe(out, ol, tr, mode_tag):
    """get_own_state / build_state_vector / rewards for controlled inputs."""
    rng = np.random.RandomState(1234)
    res = {}
    for (R, C) in [(1, 1), (2, 2), (3, 3), (4, 4), (8, 8), (2, 3)]:
        A = R * C
        tl = [f"J_{r}_{c}" for r in range(R) for c in range(C)]
        lanes = grid_all_lane_ids(R, C, random.Random(7))
        jmap = ol.order_lanes_in_edge(ol.build_junction_lane_mapping(tl, lanes))
        inc = grid_incoming_lane_ids(R, C)
        # the reference mapping must equal our [A][n,s,e,w][k] order
        lane_order_ok = all(jmap[tl[a]] == inc[a] for a in range(A))
        for case in range(3):
            halt = rng.randint(0, 24, size=(A, 12)).astype(np.int64)
            phase = rng.randint(0, 12, size=A).astype(np.int64)
            t = float(rng.randint(0, 2400))
            dur = rng.choice([2, 6, 20, 25], size=A).astype(np.int64)
            tspent = np.minimum(rng.randint(0, 30, size=A), t).astype(np.int64)
            SIM.halting = {inc[a][d][k]: int(halt[a, d * 3 + k])
                           for a in range(A) for d in range(4) for k in range(3)}
            for a in range(A):
                SIM.phase[tl[a]] = int(phase[a])
                SIM.phase_duration[tl[a]] = float(dur[a])
                SIM.next_switch[tl[a]] = float(t - tspent[a] + dur[a])
            SIM.time = t
            gstate = {j: ol.get_own_state(j, jmap, 3, t) for j in tl}
            L = np.array([gstate[j] for j in tl], dtype=np.float64)
            obs = np.stack([ol.build_state_vector(j, tl, jmap, 3, t, gstate)
                            for j in tl]).astype(np.float64)
            # rewards: train.py:159-165 and the combination at train.py:254
            g = tr.calculate_global_reward(gstate, {})
            rew = np.array([0.3 * tr.calculate_local_reward(gstate[j], None)
                            + 0.7 * g for j in tl], dtype=np.float64)
            pres = np.array([ol._get_neighbor_info(j, tl)[0] for j in tl])
            key = f"{mode_tag}_{R}x{C}_{case}"
            res[key + "_halt"] = halt
            res[key + "_phase"] = phase
            res[key + "_tspent"] = tspent
            res[key + "_t"] = np.array([t])
            res[key + "_local"] = L
            res[key + "_obs"] = obs
            res[key + "_reward"] = rew
            res[key + "_presence"] = pres
            res[key + "_lane_order_ok"] = np.array([int(lane_order_ok)])
    np.savez_compressed(os.path.join(out, f"observe_{mode_tag}.npz"), **res)


def gen_smoothed(out, tr):
    sv = tr.SmoothedValue(alpha=0.3)
    xs = [-3.0, -10.5, 4.25, 0.0, -7.0]
    ys = []
    for x in xs:
        sv.update(x)
        ys.append(sv.get_value())
    np.savez(os.path.join(out, "smoothed.npz"), x=np.array(xs), y=np.array(ys))


def _fill_buffer(dq, n, rseed):
    """n transitions whose state row encodes the index (exact small ints)."""
    g = np.random.RandomState(rseed)
    loc = g.randint(0, 40, size=n)
    glob = g.randint(0, 400, size=n)
    buf = dq.ReplayBuffer(10000)
    for i in range(n):
        s = np.zeros((1, 89), dtype=np.float32)
        s[0, 0] = i % 128
        s[0, 1] = i // 128
        s[0, 2:] = (i * 7 + np.arange(87)) % 23
        s2 = s.copy()
        s2[0, 2] = -1.0
        r = 0.3 * (-1.0 * float(loc[i])) + 0.7 * (-1.0 * float(glob[i]))
        buf.add((s, i % 4, r, s2, (i % 240) == 239))
    return buf, loc, glob


def gen_replay(out, dq):
    res = {}
    for n in [128, 129, 500, 1045, 1046, 5000, 10000, 10500]:
        buf, loc, glob = _fill_buffer(dq, n, rseed=n)
        for seed in [0, 1, 12345]:
            random.seed(seed)
            draws = []
            for rep in range(3):  # three consecutive samples on one stream
                st, ac, rw, ns, dn = buf.sample(128)
                idx = (st[:, 0] + 128 * st[:, 1]).astype(np.int64)
                first = max(0, n - 10000)
                pos = idx - first  # deque position, 0 = oldest
                draws.append((pos, ac, rw, dn, ns[:, 2]))
            key = f"n{n}_s{seed}"
            res[key + "_pos"] = np.stack([d[0] for d in draws])
            res[key + "_act"] = np.stack([d[1] for d in draws])
            res[key + "_rew"] = np.stack([d[2] for d in draws])
            res[key + "_done"] = np.stack([d[3] for d in draws])
            res[key + "_ns2"] = np.stack([d[4] for d in draws])
        res[f"n{n}_loc"] = loc
        res[f"n{n}_glob"] = glob
    np.savez_compressed(os.path.join(out, "replay_sample.npz"), **res)


def gen_rng(out):
    res = {}
    for seed in [0, 1, 42, 12345, 2**31 - 1, 4000000000]:
        random.seed(seed)
        res[f"py_{seed}_u32"] = np.array([random.getrandbits(32)
                                          for _ in range(2000)], dtype=np.uint64)
        random.seed(seed)
        res[f"py_{seed}_below"] = np.array(
            [random.randrange(n) for n in [1, 2, 3, 5, 128, 1045, 10000] * 40])
        np.random.seed(seed)
        rr, ri = [], []
        for _ in range(1000):  # dqn_agent.py:263-265 call pattern
            rr.append(np.random.rand())
            ri.append(np.random.randint(0, 4))
        res[f"np_{seed}_rand"] = np.array(rr, dtype=np.float64)
        res[f"np_{seed}_randint"] = np.array(ri, dtype=np.int64)
        # epsilon-greedy pattern: randint only when rand() < eps
        np.random.seed(seed)
        eps = 0.3
        acts = []
        for _ in range(500):
            if np.random.rand() < eps:
                acts.append(np.random.randint(0, 4))
            else:
                acts.append(-1)
        res[f"np_{seed}_eps03"] = np.array(acts, dtype=np.int64)
    np.savez_compressed(os.path.join(out, "rng.npz"), **res)


def gen_neighbors(out, ol):
    res = {}
    for (R, C) in [(1, 1), (2, 2), (3, 3), (4, 4), (8, 8), (2, 3)]:
        tl = [f"J_{r}_{c}" for r in range(R) for c in range(C)]
        pres, nb = [], []
        for j in tl:
            p, ids = ol._get_neighbor_info(j, tl)
            pres.append(p)
            nb.append([tl.index(x) if x is not None else -1 for x in ids])
        res[f"{R}x{C}_presence"] = np.array(pres)
        res[f"{R}x{C}_nbr"] = np.array(nb)
    np.savez(os.path.join(out, "neighbors.npz"), **res)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.dirname(os.path.abspath(__file__)))
    args = ap.parse_args()
    out = os.path.abspath(args.out)
    scratch = "/tmp/dmdqn_golden_scratch"
    os.makedirs(scratch, exist_ok=True)
    os.chdir(scratch)  # log_config.py truncates ./replay_buffer.log
    sys.dont_write_bytecode = True

    ol, dq, tr = _import_reference(junction_has_get_type=False)
    gen_observe(out, ol, tr, "refpad")  # traci.junction has no getType (A-5)
    gen_neighbors(out, ol)
    gen_replay(out, dq)
    gen_smoothed(out, tr)
    ol, dq, tr = _import_reference(junction_has_get_type=True)
    gen_observe(out, ol, tr, "intended")
    gen_rng(out)
    meta = {"python": sys.version.split()[0], "numpy": np.__version__,
            "reference": REF, "generator": "tests/golden/make_golden.py"}
    with open(os.path.join(out, "META.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print("golden fixtures written to", out)


if __name__ == "__main__":
    main()
