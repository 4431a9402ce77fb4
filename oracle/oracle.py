"""ctypes binding of oracle/liboracle.so (TEST INFRASTRUCTURE ONLY)."""
import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def build():
    """Compile liboracle.so (gcc) if missing or stale.  ORACLE_LIB names another
    build of the same sources to load instead (the sanitizer test's
    liboracle_asan.so)."""
    if os.environ.get("ORACLE_LIB"):
        return os.environ["ORACLE_LIB"]
    so = os.path.join(_HERE, "liboracle.so")
    srcs = [os.path.join(_HERE, f) for f in os.listdir(_HERE)
            if f.startswith("oracle_") and f.endswith(".c")] + [os.path.join(_HERE, "oracle.h")]
    if (not os.path.exists(so)) or any(os.path.getmtime(s) > os.path.getmtime(so) for s in srcs):
        subprocess.check_call(["make", "-s", "-C", _HERE])
    return so


def lib():
    global _LIB
    if _LIB is None:
        _LIB = C.CDLL(build())
        _declare(_LIB)
    return _LIB


class MT(C.Structure):
    _fields_ = [("mt", C.c_uint32 * 624), ("mti", C.c_int32)]

    def state_array(self):
        """[625] uint32: 624 words + position (the device stream layout)."""
        return np.array(list(self.mt) + [self.mti & 0xffffffff], dtype=np.uint32)


_P = np.ctypeslib.ndpointer
_i32 = _P(np.int32, flags="C_CONTIGUOUS")
_f32 = _P(np.float32, flags="C_CONTIGUOUS")
_f64 = _P(np.float64, flags="C_CONTIGUOUS")
_u8 = _P(np.uint8, flags="C_CONTIGUOUS")
_u16 = _P(np.uint16, flags="C_CONTIGUOUS")


def _declare(L):
    M = C.POINTER(MT)
    sig = {
        "orc_py_seed": (None, [M, C.c_uint64]),
        "orc_np_seed": (None, [M, C.c_uint32]),
        "orc_mt_u32": (C.c_uint32, [M]),
        "orc_py_randbelow": (C.c_uint32, [M, C.c_uint32]),
        "orc_py_sample": (C.c_int, [M, C.c_uint32, C.c_uint32, _i32]),
        "orc_np_rand": (C.c_double, [M]),
        "orc_np_randint": (C.c_uint32, [M, C.c_uint32]),
        "orc_np_sum": (C.c_double, [_f64, C.c_long]),
        "orc_zscore": (None, [_f64, C.c_long, _f32]),
        "orc_act": (None, [M, C.c_int, C.c_double, C.c_void_p, _i32]),
        "orc_neighbors": (None, [C.c_int, C.c_int, _i32]),
        "orc_local_state": (None, [C.c_int, _i32, _i32, _i32, C.c_int, _f32]),
        "orc_build_obs": (None, [C.c_int, C.c_int, _f32, _f32]),
        "orc_reward": (None, [C.c_int, _f32, _f64]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype, f.argtypes = res, args


# ---------------------------------------------------------------- streams
def py_stream(seed):
    s = MT()
    lib().orc_py_seed(C.byref(s), seed)
    return s


def np_stream(seed):
    s = MT()
    lib().orc_np_seed(C.byref(s), seed & 0xffffffff)
    return s


def u32(s, n):
    f = lib().orc_mt_u32
    return np.array([f(C.byref(s)) for _ in range(n)], dtype=np.uint64)


def py_randbelow(s, n):
    return lib().orc_py_randbelow(C.byref(s), n)


def py_sample(s, n, k=128):
    out = np.zeros(k, dtype=np.int32)
    rc = lib().orc_py_sample(C.byref(s), n, k, out)
    if rc != 0:
        raise ValueError(f"orc_py_sample rc={rc}")
    return out


def np_rand(s):
    return lib().orc_np_rand(C.byref(s))


def np_randint(s, hi):
    return lib().orc_np_randint(C.byref(s), hi)


def np_sum(a):
    a = np.ascontiguousarray(a, dtype=np.float64)
    return lib().orc_np_sum(a, a.size)


def zscore(r):
    r = np.ascontiguousarray(r, dtype=np.float64)
    out = np.zeros(r.size, dtype=np.float32)
    lib().orc_zscore(r, r.size, out)
    return out


def act(s, nagents, eps, greedy=None):
    out = np.zeros(nagents, dtype=np.int32)
    g = None if greedy is None else np.ascontiguousarray(greedy, dtype=np.int32)
    lib().orc_act(C.byref(s), nagents, eps, None if g is None else g.ctypes.data, out)
    return out


# ---------------------------------------------------------------- observe
def neighbors(R, Cc):
    out = np.zeros((R * Cc, 4), dtype=np.int32)
    lib().orc_neighbors(R, Cc, out)
    return out


def local_state(halt, phase, tspent, mode):
    halt = np.ascontiguousarray(halt, dtype=np.int32)
    A = halt.shape[0]
    out = np.zeros((A, 17), dtype=np.float32)
    lib().orc_local_state(A, halt, np.ascontiguousarray(phase, dtype=np.int32),
                          np.ascontiguousarray(tspent, dtype=np.int32), int(mode), out)
    return out


def build_obs(R, Cc, local):
    local = np.ascontiguousarray(local, dtype=np.float32)
    out = np.zeros((R * Cc, 89), dtype=np.float32)
    lib().orc_build_obs(R, Cc, local, out)
    return out


def reward(local):
    local = np.ascontiguousarray(local, dtype=np.float32)
    out = np.zeros(local.shape[0], dtype=np.float64)
    lib().orc_reward(local.shape[0], local, out)
    return out


# ---------------------------------------------------------------- simulator
class CIdmO(C.Structure):
    _fields_ = [(n, C.c_float) for n in ["length", "min_gap", "accel", "decel", "tau", "vmax",
                                         "two_sqrt_ab", "halt_speed", "len_inner", "len_outer",
                                         "det_dist", "max_gap"]]


def idm_default():
    f = np.float32
    return CIdmO(f(5.0), f(2.5), f(2.6), f(4.5), f(1.0), f(13.89),
                 f(2.0) * np.sqrt(f(2.6) * f(4.5), dtype=np.float32), f(0.1), f(172.8), f(86.4),
                 f(2.0) * f(13.89), f(3.0))


def _declare_env(L):
    L.orc_env_create.restype = C.c_void_p
    L.orc_env_create.argtypes = [C.c_int, C.c_int, C.c_int, C.c_uint64, C.c_long, C.c_int,
                                 C.POINTER(CIdmO)]
    L.orc_env_free.argtypes = [C.c_void_p]
    L.orc_env_reset.argtypes = [C.c_void_p]
    L.orc_env_step.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int,
                               _i32, _i32, _i32, _u8]
    L.orc_env_info.argtypes = [C.c_void_p, _i32]
    L.orc_env_lanes.argtypes = [C.c_void_p, _f32, _f32, _i32, _i32, _i32]
    L.orc_env_demand.argtypes = [C.c_void_p, _u16, _i32, _u16]
    L.orc_env_set_demand.argtypes = [C.c_void_p, C.c_int, C.c_int, _u16, _i32, _u16]
    L.orc_env_enable_trace.argtypes = [C.c_void_p, C.c_int]
    L.orc_env_set_actuated.argtypes = [C.c_void_p, C.c_int]
    L.orc_env_trace.restype = C.c_int
    L.orc_env_trace.argtypes = [C.c_void_p, C.c_void_p]


class OracleEnv:
    """One replica of the grid microsimulation on the CPU (oracle_sim.c)."""

    def __init__(self, R, Cc, seed, cap=24, end_ms=2_500_000, period_ms=0, idm=None,
                 actuated=False):
        L = lib()
        if not hasattr(L, "_env_declared"):
            _declare_env(L)
            L._env_declared = True
        self.R, self.C, self.A, self.cap = R, Cc, R * Cc, cap
        self.idm = idm or idm_default()
        self.h = L.orc_env_create(R, Cc, cap, seed, end_ms, period_ms or 0, C.byref(self.idm))
        info = self.info()
        self.NL, self.nveh = int(info[0]), int(info[1])
        if actuated:
            L.orc_env_set_actuated(self.h, 1)

    def __del__(self):
        try:
            lib().orc_env_free(self.h)
        except Exception:
            pass

    def info(self):
        out = np.zeros(8, dtype=np.int32)
        lib().orc_env_info(self.h, out)
        return out

    def reset(self):
        lib().orc_env_reset(self.h)

    def step(self, actions, stride, t0, K, max_time):
        halt = np.zeros(self.A * 12, dtype=np.int32)
        ph = np.zeros(self.A, dtype=np.int32)
        ts = np.zeros(self.A, dtype=np.int32)
        done = np.zeros(1, dtype=np.uint8)
        a = None
        if actions is not None:
            a = np.ascontiguousarray(actions, dtype=np.int32)
        lib().orc_env_step(self.h, None if a is None else a.ctypes.data, stride, t0, K, max_time,
                           halt, ph, ts, done)
        return halt.reshape(self.A, 12), ph, ts, bool(done[0])

    def lanes(self):
        ns = self.NL * self.cap
        x, v = np.zeros(ns, np.float32), np.zeros(ns, np.float32)
        d = np.zeros(ns, np.int32)
        hd, cn = np.zeros(self.NL, np.int32), np.zeros(self.NL, np.int32)
        lib().orc_env_lanes(self.h, x, v, d, hd, cn)
        return x.reshape(self.NL, self.cap), v.reshape(self.NL, self.cap), d.reshape(self.NL, self.cap), hd, cn

    def set_demand(self, q_ids, q_off, vdst, period_ms):
        """Explicit departures (a loaded SUMO scenario); resets the replica."""
        q = np.ascontiguousarray(q_ids, np.uint16)
        lib().orc_env_set_demand(self.h, len(q), int(period_ms), q,
                                 np.ascontiguousarray(q_off, np.int32),
                                 np.ascontiguousarray(vdst, np.uint16))
        self.nveh = len(q)

    def enable_trace(self, max_events=1 << 20):
        """Record every edge entry (insertion or junction crossing) from now on."""
        lib().orc_env_enable_trace(self.h, int(max_events))
        self._max_trace = int(max_events)

    def trace(self):
        """[n, 2] int32 (vehicle id, simulator edge) in the order they happened."""
        n = lib().orc_env_trace(self.h, None)
        if n > self._max_trace:
            raise RuntimeError(f"trace overflow: {n} events > {self._max_trace}")
        out = np.zeros((n, 2), np.int32)
        lib().orc_env_trace(self.h, out.ctypes.data)
        return out

    def demand(self):
        q = np.zeros(self.nveh, np.uint16)
        off = np.zeros(4 * self.A + 1, np.int32)
        vd = np.zeros(self.nveh, np.uint16)
        lib().orc_env_demand(self.h, q, off, vd)
        return q, off, vd


# ---------------------------------------------------------------- learn
def _declare_learn(L):
    L.orc_qnet_nparams.restype = C.c_long
    L.orc_qnet_nparams.argtypes = [C.c_int, C.c_int, C.c_int]
    L.orc_qnet_forward.argtypes = [_f32, C.c_int, C.c_int, C.c_int, _f32, C.c_int, _f32,
                                   C.c_void_p, C.c_void_p]
    L.orc_learn.restype = C.c_float
    L.orc_learn.argtypes = [_f32, _f32, _f32, _f32, C.c_int, C.c_int, C.c_int, C.c_int, _f32, _i32,
                            _f32, _f32, _f32, _f32, C.c_void_p, C.c_int]


def _L():
    L = lib()
    if not hasattr(L, "_learn_declared"):
        _declare_learn(L)
        L._learn_declared = True
    return L


def qnet_nparams(H1=128, H2=128, NA=4):
    return int(_L().orc_qnet_nparams(H1, H2, NA))


def qnet_forward(p, x, H1=128, H2=128, NA=4):
    p = np.ascontiguousarray(p, np.float32)
    x = np.ascontiguousarray(x, np.float32)
    q = np.zeros((x.shape[0], NA), np.float32)
    _L().orc_qnet_forward(p, H1, H2, NA, x, x.shape[0], q, None, None)
    return q


def keras_adam_consts(t, lr=1e-3, b1=0.9, b2=0.999, eps=1e-7):
    """Keras-3 Adam constants for step t (1-based) computed in float32 ops."""
    f = np.float32
    b1p = np.power(f(b1), f(t), dtype=np.float32)
    b2p = np.power(f(b2), f(t), dtype=np.float32)
    alpha = f(f(lr) * np.sqrt(f(1) - b2p, dtype=np.float32)) / f(f(1) - b1p)
    return f(alpha), f(1 - b1), f(1 - b2), f(eps)


def learn(p, target, m, v, S, A, Rn, S2, Dn, t, gamma=0.99, lr=1e-3, H1=128, H2=128, NA=4,
          want_grad=False, loss_kind=0):
    """In-place Keras-semantics learn step on float32 numpy arrays; returns loss (and grad).
    loss_kind 0 = MSE (dqn_agent.py:352), 1 = Huber delta 1 (experimental/agent.py:99)."""
    alpha, c1, c2, eps = keras_adam_consts(t, lr)
    hyper = np.array([np.float32(gamma), alpha, c1, c2, eps], np.float32)
    grad = np.zeros(p.size, np.float32) if want_grad else None
    B = S.shape[0]
    loss = _L().orc_learn(p, np.ascontiguousarray(target, np.float32), m, v, H1, H2, NA, B,
                          np.ascontiguousarray(S, np.float32), np.ascontiguousarray(A, np.int32),
                          np.ascontiguousarray(Rn, np.float32), np.ascontiguousarray(S2, np.float32),
                          np.ascontiguousarray(Dn, np.float32), hyper,
                          None if grad is None else grad.ctypes.data, int(loss_kind))
    return (loss, grad) if want_grad else loss


def round_f16(x):
    """f32 -> IEEE half -> f32, round to nearest even."""
    return np.asarray(x, np.float32).astype(np.float16).astype(np.float32)


def round_bf16(x):
    """f32 -> bfloat16 -> f32, round to nearest even (finite inputs)."""
    u = np.ascontiguousarray(x, dtype=np.float32).view(np.uint32).astype(np.uint64)
    u = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16
    return u.astype(np.uint32).view(np.float32)


MIXED_ROUND = {"fp16": round_f16, "bf16": round_bf16}


def _mixed_split(w, rnd, H):
    sizes = [89 * H, H, H * H, H, H * 4, 4]
    offs = np.cumsum([0] + sizes)
    W1, b1, W2, b2, W3, b3 = (np.asarray(w[offs[i]:offs[i + 1]], np.float32) for i in range(6))
    return (rnd(W1.reshape(89, H)), rnd(b1), rnd(W2.reshape(H, H)), rnd(b2),
            rnd(W3.reshape(H, 4)), rnd(b3))


def _mixed_fwd(ws, X, rnd):
    def dense(x, W, b):
        return rnd(rnd(np.matmul(x, W, dtype=np.float32)) + b)
    W1, b1, W2, b2, W3, b3 = ws
    h1 = np.maximum(dense(X, W1, b1), 0)
    h2 = np.maximum(dense(h1, W2, b2), 0)
    return h1, h2, dense(h2, W3, b3)


def qnet_forward_mixed(p, x, precision="fp16", H=128):
    """The Keras Sequential forward under mixed_float16 / mixed_bfloat16 on
    Keras-order flat f32 weights: 16-bit Q [B, 4] (as f32 values); see learn_mixed."""
    rnd = MIXED_ROUND[precision]
    return _mixed_fwd(_mixed_split(p, rnd, H), rnd(np.asarray(x, np.float32)), rnd)[2]


def learn_mixed(p, target, m, v, S, A, Rn, S2, Dn, t, precision="fp16", gamma=0.99, lr=1e-3,
                H=128, loss_kind=0, round_grad=True, want_grad=False, w3_bwd=None):
    """DQNAgent.learn (dqn_agent.py:328-380) under Keras 3's mixed precision
    policy (train.py:61 sets mixed_float16; "bf16" = mixed_bfloat16), in numpy,
    on Keras-order flat f32 parameters (TEST INFRASTRUCTURE, the checker of the
    16-bit learn kernels).  In place on p, m, v; returns the f32 loss (and the
    f32-widened gradient with want_grad).

    Rounding points (rnd = round to the 16-bit compute type; every matmul is
    f32 products + f32 sums, rounded once; tests/golden/tf_shim.py states the
    Keras / TF sources):
      Dense:   z = rnd(rnd(x @ rnd(W)) + rnd(b)), h = relu(z)      (3 layers)
      Q (f16) -> argmax (first max) of online(S'); target(S')[a*] widened;
      y = Rn + (gamma (1 - d)) q_t  and  the MSE / Huber loss in f32;
      dQ = rnd(dL/dq) at the taken action (the gradient of tf.cast);
      dW = rnd(h_in^T @ dZ), db = rnd(sum_batch dZ), dh_in = rnd(dZ @ rnd(W)^T),
      dZ = dh * (h > 0);  Adam (Keras 3) in f32 on the widened gradients.
    round_grad=False keeps dW / db in f32 (the shared-network configuration
    C5 sums its per-agent gradients before any rounding).  w3_bwd [H, 4]
    replaces the W3 backprop multiplies dQ by (a test hook)."""
    rnd = MIXED_ROUND[precision]
    f32 = np.float32

    def split(w):
        return _mixed_split(w, rnd, H)

    def fwd(ws, X):
        return _mixed_fwd(ws, X, rnd)

    S, S2 = rnd(np.asarray(S, f32)), rnd(np.asarray(S2, f32))
    Rn, Dn = np.asarray(Rn, f32), np.asarray(Dn, f32)
    A = np.asarray(A, np.int64)
    B = S.shape[0]
    rows = np.arange(B)
    wo, wt = split(np.asarray(p, f32)), split(np.asarray(target, f32))
    a_star = fwd(wo, S2)[2].argmax(1)
    q_t = fwd(wt, S2)[2][rows, a_star]
    y = Rn + (f32(gamma) * (f32(1.0) - Dn)) * q_t
    h1, h2, q = fwd(wo, S)
    e = q[rows, A] - y
    if loss_kind == 1:
        ae = np.abs(e)
        loss = np.mean(np.where(ae <= 1, f32(0.5) * e * e, ae - f32(0.5)), dtype=f32)
        dq = np.where(ae <= 1, e, np.sign(e)).astype(f32) * f32(1.0 / B)
    else:
        loss = np.mean(e * e, dtype=f32)
        dq = f32(2.0) * e * f32(1.0 / B)
    DQ = np.zeros((B, 4), f32)
    DQ[rows, A] = rnd(dq)
    W1, b1, W2, b2, W3, b3 = wo
    gr = rnd if round_grad else (lambda x: np.asarray(x, f32))
    gW3, gb3 = gr(np.matmul(h2.T, DQ, dtype=f32)), gr(DQ.sum(0, dtype=f32))
    if w3_bwd is not None:
        W3 = rnd(np.asarray(w3_bwd, f32))
    dz2 = np.where(h2 > 0, rnd(np.matmul(DQ, W3.T, dtype=f32)), f32(0))
    gW2, gb2 = gr(np.matmul(h1.T, dz2, dtype=f32)), gr(dz2.sum(0, dtype=f32))
    dz1 = np.where(h1 > 0, rnd(np.matmul(dz2, W2.T, dtype=f32)), f32(0))
    gW1, gb1 = gr(np.matmul(S.T, dz1, dtype=f32)), gr(dz1.sum(0, dtype=f32))
    g = np.concatenate([gW1.ravel(), gb1, gW2.ravel(), gb2, gW3.ravel(), gb3]).astype(f32)
    alpha, c1, c2, eps = keras_adam_consts(t, lr)
    m += (g - m) * c1
    v += (g * g - v) * c2
    p -= (m * alpha) / (np.sqrt(v) + eps)
    return (f32(loss), g) if want_grad else f32(loss)


def keras_init(rng, H1=128, H2=128, NA=4):
    """HeNormal (truncated, stddev sqrt(2/fan_in)/0.8796) hidden kernels,
    GlorotUniform output kernel, zero biases (dqn_agent.py:160-181)."""
    def he(fi, fo):
        std = np.sqrt(2.0 / fi) / 0.87962566103423978
        w = rng.normal(0, std, size=(fi, fo))
        bad = np.abs(w) > 2 * std
        while bad.any():
            w[bad] = rng.normal(0, std, size=bad.sum())
            bad = np.abs(w) > 2 * std
        return w
    lim = np.sqrt(6.0 / (H2 + NA))
    parts = [he(89, H1), np.zeros(H1), he(H1, H2), np.zeros(H2),
             rng.uniform(-lim, lim, size=(H2, NA)), np.zeros(NA)]
    return np.concatenate([x.reshape(-1) for x in parts]).astype(np.float32)


# ---------------------------------------------------------------- CPU baseline loop
def train_loop(R, Cc, E, fill, steps, seed=0, threads=1):
    """The training loop body for E replicas in C (oracle_loop.c), OpenMP over
    replicas.  Returns (timed seconds, agent-env steps timed)."""
    L = lib()
    if not hasattr(L, "_loop_declared"):
        L.orc_train_loop.restype = C.c_double
        L.orc_train_loop.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_uint64,
                                     C.c_int, C.POINTER(C.c_long)]
        L._loop_declared = True
    n = C.c_long(0)
    el = L.orc_train_loop(R, Cc, E, fill, steps, seed, threads, C.byref(n))
    return el, n.value


# ---------------------------------------------------------------- the loop body, one replica
class OracleLoop:
    """src/scripts/train.py:188-310 for ONE env replica on the CPU oracle (TEST
    INFRASTRUCTURE): env step (oracle_sim.c), observe / reward from the pre-step
    local state, act on the replica's numpy stream (epsilon 1, A-1), remember
    into a per-agent deque of maxlen `cap`, then per agent in junction order
    random.sample on the replica's CPython stream, z-score and (learn=True) the
    fp32 learn of oracle_learn.c, with the hard target sync every `tuf` learns.
    Episode end (done: t >= max_time or no vehicle left, train.py:233-236)
    reloads the replica (train.py:190).  With learn=False the replay draws
    still run (they advance the stream exactly as the training loop does)."""

    def __init__(self, R, Cc, seed, cap=10000, tuf=500, weights=None, mode=0, max_time=2400,
                 learn=True, loss_kind=0, H=128, gamma=0.99, lr=1e-3, env=None, track_ties=False):
        self.R, self.C, self.A = R, Cc, R * Cc
        self.env = env or OracleEnv(R, Cc, seed)
        self.nps, self.pys = np_stream(seed), py_stream(seed)
        self.cap, self.tuf, self.mode, self.max_time = cap, tuf, mode, max_time
        self.learn, self.loss_kind, self.H, self.gamma, self.lr = learn, loss_kind, H, gamma, lr
        self.dq = [[] for _ in range(self.A)]
        if learn:
            self.params = np.array(weights, np.float32).reshape(self.A, -1).copy()
            self.target = self.params.copy()
            self.m = np.zeros_like(self.params)
            self.v = np.zeros_like(self.params)
        self.learn_steps = 0
        # track_ties: per learn and agent, the smallest relative gap between the
        # two largest online Q(S') of the batch -- below ~1e-6 the Double-DQN
        # argmax (dqn_agent.py:342) can go either way under another fp32
        # summation order, and two correct implementations part ways there
        self.track_ties, self.tie_gaps = track_ties, []
        self._reset()

    def _reset(self):
        A = self.A
        self.t = 0
        self.L = local_state(np.zeros((A, 12)), np.zeros(A), np.zeros(A), self.mode)
        self.obs = build_obs(self.R, self.C, self.L)

    def step(self):
        A = self.A
        acts = act(self.nps, A, 1.0)
        halt, ph, ts, done = self.env.step(acts, 3, self.t, 10, self.max_time)
        self.t += 10
        rew = reward(self.L)
        L2 = local_state(halt, ph, ts, self.mode)
        obs2 = build_obs(self.R, self.C, L2)
        for j in range(A):
            self.dq[j].append((self.obs[j].astype(np.int8), int(acts[j]), float(rew[j]),
                               obs2[j].astype(np.int8), float(done)))
            if len(self.dq[j]) > self.cap:
                self.dq[j].pop(0)
        out = {"actions": acts, "halt": halt, "phase": ph, "tspent": ts, "reward": rew,
               "obs": obs2, "done": done, "idx": None, "loss": None}
        n = len(self.dq[0])
        if n >= 128:
            idx = np.zeros((A, 128), np.int32)
            loss = np.zeros(A, np.float32)
            if self.learn:
                self.learn_steps += 1
            gaps = np.full(A, np.inf)
            for j in range(A):
                idx[j] = py_sample(self.pys, n, 128)
                if self.learn:
                    d = self.dq[j]
                    S = np.stack([d[i][0] for i in idx[j]]).astype(np.float32)
                    Aa = np.array([d[i][1] for i in idx[j]], np.int32)
                    Rn = zscore(np.array([d[i][2] for i in idx[j]]))
                    S2 = np.stack([d[i][3] for i in idx[j]]).astype(np.float32)
                    Dn = np.array([d[i][4] for i in idx[j]], np.float32)
                    if self.track_ties:
                        q = np.sort(qnet_forward(self.params[j], S2, self.H, self.H), axis=1)
                        gaps[j] = float(((q[:, -1] - q[:, -2]) / (np.abs(q[:, -1]) + 1e-30)).min())
                    loss[j] = learn(self.params[j], self.target[j], self.m[j], self.v[j], S, Aa, Rn,
                                    S2, Dn, self.learn_steps, gamma=self.gamma, lr=self.lr,
                                    H1=self.H, H2=self.H, loss_kind=self.loss_kind)
            if self.learn and self.track_ties:
                self.tie_gaps.append(gaps)
            if self.learn and self.learn_steps % self.tuf == 0:
                self.target = self.params.copy()
            out["idx"], out["loss"] = idx, (loss if self.learn else None)
        if done:
            self.env.reset()
            self._reset()
        else:
            self.L, self.obs = L2, obs2
        return out
