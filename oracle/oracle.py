"""ctypes binding of oracle/liboracle.so (TEST INFRASTRUCTURE ONLY)."""
import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def build():
    """Compile liboracle.so (gcc) if missing or stale."""
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
