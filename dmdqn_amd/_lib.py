"""ctypes binding of libdmdqn_hip.so (the C ABI declared in include/dmdqn.h).

The product path calls the HIP library only; if the library is missing or a
call fails, it raises -- there is no CPU fallback.
"""
import contextlib
import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# DMDQN_VARIANT=debug loads the debug-bounds build (libdmdqn_hip_debug.so and
# its operator library): kernels check the indices they derive (common.hpp)
VARIANT = os.environ.get("DMDQN_VARIANT", "")
if VARIANT not in ("", "debug", "prof", "exp"):
    raise ValueError(f"DMDQN_VARIANT must be '', 'debug', 'prof' or 'exp', got {VARIANT!r}")
_SUFFIX = f"_{VARIANT}" if VARIANT else ""
LIB_PATH = os.path.join(_HERE, "lib", f"libdmdqn_hip{_SUFFIX}.so")
_LIB = None

vp, i32, u32, u64, f64 = C.c_void_p, C.c_int, C.c_uint32, C.c_uint64, C.c_double

# name -> argtypes (all return int status)
SIGNATURES = {
    "dmdqn_mt_seed_np": [vp, vp, i32, vp],
    "dmdqn_mt_seed_py": [vp, vp, i32, vp],
    "dmdqn_mt_draw_u32": [vp, i32, i32, vp, vp],
    "dmdqn_act": [vp, i32, i32, f64, i32, vp, vp, vp],
    "dmdqn_act_uniform": [vp, i32, i32, i32, vp, vp],
    "dmdqn_observe": [i32, i32, i32, vp, vp, vp, i32, vp, vp, vp, vp, vp],
    "dmdqn_replay_store": [i32, i32, i32, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp],
    "dmdqn_replay_sample": [vp, i32, i32, i32, i32, vp, vp],
    "dmdqn_replay_sample_budget": [vp, i32, i32, i32, i32, C.c_size_t, vp, vp],
    "dmdqn_replay_store_f32": [i32, i32, i32, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp],
    "dmdqn_replay_gather_f32": [vp, vp, vp, i32, i32, i32, i32, vp, vp, vp],
    "dmdqn_stream_create_cumask": [u32, vp, vp],
    "dmdqn_stream_destroy": [vp],
    "dmdqn_set_option": [i32, i32],
    "dmdqn_get_option": [i32],
    "dmdqn_timing_event_create": [vp],
    "dmdqn_order_event_create": [vp],
    "dmdqn_stream_wait_event": [vp, vp],
    "dmdqn_event_record": [vp, vp],
    "dmdqn_event_synchronize": [vp],
    "dmdqn_event_elapsed_ms": [vp, vp, vp],
    "dmdqn_event_destroy": [vp],
    "dmdqn_stream_probe": [vp, vp, C.c_size_t, i32, vp],
    "dmdqn_device_lds_per_cu": [i32, vp],
}


class DmdqnError(RuntimeError):
    pass


def register(sigs):
    """Add entry-point signatures (modules that define the ctypes structs call
    this); applied at once if the library is already loaded."""
    SIGNATURES.update(sigs)
    if _LIB is not None:
        _apply(_LIB, sigs)


def _apply(lib, sigs):
    for name, args in sigs.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = C.c_int


def tree_digest(root=None):
    """The digest of the sources in this tree (build.tree_digest)."""
    from .build import tree_digest as td
    return td(root)


def verify_digest(lib, what, root=None, symbol="dmdqn_source_digest"):
    """Raise DmdqnError unless the library `lib` (its path in `what`) was
    built from the sources of this tree: the digest it embeds at build time
    (include/dmdqn.h dmdqn_source_digest) against build.tree_digest().  A
    prebuilt library that no longer matches its sources -- a kernel edited
    after the build, a library from another revision -- never runs as the
    current code.  Returns the digest.  DMDQN_ALLOW_FOREIGN_LIB=1 (same-box
    A/B of another revision's library, tools/ab_swap.sh) turns the refusal
    into a warning and records it in LIB_DIGEST_MATCHES (bench.py prints it)."""
    fn = getattr(lib, symbol, None)
    if fn is None:
        raise DmdqnError(f"{what} has no {symbol}(): built before round 6; rebuild with "
                         "`python -m dmdqn_amd.build`")
    fn.restype, fn.argtypes = C.c_char_p, []
    built = fn().decode()
    tree = tree_digest(root)
    global LIB_DIGEST_MATCHES
    if built != tree:
        if os.environ.get("DMDQN_ALLOW_FOREIGN_LIB") == "1":
            import warnings
            warnings.warn(f"{what}: digest {built} != tree {tree} (DMDQN_ALLOW_FOREIGN_LIB=1)")
            LIB_DIGEST_MATCHES = False
            return built
        raise DmdqnError(f"{what} is stale: built from sources with digest {built}, this tree's "
                         f"is {tree} -- rebuild with `python -m dmdqn_amd.build`")
    return built


LIB_DIGEST = None  # the loaded library's source digest (== the tree's)
LIB_DIGEST_MATCHES = True  # False only under DMDQN_ALLOW_FOREIGN_LIB=1 with another build


def load(path=None):
    """Load the HIP library (raises if it is absent or stale: no fallback path)."""
    global _LIB, LIB_DIGEST
    if _LIB is not None:
        return _LIB
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise DmdqnError(f"{p} not found: build it with `python -m dmdqn_amd.build` "
                         "(the HIP path has no CPU fallback)")
    lib = C.CDLL(p)
    LIB_DIGEST = verify_digest(lib, p)
    lib.dmdqn_last_error.restype = C.c_char_p
    lib.dmdqn_last_error.argtypes = []
    lib.dmdqn_version.restype = C.c_int
    lib.dmdqn_debug_status.restype = C.c_int
    lib.dmdqn_debug_status.argtypes = []
    lib.dmdqn_debug_build.restype = C.c_int
    lib.dmdqn_debug_build.argtypes = []
    lib.dmdqn_learn_shared_lds_bytes.restype = C.c_size_t
    lib.dmdqn_learn_shared_lds_bytes.argtypes = []
    _apply(lib, SIGNATURES)
    _LIB = lib
    return lib


def device_lds_per_cu(device=None):
    """LDS bytes of one CU of `device` (dmdqn_device_lds_per_cu)."""
    import torch
    d = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    idx = d.index if d.index is not None else torch.cuda.current_device()
    out = C.c_size_t()
    call("dmdqn_device_lds_per_cu", idx, C.byref(out))
    return int(out.value)


def learn_shared_lds_bytes():
    """LDS of one workgroup of the shared learn's S' pass (include/dmdqn.h)."""
    return int(load().dmdqn_learn_shared_lds_bytes())


def call(name, *args):
    lib = load()
    rc = getattr(lib, name)(*args)
    if rc != 0:
        raise DmdqnError(f"{name} failed (rc={rc}): {lib.dmdqn_last_error().decode()}")
    return rc


# include/dmdqn.h DMDQN_OPT_*: the launchers' test / A-B hooks, read from the
# environment once at library load and changed only through set_option
OPTIONS = {"sim_path": (0, {"auto": 0, "reg": 1, "lds": 2, "global": 3}),
           "sample_tlog": (1, {None: 32})}


def set_option(name, value):
    """Set a run-time option (sim_path: auto | reg | lds | global; sample_tlog:
    0..20 or None = no cap); returns the previous value in the same form."""
    which, names = OPTIONS[name]
    inv = {v: k for k, v in names.items()}
    lib = load()
    old = lib.dmdqn_get_option(which)
    call("dmdqn_set_option", which, names.get(value, value))
    return inv.get(old, old)


@contextlib.contextmanager
def option(name, value):
    """set_option for the duration of a with-block."""
    old = set_option(name, value)
    try:
        yield
    finally:
        set_option(name, old)


DEBUG_BITS = {1: "sim ring slot", 2: "sim route leaves the grid", 4: "replay index >= n",
              8: "learn deque position >= cap", 16: "stored action >= 4"}


def debug_check():
    """Debug-bounds build: wait for the device, raise if a kernel recorded an
    out-of-range index since the last check (the flags are cleared).  A no-op
    in the product build."""
    lib = load()
    if not lib.dmdqn_debug_build():
        return
    import torch
    torch.cuda.synchronize()
    v = lib.dmdqn_debug_status()
    if v != 0:
        what = "HIP error reading the flags" if v < 0 else ", ".join(
            n for b, n in DEBUG_BITS.items() if v & b)
        raise DmdqnError(f"debug-bounds check failed ({v}): {what}")


def ptr(t):
    """Device pointer of a tensor (or None -> NULL)."""
    if t is None:
        return None
    return C.c_void_p(t.data_ptr())


def stream_of(device=None):
    import torch
    return C.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def cu_masked_stream(cus, device=None):
    """A torch ExternalStream whose kernels run only on the CU indices `cus`
    (dmdqn_stream_create_cumask).  The stream lives until interpreter exit."""
    import torch
    cus = sorted(set(int(c) for c in cus))
    if not cus or cus[0] < 0:
        raise ValueError("cu_masked_stream: need a non-empty set of CU indices")
    words = cus[-1] // 32 + 1
    mask = (C.c_uint32 * words)()
    for c in cus:
        mask[c // 32] |= 1 << (c % 32)
    out = C.c_void_p()
    call("dmdqn_stream_create_cumask", words, mask, C.byref(out))
    if not _CU_STREAMS:
        import atexit
        atexit.register(_destroy_cu_streams)
    _CU_STREAMS.append(out.value)
    return torch.cuda.ExternalStream(out.value, device=device)


_CU_STREAMS = []


def _destroy_cu_streams():
    """Destroy the CU-masked streams at interpreter exit, after their work,
    before the HIP runtime's own teardown (left to it, the teardown crashed
    under rocprofv3 once the tool had finalized)."""
    import torch
    try:
        torch.cuda.synchronize()
    except Exception:  # noqa: BLE001 -- exiting anyway; still release the streams
        pass
    while _CU_STREAMS:
        load().dmdqn_stream_destroy(C.c_void_p(_CU_STREAMS.pop()))


class TimingEvent:
    """A HIP timing event without the system-scope fence
    (dmdqn_timing_event_create): recording it between two kernels costs no
    cache write-back.  For timing only (bench.py's per-learn events), never
    for ordering streams."""

    def __init__(self):
        out = C.c_void_p()
        call("dmdqn_timing_event_create", C.byref(out))
        self._ev = out.value
        self._lib = load()

    def record(self, stream):
        call("dmdqn_event_record", C.c_void_p(self._ev), C.c_void_p(stream.cuda_stream))

    def synchronize(self):
        call("dmdqn_event_synchronize", C.c_void_p(self._ev))

    def elapsed_time(self, end):
        """ms from this event's record to end's (both complete)."""
        ms = C.c_float()
        call("dmdqn_event_elapsed_ms", C.c_void_p(self._ev), C.c_void_p(end._ev), C.byref(ms))
        return ms.value

    def __del__(self):
        ev, self._ev = getattr(self, "_ev", None), None
        if ev:
            try:
                self._lib.dmdqn_event_destroy(C.c_void_p(ev))
            except Exception:  # noqa: BLE001 -- interpreter shutdown
                pass


class OrderEvent:
    """An ordering-only HIP event (dmdqn_order_event_create): a stream that
    waits on it starts after the recorded work completed, without that work's
    writes being released to it -- write-after-read ordering only (the
    trainer's side stream may overwrite ring slots once a learn has read
    them), never a data hand-over.  Recording it between dependent kernels
    costs no cache write-back."""

    def __init__(self):
        out = C.c_void_p()
        call("dmdqn_order_event_create", C.byref(out))
        self._ev = out.value
        self._lib = load()

    def record(self, stream):
        call("dmdqn_event_record", C.c_void_p(self._ev), C.c_void_p(stream.cuda_stream))

    def wait(self, stream):
        """Make `stream` wait for the last record."""
        call("dmdqn_stream_wait_event", C.c_void_p(stream.cuda_stream), C.c_void_p(self._ev))

    def synchronize(self):
        call("dmdqn_event_synchronize", C.c_void_p(self._ev))

    def __del__(self):
        ev, self._ev = getattr(self, "_ev", None), None
        if ev:
            try:
                self._lib.dmdqn_event_destroy(C.c_void_p(ev))
            except Exception:  # noqa: BLE001 -- interpreter shutdown
                pass
