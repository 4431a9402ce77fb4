"""The C-ABI library loads and exports every entry point include/dmdqn.h declares
(no compute calls: runs without a GPU)."""
import ctypes
import os
import re

import pytest

from conftest import ROOT


def _declared():
    names = set()
    for h in os.listdir(os.path.join(ROOT, "include")):
        if h.endswith(".h"):
            txt = open(os.path.join(ROOT, "include", h)).read()
            names |= set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(dmdqn_\w+)\s*\(", txt, re.M))
    return sorted(names)


@pytest.fixture(scope="module")
def lib():
    from dmdqn_amd import build
    build.build(verbose=False)
    from dmdqn_amd import _lib
    return _lib.load()


def test_header_declares_entry_points():
    names = _declared()
    assert "dmdqn_act" in names and "dmdqn_observe" in names and len(names) >= 8


def test_all_declared_symbols_exported(lib):
    missing = [n for n in _declared() if not hasattr(lib, n)]
    assert not missing, f"symbols declared in include/*.h but not exported: {missing}"


def test_python_bindings_cover_header(lib):
    """Every compute entry point is wrapped by a torch.ops.dmdqn operator (the
    product path) and every entry point but the sim's struct calls has a
    ctypes signature (the C-ABI tests' path)."""
    from dmdqn_amd import _lib, agent, env, ops  # noqa: F401  (agent registers its signatures)
    declared = set(_declared()) - {"dmdqn_last_error", "dmdqn_version", "dmdqn_debug_status",
                                   "dmdqn_debug_build", "dmdqn_learn_shared_work_bytes",
                                   "dmdqn_learn_shared_lds_bytes", "dmdqn_source_digest"}
    host_only = {"dmdqn_stream_create_cumask", "dmdqn_stream_destroy", "dmdqn_set_option",
                 "dmdqn_get_option", "dmdqn_timing_event_create", "dmdqn_event_record",
                 "dmdqn_event_synchronize", "dmdqn_event_elapsed_ms", "dmdqn_event_destroy",
                 "dmdqn_order_event_create", "dmdqn_stream_wait_event",
                 "dmdqn_stream_probe",  # bench.py's HBM probe, not on the path
                 "dmdqn_device_lds_per_cu"}  # the trainer's sampler budget
    assert declared - host_only <= set(ops.ENTRY_POINTS), sorted(declared - host_only -
                                                                 set(ops.ENTRY_POINTS))
    ctypes_only = declared - {"dmdqn_sim_reset", "dmdqn_sim_reset_envs", "dmdqn_sim_step",
                              "dmdqn_env_step"}
    assert ctypes_only <= set(_lib.SIGNATURES), sorted(ctypes_only - set(_lib.SIGNATURES))


def test_torch_ops_registered_without_gpu(lib):
    """libdmdqn_torch.so loads on a CPU-only host and registers every op with
    a schema; a CPU tensor is refused (no CPU kernel, no fallback)."""
    import torch
    from dmdqn_amd import ops
    D = ops.load()
    for name in set(ops.ENTRY_POINTS.values()):
        assert getattr(D, name).default._schema.name == f"dmdqn::{name}"
    with pytest.raises(NotImplementedError):
        D.mt_seed(torch.zeros((1, 625), dtype=torch.int32), torch.zeros(1, dtype=torch.int64), "np")


def test_version_and_error_string(lib):
    # 4: dmdqn_source_digest, dmdqn_device_lds_per_cu (3: dmdqn_adam_slabs;
    # cap = physical ring slots; include/dmdqn.h)
    assert lib.dmdqn_version() == 4
    import ctypes
    lib.dmdqn_learn_shared_work_bytes.restype = ctypes.c_size_t
    assert lib.dmdqn_learn_shared_work_bytes(16384) == 16384 * 128 * 5
    from dmdqn_amd import _lib
    # the S' pass's workgroup: both nets (2 x 58,896 B) + 8 waves' scratch
    assert _lib.learn_shared_lds_bytes() == 2 * 58896 + 8 * 128 * 20
    assert isinstance(lib.dmdqn_last_error(), bytes)


def test_host_side_argument_check_without_gpu(lib):
    """Argument validation happens on the host before any launch."""
    rc = lib.dmdqn_act(None, 0, 0, ctypes.c_double(1.0), 4, None, None, None)
    assert rc == -1
    assert b"dmdqn_act" in lib.dmdqn_last_error()


def test_env_step_argument_check_without_gpu(lib):
    """dmdqn_env_step (the fused act / sim / observe / store launch) refuses a
    missing fuse block, a missing sim and incomplete act arguments on the host."""
    rc = lib.dmdqn_env_step(None, None, None, 3, 0, 10, 2400, None, None, None, None, None)
    assert rc == -1 and b"null fuse" in lib.dmdqn_last_error()
    fuse = ctypes.create_string_buffer(512)  # all-zero dmdqn_env_fuse
    rc = lib.dmdqn_env_step(None, None, fuse, 3, 0, 10, 2400, None, None, None, None, None)
    assert rc == -1 and b"junctions" in lib.dmdqn_last_error()


def test_replay_sample_lds_limit_checked_on_host(lib):
    """The sampler's LDS plan (MT state + n-bit bitmap + first-lane table) is
    checked before launch: an n whose bitmap alone exceeds LDS is refused."""
    dummy = ctypes.c_void_p(16)  # never dereferenced: the check fails first
    rc = lib.dmdqn_replay_sample(dummy, 1, 1, 2_000_000, 128, dummy, None)
    assert rc == -1
    assert b"too large for LDS" in lib.dmdqn_last_error()
    rc = lib.dmdqn_replay_sample(dummy, 1, 1, 100, 128, dummy, None)  # k > n
    assert rc == -1 and b"1 <= k <= n" in lib.dmdqn_last_error()


def test_debug_build_exports_and_reports_its_variant():
    """Both library variants export the debug entry points; only the
    debug-bounds build says so (no GPU call: the flags are not read here)."""
    import ctypes
    from dmdqn_amd import build
    build.build(verbose=False, variant="debug")
    for variant, want in (("", 0), ("debug", 1)):
        lib = ctypes.CDLL(os.path.join(build.LIBDIR, build.libname(variant)))
        assert lib.dmdqn_debug_build() == want
        assert hasattr(lib, "dmdqn_debug_status")


def test_learn_args_layout_matches_header(tmp_path):
    """agent.CLearn (the ctypes mirror the C-ABI tests pass) has the size and
    field offsets gcc gives include/dmdqn.h's dmdqn_learn_args."""
    import ctypes
    import subprocess
    from dmdqn_amd.agent import CLearn
    fields = [f for f, _ in CLearn._fields_]
    src = tmp_path / "lay.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "dmdqn.h"\nint main(void){'
                   'printf("%zu", sizeof(dmdqn_learn_args));' +
                   "".join(f'printf(" %zu", offsetof(dmdqn_learn_args, {f}));' for f in fields) +
                   "return 0;}\n")
    exe = tmp_path / "lay"
    inc = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include")
    subprocess.run(["gcc", f"-I{inc}", str(src), "-o", str(exe)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True,
                                          check=True).stdout.split()]
    assert got[0] == ctypes.sizeof(CLearn)
    assert got[1:] == [getattr(CLearn, f).offset for f in fields]


def test_options_read_once_not_per_launch(lib):
    """The launchers' test / A-B hooks (DMDQN_OPT_*) are read from the
    environment once at load (capi.cpp) and set through dmdqn_set_option: no
    other source calls getenv, so a stray variable cannot switch a launch."""
    csrc = os.path.join(ROOT, "dmdqn_amd", "csrc")
    for f in os.listdir(csrc):
        txt = open(os.path.join(csrc, f)).read()
        if f != "capi.cpp":
            assert "getenv" not in txt, f
    from dmdqn_amd import _lib
    with _lib.option("sim_path", "reg"):
        assert lib.dmdqn_get_option(0) == 1
        with _lib.option("sample_tlog", 3):
            assert lib.dmdqn_get_option(1) == 3
        assert lib.dmdqn_get_option(1) == 32
    assert lib.dmdqn_get_option(0) == 0
    assert lib.dmdqn_set_option(0, 7) == -1 and lib.dmdqn_set_option(5, 0) == -1
    assert lib.dmdqn_set_option(1, 21) == -1 and lib.dmdqn_get_option(1) == 32
