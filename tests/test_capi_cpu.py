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


def test_python_signatures_cover_header(lib):
    from dmdqn_amd import _lib, agent, env  # noqa: F401  (agent / env register theirs)
    declared = set(_declared()) - {"dmdqn_last_error", "dmdqn_version"}
    assert declared <= set(_lib.SIGNATURES), sorted(declared - set(_lib.SIGNATURES))


def test_version_and_error_string(lib):
    assert lib.dmdqn_version() >= 1
    assert isinstance(lib.dmdqn_last_error(), bytes)


def test_host_side_argument_check_without_gpu(lib):
    """Argument validation happens on the host before any launch."""
    rc = lib.dmdqn_act(None, 0, 0, ctypes.c_double(1.0), 4, None, None, None)
    assert rc == -1
    assert b"dmdqn_act" in lib.dmdqn_last_error()
