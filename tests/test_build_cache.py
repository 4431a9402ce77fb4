"""dmdqn_amd.build's object cache: an object is reused only when it is newer
than its sources AND was built with the same flags, so an experiment build
(DMDQN_EXTRA_FLAGS=-D...) never leaves its objects behind for the next plain
build.  hipcc is mocked: no compiler or GPU is needed."""
import os
import subprocess

from dmdqn_amd import build


def _fake_hipcc(calls):
    def run(cmd, capture_output=True, text=True):
        calls.append(cmd)
        with open(cmd[cmd.index("-o") + 1], "w") as f:
            f.write("obj")
        return subprocess.CompletedProcess(cmd, 0, "", "")
    return run


def test_object_rebuilt_when_flags_change(tmp_path, monkeypatch):
    src = tmp_path / "k.hip"
    src.write_text("// kernel\n")
    os.utime(src, (1_000_000, 1_000_000))
    calls = []
    monkeypatch.setattr(build, "objdir", lambda variant="": str(tmp_path))
    monkeypatch.setattr(build, "_headers", lambda: [])
    monkeypatch.setattr(build.subprocess, "run", _fake_hipcc(calls))

    monkeypatch.setattr(build, "EXTRA", ["-DEXPERIMENT"])
    assert build._compile(str(src), False)[1] is True
    assert "-DEXPERIMENT" in calls[-1]

    # plain build after the experiment: flags differ, so it must recompile
    monkeypatch.setattr(build, "EXTRA", [])
    assert build._compile(str(src), False)[1] is True
    assert "-DEXPERIMENT" not in calls[-1]

    # same flags, object newer than the source: reused
    n = len(calls)
    assert build._compile(str(src), False)[1] is False
    assert len(calls) == n

    # a touched source is rebuilt even with the same flags
    os.utime(src, None)
    obj = tmp_path / "k.hip.o"
    os.utime(obj, (1_000_001, 1_000_001))
    assert build._compile(str(src), False)[1] is True


def test_missing_flag_stamp_forces_rebuild(tmp_path, monkeypatch):
    src = tmp_path / "k.hip"
    src.write_text("// kernel\n")
    os.utime(src, (1_000_000, 1_000_000))
    (tmp_path / "k.hip.o").write_text("old object, built before stamps existed")
    calls = []
    monkeypatch.setattr(build, "objdir", lambda variant="": str(tmp_path))
    monkeypatch.setattr(build, "_headers", lambda: [])
    monkeypatch.setattr(build, "EXTRA", [])
    monkeypatch.setattr(build.subprocess, "run", _fake_hipcc(calls))
    assert build._compile(str(src), False)[1] is True
    assert (tmp_path / "k.hip.o.flags").read_text() == " ".join(
        build.COMMON + build.DEFAULT_FP)


# ------------------------------------------------------------ source digest
def _tree_copy(tmp_path):
    """A copy of the sources the libraries are built from, laid out as in the
    repository (dmdqn_amd/{csrc,torch_ext}, include/)."""
    import shutil
    pkg = tmp_path / "dmdqn_amd"
    for d in ("csrc", "torch_ext"):
        shutil.copytree(os.path.join(build.HERE, d), pkg / d)
    shutil.copytree(os.path.join(build.HERE, "..", "include"), tmp_path / "include")
    return str(pkg)


def test_shipped_library_matches_tree():
    """The built libraries embed the digest of the sources they were built
    from (dmdqn_source_digest), and it is this tree's: load() accepts them."""
    from dmdqn_amd import _lib, ops
    _lib.load()
    assert _lib.LIB_DIGEST == build.tree_digest() and _lib.LIB_DIGEST_MATCHES
    ops.load()


def test_stale_library_refused(tmp_path, monkeypatch):
    """Touching a kernel source (here: one comment line in a copy of the tree)
    changes the tree digest, and the library built before it is refused with
    a message naming the rebuild command."""
    import ctypes
    import pytest
    from dmdqn_amd import _lib
    _lib.load()
    lib = ctypes.CDLL(_lib.LIB_PATH)
    root = _tree_copy(tmp_path)
    assert _lib.verify_digest(lib, "libdmdqn_hip.so", root=root) == build.tree_digest()
    with open(os.path.join(root, "csrc", "learn_h16.hpp"), "a") as f:
        f.write("// edited after the build\n")
    assert build.tree_digest(root) != build.tree_digest()
    monkeypatch.delenv("DMDQN_ALLOW_FOREIGN_LIB", raising=False)
    with pytest.raises(_lib.DmdqnError, match=r"stale.*python -m dmdqn_amd\.build"):
        _lib.verify_digest(lib, "libdmdqn_hip.so", root=root)
    # the operator library carries the same digest
    tl = ctypes.CDLL(os.path.join(os.path.dirname(_lib.LIB_PATH), "libdmdqn_torch.so"))
    with pytest.raises(_lib.DmdqnError, match="stale"):
        _lib.verify_digest(tl, "libdmdqn_torch.so", root=root, symbol="dmdqn_torch_source_digest")


def test_digest_covers_every_source():
    """Every kernel, header, C-ABI and operator source is in the digest."""
    names = {os.path.basename(p) for p in build.tree_files()}
    for d, ext in (("csrc", (".hip", ".hpp", ".cpp")), ("torch_ext", (".cpp",))):
        for f in os.listdir(os.path.join(build.HERE, d)):
            if f.endswith(ext):
                assert f in names, f
    assert "dmdqn.h" in names
