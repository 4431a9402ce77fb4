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
