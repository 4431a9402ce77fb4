"""Tuning aid: build libdmdqn_hip.so of an earlier git revision (its own csrc/,
include/ and build flags) into exp/libdmdqn_hip_<name>.so, so that a learn
kernel of that revision can be timed beside HEAD's on one box
(tools/ab_learn_lib.py, which calls dmdqn_learn through the C ABI -- the
dmdqn_learn_args of every revision since round 2 is a prefix of HEAD's).
usage: python tools/build_rev.py <rev> <name> [-DFOO ...]
  Extra arguments are appended to every hipcc line (e.g. -fslp-vectorize).
Output goes under exp/ (git-ignored; travels to the GPU box)."""
import concurrent.futures as cf
import importlib.util
import io
import os
import subprocess
import sys
import tarfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    rev, name, extra = sys.argv[1], sys.argv[2], sys.argv[3:]
    dst = os.path.join(ROOT, "exp", f"rev_{name}")
    os.makedirs(dst, exist_ok=True)
    tar = subprocess.run(["git", "-C", ROOT, "archive", rev, "dmdqn_amd/csrc", "dmdqn_amd/build.py",
                          "include"], check=True, capture_output=True).stdout
    tarfile.open(fileobj=io.BytesIO(tar)).extractall(dst)
    spec = importlib.util.spec_from_file_location(f"build_{name}",
                                                  os.path.join(dst, "dmdqn_amd", "build.py"))
    B = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(B)
    srcs = B._sources()

    def compile_one(src):
        base = os.path.basename(src)
        obj = os.path.join(dst, base + ".o")
        flags = B.COMMON + B.PER_FILE.get(base, B.DEFAULT_FP) + extra
        lang = ["-x", "hip"] if base.endswith(".hip") else []
        subprocess.run([B.HIPCC] + flags + lang + ["-c", src, "-o", obj], check=True)
        return obj

    with cf.ThreadPoolExecutor(max_workers=8) as ex:
        objs = list(ex.map(compile_one, srcs))
    # dmdqn_source_digest(), tagged with the revision: _lib.load() refuses it
    # as stale unless DMDQN_ALLOW_FOREIGN_LIB=1 (tools/ab_swap.sh sets it)
    dsrc = os.path.join(dst, "source_digest.cpp")
    with open(dsrc, "w") as f:
        f.write(f'extern "C" const char *dmdqn_source_digest(void) {{ return "rev-{rev}"; }}\n')
    subprocess.run(["g++", "-c", "-fPIC", dsrc, "-o", dsrc + ".o"], check=True)
    objs.append(dsrc + ".o")
    so = os.path.join(ROOT, "exp", f"libdmdqn_hip_{name}.so")
    subprocess.run([B.HIPCC, "-shared", "-fPIC", f"--offload-arch={B.ARCH}", "-o", so] + objs,
                   check=True)
    print(so)


if __name__ == "__main__":
    main()
