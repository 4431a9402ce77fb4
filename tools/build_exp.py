"""Tuning aid: build experiment copies of libdmdqn_hip.so that differ from the
product build only in learn_shared.hip, compiled with extra -D switches, so
several variants of the shared-learn kernels can be timed in one GPU call
(tools/stamp_shared.py <lib>).  Output: exp/libdmdqn_hip_<name>.so (git-ignored,
travels with the snapshot).
usage: python tools/build_exp.py <name> [-DFOO=1 ...]"""
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dmdqn_amd import build as B  # noqa: E402


def main():
    name, flags = sys.argv[1], sys.argv[2:]
    B.build(verbose=False)  # the product objects this links against
    root = os.path.dirname(B.HERE)
    out = os.path.join(root, "exp")
    os.makedirs(out, exist_ok=True)
    src = os.path.join(B.CSRC, "learn_shared.hip")
    obj = os.path.join(out, f"learn_shared_{name}.o")
    cmd = [B.HIPCC] + B.COMMON + B.DEFAULT_FP + flags + ["-x", "hip", "-c", src, "-o", obj]
    subprocess.run(cmd, check=True)
    objs = [os.path.join(B.objdir(), os.path.basename(s) + ".o") for s in B._sources()
            if os.path.basename(s) != "learn_shared.hip"] + [obj]
    so = os.path.join(out, f"libdmdqn_hip_{name}.so")
    subprocess.run([B.HIPCC, "-shared", "-fPIC", f"--offload-arch={B.ARCH}", "-o", so] + objs,
                   check=True)
    print(so)


if __name__ == "__main__":
    main()
