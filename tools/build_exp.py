"""Tuning aid: build experiment copies of libdmdqn_hip.so that differ from the
product build only in learn_shared.hip, compiled with extra -D switches, so
several variants of the shared-learn kernels can be timed in one GPU call
(tools/stamp_shared.py <lib>).  Output: exp/libdmdqn_hip_<name>.so (git-ignored,
travels with the snapshot).
usage: python tools/build_exp.py <name> [--src sim.hip] [--from FILE] [-DFOO=1 ...]
(--src: the one source rebuilt with the switches; default learn_shared.hip;
--from: compile FILE in its place, e.g. an earlier revision from `git show`)"""
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dmdqn_amd import build as B  # noqa: E402


def main():
    name, flags = sys.argv[1], sys.argv[2:]
    srcname = "learn_shared.hip"
    if "--src" in flags:
        k = flags.index("--src")
        srcname = flags[k + 1]
        flags = flags[:k] + flags[k + 2:]
    alt = None
    if "--from" in flags:
        k = flags.index("--from")
        alt = flags[k + 1]
        flags = flags[:k] + flags[k + 2:]
    B.build(verbose=False)  # the product objects this links against
    root = os.path.dirname(B.HERE)
    out = os.path.join(root, "exp")
    os.makedirs(out, exist_ok=True)
    src = os.path.abspath(alt) if alt else os.path.join(B.CSRC, srcname)
    obj = os.path.join(out, f"{srcname.split('.')[0]}_{name}.o")
    cmd = ([B.HIPCC] + B.COMMON + B.PER_FILE.get(srcname, B.DEFAULT_FP) + flags + ["-I", B.CSRC] +
           ["-x", "hip", "-c", src, "-o", obj])
    subprocess.run(cmd, check=True)
    objs = [os.path.join(B.objdir(), os.path.basename(s) + ".o") for s in B._sources()
            if os.path.basename(s) != srcname] + [obj]
    # the tree's source digest (dmdqn_source_digest): the variant is this tree
    # plus switches, and loads only under DMDQN_ALLOW_FOREIGN_LIB=1 when swapped
    # in (tools/ab_swap.sh) if its -D switches change the code
    objs.append(B._digest_object("", B.tree_digest())[0])
    so = os.path.join(out, f"libdmdqn_hip_{name}.so")
    subprocess.run([B.HIPCC, "-shared", "-fPIC", f"--offload-arch={B.ARCH}", "-o", so] + objs,
                   check=True)
    print(so)


if __name__ == "__main__":
    main()
