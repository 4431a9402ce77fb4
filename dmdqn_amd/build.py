"""Build libdmdqn_hip.so (all HIP kernels + the C ABI) for gfx950 with hipcc.

The library is built in-tree (dmdqn_amd/lib/) so it travels to the GPU box with
the repository snapshot.  Usage:  python -m dmdqn_amd.build [--force]
"""
import concurrent.futures as cf
import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIBDIR = os.path.join(HERE, "lib")
# variants: "" (the product build) and "debug" (-DDMDQN_DEBUG_BOUNDS: kernels
# check and clamp the indices they derive, dmdqn_debug_status reports them)
# ("prof": the sim's per-pass timers, tools/sim_profile.py; built on demand)
# ("exp": an A/B build whose only flags are DMDQN_EXTRA_FLAGS; loaded with
# DMDQN_VARIANT=exp through the torch operators like the product library)
VARIANT_FLAGS = {"": [], "debug": ["-DDMDQN_DEBUG_BOUNDS"], "prof": ["-DDMDQN_SIM_PROFILE"],
                 "exp": []}


def _suffix(variant):
    return f"_{variant}" if variant else ""


def objdir(variant=""):
    return os.path.join(LIBDIR, "obj" + _suffix(variant))


def libname(variant=""):
    return f"libdmdqn_hip{_suffix(variant)}.so"


LIBNAME = libname()
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("DMDQN_ARCH", "gfx950")

# Exact-arithmetic kernels (RNG, observe, sim, replay) must not contract a*b+c
# into an fma: the oracle (gcc, -ffp-contract=off) computes the same IEEE
# sequence.  The learn kernel is tolerance-checked and may contract.
#
# -fno-slp-vectorize everywhere: the SLP vectorizer formed
# `v_pk_mul_f32 v[4:5], v[4:5], v[8:9] op_sel:[0,1]` in the sim (the IDM terms
# v*tau and v*dv as one packed op, v taken from the high half of the second
# operand).  With another kernel's MFMA waves co-executing on the SIMD that
# encoding returns 0 in about 0.1 % of executions (tools/pk_hazard.hip: only
# op_sel with the second operand's high half; the plain, neg, op_sel:[1,0] and
# op_sel_hi forms measured exact), so one follower's desired gap collapsed to
# min_gap and the full overlap schedule diverged (tools/sim_contention.py).
# Without SLP no kernel has a packed-f32 op at all; the learn kernels (whose
# packed ops never used that form) measured the same with and without it
# (same-box A/B, tools/ab_learn.sh: 2.41-2.63 vs 2.46-2.67 ms, box drift
# larger than any difference).  tests/test_isa_cpu.py checks the built code.
COMMON = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-Wall",
          "-Wno-unused-result", "-munsafe-fp-atomics", "-fno-slp-vectorize"]
PER_FILE = {
    "learn.hip": ["-ffp-contract=fast"],
    "learn_f16.hip": ["-ffp-contract=fast"],
    "learn_bf16.hip": ["-ffp-contract=fast"],
}
DEFAULT_FP = ["-ffp-contract=off"]
# experiment hook: extra flags for every file (e.g. -D switches while tuning)
EXTRA = os.environ.get("DMDQN_EXTRA_FLAGS", "").split()


# The sources whose code a PMC traffic figure describes (profiles/learn_pmc.json
# records their digest; bench.py flags a figure measured on other sources as
# stale): the learn kernels, and the env step (sim + fused observe / store).
KERNEL_SOURCES = {
    "learn": ["learn.hip", "learn_f16.hip", "learn_bf16.hip", "learn_h16.hpp", "learn_shared.hip",
              "qnet_layout.hpp", "common.hpp"],
    "sim": ["sim.hip", "sim.hpp", "observe.hpp", "common.hpp"],
}


def source_digest(kind):
    """sha256 (hex, 16 chars) over the KERNEL_SOURCES of `kind` and the compile
    flags, in a fixed order."""
    import hashlib
    h = hashlib.sha256(" ".join(COMMON).encode())
    for name in KERNEL_SOURCES[kind]:
        h.update(name.encode())
        with open(os.path.join(CSRC, name), "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def tree_files(root=None):
    """Every file the two libraries are built from, in a fixed order: the
    kernels, headers and C ABI (csrc/), include/*.h and the torch operator
    library's source.  root: another copy of the package directory (tests)."""
    here = root or HERE
    pats = [os.path.join(here, "csrc", "*"), os.path.join(here, "..", "include", "*.h"),
            os.path.join(here, "torch_ext", "*.cpp")]
    files = [p for pat in pats for p in glob.glob(pat)
             if os.path.isfile(p) and p.endswith((".hip", ".hpp", ".cpp", ".h"))]
    return sorted(files, key=lambda p: (os.path.basename(os.path.dirname(p)), os.path.basename(p)))


def tree_digest(root=None):
    """sha256 (hex, 16 chars) over tree_files() (names and contents) and the
    common compile flags: what libdmdqn_hip.so / libdmdqn_torch.so embed at
    build time (dmdqn_source_digest) and what _lib.load() checks them against,
    so a library built from other sources than the tree's is refused."""
    import hashlib
    h = hashlib.sha256(" ".join(COMMON).encode())
    for p in tree_files(root):
        h.update(os.path.basename(p).encode())
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def _digest_object(variant, digest):
    """The object that exports dmdqn_source_digest(): regenerated (and the
    library relinked) whenever the tree digest changes."""
    src = os.path.join(objdir(variant), "source_digest.cpp")
    obj = src + ".o"
    text = ("// generated by dmdqn_amd/build.py: the digest of the sources this library\n"
            "// was built from (build.tree_digest; _lib.load() compares it with the tree)\n"
            f'extern "C" const char *dmdqn_source_digest(void) {{ return "{digest}"; }}\n')
    try:
        with open(src) as f:
            same = f.read() == text
    except OSError:
        same = False
    if same and os.path.exists(obj):
        return obj, False
    with open(src, "w") as f:
        f.write(text)
    r = subprocess.run(["g++", "-O2", "-fPIC", "-c", src, "-o", obj], capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"digest object failed:\n{r.stdout}\n{r.stderr}")
    return obj, True


def _sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.cpp")))


def _headers():
    return glob.glob(os.path.join(CSRC, "*.hpp")) + glob.glob(
        os.path.join(HERE, "..", "include", "*.h"))


def _compile(src, force, variant=""):
    name = os.path.basename(src)
    obj = os.path.join(objdir(variant), name + ".o")
    flags = COMMON + PER_FILE.get(name, DEFAULT_FP) + VARIANT_FLAGS[variant] + EXTRA
    # the flags an object was built with sit beside it: a changed flag set
    # (e.g. an experiment's -D switches, then none) forces a rebuild
    stamp = obj + ".flags"
    try:
        with open(stamp) as f:
            same_flags = f.read() == " ".join(flags)
    except OSError:
        same_flags = False
    newest = max([os.path.getmtime(src)] + [os.path.getmtime(h) for h in _headers()])
    if (not force and same_flags and os.path.exists(obj)
            and os.path.getmtime(obj) >= newest):
        return obj, False
    lang = ["-x", "hip"] if name.endswith(".hip") else []
    cmd = [HIPCC] + flags + lang + ["-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {name}:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    if r.stderr.strip():
        sys.stderr.write(r.stderr)
    with open(stamp, "w") as f:
        f.write(" ".join(flags))
    return obj, True


TORCH_EXT = os.path.join(HERE, "torch_ext", "dmdqn_torch.cpp")
TORCH_LIBNAME = "libdmdqn_torch.so"


def torch_libname(variant=""):
    return f"libdmdqn_torch{_suffix(variant)}.so"


def build_torch_ext(force=False, verbose=True, variant=""):
    """libdmdqn_torch.so: the C ABI registered as torch.ops.dmdqn.* (TORCH_LIBRARY),
    linked against libdmdqn_hip.so (same directory) and the installed PyTorch."""
    import torch
    tdir = os.path.dirname(torch.__file__)
    so = os.path.join(LIBDIR, torch_libname(variant))
    deps = [TORCH_EXT, os.path.join(LIBDIR, libname(variant))] + _headers()
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    flags = ["-O2", "-fPIC", "-std=c++17", "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
             f'-DDMDQN_SOURCE_DIGEST="{tree_digest()}"',
             f"-D_GLIBCXX_USE_CXX11_ABI={abi}", f"-I{tdir}/include",
             f"-I{tdir}/include/torch/csrc/api/include", "-I/opt/rocm/include"]
    stamp = so + ".flags"
    try:
        with open(stamp) as f:
            same = f.read() == " ".join(flags)
    except OSError:
        same = False
    if (not force and same and os.path.exists(so)
            and os.path.getmtime(so) >= max(os.path.getmtime(d) for d in deps)):
        return so
    cmd = (["g++"] + flags + ["-shared", TORCH_EXT, "-o", so, f"-L{tdir}/lib", "-lc10", "-lc10_hip",
                              "-ltorch", "-ltorch_cpu", "-ltorch_hip", f"-L{LIBDIR}",
                              f"-ldmdqn_hip{_suffix(variant)}",
                              "-Wl,-rpath,$ORIGIN", f"-Wl,-rpath,{tdir}/lib"])
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"torch extension build failed:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    with open(stamp, "w") as f:
        f.write(" ".join(flags))
    if verbose:
        print(f"built {so}")
    return so


def build(force=False, verbose=True, variant=""):
    os.makedirs(objdir(variant), exist_ok=True)
    srcs = _sources()
    with cf.ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        results = list(ex.map(lambda s: _compile(s, force, variant), srcs))
    so = os.path.join(LIBDIR, libname(variant))
    results.append(_digest_object(variant, tree_digest()))
    objs = [o for o, _ in results]
    if force or any(ch for _, ch in results) or not os.path.exists(so):
        cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", so] + objs
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
        if verbose:
            print(f"built {so}")
    build_torch_ext(force, verbose, variant)
    return so


def build_all(force=False, verbose=True):
    """The product build and the debug-bounds build (both travel to the GPU box)."""
    so = build(force, verbose)
    build(force, verbose, "debug")
    return so


if __name__ == "__main__":
    named = [v for v in VARIANT_FLAGS if v and f"--{v}" in sys.argv]
    if named:
        build(force="--force" in sys.argv, variant=named[0])
    else:
        build_all(force="--force" in sys.argv)
