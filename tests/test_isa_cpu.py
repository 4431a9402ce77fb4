"""ISA guard on the built gfx950 code objects (no GPU needed).

`v_pk_mul_f32 ... op_sel:[0,1]` (the second operand's high half feeding the
low lane) returns 0 in about 0.1 % of executions while another kernel's MFMA
waves co-execute on the SIMD (tools/pk_hazard.hip; the plain, neg,
op_sel:[1,0] and op_sel_hi forms measured exact).  The SLP vectorizer formed
it in the sim, and the full overlap schedule diverged (tools/sim_contention.py).
dmdqn_amd/build.py compiles every kernel with -fno-slp-vectorize; this test
checks the machine code itself:
  * no packed-f32 op with an op_sel whose second-operand bit is set, anywhere;
  * no packed-f32 op at all in the sim, observe, RNG and replay kernels (the
    learn kernels may use the measured-exact forms, should a later change
    write packed vector code by hand)."""
import os
import re
import subprocess

import pytest

from dmdqn_amd import build

LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
TARGET = f"hipv4-amdgcn-amd-amdhsa--{build.ARCH}"


def _code_objects(so, tmp_path):
    """Every gfx950 code object in the library's .hip_fatbin section (one
    offload bundle per translation unit)."""
    fb = tmp_path / "fatbin.bin"
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", so,
                    str(tmp_path / "stripped.so")], check=True, capture_output=True)
    data = fb.read_bytes()
    starts = [m.start() for m in re.finditer(re.escape(MAGIC), data)] + [len(data)]
    out = []
    for k, (a, b) in enumerate(zip(starts, starts[1:])):
        part = tmp_path / f"bundle{k}.bin"
        part.write_bytes(data[a:b])
        co = tmp_path / f"bundle{k}.co"
        r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o",
                            f"--input={part}", f"--targets={TARGET}", f"--output={co}"],
                           capture_output=True)
        if r.returncode == 0 and co.exists() and co.stat().st_size:
            out.append(co)
    return out


EXACT = ("k_sim_step", "k_sim_reset", "k_observe", "k_seed", "k_act", "k_sample", "k_draw",
         "k_replay")
PK = re.compile(r"\bv_pk_\w+_f32\b")
OPSEL_SRC1 = re.compile(r"\bop_sel:\[\d,1")


@pytest.mark.parametrize("variant", ["", "debug"])
def test_packed_f32_forms(variant, tmp_path):
    if not os.path.exists(f"{LLVM}/llvm-objdump"):
        pytest.skip("ROCm LLVM tools not installed")
    so = os.path.join(build.LIBDIR, build.libname(variant))
    if not os.path.exists(so):
        build.build(verbose=False, variant=variant)
    cos = _code_objects(so, tmp_path)
    assert len(cos) >= 6, f"expected one code object per HIP source, found {len(cos)}"
    kernels, opsel, exact = set(), [], []
    for co in cos:
        dis = subprocess.run([f"{LLVM}/llvm-objdump", "-d", str(co)], check=True,
                             capture_output=True, text=True).stdout
        fn = ""
        for ln in dis.splitlines():
            m = re.match(r"^[0-9a-f]+ <(\w+)>:", ln)
            if m:
                fn = m.group(1)
                kernels.add(fn)
            elif PK.search(ln):
                if OPSEL_SRC1.search(ln):
                    opsel.append((fn, ln.strip()))
                if any(k in fn for k in EXACT):
                    exact.append((fn, ln.strip()))
    assert any("k_sim_step" in k for k in kernels) and any("k_learn_f16" in k for k in kernels)
    assert not opsel, f"{len(opsel)} packed-f32 ops with op_sel on the second operand: {opsel[:3]}"
    assert not exact, f"{len(exact)} packed-f32 ops in exact-arithmetic kernels: {exact[:3]}"
