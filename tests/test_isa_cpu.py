"""ISA guard on the built gfx950 code objects (no GPU needed).

The product and debug libraries are compiled with -fno-slp-vectorize
(dmdqn_amd/build.py): no packed-f32 VALU op (v_pk_{add,mul,fma}_f32) may
appear in any kernel.  An SLP-formed v_pk_mul_f32 in the sim read a VGPR
written by the instruction just before it as its stale value while another
kernel's MFMA waves co-executed on the SIMD (tools/sim_contention.py), so the
guard is on the machine code itself, not on the flag."""
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


@pytest.mark.parametrize("variant", ["", "debug"])
def test_no_packed_f32_valu_ops(variant, tmp_path):
    if not os.path.exists(f"{LLVM}/llvm-objdump"):
        pytest.skip("ROCm LLVM tools not installed")
    so = os.path.join(build.LIBDIR, build.libname(variant))
    if not os.path.exists(so):
        build.build(verbose=False, variant=variant)
    cos = _code_objects(so, tmp_path)
    assert len(cos) >= 6, f"expected one code object per HIP source, found {len(cos)}"
    kernels, bad = set(), []
    for co in cos:
        dis = subprocess.run([f"{LLVM}/llvm-objdump", "-d", str(co)], check=True,
                             capture_output=True, text=True).stdout
        kernels.update(re.findall(r"^[0-9a-f]+ <(\w+)>:", dis, re.M))
        bad += [ln.strip() for ln in dis.splitlines() if re.search(r"\bv_pk_\w+_f32\b", ln)]
    assert any("k_sim_step" in k for k in kernels) and any("k_learn_f16" in k for k in kernels)
    assert not bad, f"{len(bad)} packed-f32 VALU ops, e.g. {bad[:3]}"
