"""Disassemble the gfx950 code objects of libdmdqn_hip.so: one .s per
translation unit under the output directory (default /tmp/dmdqn_isa).
usage: python tools/disasm.py [outdir]"""
import os
import re
import subprocess
import sys
import tempfile

from dmdqn_amd import build

LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def main(out="/tmp/dmdqn_isa"):
    os.makedirs(out, exist_ok=True)
    so = os.path.join(build.LIBDIR, build.libname())
    with tempfile.TemporaryDirectory() as td:
        fb = os.path.join(td, "fb.bin")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", so,
                        os.path.join(td, "s.so")], check=True, capture_output=True)
        data = open(fb, "rb").read()
        starts = [m.start() for m in re.finditer(re.escape(MAGIC), data)] + [len(data)]
        for k, (a, b) in enumerate(zip(starts, starts[1:])):
            part, co = os.path.join(td, f"b{k}.bin"), os.path.join(td, f"b{k}.co")
            open(part, "wb").write(data[a:b])
            r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o",
                                f"--input={part}", f"--targets=hipv4-amdgcn-amd-amdhsa--{build.ARCH}",
                                f"--output={co}"], capture_output=True)
            if r.returncode or not os.path.exists(co):
                continue
            dis = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", co],
                                 check=True, capture_output=True, text=True).stdout
            names = re.findall(r"^[0-9a-f]+ <(\w+)>:", dis, re.M)
            tag = names[0][:40] if names else f"tu{k}"
            open(os.path.join(out, f"{k:02d}_{tag}.s"), "w").write(dis)
            print(k, len(names), tag)


if __name__ == "__main__":
    main(*sys.argv[1:])
