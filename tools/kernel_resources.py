"""Per-kernel resources of the built gfx950 code objects (VGPRs, AGPRs,
SGPRs, static LDS, scratch per lane, occupancy bound), from the AMDGPU
metadata notes.  usage: python tools/kernel_resources.py [lib.so] [name-filter]"""
import os
import re
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
LLVM = "/opt/rocm/lib/llvm/bin"
so = sys.argv[1] if len(sys.argv) > 1 and sys.argv[1] else str(ROOT / "dmdqn_amd/lib/libdmdqn_hip.so")
filt = sys.argv[2] if len(sys.argv) > 2 else ""
sys.path[:0] = [str(ROOT), str(ROOT / "tests")]
from test_isa_cpu import _code_objects  # noqa: E402

KEYS = {".vgpr_count": "vgpr", ".agpr_count": "agpr", ".sgpr_count": "sgpr",
        ".group_segment_fixed_size": "lds", ".private_segment_fixed_size": "scratch",
        ".max_flat_workgroup_size": "wg"}
with tempfile.TemporaryDirectory() as td:
    rows = []
    for co in _code_objects(so, Path(td)):
        notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", str(co)], check=True,
                               capture_output=True, text=True).stdout
        for block in notes.split("  - .agpr_count")[1:]:
            block = "  - .agpr_count" + block
            name = re.search(r"\.name:\s+(\S+)", block).group(1)
            if filt not in name:
                continue
            vals = {v: int(m.group(1)) for k, v in KEYS.items()
                    if (m := re.search(re.escape(k) + r":\s+(\d+)", block))}
            rows.append((name, vals))
for name, v in sorted(rows):
    print(f"{name[:70]:70s} " + " ".join(f"{k}={v.get(k, '-')}" for k in KEYS.values()))
