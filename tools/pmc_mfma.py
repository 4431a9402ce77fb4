"""MFMA utilisation of a kernel from a rocprofv3 --pmc pass of
SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES (tools/profile_configs.sh).

Per dispatch: busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x CUs x
4 SIMDs) -- the share of SIMD-cycles of the dispatch in which a matrix core was
busy (rocprofv3 sums GRBM_GUI_ACTIVE over the 8 XCDs, MI355X_MICROARCH.md DVFS
note; SQ_VALU_MFMA_BUSY_CYCLES counts cycles).  Prints the mean over the
kernel's dispatches as JSON.
usage: python tools/pmc_mfma.py <counter_collection.csv> <kernel_substr> [n_cu]"""
import csv
import json
import sys
from collections import defaultdict


def main():
    path, substr = sys.argv[1], sys.argv[2]
    n_cu = int(sys.argv[3]) if len(sys.argv) > 3 else 256
    per = defaultdict(dict)
    with open(path) as f:
        for row in csv.DictReader(f):
            if substr not in row.get("Kernel_Name", ""):
                continue
            key = row.get("Dispatch_Id") or row.get("Correlation_Id")
            per[key][row["Counter_Name"]] = per[key].get(row["Counter_Name"], 0.0) + \
                float(row["Counter_Value"])
    busy = []
    for d in per.values():
        if d.get("GRBM_GUI_ACTIVE") and "SQ_VALU_MFMA_BUSY_CYCLES" in d:
            cycles = d["GRBM_GUI_ACTIVE"] / 8.0
            busy.append(d["SQ_VALU_MFMA_BUSY_CYCLES"] / (cycles * n_cu * 4))
    out = {"kernel": substr, "dispatches": len(busy),
           "mfma_busy_frac": sum(busy) / len(busy) if busy else None,
           "definition": "SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE/8 x CUs x 4 SIMDs)",
           "raw": list(per.values())[:3]}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
