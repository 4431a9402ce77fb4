"""Where the waves of a kernel spend their cycles, from one rocprofv3 --pmc pass of
SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS
SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
(tools/pmc_stalls.sh).  Per kernel substring, summed over dispatches:
  parked  = SQ_WAIT_ANY / SQ_WAVE_CYCLES       (s_waitcnt or barrier)
  stalled = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES  (issue stalls, e.g. MFMA dependencies)
  active  = SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES
  lds_issue_stall = SQ_WAIT_INST_LDS / SQ_WAVE_CYCLES
  bank_conflict_share = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x CUs x 4 SIMDs)
(MI355X_MICROARCH.md: WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ~ WAVE_CYCLES.)
usage: python tools/pmc_stalls.py <counter_collection.csv> <kernel_substr>... [--cus N]"""
import csv
import json
import sys
from collections import defaultdict


def main():
    args = sys.argv[1:]
    n_cu = 256
    if "--cus" in args:
        k = args.index("--cus")
        n_cu = int(args[k + 1])
        del args[k:k + 2]
    path, names = args[0], args[1:]
    per = {n: defaultdict(float) for n in names}
    for row in csv.DictReader(open(path)):
        for n in names:
            if n in row.get("Kernel_Name", ""):
                per[n][row["Counter_Name"]] += float(row["Counter_Value"])
    out = {}
    for n, d in per.items():
        wc = d.get("SQ_WAVE_CYCLES", 0.0)
        if not wc:
            continue
        out[n] = {
            "parked": round(d["SQ_WAIT_ANY"] / wc, 3),
            "stalled": round(d["SQ_WAIT_INST_ANY"] / wc, 3),
            "active": round(d["SQ_ACTIVE_INST_ANY"] / wc, 3),
            "lds_issue_stall": round(d["SQ_WAIT_INST_LDS"] / wc, 3),
            "bank_conflict_share": round(d["SQ_LDS_BANK_CONFLICT"] / max(1.0, d["SQ_LDS_IDX_ACTIVE"]), 3),
            "mfma_busy": round(d["SQ_VALU_MFMA_BUSY_CYCLES"] / (d["GRBM_GUI_ACTIVE"] / 8 * n_cu * 4), 3),
        }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
