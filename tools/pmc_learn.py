"""Reduce rocprofv3 --pmc counter CSVs of a bench run to per-launch HBM bytes of
the learn kernel, with the gfx950 corrections of MI355X_MICROARCH.md (HBM):
  * FETCH_SIZE (KB) reports 1/2 of the bytes of a wide coalesced stream -> x2
  * WRITE_SIZE (KB) is exact for 16-byte stores
FETCH_SIZE and WRITE_SIZE are collected in separate passes (TCC slots).
Usage: python tools/pmc_learn.py <fetch_csv> <write_csv> <workload_key> [kernel_substr] [source]
(kernel_substr: one name, or a '|' list of the kernels one learn launches --
their per-dispatch means are summed (template names hold commas); source: where the passes were run, e.g.
"profiles/r03/c3 @ <commit>").
Writes/updates profiles/learn_pmc.json."""
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dmdqn_amd.build import source_digest  # noqa: E402


def per_kernel(path, counter, substr):
    vals = []
    with open(path) as f:
        for row in csv.DictReader(f):
            if substr in row.get("Kernel_Name", "") and row.get("Counter_Name") == counter:
                vals.append(float(row["Counter_Value"]))
    return vals


def main():
    fetch_csv, write_csv, key = sys.argv[1:4]
    substr = sys.argv[4] if len(sys.argv) > 4 else "k_learn"
    source = sys.argv[5] if len(sys.argv) > 5 else None
    fetch_kb = write_kb = 0.0
    counts = []
    for name in substr.split("|"):
        fv = per_kernel(fetch_csv, "FETCH_SIZE", name)
        wv = per_kernel(write_csv, "WRITE_SIZE", name)
        if not fv or not wv:
            raise SystemExit(f"no {name} rows: fetch {len(fv)} write {len(wv)}")
        fetch_kb += sum(fv) / len(fv)
        write_kb += sum(wv) / len(wv)
        counts += [len(fv), len(wv)]
    out = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles",
                       "learn_pmc.json")
    d = {}
    if os.path.exists(out):
        with open(out) as f:
            d = json.load(f)
    d[key] = {"kernel": substr, "dispatches": counts,
              "FETCH_SIZE_KB_raw": fetch_kb, "WRITE_SIZE_KB_raw": write_kb,
              "hbm_bytes_per_launch": int(round((2.0 * fetch_kb + write_kb) * 1024)),
              "correction": "fetch x2 (gfx950 FETCH_SIZE reads 1/2 of wide streams), write x1"}
    if source:
        d[key]["source"] = source
    # the kernel sources the passes measured (bench.py: traffic_stale when HEAD's differ)
    kind = "sim" if key.endswith("_sim") or key.endswith("_envstep") else "learn"
    d[key]["sources_digest"] = {"kind": kind, "sha256_16": source_digest(kind)}
    with open(out, "w") as f:
        json.dump(d, f, indent=1)
    print(json.dumps(d[key]))


if __name__ == "__main__":
    main()
