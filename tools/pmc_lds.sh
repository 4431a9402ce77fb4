#!/bin/bash
# LDS bank-conflict counters per kernel of the default bench (own --pmc pass):
#   SQ_LDS_BANK_CONFLICT (extra cycles) vs SQ_LDS_IDX_ACTIVE (all LDS-array cycles)
# usage (GPU box, repo root): bash tools/pmc_lds.sh <tag> [extra bench args]
set -e
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv \
    -d $O/pmcL_$TAG -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline "$@" \
    > $O/pmcL_$TAG.log 2>&1
F=$(find $O/pmcL_$TAG -name '*counter_collection.csv' | head -n 1)
python3 - "$F" <<'PY'
import csv, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.Counter()
for row in csv.DictReader(open(sys.argv[1])):
    k = row["Kernel_Name"].split("(")[0][:60]
    acc[k][row["Counter_Name"]] += float(row["Counter_Value"])
    n[(k, row["Counter_Name"])] += 1
for k, d in acc.items():
    c, a = d.get("SQ_LDS_BANK_CONFLICT", 0), d.get("SQ_LDS_IDX_ACTIVE", 0)
    if a:
        print(f"{k:60s} conflict/active = {c / a:.3f}  (active {a:.3g})")
PY
