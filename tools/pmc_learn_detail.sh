#!/bin/bash
# Counter passes over tools/learn_bench.py (the learn kernel alone, C3 size):
# FETCH_SIZE, WRITE_SIZE, and TCC request/hit counters, each in its own pass.
# usage (GPU box, repo root): bash tools/pmc_learn_detail.sh <tag>
set -e
TAG=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pmcd_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for C in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_HIT_sum TCC_MISS_sum" \
         "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/p$i -o run \
      -- python3 $R/tools/learn_bench.py 8 > $O/p$i.log 2>&1
done
cd $R
python3 - "$O" <<'PY'
import csv, glob, sys, collections
O = sys.argv[1]
acc = collections.defaultdict(list)
for f in glob.glob(O + "/p*/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        if "k_learn" in row.get("Kernel_Name", ""):
            acc[row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, v in sorted(acc.items()):
    print(f"{k}: per launch {sum(v) / len(v):.6g} over {len(v)} launches")
PY
