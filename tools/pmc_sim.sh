#!/bin/bash
# SQ counters of k_sim_step (4x4 x 1024, tools/sim_bench.py) -- two passes of
# at most 8 SQ counters each (run via gpurun from the repo root).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pmc_sim
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY --output-format csv -d $O/p1 -o run -- python3 $R/tools/sim_bench.py 4 4 1024 > $O/p1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA --output-format csv -d $O/p2 -o run -- python3 $R/tools/sim_bench.py 4 4 1024 > $O/p2.log 2>&1
cd $R
python3 - <<'PY'
import csv, glob, collections
for p in ["p1", "p2"]:
    f = glob.glob(f"gpurun_out/pmc_sim/{p}/**/*counter_collection.csv", recursive=True)[0]
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if "k_sim_step" in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in sorted(acc.items()):
        print(p, k, "per launch", round(sum(v) / max(1, len(set(range(len(v))))) , 1), "n", len(v))
PY
