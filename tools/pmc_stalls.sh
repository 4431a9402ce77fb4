#!/bin/bash
# One PMC pass (8 SQ + 1 GRBM counters) over the C5 shared learn alone
# (tools/learn_bench.py --shared), reduced by tools/pmc_stalls.py.
# usage (via gpurun, repo root): bash tools/pmc_stalls.sh <out_dir> [env assignments...]
set -e
R=$(pwd)
O=$R/$1; shift
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
env "$@" timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE \
    --output-format csv -d $O/pmc -o run -- python3 $R/tools/learn_bench.py 5 --shared > $O/pmc.log 2>&1
cp "$(find $O/pmc -name '*counter_collection.csv' | head -n 1)" $O/stalls_counter_collection.csv
rm -rf $O/pmc
# pass 2: instruction counts (LDS, VALU) per kernel, summed over dispatches
env "$@" timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES \
    --output-format csv -d $O/pmc2 -o run -- python3 $R/tools/learn_bench.py 5 --shared > $O/pmc2.log 2>&1
cp "$(find $O/pmc2 -name '*counter_collection.csv' | head -n 1)" $O/insts_counter_collection.csv
rm -rf $O/pmc2
cd $R && python3 tools/pmc_stalls.py $O/stalls_counter_collection.csv k_shared_next k_shared_grad > $O/stalls.json
python3 - $O/insts_counter_collection.csv > $O/insts.json <<'PY'
import csv, json, sys
from collections import defaultdict
tot = defaultdict(lambda: defaultdict(float))
for row in csv.DictReader(open(sys.argv[1])):
    k = row.get("Kernel_Name", "")
    for name in ("k_shared_next", "k_shared_grad"):
        if name in k:
            tot[name][row["Counter_Name"]] += float(row["Counter_Value"])
print(json.dumps({k: dict(v) for k, v in tot.items()}, indent=1))
PY
