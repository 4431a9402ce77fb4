#!/bin/bash
# Kernel stats of one bench configuration (quick: short prefill), for A/Bs.
# usage: bash tools/prof_quick.sh <outdir> <bench args...>
set -e
O=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/$O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/stats -o run \
    -- python3 $R/bench.py --no-cpu-baseline "$@" > $R/$O/bench.json 2> $R/$O/bench.err
cp "$(find $R/$O/stats -name '*kernel_stats.csv' | head -n 1)" $R/$O/kernel_stats.csv
rm -rf $R/$O/stats
python3 - "$R/$O/kernel_stats.csv" <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:12]:
    print(r['Name'][:70].ljust(70), r['Calls'], round(float(r['AverageNs']) / 1e3, 2), 'us')
PY
