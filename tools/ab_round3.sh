#!/bin/bash
# Round-3 A/Bs on one box (run via gpurun from the repo root):
#   1. learn kernel alone, round-2 build (_ab_old) vs this tree, fp16 C3 size
#   2. the C5 shared learn: one-pass kernel (DMDQN_SHARED_V1=1) vs the two passes
#   3. rocprofv3 kernel stats of the two-pass shared learn
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ab3
mkdir -p $O
bash tools/ab_learn.sh 4 > $O/ab_learn_fp16.txt
for i in 1 2 3; do
    DMDQN_SHARED_V1=1 timeout -k 10 120 python3 tools/learn_bench.py 40 --shared | sed "s/^/v1 /" >> $O/ab_shared.txt
    timeout -k 10 120 python3 tools/learn_bench.py 40 --shared | sed "s/^/v2 /" >> $O/ab_shared.txt
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_shared -o run \
    -- python3 $R/tools/learn_bench.py 20 --shared > $O/prof_shared.log 2>&1
cp "$(find $O/prof_shared -name '*kernel_stats.csv' | head -n 1)" $O/shared_kernel_stats.csv
rm -rf $O/prof_shared
