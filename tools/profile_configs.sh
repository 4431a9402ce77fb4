#!/bin/bash
# rocprofv3 --kernel-trace --stats of the C2 and C5 bench configurations (run via
# gpurun from the repo root); summaries land in gpurun_out/cfgprof/<name>.csv.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/cfgprof
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c2 -o run \
    -- python3 $R/bench.py --rows 2 --cols 2 --envs 256 --precision bf16 --steps 20 --warmup 5 \
    --no-cpu-baseline > $O/c2.json 2> $O/c2.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c5 -o run \
    -- python3 $R/bench.py --shared --rows 8 --cols 8 --envs 256 --steps 20 --warmup 5 \
    --no-cpu-baseline > $O/c5.json 2> $O/c5.err
cp "$(find $O/c2 -name '*kernel_stats.csv' | head -n 1)" $O/c2_kernel_stats.csv
cp "$(find $O/c5 -name '*kernel_stats.csv' | head -n 1)" $O/c5_kernel_stats.csv
