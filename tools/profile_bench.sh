#!/bin/bash
# Profile the default bench on the GPU box (run via gpurun from the repo root):
#   1. rocprofv3 --kernel-trace --stats      -> gpurun_out/prof_<tag>/
#   2. rocprofv3 --pmc FETCH_SIZE (own pass)  -> gpurun_out/pmcF_<tag>/
#   3. rocprofv3 --pmc WRITE_SIZE (own pass)  -> gpurun_out/pmcW_<tag>/
#   4. tools/pmc_learn.py reduces 2+3 into profiles/learn_pmc.json (key $2)
# then copies the summaries to gpurun_out/keep_<tag>/ for committing.
# Every GPU step has its own time limit; the chain stops at the first failure.
# usage: bash tools/profile_bench.sh <tag> <pmc_key> [extra bench args]
set -e
TAG=$1; KEY=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O/keep_$TAG
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$TAG -o run \
    -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline "$@" > $O/keep_$TAG/bench_prof.log 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmcF_$TAG -o run \
    -- python3 $R/bench.py --steps 4 --warmup 1 --prefill-steps 1100 --no-cpu-baseline "$@" > $O/pmcF_$TAG.log 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmcW_$TAG -o run \
    -- python3 $R/bench.py --steps 4 --warmup 1 --prefill-steps 1100 --no-cpu-baseline "$@" > $O/pmcW_$TAG.log 2>&1
F=$(find $O/pmcF_$TAG -name '*counter_collection.csv' | head -n 1)
W=$(find $O/pmcW_$TAG -name '*counter_collection.csv' | head -n 1)
cd $R
python3 tools/pmc_learn.py "$F" "$W" "$KEY" k_learn
python3 tools/pmc_learn.py "$F" "$W" "${KEY%_*}_sim" k_sim_step
cp profiles/learn_pmc.json $O/keep_$TAG/
cp "$(find $O/prof_$TAG -name '*kernel_stats.csv' | head -n 1)" $O/keep_$TAG/kernel_stats.csv
gzip -c "$F" > $O/keep_$TAG/fetch_size_counter_collection.csv.gz
gzip -c "$W" > $O/keep_$TAG/write_size_counter_collection.csv.gz
# the un-profiled default bench line (HIP-event timing, with the CPU baseline)
timeout -k 10 400 python3 bench.py "$@" > $O/keep_$TAG/bench.json 2> $O/keep_$TAG/bench.err
cat $O/keep_$TAG/bench.json
