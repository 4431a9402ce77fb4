#!/bin/bash
# bench.py lines for the one-GPU BASELINE configurations, same box, one call
# (run via gpurun from the repo root).  Each run has its own time limit; the
# chain stops at the first failure.  Output: gpurun_out/<tag>/<cfg>.json
# usage: bash tools/bench_configs.sh <tag> [c3] [c2] [c5] [c5v1] [c3full] ...
set -e
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
for CFG in "$@"; do
    ENVV=""
    case $CFG in
        c3) ARGS="" ;;
        c3full) ARGS="--overlap full --no-cpu-baseline" ;;
        c2) ARGS="--rows 2 --cols 2 --envs 256 --precision bf16 --no-cpu-baseline" ;;
        c2full) ARGS="--rows 2 --cols 2 --envs 256 --precision bf16 --overlap full --no-cpu-baseline" ;;
        c5) ARGS="--shared --rows 8 --cols 8 --envs 256 --no-cpu-baseline" ;;
        *) echo "unknown config $CFG"; exit 2 ;;
    esac
    env $ENVV timeout -k 10 300 python3 $R/bench.py $ARGS > $O/$CFG.json 2> $O/$CFG.err
    echo "$CFG: $(head -c 300 $O/$CFG.json)"
done
