#!/bin/bash
# The -m gpu suite + smoke() on one GPU (run via gpurun from the repo root).
# usage: bash tools/gpu_tests.sh <tag> [pytest selection...]
set -e
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p $O
SEL=${@:-tests}
timeout -k 10 1000 python -u -m pytest $SEL -m gpu -x -v --timeout 300 --timeout-method thread \
    --durations=20 > $O/gpu_tests.log 2>&1
tail -3 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
