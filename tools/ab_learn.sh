#!/bin/bash
# A/B the learn kernel alone: _ab_old/ (a built copy of another commit) vs the
# working tree, alternating processes on one box (box-to-box spread is larger
# than most kernel changes).  usage: bash tools/ab_learn.sh [pairs] [learn_bench args]
N=${1:-6}; shift
for i in $(seq $N); do
  (cd _ab_old && timeout -k 10 120 python3 tools/learn_bench.py 80 "$@" | sed "s/^/old /") || exit 1
  timeout -k 10 120 python3 tools/learn_bench.py 80 "$@" | sed "s/^/new /" || exit 1
done
