#!/bin/bash
# A/B of the trainer's stream schedules on one box (run via gpurun from the
# repo root): none / full / full on a 32-CU side stream, alternating, twice.
set -e
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/ab_sched
mkdir -p $O
for rep in 1 2; do
  timeout -k 10 240 python3 bench.py --no-cpu-baseline > $O/none_$rep.json 2>/dev/null
  timeout -k 10 240 python3 bench.py --no-cpu-baseline --overlap full > $O/full_$rep.json 2>/dev/null
  timeout -k 10 240 python3 bench.py --no-cpu-baseline --overlap full --cu-split 32 > $O/full32_$rep.json 2>/dev/null
done
for f in $O/*.json; do python3 -c "import json,sys; d=json.load(open('$f')); print('$f'.split('/')[-1], d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"; done
