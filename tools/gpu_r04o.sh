#!/bin/bash
# C3 schedules with the round-4 event changes: one stream vs the env step beside
# the learn (no CU mask / side stream on 16 CUs), alternating, 2 rounds.
set -e
O=gpurun_out/r04o
mkdir -p $O
summ() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); r=d['roofline']; print(d['value'], d['ms_per_step'], r['avg_launch_ms'], r['frac'], d['step_roofline']['frac'])" $1; }
for i in 1 2; do
  for v in "none" "env" "env --cu-split 16"; do
    f=$O/c3_${v// /_}_$i.json
    timeout -k 10 300 python bench.py --steps 100 --no-cpu-baseline --overlap $v > $f 2> ${f%.json}.err
    echo "c3 $v $(summ $f)"
  done
done
