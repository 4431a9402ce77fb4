#!/bin/bash
# C2 side_learn sweep: 32 / 48 / 64 / 80 / 96 agents learned on the side stream,
# alternating, 2 rounds.
set -e
O=gpurun_out/r04s
mkdir -p $O
summ() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); r=d['roofline']; print(d['value'], d['ms_per_step'], r['avg_launch_ms'], r['frac'])" $1; }
for i in 1 2; do
  for m in 32 48 64 80 96; do
    f=$O/c2_side${m}_$i.json
    timeout -k 10 300 python bench.py --rows 2 --cols 2 --envs 256 --precision bf16 --no-cpu-baseline --side-learn $m > $f 2> ${f%.json}.err
    echo "c2 side_learn=$m $(summ $f)"
  done
done
