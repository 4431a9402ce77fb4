#!/bin/bash
# C2 env schedule: side-stream CU count re-swept with the round-4 event
# changes (48 / 56 / 64 / 72 / 80), alternating, 2 rounds.
set -e
O=gpurun_out/r04q
mkdir -p $O
summ() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); r=d['roofline']; print(d['value'], d['ms_per_step'], r['avg_launch_ms'])" $1; }
for i in 1 2; do
  for k in 48 56 64 72 80; do
    f=$O/c2_cu${k}_$i.json
    timeout -k 10 300 python bench.py --rows 2 --cols 2 --envs 256 --precision bf16 --no-cpu-baseline --overlap env --cu-split $k > $f 2> ${f%.json}.err
    echo "c2 cu$k $(summ $f)"
  done
done
