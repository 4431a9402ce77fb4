#!/bin/bash
# C5 / C3 schedule A/B with the fused env step: one stream vs replay draws on a
# side stream beside the env step ("sample") vs step t+1's env work beside
# learn t ("full"), alternating processes, one box.
set -e
O=gpurun_out/r04g
mkdir -p $O
summ() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); r=d['roofline']; print(d['value'], d['ms_per_step'], r['avg_launch_ms'], r['frac'])" $1; }
for i in 1 2; do
  for v in none sample full; do
    f=$O/c5_${v}_$i.json
    timeout -k 10 300 python bench.py --shared --rows 8 --cols 8 --envs 256 --no-cpu-baseline --overlap $v > $f 2> ${f%.json}.err
    echo "c5 $v $(summ $f)"
  done
done
for v in none sample; do
  f=$O/c3_${v}.json
  timeout -k 10 300 python bench.py --steps 100 --no-cpu-baseline --overlap $v > $f 2> ${f%.json}.err
  echo "c3 $v $(summ $f)"
done
