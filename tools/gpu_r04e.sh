#!/bin/bash
# bench.py --overlap auto at C2 (env + 64-CU side stream), and the C5 "env"
# schedule A/B against one stream (alternating processes, one box).
set -e
O=gpurun_out/r04e
mkdir -p $O
summ() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); r=d['roofline']; print(d['value'], d['ms_per_step'], r['avg_launch_ms'], r['bound'], r['frac'], d['config']['schedule'])" $1; }
timeout -k 10 300 python bench.py --rows 2 --cols 2 --envs 256 --precision bf16 --no-cpu-baseline > $O/c2_auto.json 2> $O/c2_auto.err
echo "c2 auto $(summ $O/c2_auto.json)"
for i in 1 2; do
  for v in none env; do
    f=$O/c5_${v}_$i.json
    timeout -k 10 300 python bench.py --shared --rows 8 --cols 8 --envs 256 --no-cpu-baseline --overlap $v > $f 2> ${f%.json}.err
    echo "c5 $v $(summ $f)"
  done
done
