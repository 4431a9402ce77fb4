#!/bin/bash
# C3 (the headline): one stream vs the env step on a 64-CU side stream that
# also learns m agents (2048 / 3072 / 4096), and the default C2 line.
set -e
O=gpurun_out/r04t
mkdir -p $O
summ() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); r=d['roofline']; print(d['value'], d['ms_per_step'], r['avg_launch_ms'], r['frac'])" $1; }
timeout -k 10 300 python bench.py --rows 2 --cols 2 --envs 256 --precision bf16 --no-cpu-baseline > $O/c2_default.json 2> $O/c2_default.err
echo "c2 default $(summ $O/c2_default.json)"
for i in 1 2; do
  for m in none 2048 3072 4096; do
    f=$O/c3_${m}_$i.json
    if [ $m = none ]; then a="--overlap none"; else a="--overlap env --cu-split 64 --side-learn $m"; fi
    timeout -k 10 300 python bench.py --steps 100 --no-cpu-baseline $a > $f 2> ${f%.json}.err
    echo "c3 $m $(summ $f)"
  done
done
