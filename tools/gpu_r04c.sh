#!/bin/bash
# Schedule A/B at C3 (the fused env step of t+1 beside learn t, CU splits)
# and more C2 splits.  One bench process per line, alternating.
set -e
O=gpurun_out/r04c
mkdir -p $O
summ() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])" $1; }
for v in "none" "env --cu-split 16" "env --cu-split 24" "env --cu-split 32" "env"; do
  f=$O/c3_${v// /_}.json
  timeout -k 10 300 python bench.py --steps 100 --no-cpu-baseline --overlap $v > $f 2> ${f%.json}.err
  echo "c3 $v $(summ $f)"
done
for v in "env --cu-split 48" "env --cu-split 80" "env --cu-split 96" "env --cu-split 64 --cu-stride"; do
  f=$O/c2_${v// /_}.json
  timeout -k 10 300 python bench.py --rows 2 --cols 2 --envs 256 --precision bf16 --steps 200 \
      --no-cpu-baseline --overlap $v > $f 2> ${f%.json}.err
  echo "c2 $v $(summ $f)"
done
