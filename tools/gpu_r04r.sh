#!/bin/bash
# overlap env + side_learn: the parity tests, then C2 with the side stream
# learning 128 agents (the auto default) vs none, alternating, 2 rounds; and
# 64 / 192 agents once.
set -e
O=gpurun_out/r04r
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_overlap.py > $O/tests.log 2>&1
tail -1 $O/tests.log
summ() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); r=d['roofline']; print(d['value'], d['ms_per_step'], r['avg_launch_ms'], r['frac'])" $1; }
for i in 1 2; do
  for m in 128 0; do
    f=$O/c2_side${m}_$i.json
    timeout -k 10 300 python bench.py --rows 2 --cols 2 --envs 256 --precision bf16 --no-cpu-baseline --side-learn $m > $f 2> ${f%.json}.err
    echo "c2 side_learn=$m $(summ $f)"
  done
done
for m in 64 192; do
  f=$O/c2_side${m}.json
  timeout -k 10 300 python bench.py --rows 2 --cols 2 --envs 256 --precision bf16 --no-cpu-baseline --side-learn $m > $f 2> ${f%.json}.err
  echo "c2 side_learn=$m $(summ $f)"
done
