#!/bin/bash
# bench.py with fence-free timing events on every 4th learn (the default):
# C2 (auto), C5, C3 lines, and the 2-rank bench launch test.
set -e
O=gpurun_out/r04k
mkdir -p $O
summ() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); r=d['roofline']; print(d['value'], d['ms_per_step'], r['avg_launch_ms'], r['timed_launches'], r['frac'])" $1; }
for i in 1 2; do
  timeout -k 10 300 python bench.py --rows 2 --cols 2 --envs 256 --precision bf16 --no-cpu-baseline > $O/c2_$i.json 2> $O/c2_$i.err
  echo "c2 $(summ $O/c2_$i.json)"
done
timeout -k 10 300 python bench.py --shared --rows 8 --cols 8 --envs 256 --no-cpu-baseline > $O/c5.json 2> $O/c5.err
echo "c5 $(summ $O/c5.json)"
timeout -k 10 300 python bench.py --steps 100 --no-cpu-baseline > $O/c3.json 2> $O/c3.err
echo "c3 $(summ $O/c3.json)"
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_multiproc.py -k bench > $O/tests.log 2>&1
tail -1 $O/tests.log
