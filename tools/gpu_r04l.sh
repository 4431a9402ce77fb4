#!/bin/bash
# overlap env: ordering-only events for the learn -> side-stream wait (the
# default) vs default torch events (--fenced-events) at C2, alternating; then
# the overlap schedules' bit-identity tests.
set -e
O=gpurun_out/r04l
mkdir -p $O
summ() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); r=d['roofline']; print(d['value'], d['ms_per_step'], r['avg_launch_ms'])" $1; }
for i in 1 2 3; do
  for v in "" "--fenced-events"; do
    f=$O/c2${v//-/_}_$i.json
    timeout -k 10 300 python bench.py --rows 2 --cols 2 --envs 256 --precision bf16 --no-cpu-baseline $v > $f 2> ${f%.json}.err
    echo "c2 ${v:-order-events} $(summ $f)"
  done
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_overlap.py tests/test_gpu_fullsize.py -k "overlap or env_beside or schedules" > $O/tests.log 2>&1
tail -1 $O/tests.log
