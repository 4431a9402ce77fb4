#!/bin/bash
# Cross-stream events with a device-scope release (_lib.DeviceEvent, the
# trainer default) vs torch events (system scope) at C2 under --overlap auto,
# alternating processes; then the overlap schedules' bit-identity tests.
# Result: profiles/r04/ab/c2_event_scope_ab.txt -- the same 4.15-4.21 M either
# way, so the device-scope events (and --torch-events) are not in the tree.
set -e
O=gpurun_out/r04j
mkdir -p $O
summ() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); r=d['roofline']; print(d['value'], d['ms_per_step'], r['avg_launch_ms'], r['frac'])" $1; }
for i in 1 2 3; do
  for v in "" "--torch-events"; do
    f=$O/c2_dev${v//-/_}_$i.json
    timeout -k 10 300 python bench.py --rows 2 --cols 2 --envs 256 --precision bf16 --no-cpu-baseline $v > $f 2> ${f%.json}.err
    echo "c2 ${v:-device-events} $(summ $f)"
  done
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_overlap.py tests/test_gpu_fullsize.py -k "overlap or env_beside or schedules" > $O/tests.log 2>&1
tail -2 $O/tests.log
