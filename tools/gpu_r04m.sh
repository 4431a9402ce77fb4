#!/bin/bash
# C5 sim: per-pass timers of the register path (DMDQN_VARIANT=prof), then the
# register path's lane arrays a compile-time stride apart (product) vs NL apart
# (DMDQN_VARIANT=exp, built with -DSIM_LANE_STRIDE_NT=0): C5 bench lines,
# alternating; then the sim parity tests on the product build.
set -e
O=gpurun_out/r04m
mkdir -p $O
DMDQN_VARIANT=prof timeout -k 10 200 python tools/sim_profile.py 8 8 256 --fused | tee $O/sim_profile_c5.txt
summ() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['sim_roofline']['avg_launch_ms'])" $1; }
for i in 1 2; do
  for v in "" exp; do
    f=$O/c5_${v:-prod}_$i.json
    DMDQN_VARIANT=$v timeout -k 10 300 python bench.py --shared --rows 8 --cols 8 --envs 256 --no-cpu-baseline > $f 2> ${f%.json}.err
    echo "c5 ${v:-prod} $(summ $f)"
  done
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sim.py tests/test_gpu_fused.py > $O/tests.log 2>&1
tail -1 $O/tests.log
