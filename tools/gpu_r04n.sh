#!/bin/bash
# Register-path sim: staging with constant register indices and the next
# speed read one vehicle ahead in pass C (DMDQN_VARIANT=exp, built with
# -DSIM_STAGE_UNROLL=1 -DSIM_VPREF=1) vs the product build: C5 bench lines,
# alternating; then the sim parity tests on the exp build.  Result:
# profiles/r04/sim/unroll_vpref_*.json (much slower; neither switch is in the
# tree any more).
set -e
O=gpurun_out/r04n
mkdir -p $O
summ() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['sim_roofline']['avg_launch_ms'])" $1; }
for i in 1 2; do
  for v in "" exp; do
    f=$O/c5_${v:-prod}_$i.json
    DMDQN_VARIANT=$v timeout -k 10 300 python bench.py --shared --rows 8 --cols 8 --envs 256 --no-cpu-baseline > $f 2> ${f%.json}.err
    echo "c5 ${v:-prod} $(summ $f)"
  done
done
DMDQN_VARIANT=exp timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sim.py tests/test_gpu_fused.py > $O/tests.log 2>&1
tail -1 $O/tests.log
