#!/bin/bash
# The tests the r04a call did not reach, then the C2 schedule A/B and the C5 bench.
set -e
O=gpurun_out/r04b
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_sumo_env.py tests/test_gpu_split.py -m gpu -x -v \
    --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1
tail -2 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
for rep in 1 2; do
  for v in "none" "env" "env --cu-split 32" "env --cu-split 64"; do
    f=$O/c2_${v// /_}_$rep.json
    timeout -k 10 300 python bench.py --rows 2 --cols 2 --envs 256 --precision bf16 --steps 200 \
        --no-cpu-baseline --overlap $v > $f 2> ${f%.json}.err
    echo "$v $rep $(python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])" $f)"
  done
done
timeout -k 10 300 python bench.py --shared --rows 8 --cols 8 --envs 256 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err
tail -1 $O/bench_c5.json | cut -c1-400
