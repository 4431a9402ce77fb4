#!/bin/bash
# Round-4 GPU call: the -m gpu suite + smoke, then the C2 schedule A/B (one
# stream vs the fused env step beside the learn, with and without CU masks).
set -e
O=gpurun_out/r04a
mkdir -p $O
bash tools/gpu_tests.sh r04a
for rep in 1 2; do
  for v in "none" "env" "env --cu-split 32" "env --cu-split 64"; do
    f=$O/c2_${v// /_}_$rep.json
    timeout -k 10 300 python bench.py --rows 2 --cols 2 --envs 256 --precision bf16 --steps 200 \
        --no-cpu-baseline --overlap $v > $f 2> ${f%.json}.err
    echo "$v $rep $(python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])" $f)"
  done
done
