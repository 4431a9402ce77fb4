#!/bin/bash
# Round-4 GPU call: the -m gpu suite + smoke, then the C2 schedule A/B and the
# C5 bench line (the C5 shared-learn stamp A/B: tools/stamp_shared.py [lib]).
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
timeout -k 10 300 python bench.py --shared --rows 8 --cols 8 --envs 256 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err
tail -1 $O/bench_c5.json | cut -c1-300
