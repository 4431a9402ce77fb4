#!/bin/bash
# Round-end rehearsal on one GPU: the -m gpu suite, smoke(), the default bench
# (C3, with the CPU baseline) and the C2 / C5 bench lines.  Outputs under
# gpurun_out/final/.  Every GPU step has its own limit; the chain stops at the
# first failure.
set -e
O=gpurun_out/final
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
tail -2 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -2 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench_c3.json 2> $O/bench_c3.err
tail -1 $O/bench_c3.json
timeout -k 10 300 python bench.py --rows 2 --cols 2 --envs 256 --precision bf16 --no-cpu-baseline > $O/bench_c2.json 2> $O/bench_c2.err
timeout -k 10 300 python bench.py --shared --rows 8 --cols 8 --envs 256 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err
for f in $O/bench_c2.json $O/bench_c5.json; do tail -1 $f | cut -c1-200; done
bash tools/prof_quick.sh gpurun_out/final/c5prof --shared --rows 8 --cols 8 --envs 256 --steps 30 | grep -E "sim_step|sample"
