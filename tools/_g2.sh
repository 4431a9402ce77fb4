cd ${GRAFT_REPO_ROOT:-.}
timeout -k 10 300 python -u -m pytest tests/test_gpu_overlap.py -x -v --timeout 200 --timeout-method thread > gpurun_out/ovl_test.log 2>&1 && \
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/ovl_bench_on.json 2>gpurun_out/ovl_bench_on.err && \
timeout -k 10 200 python bench.py --no-cpu-baseline --no-overlap > gpurun_out/ovl_bench_off.json 2>gpurun_out/ovl_bench_off.err && \
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/ovl_bench_on2.json 2>>gpurun_out/ovl_bench_on.err
tail -3 gpurun_out/ovl_test.log
for f in on off on2; do python -c "import json;d=json.load(open('gpurun_out/ovl_bench_$f.json'));print('$f',d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'],d['sim_roofline']['avg_launch_ms'])"; done
