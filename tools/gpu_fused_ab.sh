set -o pipefail
mkdir -p gpurun_out/f1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_fused.py > gpurun_out/f1/t_fused.log 2>&1 || { tail -50 gpurun_out/f1/t_fused.log; exit 1; }
tail -3 gpurun_out/f1/t_fused.log
for i in 1 2; do
timeout -k 10 200 python bench.py --rows 2 --cols 2 --envs 256 --precision bf16 --no-cpu-baseline > gpurun_out/f1/c2_fused_$i.json 2> gpurun_out/f1/c2_fused_$i.err || exit 1
timeout -k 10 200 python bench.py --rows 2 --cols 2 --envs 256 --precision bf16 --no-cpu-baseline --no-fuse > gpurun_out/f1/c2_unfused_$i.json 2> gpurun_out/f1/c2_unfused_$i.err || exit 1
done
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/f1/c3_fused.json 2> gpurun_out/f1/c3_fused.err || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --no-fuse > gpurun_out/f1/c3_unfused.json 2> gpurun_out/f1/c3_unfused.err || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --shared --rows 8 --cols 8 --envs 256 > gpurun_out/f1/c5_fused.json 2> gpurun_out/f1/c5_fused.err || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --shared --rows 8 --cols 8 --envs 256 --no-fuse > gpurun_out/f1/c5_unfused.json 2> gpurun_out/f1/c5_unfused.err || exit 1
for f in gpurun_out/f1/*.json; do echo $f; python -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"; done
