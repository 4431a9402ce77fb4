# Round check on the GPU box: gpu tests, smoke, kernel-trace + PMC profile, default bench.
# usage (via gpurun): TAG=v9 bash tools/gpu_round_check.sh
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_${TAG:-v8}.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${TAG:-v8}.log 2>&1 && \
bash tools/profile_bench.sh ${TAG:-v8} 4x4x1024_fp16
