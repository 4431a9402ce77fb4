cd ${GRAFT_REPO_ROOT:-.}
run() { timeout -k 10 200 env $2 python bench.py --no-cpu-baseline --steps 100 $3 > gpurun_out/ab_$1.json 2>gpurun_out/ab_$1.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/ab_$1.json'));print('$1',d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'],d['sim_roofline']['avg_launch_ms'])"; }
for i in 1 2; do
run off$i "X=1" --no-overlap
run on$i "X=1" ""
run prio$i "DMDQN_WORK_PRIO=-1" ""
done
