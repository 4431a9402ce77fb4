# A/B sim variants (timing): bash tools/cmp_sim.sh "-DA" "-DB" ...
set -e
for v in "$@"; do
  DMDQN_EXTRA_FLAGS="$v" python3 -m dmdqn_amd.build > gpurun_out/build.log 2>&1
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 30 --warmup 5 "${BENCH_ARGS[@]}" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(\"$v\", d[\"ms_per_step\"], d[\"sim_roofline\"][\"avg_launch_ms\"], d[\"sim_roofline\"][\"mean_running_vehicles\"])"
done
