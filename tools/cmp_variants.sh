# A/B kernel variants in one GPU call (same box): bash tools/cmp_variants.sh "-DA" "-DB" ...
set -e
for v in "$@"; do
  DMDQN_EXTRA_FLAGS="$v" python3 -m dmdqn_amd.build > gpurun_out/build.log 2>&1
  timeout -k 10 300 python3 bench.py --no-cpu-baseline | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(\"$v\", d[\"value\"], d[\"roofline\"][\"avg_launch_ms\"], d[\"roofline\"][\"frac\"])"
done
