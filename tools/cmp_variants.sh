# A/B kernel variants in one GPU call (same box):
#   bash tools/cmp_variants.sh "-DFOO" "-DBAR=2" "file:tools/_base_learn_f16.hip"
# BENCH_ARGS (env) is appended to the bench command line; LEARN_ONLY=1 times
# the learn kernel alone (tools/learn_bench.py, median/min of 60 launches).
# A "file:" variant builds with that file in place of csrc/learn_h16.hpp.
set -e
SRC=dmdqn_amd/csrc/learn_h16.hpp
cp $SRC /tmp/_cur_learn_h16.hpp
for v in "$@"; do
  if [[ "$v" == file:* ]]; then
    cp "${v#file:}" $SRC; flags=""
  else
    cp /tmp/_cur_learn_h16.hpp $SRC; flags="$v"
  fi
  DMDQN_EXTRA_FLAGS="$flags -DDMDQN_VARIANT" python3 -m dmdqn_amd.build > gpurun_out/build.log 2>&1
  if [ -n "$LEARN_ONLY" ]; then
    timeout -k 10 300 python3 tools/learn_bench.py 60 $BENCH_ARGS | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(\"$v\", d[\"median_ms\"], d[\"min_ms\"])"
  else
    timeout -k 10 300 python3 bench.py --no-cpu-baseline $BENCH_ARGS | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(\"$v\", d[\"value\"], d[\"roofline\"][\"avg_launch_ms\"], d[\"roofline\"][\"frac\"])"
  fi
done
cp /tmp/_cur_learn_h16.hpp $SRC
DMDQN_EXTRA_FLAGS="" python3 -m dmdqn_amd.build > gpurun_out/build.log 2>&1  # leave the current source built
