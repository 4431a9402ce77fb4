#!/bin/bash
# One GPU call as a list of named steps, each under its own time limit, the
# first failure ending the call (no GPU step after a fault, abort or timeout).
# Output: gpurun_out/<tag>/<step>.{json,log}.
# usage: bash tools/gpu_steps.sh <tag> <step> [<step> ...]
#   tests[=<pytest -k expr>]   the -m gpu suite (or a subset), verbose, 120 s per test
#   bench_c2 | bench_c3 | bench_c5 [extra bench.py args via BENCH_ARGS]
#   ab_revs                    tools/ab_learn_lib.py over dmdqn_amd/lib + exp/libdmdqn_hip_*.so
#   prof_c2 | prof_c3 | prof_c5  rocprofv3 --kernel-trace --stats of a short bench run
#   smoke                      __graft_entry__.smoke()
set -u
tag=$1; shift
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
cfg() {
  case $1 in
    c2) echo "--rows 2 --cols 2 --envs 256 --precision bf16" ;;
    c3) echo "" ;;
    c5) echo "--rows 8 --cols 8 --envs 256 --shared" ;;
  esac
}
run() {  # run <seconds> <logfile> <cmd...>
  local t=$1 log=$2; shift 2
  echo "== $(date +%T) $* (limit ${t}s)"
  timeout -k 10 "$t" "$@" > "$log" 2>&1
  local rc=$?
  echo "   rc=$rc"
  if [ $rc -ne 0 ]; then tail -30 "$log"; exit $rc; fi
}
for step in "$@"; do
  case $step in
    tests)
      run 900 "$out/tests.log" python -u -m pytest tests -m gpu -x -v --timeout 300 \
        --timeout-method thread ;;
    tests=*)
      run 900 "$out/tests_${step#tests=}.log" python -u -m pytest tests -m gpu -x -v --timeout 300 \
        --timeout-method thread -k "${step#tests=}" ;;
    bench_c2|bench_c3|bench_c5)
      c=${step#bench_}
      run 400 "$out/$step.log" python -u bench.py --steps 200 --warmup 10 $(cfg $c) ${BENCH_ARGS:-}
      grep '^{' "$out/$step.log" > "$out/$step.json" ;;
    prof_c2|prof_c3|prof_c5)
      c=${step#prof_}
      run 500 "$out/$step.log" rocprofv3 --kernel-trace --stats -d "$out/$step" -o run -- \
        python3 -u bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-stream-probe $(cfg $c) ;;
    ab_revs)
      libs="dmdqn_amd/lib/libdmdqn_hip.so $(ls exp/libdmdqn_hip_*.so 2>/dev/null)"
      run 500 "$out/ab_revs.log" python -u tools/ab_learn_lib.py --rounds ${AB_ROUNDS:-6} $libs
      grep '^{' "$out/ab_revs.log" > "$out/ab_revs.json" ;;
    smoke)
      run 300 "$out/smoke.log" python -u -c "import __graft_entry__ as g; g.smoke()" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "== done $(date +%T)"
