#!/bin/bash
# rocprofv3 evidence for the one-GPU BASELINE configurations (run via gpurun
# from the repo root).  Per configuration:
#   1. --kernel-trace --stats of the default bench (steady state, n = 10000)
#   2. --pmc FETCH_SIZE and 3. --pmc WRITE_SIZE (separate passes, TCC slots),
#      reduced by tools/pmc_learn.py into profiles/learn_pmc.json for the learn
#      kernel and k_sim_step (gfx950 corrections: FETCH x2, WRITE x1)
#   4. --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES (own pass),
#      per learn kernel (C5 launches four: next, grad, slab reduction, Adam)
# Summaries are copied to gpurun_out/<tag>/<cfg>/ for committing under
# profiles/<round>/.  Every GPU step has its own time limit; `set -e` stops the
# chain at the first failure.
# usage: bash tools/profile_configs.sh <tag> c2|c3|c5 ...
set -e
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
for CFG in "$@"; do
    case $CFG in
        c2) ARGS="--rows 2 --cols 2 --envs 256 --precision bf16"; KEY=2x2x256_bf16; LK=k_learn_bf16
            SIMK="k_sim_step<true, false, false>"; ENVK="k_sim_step<true, false, true>" ;;
        c3) ARGS="--rows 4 --cols 4 --envs 1024 --precision fp16"; KEY=4x4x1024_fp16; LK=k_learn_f16
            SIMK="k_sim_step<true, false, false>"; ENVK="k_sim_step<true, false, true>" ;;
        c5) ARGS="--shared --rows 8 --cols 8 --envs 256"; KEY=8x8x256_fp16_shared; LK="k_shared_next|k_shared_grad|k_reduce_adam"
            SIMK="k_sim_step_reg<1024, false>"; ENVK="k_sim_step_reg<1024, true>" ;;
        *) echo "unknown config $CFG"; exit 2 ;;
    esac
    O=$R/gpurun_out/$TAG/$CFG
    mkdir -p $O
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run \
        -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline $ARGS > $O/bench_prof.json 2> $O/bench_prof.err
    echo "$CFG stats done"
    timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmcF -o run \
        -- python3 $R/bench.py --steps 4 --warmup 1 --prefill-steps 1100 --no-cpu-baseline --overlap none $ARGS > $O/pmcF.log 2>&1
    echo "$CFG fetch done"
    timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmcW -o run \
        -- python3 $R/bench.py --steps 4 --warmup 1 --prefill-steps 1100 --no-cpu-baseline --overlap none $ARGS > $O/pmcW.log 2>&1
    echo "$CFG write done"
    timeout -k 10 400 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES \
        --output-format csv -d $O/pmcM -o run \
        -- python3 $R/bench.py --steps 4 --warmup 1 --prefill-steps 1100 --no-cpu-baseline --overlap none $ARGS > $O/pmcM.log 2>&1
    echo "$CFG mfma done"
    F=$(find $O/pmcF -name '*counter_collection.csv' | head -n 1)
    W=$(find $O/pmcW -name '*counter_collection.csv' | head -n 1)
    M=$(find $O/pmcM -name '*counter_collection.csv' | head -n 1)
    # the sim key: the bench's sim probe (k_sim_step alone, the launches
    # sim_roofline times); the envstep key: the fused env step of the loop
    (cd $R && python3 tools/pmc_learn.py "$F" "$W" "$KEY" "$LK" "profiles/$TAG/$CFG" &&
         python3 tools/pmc_learn.py "$F" "$W" "${KEY%%_*}_sim" "$SIMK" "profiles/$TAG/$CFG" &&
         python3 tools/pmc_learn.py "$F" "$W" "${KEY%%_*}_envstep" "$ENVK" "profiles/$TAG/$CFG" &&
         for K1 in ${LK//|/ }; do python3 tools/pmc_mfma.py "$M" "$K1" > $O/mfma_busy_$K1.json; done)
    cp "$(find $O/stats -name '*kernel_stats.csv' | head -n 1)" $O/kernel_stats.csv
    # per launch size (a kernel launched at two sizes, e.g. C2's side-stream learn)
    python3 $R/tools/trace_by_grid.py "$(find $O/stats -name '*kernel_trace.csv' | head -n 1)" \
        k_learn k_shared k_sim_step k_sample > $O/kernel_stats_by_grid.json
    gzip -c "$F" > $O/fetch_size_counter_collection.csv.gz
    gzip -c "$W" > $O/write_size_counter_collection.csv.gz
    gzip -c "$M" > $O/mfma_counter_collection.csv.gz
    cp $R/profiles/learn_pmc.json $O/
    rm -rf $O/stats $O/pmcF $O/pmcW $O/pmcM
done
