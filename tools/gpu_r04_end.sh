#!/bin/bash
# Round-4 end: rocprof passes of C2 / C3 / C5 on HEAD's kernels (PMC digests
# current), then the rehearsal (-m gpu suite, smoke, the three bench lines).
set -e
bash tools/profile_configs.sh r04 c2 c3 c5 > gpurun_out/profcfg_end.log 2>&1
tail -3 gpurun_out/profcfg_end.log
bash tools/gpu_round_final.sh > gpurun_out/final_end.log 2>&1
tail -8 gpurun_out/final_end.log | cut -c1-250
