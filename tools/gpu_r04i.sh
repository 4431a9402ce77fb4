#!/bin/bash
# k_shared_next on 12 waves (3 per SIMD) with one 16-row tile per weight read
# (-DNEXT_WAVES=12 -DNEXT_NT=1) vs the default 8 waves x 2 tiles; same box,
# alternating processes, unperturbed HIP-event timing of the whole shared learn.
# Result: profiles/r04/ab/next_12waves_ab.jsonl (slower; not kept).
set -e
O=gpurun_out/r04i
mkdir -p $O
for r in 1 2 3; do
  for n in g4base n12nt1; do
    timeout -k 10 120 python3 tools/stamp_shared.py exp/libdmdqn_hip_$n.so --nostamp >> $O/ab.jsonl 2>> $O/ab.err
    tail -1 $O/ab.jsonl
  done
done
timeout -k 10 120 python3 tools/stamp_shared.py exp/libdmdqn_hip_n12nt1.so > $O/stamp_n12nt1.json 2>> $O/ab.err
cat $O/stamp_n12nt1.json
