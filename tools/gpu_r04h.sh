#!/bin/bash
# k_shared_grad4 with LDS phase counters in place of its four barriers
# (-DSH_G4_FLOW=1) vs the barrier form, same box, alternating processes;
# unperturbed HIP-event timing of the whole shared learn and the gradient sha1.
# Result: profiles/r04/ab/grad4_flow_ab.jsonl (bit-identical, 0-4 % slower);
# the variant was not kept and its source is not in the tree.
set -e
O=gpurun_out/r04h
mkdir -p $O
for r in 1 2 3; do
  for n in g4base flow; do
    timeout -k 10 120 python3 tools/stamp_shared.py exp/libdmdqn_hip_$n.so --nostamp >> $O/ab.jsonl 2>> $O/ab.err
    tail -1 $O/ab.jsonl
  done
done
