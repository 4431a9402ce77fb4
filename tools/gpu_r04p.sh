#!/bin/bash
# k_shared_grad4 with 2 row tiles per pass of L1 / L2 / dH1 (-DSH_G4_RH=2)
# vs the default 4, unperturbed HIP-event timing, alternating, 3 rounds.
# Result: profiles/r04/ab/grad4_rh2_ab.jsonl (the same; the switch is not in
# the tree).
set -e
O=gpurun_out/r04p
mkdir -p $O
for r in 1 2 3; do
  for n in g4base g4rh2; do
    timeout -k 10 120 python3 tools/stamp_shared.py exp/libdmdqn_hip_$n.so --nostamp >> $O/ab.jsonl 2>> $O/ab.err
    tail -1 $O/ab.jsonl
  done
done
