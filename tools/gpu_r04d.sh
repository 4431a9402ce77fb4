#!/bin/bash
# C5 shared-learn variant A/B, unperturbed HIP-event timing (tools/stamp_shared.py --nostamp).
# The exp/ libraries were built by tools/build_exp.py from round-4 switches
# (dH1/dW2 order, rows per pass, next-pass tiles/waves) that were measured
# without a gain and are no longer in the tree; kept as a record.
set -e
O=gpurun_out/r04d
mkdir -p $O
for rep in 1 2 3; do
  for v in g4base g4order g4rh8 g4order_rh8 next12 next16nt1; do
    timeout -k 10 120 python tools/stamp_shared.py exp/libdmdqn_hip_$v.so --nostamp >> $O/ab.jsonl
  done
done
cat $O/ab.jsonl
