#!/bin/bash
# k_shared_grad4 VALU A/B (tools/build_exp.py switches): packed relu, int8->f16
# by magic number, X staging after the dW phase, setprio for waves 4-7, packed
# dZ2 rows, all of them.  Unperturbed HIP-event timing of the whole shared learn
# (tools/stamp_shared.py --nostamp), alternating libraries, one box.  Result:
# profiles/r04/ab/grad4_valu_ab.jsonl (all within noise, bit-identical); the
# packed relu and the int8 conversion were kept, the other switches removed.
set -e
O=gpurun_out/r04f
mkdir -p $O
for r in 1 2 3; do
  for n in g4base relu xmagic latex prio pkz2 g4all; do
    timeout -k 10 120 python3 tools/stamp_shared.py exp/libdmdqn_hip_$n.so --nostamp >> $O/ab.jsonl 2>> $O/ab.err
    tail -1 $O/ab.jsonl
  done
done
