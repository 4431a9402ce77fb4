#!/bin/bash
# Same-box A/B of the C5 shared learn (dmdqn_learn_shared_grad: k_shared_next +
# k_shared_grad) across library builds, alternating (tools/stamp_shared.py
# --nostamp: HIP-event time of each launch, median of 20, and the gradient's
# sha1).  Run via gpurun from the repo root.
# usage: bash tools/ab_shared_libs.sh <tag> <rounds> lib1.so lib2.so ...
set -u
tag=$1 rounds=$2; shift 2
out=gpurun_out/$tag
mkdir -p "$out"
for r in $(seq 1 "$rounds"); do
  for lib in "$@"; do
    timeout -k 10 120 python3 -u tools/stamp_shared.py "$lib" --nostamp 2>>"$out/err.log" | grep '^{' >> "$out/ab.jsonl"
    rc=${PIPESTATUS[0]}
    if [ $rc -ne 0 ]; then echo "rc=$rc for $lib"; tail -20 "$out/err.log"; exit $rc; fi
  done
done
cat "$out/ab.jsonl"
