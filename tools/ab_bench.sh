#!/bin/bash
# Same-box A/B of bench.py configurations, alternating (run via gpurun from the
# repo root).  Each variant is one quoted string of bench.py arguments.
# usage: bash tools/ab_bench.sh <tag> <rounds> "<args A>" "<args B>" ...
# Output: gpurun_out/<tag>/v<i>_r<k>.json and a summary line per variant.
set -u
tag=$1 rounds=$2; shift 2
out=gpurun_out/$tag
mkdir -p "$out"
for r in $(seq 1 "$rounds"); do
  i=0
  for v in "$@"; do
    echo "== $(date +%T) round $r variant $i: $v"
    timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-stream-probe --steps ${AB_STEPS:-200} \
      $v > "$out/v${i}_r${r}.json" 2> "$out/v${i}_r${r}.err"
    rc=$?
    if [ $rc -ne 0 ]; then echo "rc=$rc"; tail -20 "$out/v${i}_r${r}.err"; exit $rc; fi
    i=$((i + 1))
  done
done
python3 - "$out" "$@" <<'E'
import glob, json, sys
out, variants = sys.argv[1], sys.argv[2:]
for i, v in enumerate(variants):
    rows = []
    for f in sorted(glob.glob(f"{out}/v{i}_r*.json")):
        d = json.loads([l for l in open(f) if l.startswith("{")][-1])
        rows.append((d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"]))
    print(json.dumps({"variant": v, "values": [r[0] for r in rows],
                      "ms_per_step": [r[1] for r in rows], "learn_ms": [r[2] for r in rows]}))
E
