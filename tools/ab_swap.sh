#!/bin/bash
# Same-box A/B of whole libdmdqn_hip.so builds under bench.py (run via gpurun
# from the repo root): each library (e.g. exp/libdmdqn_hip_<rev>.so from
# tools/build_rev.py) is copied over dmdqn_amd/lib/libdmdqn_hip.so in turn --
# libdmdqn_torch.so loads it by name -- and bench.py runs with the given
# arguments; alternating rounds; the product library is restored at the end.
# usage: bash tools/ab_swap.sh <tag> <rounds> "<bench args>" lib1.so lib2.so ...
set -u
tag=$1 rounds=$2 bargs=$3; shift 3
out=gpurun_out/$tag
mkdir -p "$out"
prod=dmdqn_amd/lib/libdmdqn_hip.so
export DMDQN_ALLOW_FOREIGN_LIB=1  # the swapped-in libraries are other revisions (_lib.verify_digest)
cp "$prod" "$out/_product.so"
restore() { cp "$out/_product.so" "$prod"; rm -f "$out/_product.so"; }
trap restore EXIT
for r in $(seq 1 "$rounds"); do
  for lib in "$@"; do
    name=$(basename "$lib" .so)
    cp "$lib" "$prod"
    echo "== $(date +%T) round $r $name"
    timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-stream-probe --steps ${AB_STEPS:-200} \
      $bargs > "$out/${name}_r${r}.json" 2> "$out/${name}_r${r}.err"
    rc=$?
    if [ $rc -ne 0 ]; then echo "rc=$rc"; tail -20 "$out/${name}_r${r}.err"; exit $rc; fi
  done
done
python3 - "$out" "$@" <<'E'
import glob, json, os, sys
out, libs = sys.argv[1], sys.argv[2:]
for lib in libs:
    name = os.path.basename(lib)[:-3]
    rows = []
    for f in sorted(glob.glob(f"{out}/{name}_r*.json")):
        d = json.loads([l for l in open(f) if l.startswith("{")][-1])
        sim = (d.get("sim_roofline") or {}).get("avg_launch_ms")
        rows.append((d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"], sim))
    print(json.dumps({"lib": name, "values": [r[0] for r in rows], "ms_per_step": [r[1] for r in rows],
                      "learn_ms": [r[2] for r in rows], "sim_ms": [r[3] for r in rows]}))
E
