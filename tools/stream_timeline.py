"""Diagnostic: where the GPU's streams idle in the steady state, from a
rocprofv3 kernel trace CSV (--kernel-trace).  Kernels are grouped by the
trace's queue / stream id; for the last N launches of the learn kernel on
the learn stream it prints, per step (learn start to the next learn start):
the learn's duration, the gap before it, and what the other stream ran in
that step (kernel, grid, start offset and duration, us).
usage: python tools/stream_timeline.py run_kernel_trace.csv [learn-substring] [N] [skip]
  skip: leave out the last `skip` learns (bench.py runs SIM_PROBE_STEPS = 10
  untimed steps after its timed region, with a V-bar reduction on the learn
  stream between them: pass 10 to see the timed steps only)"""
import csv
import json
import statistics
import sys

path = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else "k_learn"
N = int(sys.argv[3]) if len(sys.argv) > 3 else 12
SKIP = int(sys.argv[4]) if len(sys.argv) > 4 else 0
rows = list(csv.DictReader(open(path)))
qkey = next((k for k in ("Stream_Id", "Queue_Id") if k in rows[0]), None)
ks = sorted(({"name": r["Kernel_Name"].split("(")[0][-48:], "q": r.get(qkey, "?"),
              "grid": int(r["Grid_Size_X"]), "t0": int(r["Start_Timestamp"]) / 1e3,
              "t1": int(r["End_Timestamp"]) / 1e3} for r in rows), key=lambda k: k["t0"])
learn = [k for k in ks if pat in k["name"]]
# the learn stream: the queue of the biggest learn launches
big = max(k["grid"] for k in learn)
lq = next(k["q"] for k in learn if k["grid"] == big)
main = [k for k in learn if k["q"] == lq and k["grid"] == big]
main = main[:len(main) - SKIP][-N - 1:]
steps = []
for a, b in zip(main, main[1:]):
    other = [{"name": k["name"], "q": k["q"], "grid": k["grid"], "start": round(k["t0"] - a["t0"], 1),
              "us": round(k["t1"] - k["t0"], 1)}
             for k in ks if a["t0"] <= k["t0"] < b["t0"] and k is not a]
    steps.append({"step_us": round(b["t0"] - a["t0"], 1), "learn_us": round(a["t1"] - a["t0"], 1),
                  "gap_after_learn_us": round(b["t0"] - a["t1"], 1), "others": other})
out = {"queue_key": qkey, "learn_queue": lq, "learn_grid": big,
       "median_step_us": round(statistics.median(s["step_us"] for s in steps), 1),
       "median_learn_us": round(statistics.median(s["learn_us"] for s in steps), 1),
       "median_gap_us": round(statistics.median(s["gap_after_learn_us"] for s in steps), 1),
       "steps": steps[-4:]}
print(json.dumps(out, indent=1))
