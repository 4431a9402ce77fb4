"""Per (kernel, grid size) launch count and mean / median duration (us) from a
rocprofv3 kernel trace CSV -- the launches of one kernel at different sizes
(e.g. C2's learn: the learn stream's 960 agents and the side stream's 64)
that kernel_stats.csv averages together.
usage: python tools/trace_by_grid.py run_kernel_trace.csv [name-substring ...] > out.json"""
import csv
import json
import statistics
import sys

path, pats = sys.argv[1], sys.argv[2:]
groups = {}
for r in csv.DictReader(open(path)):
    name = r["Kernel_Name"]
    if pats and not any(p in name for p in pats):
        continue
    key = f"{name[:80]} | grid {r['Grid_Size_X']}x{r['Grid_Size_Y']}x{r['Grid_Size_Z']}"
    groups.setdefault(key, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
out = {k: {"calls": len(v), "mean_us": round(statistics.fmean(v), 2),
           "median_us": round(statistics.median(v), 2)} for k, v in sorted(groups.items())}
print(json.dumps(out, indent=1))
