"""Summarise tools/ab_learn.sh output: python tools/ab_summary.py <file>"""
import collections
import json
import sys

d = collections.defaultdict(list)
for line in open(sys.argv[1]):
    if line.startswith(("old ", "new ")):
        k, j = line.split(" ", 1)
        d[k].append(json.loads(j)["median_ms"])
for k, v in d.items():
    v = sorted(v)
    print(k, " ".join(f"{x:.3f}" for x in v), f"| median {v[len(v) // 2]:.4f} min {v[0]:.4f}")
