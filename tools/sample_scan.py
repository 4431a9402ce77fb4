"""Diagnostic: k_sample duration vs agents per env and draws per agent (set
branch, n = 10000, 1024 envs), HIP events around back-to-back launches queued
behind a GPU sleep.  Separates the per-launch fixed cost (MT state load /
store, table init) from the per-draw chunk loop.  usage: python tools/sample_scan.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dmdqn_amd import kernels as K  # noqa: E402

E, n, reps = 1024, 10000, 20
st = K.seed_streams(list(range(E)), "py", "cuda")
res = {}
for A, k in ((1, 1), (1, 128), (4, 128), (16, 128), (16, 256)):
    out = torch.empty((E * A, k), dtype=torch.int32, device="cuda")
    K.replay_sample(st, A, n, k, out=out)
    torch.cuda.synchronize()
    torch.cuda._sleep(int(3e6))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        K.replay_sample(st, A, n, k, out=out)
    e1.record()
    torch.cuda.synchronize()
    res[f"A{A}_k{k}_us"] = round(e0.elapsed_time(e1) * 1000 / reps, 1)
print(json.dumps(res))
