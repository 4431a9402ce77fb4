"""Diagnostic: the replay sampler (k_sample) alone at C3 size (1024 envs x 16
agents x 128 draws), HIP-event timed, for a pool-branch n (the bench's early
training) and a set-branch n.  usage: python tools/sample_bench.py [reps]"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dmdqn_amd import kernels as K  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
E, A = 1024, 16
st = K.seed_streams(np.arange(E), "py", "cuda")
out = torch.empty((E * A, 128), dtype=torch.int32, device="cuda")
res = {}
for n in (200, 10000):
    for _ in range(3):
        K.replay_sample(st, A, n, 128, out=out)
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        K.replay_sample(st, A, n, 128, out=out)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1000)
    res[f"n{n}_us"] = round(float(np.median(ts)), 1)
print(json.dumps(res))
