"""Diagnostic: the fp16 (or --bf16) learn kernel alone at C3 size (16 agents x 1024 envs)
on random replay contents, timed with HIP events on one stream.  Prints the
median and min of N launches (ms) -- a tighter A/B signal than bench.py.
usage: python tools/learn_bench.py [N] [--shared] [--bf16] [--envs E] [--agents A]
(default E = 1024, A = 16: C3; C2 is --envs 256 --agents 4 --bf16)"""
import json
import sys

import numpy as np
import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from dmdqn_amd.agent import AgentConfig, BatchedDQN  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 40
shared = "--shared" in sys.argv
prec = "bf16" if "--bf16" in sys.argv else "fp16"
def _opt(name, default):
    return int(sys.argv[sys.argv.index(name) + 1]) if name in sys.argv else default


E, A = _opt("--envs", 1024), _opt("--agents", 16)
ag = BatchedDQN(E, A, AgentConfig(precision=prec, seed=0, shared_params=shared,
                                  replay_buffer_size=1000))
g = torch.Generator(device="cuda").manual_seed(0)
for t in range(200):
    s = torch.randint(-1, 24, (E, A, 89), device="cuda", generator=g).float()
    a = torch.randint(0, 4, (E, A), device="cuda", generator=g, dtype=torch.int32)
    r = -torch.rand((E, A), device="cuda", generator=g, dtype=torch.float64) * 100
    ag.remember(s, a, r, s, t % 60 == 59)
torch.cuda.synchronize()
for _ in range(5):
    ag.learn()
ts = []
for _ in range(N):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    ag.learn()
    e1.record()
    torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1))
print(json.dumps({"median_ms": round(float(np.median(ts)), 4), "min_ms": round(float(min(ts)), 4),
                  "n": N, "shared": shared, "precision": prec}))
