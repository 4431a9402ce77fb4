"""Diagnostic: the C5 shared learn with the slab reduction and Adam as one
launch (dmdqn_adam_slabs, BatchedDQN's one-rank path) against the separate
reduce + dmdqn_adam launches, same process, alternating, at C5 size (256 envs
x 64 agents) on random replay contents.  Prints the median ms per learn of
each (HIP events around whole learns)."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dmdqn_amd.agent import LOSSES, AgentConfig, BatchedDQN  # noqa: E402

E, A = 256, 64
ag = BatchedDQN(E, A, AgentConfig(precision="fp16", seed=0, shared_params=True,
                                  replay_buffer_size=1000))
g = torch.Generator(device="cuda").manual_seed(0)
for t in range(200):
    s = torch.randint(-1, 24, (E, A, 89), device="cuda", generator=g).float()
    a = torch.randint(0, 4, (E, A), device="cuda", generator=g, dtype=torch.int32)
    r = -torch.rand((E, A), device="cuda", generator=g, dtype=torch.float64) * 100
    ag.remember(s, a, r, s, t % 60 == 59)


def separate():
    assert ag.learn_begin()
    alpha, c1, c2, eps, sync, qstats = ag._last_learn
    ring, cfg = ag.ring, ag.cfg
    ag._ops.learn_shared_grad(ring.s, ring.n, ring.a, ring.d, ring.r, ag.idx, ag.params, ag.target,
                              ag.target_h, ag.params_h, ag.loss, ring.start, cfg.gamma,
                              LOSSES[cfg.loss], qstats, ag.rn_out, ag.slab, ag.grad, 1.0 / ag.NA,
                              work=ag.shared_work)
    ag._ops.adam(ag.params, ag.adam_m, ag.adam_v, ag.target, ag.target_h, ag.params_h, ag.grad,
                 1.0, alpha, c1, c2, eps, sync)


def timed(fn, reps=20):
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return ts


for _ in range(3):
    ag.learn()
res = {"fused": [], "separate": []}
for rnd in range(int(sys.argv[1]) if len(sys.argv) > 1 else 6):
    res["fused"] += timed(ag.learn)
    res["separate"] += timed(separate)
print(json.dumps({k: {"median_ms": round(float(np.median(v)), 4), "min_ms": round(min(v), 4),
                      "n": len(v)} for k, v in res.items()}))
