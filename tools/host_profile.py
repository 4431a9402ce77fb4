"""Diagnostic: host-side cost of Trainer.step at the bench workload.
Prints wall ms/step for the plain loop, the loop with bench's timing hooks,
and a cProfile summary of the plain loop."""
import cProfile
import pstats
import sys
import time

import torch

sys.path.insert(0, ".")
from dmdqn_amd.agent import AgentConfig  # noqa: E402
from dmdqn_amd.env import EnvConfig  # noqa: E402
from dmdqn_amd.trainer import Trainer  # noqa: E402

dev = torch.device("cuda", 0)
tr = Trainer(EnvConfig(rows=4, cols=4, num_envs=1024, seed=1000), AgentConfig(precision="fp16", seed=1000), device=dev)
for _ in range(137):
    tr.step()
torch.cuda.synchronize()


def run(n, hooks=False, learn_only=False):
    if hooks:
        pool = [torch.cuda.Event(enable_timing=True) for _ in range(4 * n)]
        it = iter(pool)
        tr.agent.learn_hook = lambda b: next(it).record()
        if not learn_only:
            tr.env.sim_hook = lambda b: next(it).record()
    vs = torch.zeros(1024, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    th = 0.0
    for _ in range(n):
        a = time.perf_counter()
        tr.step()
        if hooks:
            vs += tr.env.t_stats[:, 2]
        th += time.perf_counter() - a
    torch.cuda.synchronize()
    tr.agent.learn_hook = None
    tr.env.sim_hook = None
    return (time.perf_counter() - t0) / n * 1e3, th / n * 1e3


print("plain  wall/host ms per step: %.3f %.3f" % run(20))
print("hooks  wall/host ms per step: %.3f %.3f" % run(20, True))
print("learn-only hooks wall/host ms per step: %.3f %.3f" % run(20, True, True))
side = torch.cuda.Stream(dev)
with torch.cuda.stream(side):
    print("side stream plain  wall/host ms per step: %.3f %.3f" % run(20))
    print("side stream hooks  wall/host ms per step: %.3f %.3f" % run(20, True))
    print("side stream learn-only hooks: %.3f %.3f" % run(20, True, True))
