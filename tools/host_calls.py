"""Diagnostic: host time of each call inside Trainer.step (act, env.step,
remember, learn) in steady state, on a dedicated stream as bench.py runs.
usage: python tools/host_calls.py [rows cols envs precision]"""
import sys
import time

import torch

sys.path.insert(0, ".")
from dmdqn_amd.agent import AgentConfig  # noqa: E402
from dmdqn_amd.env import EnvConfig  # noqa: E402
from dmdqn_amd.trainer import Trainer  # noqa: E402

R, C, E, prec = (int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]) \
    if len(sys.argv) > 4 else (2, 2, 256, "bf16")
dev = torch.device("cuda", 0)
work = torch.cuda.Stream(dev)
torch.cuda.set_stream(work)
tr = Trainer(EnvConfig(rows=R, cols=C, num_envs=E, seed=1000), AgentConfig(precision=prec, seed=1000),
             device=dev)
for _ in range(140):
    tr.step()
torch.cuda.synchronize()
env, ag = tr.env, tr.agent
acc = {k: 0.0 for k in ["act", "env.step", "remember", "learn", "rest"]}
n = 100
t0 = time.perf_counter()
for _ in range(n):
    a = time.perf_counter()
    actions = ag.act(tr.obs)
    b = time.perf_counter()
    nxt, rew, done, info = env.step(actions)
    c = time.perf_counter()
    ag.remember(tr.obs, actions, rew, nxt, info["done"])
    d = time.perf_counter()
    ag.learn()
    e = time.perf_counter()
    tr.obs = tr._after_step(done, nxt, info)
    f = time.perf_counter()
    for k, x in zip(acc, (b - a, c - b, d - c, e - d, f - e)):
        acc[k] += x
issue = time.perf_counter() - t0
torch.cuda.synchronize()
wall = time.perf_counter() - t0
print({k: round(v / n * 1e3, 4) for k, v in acc.items()}, "issue ms/step", round(issue / n * 1e3, 4),
      "wall ms/step", round(wall / n * 1e3, 4))
