"""Diagnostic: C2 (2x2 x 256, bf16) under bench.py's --overlap auto layout
(env step beside the learn, side stream on 64 CUs): ms per step over K steps
with bench.py's per-learn timing events as torch timing events, as fence-free
timing events (_lib.TimingEvent), and without, alternating.
usage: python tools/hook_cost.py [K]"""
import json
import sys
import time

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from dmdqn_amd._lib import cu_masked_stream  # noqa: E402
from dmdqn_amd.agent import AgentConfig  # noqa: E402
from dmdqn_amd.env import EnvConfig  # noqa: E402
from dmdqn_amd.trainer import Trainer  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 300
dev = torch.device("cuda", 0)
n_cu = torch.cuda.get_device_properties(dev).multi_processor_count
work = cu_masked_stream(range(64, n_cu), dev)
side = cu_masked_stream(range(64), dev)
torch.cuda.set_stream(work)
tr = Trainer(EnvConfig(rows=2, cols=2, num_envs=256, seed=1000),
             AgentConfig(precision="bf16", seed=1000), device=dev, overlap="env", side_stream=side)
for _ in range(10010):
    tr.step()
torch.cuda.synchronize()


def timed(hooked):
    from dmdqn_amd._lib import TimingEvent
    pool = [(TimingEvent() if hooked == "fencefree" else torch.cuda.Event(enable_timing=True))
            for _ in range(2 * K)]
    for ev in pool:
        ev.record(work)
    torch.cuda.synchronize()
    it = iter(pool)

    def hook(before):
        next(it).record(torch.cuda.current_stream(dev))
    tr.agent.learn_hook = hook if hooked else None
    t0 = time.perf_counter()
    for _ in range(K):
        tr.step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    tr.agent.learn_hook = None
    return el / K * 1e3


res = {"torch_events": [], "fencefree_events": [], "plain": []}
for _ in range(3):
    res["torch_events"].append(round(timed("torch"), 4))
    res["fencefree_events"].append(round(timed("fencefree"), 4))
    res["plain"].append(round(timed(None), 4))
print(json.dumps({"ms_per_step": res, "steps": K}))
