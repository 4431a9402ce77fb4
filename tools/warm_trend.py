"""Diagnostic: wall ms/step of the bench workload in chunks of 20 steps from
the first learn-active step on, to see whether a fresh process (or a fresh
box) settles.  usage: python tools/warm_trend.py [n_chunks] [--overlap MODE]"""
import sys
import time

import torch

sys.path.insert(0, ".")
from dmdqn_amd.agent import AgentConfig  # noqa: E402
from dmdqn_amd.env import EnvConfig  # noqa: E402
from dmdqn_amd.trainer import Trainer  # noqa: E402

n_chunks = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 20
mode = sys.argv[sys.argv.index("--overlap") + 1] if "--overlap" in sys.argv else "none"
dev = torch.device("cuda", 0)
work = torch.cuda.Stream(dev)
torch.cuda.set_stream(work)
t0 = time.perf_counter()
tr = Trainer(EnvConfig(rows=4, cols=4, num_envs=1024, seed=1000),
             AgentConfig(precision="fp16", seed=1000), device=dev, overlap=mode)
torch.cuda.synchronize()
print(f"setup {time.perf_counter() - t0:.2f} s", flush=True)
t0 = time.perf_counter()
for _ in range(127):
    tr.step()
torch.cuda.synchronize()
print(f"fill 127 steps {time.perf_counter() - t0:.2f} s", flush=True)
out = []
for c in range(n_chunks):
    t0 = time.perf_counter()
    for _ in range(20):
        tr.step()
    torch.cuda.synchronize()
    out.append((time.perf_counter() - t0) / 20 * 1e3)
print("ms/step per 20-step chunk:", " ".join(f"{x:.3f}" for x in out), flush=True)
