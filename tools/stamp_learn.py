"""Diagnostic: phase timing of the fp16 learn kernel from in-kernel
s_memrealtime stamps (100 MHz).  Runs the learn kernel alone at C3 size on
random replay contents.  Prints median phase durations (us) over agents."""
import json
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from dmdqn_amd.agent import AgentConfig, BatchedDQN  # noqa: E402

E, A = int(sys.argv[1]) if len(sys.argv) > 1 else 1024, 16
ag = BatchedDQN(E, A, AgentConfig(precision="fp16", seed=0))
NA = E * A
g = torch.Generator(device="cuda").manual_seed(0)
for t in range(130):
    s = torch.randint(-1, 24, (E, A, 89), device="cuda", generator=g).float()
    a = torch.randint(0, 4, (E, A), device="cuda", generator=g, dtype=torch.int32)
    r = -torch.rand((E, A), device="cuda", generator=g, dtype=torch.float64) * 100
    ag.remember(s, a, r, s, t % 60 == 59)
torch.cuda.synchronize()
names = ["slots + gather S' + metadata + zscore", "-", "fwd target (+online frag loads)",
         "fwd online S' (+S gather)", "-", "argmax+y", "fwd online S", "loss+dW3+Adam W3",
         "dZ2", "dW2+Adam W2+image+dH1+gather S", "dZ1", "dW1+Adam W1"]
ag.stamps = torch.zeros((NA, 16), dtype=torch.int64, device="cuda")
res = {}
for rep in range(3):
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    ag.learn()
    ev1.record()
    torch.cuda.synchronize()
    st = ag.stamps.cpu().numpy().astype(np.float64) / 100.0  # us
    d = np.diff(st[:, :13], axis=1)
    res = {n: round(float(np.median(d[:, i])), 2) for i, n in enumerate(names)}
    res["block_total_median_us"] = round(float(np.median(st[:, 12] - st[:, 0])), 2)
    res["kernel_ms"] = round(ev0.elapsed_time(ev1), 3)
    res["span_ms"] = round(float(st[:, 12].max() - st[:, 0].min()) / 1000, 3)
print(json.dumps(res, indent=1))
