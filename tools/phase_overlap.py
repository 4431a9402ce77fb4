"""Diagnostic: are co-running learn workgroups phase-locked?  Runs the fp16
learn kernel at C3 size with phase stamps and reports, over the kernel's
lifetime, how many workgroups are inside an Adam-heavy phase vs active."""
import json
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from dmdqn_amd.agent import AgentConfig, BatchedDQN  # noqa: E402

E, A = 1024, 16
ag = BatchedDQN(E, A, AgentConfig(precision="fp16", seed=0))
g = torch.Generator(device="cuda").manual_seed(0)
for t in range(130):
    s = torch.randint(-1, 24, (E, A, 89), device="cuda", generator=g).float()
    a = torch.randint(0, 4, (E, A), device="cuda", generator=g, dtype=torch.int32)
    r = -torch.rand((E, A), device="cuda", generator=g, dtype=torch.float64) * 100
    ag.remember(s, a, r, s, t % 60 == 59)
ag.stamps = torch.zeros((E * A, 16), dtype=torch.int64, device="cuda")
ag.learn()
ag.learn()
torch.cuda.synchronize()
st = ag.stamps.cpu().numpy().astype(np.float64) / 100.0  # us
st -= st[:, 0].min()
T = st[:, 12].max()
grid = np.linspace(0, T, 400)
act = ((st[:, 0][None] <= grid[:, None]) & (st[:, 12][None] > grid[:, None])).sum(1)
# adam-heavy: stamps 9->10 (dW2 + Adam W2 + dH1) and 11->12 (dW1 + Adam W1)
ad = (((st[:, 9][None] <= grid[:, None]) & (st[:, 10][None] > grid[:, None])) |
      ((st[:, 11][None] <= grid[:, None]) & (st[:, 12][None] > grid[:, None]))).sum(1)
frac = ad / np.maximum(act, 1)
mid = (grid > 0.1 * T) & (grid < 0.9 * T)
print(json.dumps({"kernel_us": round(T, 1), "active_mean": round(float(act[mid].mean()), 1),
                  "adam_frac_mean": round(float(frac[mid].mean()), 3),
                  "adam_frac_std": round(float(frac[mid].std()), 3),
                  "adam_frac_min_max": [round(float(frac[mid].min()), 3),
                                        round(float(frac[mid].max()), 3)],
                  "adam_frac_series": [round(float(x), 2) for x in frac[mid][::8]]}))
# per-slot start times of the first 512 workgroups
print("first-round start spread us:", np.percentile(st[:512, 0], [0, 50, 100]).round(1).tolist())
print("start of blocks 256..511 median us:", float(np.median(st[256:512, 0])))
