"""Diagnostic: first step where the "full" / "sample" stream schedules differ
from the one-stream order at C3 size.  No host sync inside the loop (a sync
per step would serialise the streams and hide a race): per-step clones are
taken on the main stream and compared after the run."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dmdqn_amd.agent import AgentConfig  # noqa: E402
from dmdqn_amd.env import EnvConfig  # noqa: E402
from dmdqn_amd.trainer import Trainer  # noqa: E402

E = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
STEPS = 140
runs = {}
for sched in sys.argv[2:] or ["none", "full"]:
    tr = Trainer(EnvConfig(rows=4, cols=4, num_envs=E, seed=2),
                 AgentConfig(precision="fp16", replay_buffer_size=500, seed=2), overlap=sched)
    rec = []
    for t in range(STEPS):
        tr.step()
        a = tr.agent
        slot = (a.ring.total - 1) % a.ring.slots
        rec.append({"actions": a.actions.clone(), "obs": tr.obs.clone(),
                    "ring_s": a.ring.s[:, slot].clone(), "ring_n": a.ring.n[:, slot].clone(),
                    "ring_r": a.ring.r[:, slot].clone(),
                    "idx": a.idx.clone() if tr.last_loss is not None else None,
                    "loss": tr.last_loss.clone() if tr.last_loss is not None else None,
                    "params": a.params[::97].clone()})
    torch.cuda.synchronize()
    runs[sched] = [{k: (None if v is None else v.cpu()) for k, v in r.items()} for r in rec]
    del tr, rec
    torch.cuda.empty_cache()
ref = runs.get("none")
for sched, rec in runs.items():
    if sched == "none":
        continue
    first = None
    for t in range(STEPS):
        diff = [k for k in ref[t] if (ref[t][k] is None) != (rec[t][k] is None) or
                (ref[t][k] is not None and not torch.equal(ref[t][k], rec[t][k]))]
        if diff:
            detail = {}
            for k in diff:
                if ref[t][k] is not None and rec[t][k] is not None:
                    m = (ref[t][k] != rec[t][k])
                    detail[k] = (int(m.sum()), m.nonzero()[:3].tolist())
            first = (t, diff, detail)
            break
    print(sched, "first divergence:", first, flush=True)
