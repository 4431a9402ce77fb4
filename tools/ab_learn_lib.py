"""Diagnostic: the per-agent learn (dmdqn_learn, one k_learn_f16 launch) of
several libraries on the same box and the same inputs, alternating, at C3 size
(16 agents x 1024 envs, fp16) on random replay contents.  Each library is a
build of tools/build_exp.py (or the product library) called through the C ABI
with the args of one product learn.  Prints per library the median / min of
all its launches (ms) and the sha1 of the weights after one launch from the
same starting weights (a timing-only variant differs there, by design).
usage: python tools/ab_learn_lib.py [--rounds R] [--reps N] [--envs E --agents A] [--bf16]
       lib.so [lib.so ...]   (default C3: 1024 envs x 16 agents, fp16; C2: --envs 256
       --agents 4 --bf16)"""
import ctypes as C
import hashlib
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dmdqn_amd.agent import AgentConfig, BatchedDQN  # noqa: E402


def _opt(name, default):
    if name in sys.argv:
        i = sys.argv.index(name)
        v = int(sys.argv[i + 1])
        del sys.argv[i:i + 2]
        return v
    return default


R, N = _opt("--rounds", 6), _opt("--reps", 20)
E, A = _opt("--envs", 1024), _opt("--agents", 16)
PREC = "fp16"
if "--bf16" in sys.argv:
    sys.argv.remove("--bf16")
    PREC = "bf16"
libs = sys.argv[1:]
ag = BatchedDQN(E, A, AgentConfig(precision=PREC, seed=0, replay_buffer_size=1000))
g = torch.Generator(device="cuda").manual_seed(0)
for t in range(200):
    s = torch.randint(-1, 24, (E, A, 89), device="cuda", generator=g).float()
    a = torch.randint(0, 4, (E, A), device="cuda", generator=g, dtype=torch.int32)
    r = -torch.rand((E, A), device="cuda", generator=g, dtype=torch.float64) * 100
    ag.remember(s, a, r, s, t % 60 == 59)
for _ in range(3):
    ag.learn()
torch.cuda.synchronize()
args = ag.c_learn_args()
fns = []
for p in libs:
    fn = C.CDLL(os.path.abspath(p)).dmdqn_learn
    fn.argtypes = [C.c_void_p, C.c_void_p]
    fn.restype = C.c_int
    fns.append(fn)

state = [t.clone() for t in (ag.params, ag.target, ag.adam_m, ag.adam_v)]


def restore():
    for dst, src in zip((ag.params, ag.target, ag.adam_m, ag.adam_v), state):
        dst.copy_(src)


out = {os.path.basename(p): {"ms": []} for p in libs}
for k, (p, fn) in enumerate(zip(libs, fns)):
    restore()
    assert fn(C.addressof(args), None) == 0
    torch.cuda.synchronize()
    out[os.path.basename(p)]["params_sha1"] = hashlib.sha1(
        ag.params.cpu().numpy().tobytes()).hexdigest()[:16]
for rnd in range(R):
    for p, fn in zip(libs, fns):
        restore()
        for _ in range(N):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            rc = fn(C.addressof(args), None)
            e1.record()
            torch.cuda.synchronize()
            assert rc == 0, rc
            out[os.path.basename(p)]["ms"].append(e0.elapsed_time(e1))
for name, d in out.items():
    ms = d.pop("ms")
    d["median_ms"] = round(float(np.median(ms)), 4)
    d["min_ms"] = round(float(min(ms)), 4)
    d["n"] = len(ms)
print(json.dumps(out))
