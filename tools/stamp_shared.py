"""Diagnostic: phase timing of the C5 shared learn (k_shared_next,
k_shared_grad) from in-kernel s_memrealtime stamps (100 MHz), at C5 size
(16384 agents) on random replay contents.  Calls dmdqn_learn_shared_grad
through the C ABI with a stamps buffer; prints the median per-agent phase
durations (us) and the kernel spans.
usage: python tools/stamp_shared.py [lib.so] [--nostamp]  (default: the product
library; an experiment build of tools/build_exp.py is called through the same C
ABI; --nostamp: no stamps buffer -- the kernels unperturbed -- and only the
HIP-event time of each launch, median of 20)"""
import ctypes as C
import hashlib
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dmdqn_amd import _lib  # noqa: E402
from dmdqn_amd.agent import AgentConfig, BatchedDQN  # noqa: E402

E, A = 1024, 16
ag = BatchedDQN(E, A, AgentConfig(precision="fp16", seed=0, shared_params=True,
                                  replay_buffer_size=1000))
NA = E * A
g = torch.Generator(device="cuda").manual_seed(0)
for t in range(200):
    s = torch.randint(-1, 24, (E, A, 89), device="cuda", generator=g).float()
    a = torch.randint(0, 4, (E, A), device="cuda", generator=g, dtype=torch.int32)
    r = -torch.rand((E, A), device="cuda", generator=g, dtype=torch.float64) * 100
    ag.remember(s, a, r, s, t % 60 == 59)
for _ in range(3):
    ag.learn()
torch.cuda.synchronize()
NOSTAMP = "--nostamp" in sys.argv
argv = [x for x in sys.argv if x != "--nostamp"]
ag.stamps = None if NOSTAMP else torch.zeros((NA, 16), dtype=torch.int64, device="cuda")
args = ag.c_learn_args()
lib = C.CDLL(argv[1]) if len(argv) > 1 else _lib.load()
fn = lib.dmdqn_learn_shared_grad
fn.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_float, C.c_void_p, C.c_void_p]
fn.restype = C.c_int
GRAD3 = "grad3" in (argv[1] if len(argv) > 1 else "")
names_g = (["L1", "B1+L2+L3", "B2+loss+next X", "B3+dW3+dZ2", "B4+dH1", "dW2+dW1", "B5"] if GRAD3
           else ["L1", "B1+L2", "B2+RQ (Q, loss, dZ2 rows)+next X", "B3+dW3", "dH1", "dW2+dW1", "B4"])
if NOSTAMP:
    ts = []
    for rep in range(20):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        rc = fn(C.addressof(args), ag.slab.data_ptr(), ag.n_slabs, ag.grad.data_ptr(),
                C.c_float(1.0 / NA), ag.shared_work.data_ptr(), None)
        e1.record()
        torch.cuda.synchronize()
        assert rc == 0, rc
        ts.append(e0.elapsed_time(e1))
    print(json.dumps({"lib": os.path.basename(argv[1]) if len(argv) > 1 else "product",
                      "median_ms": round(float(np.median(ts)), 4), "min_ms": round(min(ts), 4),
                      "grad_sha1": hashlib.sha1(ag.grad.cpu().numpy().tobytes()).hexdigest()[:16]}))
    sys.exit(0)
out = {}
hashes = []
for rep in range(3):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    rc = fn(C.addressof(args), ag.slab.data_ptr(), ag.n_slabs, ag.grad.data_ptr(),
            C.c_float(1.0 / NA), ag.shared_work.data_ptr(), None)
    e1.record()
    torch.cuda.synchronize()
    assert rc == 0, rc
    hashes.append(hashlib.sha1(ag.grad.cpu().numpy().tobytes()).hexdigest()[:16])
    st = ag.stamps.cpu().numpy().astype(np.float64) / 100.0  # us
    dg = np.diff(st[:, 0:len(names_g) + 1], axis=1)
    out = {"grad_" + n: round(float(np.median(dg[:, k])), 3) for k, n in enumerate(names_g)}
    last = len(names_g)
    out["grad_per_agent_us"] = round(float(np.median(st[:, last] - st[:, 0])), 3)
    out["grad_span_ms"] = round(float(st[:, last].max() - st[:, 0].min()) / 1000, 4)
    out["next_zscore_us"] = round(float(np.median(st[:, 11] - st[:, 10])), 3)
    out["next_tiles_us"] = round(float(np.median(st[:, 12] - st[:, 11])), 3)
    out["next_span_ms"] = round(float(st[:, 12].max() - st[:, 10].min()) / 1000, 4)
    out["gap_next_to_grad_us"] = round(float(st[:, 0].min() - st[:, 12].max()), 2)
    out["total_ms_events"] = round(e0.elapsed_time(e1), 4)
out["grad_sha1"] = hashes
tag = os.path.basename(argv[1])[:-3] if len(argv) > 1 else "product"
os.makedirs("gpurun_out", exist_ok=True)
np.save(f"gpurun_out/grad_{tag}.npy", ag.grad.cpu().numpy())
out["lib"] = (os.path.basename(argv[1]) if len(argv) > 1 else "product") + \
    (" k_shared_grad3" if GRAD3 else " k_shared_grad4")
print(json.dumps(out))
