"""Diagnostic: the replay sampler alone (dmdqn_replay_sample, set branch) at a
configuration's shape, per first-lane table size (DMDQN_OPT_SAMPLE_TLOG cap)
and LDS budget (160 KB: a table of 2^14 entries, no slot shared by two values
below n = 10000, so one dedupe round per chunk; default budget: 2^13):
median launch time over R launches (HIP events), and whether
the draws match the uncapped ones (they must: the table changes only the
speed).  usage: python tools/sample_bench.py [E A n] [reps]
(default C5: 256 envs x 64 agents, n = 10000; C3: 1024 16 10000)"""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dmdqn_amd import _lib  # noqa: E402
from dmdqn_amd import kernels as K  # noqa: E402

E, A, n = (int(x) for x in sys.argv[1:4]) if len(sys.argv) > 3 else (256, 64, 10000)
R = int(sys.argv[4]) if len(sys.argv) > 4 else 40
OPT_TLOG = 1  # include/dmdqn.h DMDQN_OPT_SAMPLE_TLOG
lib = _lib.load()
st0 = K.seed_streams(np.arange(E) + 7, "py")
for _ in range(3):  # past the first blocks of the streams
    K.replay_sample(st0, A, n)
ref = None
rows = []
for tlog, budget in [(32, 0), (32, 160 * 1024), (13, 160 * 1024), (11, 0), (10, 0), (9, 0), (32, 25568)]:
    assert lib.dmdqn_set_option(OPT_TLOG, tlog) == 0
    st = st0.clone()
    out = K.replay_sample(st, A, n, lds_budget=budget)
    if ref is None:
        ref = out.clone()
    same = bool(torch.equal(out, ref))
    ms = []
    for _ in range(R):
        st = st0.clone()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        K.replay_sample(st, A, n, out=out, lds_budget=budget)
        e1.record()
        torch.cuda.synchronize()
        ms.append(e0.elapsed_time(e1))
    rows.append({"tlog_cap": tlog, "lds_budget": budget, "median_us": round(1e3 * float(np.median(ms)), 1),
                 "min_us": round(1e3 * min(ms), 1), "draws_equal": same})
    print(json.dumps(rows[-1]), flush=True)
assert lib.dmdqn_set_option(OPT_TLOG, 32) == 0
print(json.dumps({"E": E, "A": A, "n": n, "reps": R, "rows": rows}))
