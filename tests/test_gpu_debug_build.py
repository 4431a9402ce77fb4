"""The debug-bounds build ("bounds checks in debug builds of
kernels"; DMDQN_VARIANT=debug loads libdmdqn_hip_debug.so): kernels check
the ring slots, edges, replay indices and stored actions they derive and
record violations, which Trainer.step turns into an error after every step.

Runs in a child process (one library variant per process): a clean run of
the loop in every precision, the shipped scenario with routes and the
actuated mode, and a negative control -- a learn fed deque positions past the
ring must be reported, not read out of range."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import numpy as np, torch
from dmdqn_amd import _lib
from dmdqn_amd.agent import AgentConfig
from dmdqn_amd.env import EnvConfig
from dmdqn_amd.trainer import Trainer
assert _lib.load().dmdqn_debug_build() == 1
for prec in ("fp32", "fp16", "bf16"):
    tr = Trainer(EnvConfig(rows=2, cols=2, num_envs=16, seed=3),
                 AgentConfig(precision=prec, replay_buffer_size=200, loss="huber"))
    for _ in range(260):   # the ring wraps; every step is range-checked
        tr.step()
tr = Trainer(EnvConfig(rows=4, cols=4, num_envs=8, seed=5, actuated=True),
             AgentConfig(precision="fp16", replay_buffer_size=1200, shared_params=False))
for _ in range(140):
    tr.step()
sc = ROOT + "/config/scenarios/grid_3x3_p06.npz"
tr = Trainer(EnvConfig(num_envs=4, scenario=sc), AgentConfig(precision="fp16"))
for _ in range(240):
    tr.step()
print("CLEAN")
# negative control: positions >= the ring's physical slot count
ag = tr.agent
ag.idx.fill_(ag.ring.slots + 3)  # past the physical slots
torch.ops.dmdqn.learn_step(ag.ring.s, ag.ring.n, ag.ring.a, ag.ring.d, ag.ring.r, ag.idx,
                           ag.params, ag.adam_m, ag.adam_v, ag.target, ag.target_h, ag.loss,
                           ag.ring.start, 128, 1, False, 0.99, 1e-3, 0.1, 1e-3, 1e-7, 0,
                           None, None, None)
try:
    _lib.debug_check()
except _lib.DmdqnError as e:
    print("CAUGHT", e)
"""


def test_debug_bounds_build_clean_run_and_negative_control():
    env = dict(os.environ, DMDQN_VARIANT="debug", PYTHONPATH=ROOT)
    code = "ROOT = %r\n" % ROOT + CHILD
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env,
                       timeout=400, cwd=ROOT)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    assert "CLEAN" in r.stdout
    assert "CAUGHT" in r.stdout and "learn deque position" in r.stdout, r.stdout[-2000:]
