"""Sanitizer builds: the CPU restatement under AddressSanitizer +
UndefinedBehaviorSanitizer (oracle/Makefile `asan`), driven through every
oracle entry point the parity tests use -- simulator (synthetic, scenario,
actuated, trace), observe / reward, MT19937 streams, random.sample in both
branches, z-score, the learn step (MSE and Huber) and the OpenMP training
loop.  It runs in a child process with libasan preloaded (a sanitized
shared library cannot be loaded into an uninstrumented interpreter
otherwise); any report fails the child."""
import os
import subprocess
import sys

import pytest

from conftest import ROOT

CHILD = r"""
import numpy as np, oracle as O
from dmdqn_amd.sumo_scenario import load_scenario, scenario_tables
for act in (False, True):
    env = O.OracleEnv(3, 3, 5, actuated=act)
    env.enable_trace(1 << 15)
    t = 0
    for _ in range(40):
        env.step(np.random.RandomState(t).randint(0, 4, 9).astype(np.int32), 3, t, 10, 2400)
        t += 10
    env.lanes(); env.demand(); env.trace()
sc = load_scenario(os.path.join(ROOT, "tests", "golden", "grid_3x3_p06_scenario.npz"))
q, off, vd, N, period = scenario_tables(sc, 1)
env = O.OracleEnv(3, 3, 100); env.set_demand(q[0], off[0], vd[0], period)
for k in range(30):
    env.step(np.zeros(9, np.int32), 3, 10 * k, 10, 2400)
L = O.local_state(np.arange(48).reshape(4, 12) % 7, np.arange(4), np.arange(4), 1)
O.build_obs(2, 2, L); O.reward(L); O.neighbors(8, 8)
s = O.py_stream(3)
for n in (128, 1045, 1046, 10000):
    O.py_sample(s, n, 128)
O.zscore(np.arange(128.0)); O.np_sum(np.arange(1000.0))
nps = O.np_stream(1); O.act(nps, 16, 0.5, np.zeros(16, np.int32))
rng = np.random.RandomState(0)
p = O.keras_init(rng)
for lk in (0, 1):
    S = rng.randint(-1, 24, size=(128, 89)).astype(np.float32)
    O.learn(p, p.copy(), np.zeros_like(p), np.zeros_like(p), S, rng.randint(0, 4, 128).astype(np.int32),
            rng.normal(size=128).astype(np.float32), S, np.zeros(128, np.float32), 1, loss_kind=lk)
O.train_loop(2, 2, 2, 127, 3, 0, 2)
print("SANITIZED-OK")
"""


def _run_sanitized(code):
    libasan = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True,
                             text=True).stdout.strip()
    if not os.path.isabs(libasan) or not os.path.exists(libasan):
        pytest.skip("libasan not available")
    r = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "asan"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    env = dict(os.environ, LD_PRELOAD=libasan,
               ORACLE_LIB=os.path.join(ROOT, "oracle", "liboracle_asan.so"),
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=0:exitcode=23",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1",
               PYTHONPATH=ROOT, OMP_NUM_THREADS="2")
    return subprocess.run([sys.executable, "-c", "import os\nROOT = %r\n" % ROOT + code],
                          capture_output=True, text=True, env=env, timeout=600)


def test_oracle_under_asan_and_ubsan():
    r = _run_sanitized(CHILD)
    assert r.returncode == 0 and "SANITIZED-OK" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-4000:]


def test_sanitizer_setup_catches_an_overflow():
    """Negative control: the same harness reports a heap overflow (a sum over
    64 elements past a malloc'd buffer), so a clean run above means clean."""
    r = _run_sanitized("import numpy as np, oracle as O\n"
                       "a = np.arange(4096.0)\n"
                       "O.lib().orc_np_sum(a, a.size + 64)\n")
    assert r.returncode == 23 and "heap-buffer-overflow" in r.stderr, r.stderr[-3000:]
