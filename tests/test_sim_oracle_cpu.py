"""Simulator semantics on the CPU restatement (oracle/oracle_sim.c): the
actuated gap-out option (SURVEY A-14) against hand-worked timelines.  The HIP
sim matches the oracle bit for bit (tests/test_gpu_sim.py)."""
import numpy as np

import oracle as O


def _phases(actuated, end_ms, steps, action=0):
    env = O.OracleEnv(2, 2, 7, end_ms=end_ms, actuated=actuated)
    out, t = [], 0
    for _ in range(steps):
        _, ph, ts, _ = env.step(np.full(4, action, np.int32), 3, t, 10, 2400)
        t += 10
        out.append((ph.copy(), ts.copy()))
    return out


def test_fixed_durations_keep_phase_0_under_set_phase_every_10s():
    # setPhase every RL step restarts the 25 s phase 0: it never expires (A-14)
    for ph, ts in _phases(False, 2_500_000, 5):
        assert (ph == 0).all() and (ts == 10).all()


def test_gap_out_on_an_empty_network():
    # no vehicle ever reaches a detector: phase 0 ends at minDur = 5 s, then the
    # 6 s yellow (phase 1) runs from t = 5 to 11; at t = 10 the agent's next
    # setPhase restarts phase 0
    ph, ts = _phases(True, 1, 1)[0]   # one vehicle departing at t = 0 at most
    assert (ph == 1).all() and (ts == 5).all()


def test_gap_out_waits_for_traffic():
    # with steady demand the phase is held while vehicles keep crossing the
    # detectors: some junctions are still in phase 0 after 10 s, others gapped out
    res = _phases(True, 2_500_000, 30)
    seen = np.concatenate([ph for ph, _ in res])
    assert (seen == 0).any() and (seen == 1).any()
