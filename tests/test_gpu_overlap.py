"""GPU: the two-stream Trainer (side stream: act -> sim -> observe -> replay
draws, overlapped with the learn) is bit-identical to the sequential loop of
src/scripts/train.py:207-310 -- per-step losses, observations, rewards and the
final networks, Adam slots, rings and random streams -- across episode resets,
target syncs, the shared-network configuration and a greedy (epsilon < 1) act
that must wait for the learn's weights."""
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from dmdqn_amd.agent import AgentConfig  # noqa: E402
from dmdqn_amd.env import EnvConfig  # noqa: E402
from dmdqn_amd.trainer import Trainer  # noqa: E402


def _trainer(overlap, precision, shared, greedy, side_stream=None, cap=200, side_learn=0,
             spare=16):
    tr = Trainer(EnvConfig(rows=2, cols=2, num_envs=8, seed=11, max_sim_time=500),
                 AgentConfig(replay_buffer_size=cap, target_update_frequency=9, seed=4,
                             precision=precision, shared_params=shared,
                             count_env_steps=greedy, ring_spare=spare),
                 overlap=overlap, side_stream=side_stream, side_learn=side_learn)
    if greedy:  # past the 8000-step epsilon floor (dqn_agent.py:258-261)
        tr.agent.global_step_count = 12000
    return tr


def _run(tr, n):
    out = []
    for _ in range(n):
        st = tr.step()
        out.append((None if tr.last_loss is None else tr.last_loss.clone(),
                    tr.obs.clone(), tr.last_reward.clone(), tr.agent.actions.clone(), st.done))
    torch.cuda.synchronize()
    return out


@pytest.mark.parametrize("mode", ["sample", "full", "env", "learn"])
@pytest.mark.parametrize("precision,shared,greedy", [
    ("fp16", False, False), ("fp32", False, False), ("bf16", False, False), ("fp16", True, False),
    ("fp16", False, True)])
def test_overlap_matches_sequential(mode, precision, shared, greedy):
    ref = _trainer("none", precision, shared, greedy)
    ovl = _trainer(mode, precision, shared, greedy)
    assert ovl.side is not None and ref.side is None
    a, b = _run(ref, 170), _run(ovl, 170)   # 3 episodes of 50 steps, learn from step 128
    _compare(ref, ovl, a, b)


@pytest.mark.parametrize("precision,greedy,masked", [
    ("fp16", False, True), ("bf16", False, False), ("fp32", False, True), ("fp16", True, True)])
def test_side_learn_matches_sequential(precision, greedy, masked):
    """overlap "env" with side_learn: the last 12 of 32 agents learn on the side
    stream behind the env step (the rest on the learn stream), across episode
    resets, target syncs and a greedy act that reads both parts' weights:
    bit-identical to the sequential loop."""
    side = None
    if masked:
        from dmdqn_amd._lib import cu_masked_stream
        side = cu_masked_stream(range(32))
        main = cu_masked_stream(range(32, torch.cuda.get_device_properties(0).multi_processor_count))
        torch.cuda.set_stream(main)
    try:
        ref = _trainer("none", precision, False, greedy)
        ovl = _trainer("env", precision, False, greedy, side_stream=side, side_learn=12)
        a, b = _run(ref, 170), _run(ovl, 170)
        _compare(ref, ovl, a, b)
    finally:
        torch.cuda.set_stream(torch.cuda.default_stream())


def test_overlap_on_cu_masked_streams_matches_sequential():
    """bench --cu-split: the learn on one CU-masked stream, the side work on
    another (dmdqn_stream_create_cumask) -- still bit-identical."""
    from dmdqn_amd._lib import cu_masked_stream
    n_cu = torch.cuda.get_device_properties(0).multi_processor_count
    main = cu_masked_stream(range(32, n_cu))
    side = cu_masked_stream(range(32))
    ref = _trainer("none", "fp16", False, False)
    a = _run(ref, 170)
    with torch.cuda.stream(main):
        ovl = _trainer("full", "fp16", False, False, side_stream=side)
        assert ovl.side is side
        b = _run(ovl, 170)
    _compare(ref, ovl, a, b)


@pytest.mark.parametrize("masked,spare", [(False, 2), (True, 2), (False, 16), (True, 16)])
def test_env_beside_learn_on_a_wrapped_ring(masked, spare):
    """overlap "env": the fused env step of t+1 beside learn t (the side
    stream up to `spare` steps ahead), with the deque wrapped (replay 150 <
    170 steps, learns from step 128) and, with 2 spare slots, the physical
    ring too, so every store lands in a spare slot the running learns cannot
    sample (kernels.ReplayRing) -- bit-identical to the one-stream order, also
    with the two streams CU-masked (bench --cu-split)."""
    from dmdqn_amd._lib import cu_masked_stream
    ref = _trainer("none", "bf16", False, False, cap=150, spare=spare)
    a = _run(ref, 170)
    if masked:
        n_cu = torch.cuda.get_device_properties(0).multi_processor_count
        main, side = cu_masked_stream(range(64, n_cu)), cu_masked_stream(range(64))
        with torch.cuda.stream(main):
            ovl = _trainer("env", "bf16", False, False, side_stream=side, cap=150, spare=spare)
            b = _run(ovl, 170)
    else:
        ovl = _trainer("env", "bf16", False, False, cap=150, spare=spare)
        b = _run(ovl, 170)
    assert ovl.agent.ring.start != 0 and ovl.agent.learn_launches == 170 - 127
    _compare(ref, ovl, a, b)


def _compare(ref, ovl, a, b):
    assert sum(x[4] for x in a) == 3 and ref.episode == ovl.episode == 3
    for t, (x, y) in enumerate(zip(a, b)):
        assert (x[0] is None) == (y[0] is None), t
        if x[0] is not None:
            assert torch.equal(x[0], y[0]), f"loss differs at step {t}"
        assert torch.equal(x[1], y[1]), f"obs differs at step {t}"
        assert torch.equal(x[2], y[2]), f"reward differs at step {t}"
        assert torch.equal(x[3], y[3]), f"actions differ at step {t}"
    ra, rb = ref.agent, ovl.agent
    for name in ["params", "target", "adam_m", "adam_v", "np_state", "py_state", "idx"]:
        assert torch.equal(getattr(ra, name), getattr(rb, name)), name
    for name in ["s", "n", "a", "r", "d"]:
        assert torch.equal(getattr(ra.ring, name), getattr(rb.ring, name)), "ring." + name
    if ra.target_h is not None:
        assert torch.equal(ra.target_h, rb.target_h)


def test_fence_free_timing_and_ordering_events():
    """_lib.TimingEvent (bench.py's per-learn timing) measures what a torch
    timing event measures around the same GPU sleep, and _lib.OrderEvent (the
    env schedule's learn -> side-stream wait) orders: the side stream's work
    recorded after waiting on it starts only after the main stream's sleep."""
    from dmdqn_amd._lib import OrderEvent, TimingEvent
    main, side = torch.cuda.Stream(), torch.cuda.Stream()
    cycles = 2_000_000
    t0, t1 = TimingEvent(), TimingEvent()
    r0, r1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(main):
        r0.record(main)
        t0.record(main)
        torch.cuda._sleep(cycles)
        t1.record(main)
        r1.record(main)
    torch.cuda.synchronize()
    ours, ref = t0.elapsed_time(t1), r0.elapsed_time(r1)
    assert ours > 0.1 and abs(ours - ref) <= 0.05 * ref + 0.02, (ours, ref)
    # ordering: side waits for main's sleep through an OrderEvent (the sleep's
    # own end, timed on main, bounds the side's first record from below)
    start, slept, after = TimingEvent(), TimingEvent(), TimingEvent()
    ev = OrderEvent()
    with torch.cuda.stream(main):
        start.record(main)
        torch.cuda._sleep(cycles)
        slept.record(main)
        ev.record(main)
    ev.wait(side)
    after.record(side)
    torch.cuda.synchronize()
    t_sleep, t_after = start.elapsed_time(slept), start.elapsed_time(after)
    assert t_sleep > 0.1 and t_after >= t_sleep - 0.005, (t_after, t_sleep)


@pytest.mark.parametrize("spare", [2, 4])
def test_env_schedule_with_a_lagging_learn_stream(spare):
    """overlap "env" with the learn stream held back (a GPU sleep queued on it
    every step): the side stream then runs as far ahead as the schedule allows
    (`spare` env steps past the newest marked call), before the first learn
    too, while the caller's clones of each step's actions / observations /
    rewards / losses are queued on the learn stream.  Every output and the
    final state stay bit-identical to the one-stream order -- the marks order
    both the ring slots' reuse and the output buffers' (OUT_BUFS = spare + 2)."""
    ref = _trainer("none", "fp16", False, False, cap=150, spare=spare)
    a = _run(ref, 170)
    ovl = _trainer("env", "fp16", False, False, cap=150, spare=spare)
    assert ovl.agent.OUT_BUFS == spare + 2
    main = torch.cuda.current_stream()
    out = []
    for _ in range(170):
        torch.cuda._sleep(200_000)  # ~0.1 ms of GPU time on the learn stream per step
        st = ovl.step()
        out.append((None if ovl.last_loss is None else ovl.last_loss.clone(), ovl.obs.clone(),
                    ovl.last_reward.clone(), ovl.agent.actions.clone(), st.done))
    assert torch.cuda.current_stream() == main
    torch.cuda.synchronize()
    _compare(ref, ovl, a, out)
