"""GPU: the fused env step (dmdqn_env_step: select_action's draws, setPhase + K
substeps, observation / reward and ReplayBuffer.add in ONE launch per replica,
train.py:211-282) is bit-identical to the four launches it replaces (dmdqn_act,
dmdqn_sim_step, dmdqn_observe, dmdqn_replay_store) -- per step the actions,
observations, rewards, losses, and at the end every sim array, ring, network and
random stream -- on every sim path (LDS image, register lanes, global rings),
grid sizes whose MT stream / epilogue scratch take the extra-LDS branch (1x1),
actuated signals, replicas that restart on their own `done`, a greedy act and
the shared network.  The Trainer's default one-stream schedule uses it, so every
Trainer-vs-oracle test also runs it."""
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from dmdqn_amd.agent import AgentConfig  # noqa: E402
from dmdqn_amd.env import EnvConfig  # noqa: E402
from dmdqn_amd.trainer import Trainer  # noqa: E402


def _trainer(fused, rows=2, cols=2, E=6, greedy=False, shared=False, overlap="none", **env_kw):
    kw = dict(rows=rows, cols=cols, num_envs=E, seed=21, max_sim_time=400)
    kw.update(env_kw)
    tr = Trainer(EnvConfig(**kw),
                 AgentConfig(replay_buffer_size=150, target_update_frequency=7, seed=3,
                             precision="fp16", shared_params=shared, count_env_steps=greedy),
                 overlap=overlap, fused=fused)
    assert tr.fused == fused
    if greedy:  # past the 8000-step epsilon floor (dqn_agent.py:258-261)
        tr.agent.global_step_count = 12000
    return tr


def _run(tr, n):
    out = []
    for _ in range(n):
        st = tr.step()
        out.append((None if tr.last_loss is None else tr.last_loss.clone(), tr.obs.clone(),
                    tr.last_reward.clone(), tr.agent.actions.clone(), st.done))
    torch.cuda.synchronize()
    return out


def _compare(ref, fus, a, b):
    for t, (x, y) in enumerate(zip(a, b)):
        assert (x[0] is None) == (y[0] is None), t
        if x[0] is not None:
            assert torch.equal(x[0], y[0]), f"loss differs at step {t}"
        assert torch.equal(x[1], y[1]), f"obs differs at step {t}"
        assert torch.equal(x[2], y[2]), f"reward differs at step {t}"
        assert torch.equal(x[3], y[3]), f"actions differ at step {t}"
        assert x[4] == y[4], f"done differs at step {t}"
    ra, rb = ref.agent, fus.agent
    for name in ["params", "target", "adam_m", "adam_v", "np_state", "py_state"]:
        assert torch.equal(getattr(ra, name), getattr(rb, name)), name
    for name in ["s", "n", "a", "r", "d"]:
        assert torch.equal(getattr(ra.ring, name), getattr(rb.ring, name)), "ring." + name
    assert ra.ring.total == rb.ring.total and int(rb.ring.err[0]) == 0
    ea, eb = ref.env, fus.env
    for x, y in zip(ea._sim_state, eb._sim_state):
        assert torch.equal(x, y)
    for name in ["halt", "phase", "tspent", "done_u8", "local"]:
        assert torch.equal(getattr(ea, name), getattr(eb, name)), name
    assert ref.episode == fus.episode and ref.total_steps == fus.total_steps


@pytest.mark.parametrize("path", ["lds", "reg", "global"])
@pytest.mark.parametrize("rows,cols", [(1, 1), (2, 2), (3, 3)])
def test_fused_step_matches_four_launches(lib_option, path, rows, cols):
    lib_option("sim_path", path)
    ref, fus = _trainer(False, rows, cols), _trainer(True, rows, cols)
    a, b = _run(ref, 140), _run(fus, 140)  # episodes of 40 steps; learns from step 128
    _compare(ref, fus, a, b)


def test_fused_step_4x4_and_8x8_default_paths():
    """4x4 takes the LDS image (four blocks per CU), 8x8 the register path
    (1024-thread blocks): the bench's C3 and C5 shapes, few replicas."""
    for rows in (4, 8):
        ref, fus = _trainer(False, rows, rows, E=3), _trainer(True, rows, rows, E=3)
        _compare(ref, fus, _run(ref, 45), _run(fus, 45))


@pytest.mark.parametrize("kind", ["actuated", "greedy", "shared", "sample_schedule"])
def test_fused_step_variants(kind):
    kw = {}
    if kind == "actuated":
        kw = dict(env_kw=dict(actuated=True))
    elif kind == "greedy":
        kw = dict(greedy=True)
    elif kind == "shared":
        kw = dict(shared=True)
    env_kw = kw.pop("env_kw", {})
    ovl = "sample" if kind == "sample_schedule" else "none"
    ref = _trainer(False, **kw, **env_kw)
    fus = _trainer(True, overlap=ovl, **kw, **env_kw)
    _compare(ref, fus, _run(ref, 170), _run(fus, 170))


def test_fused_step_replicas_restart_on_their_own_done():
    """Demand that drains before max_sim_time (end_ms 60 s): replicas end at
    different steps and restart alone; the fused store carries each one's flag."""
    kw = dict(E=3, max_sim_time=2400, end_ms=60_000)
    ref, fus = _trainer(False, **kw), _trainer(True, **kw)
    assert fus.env.drains_early
    a, b = _run(ref, 160), _run(fus, 160)
    _compare(ref, fus, a, b)
    assert fus.env.env_episodes.sum() > 0


def test_fused_step_flags_a_non_integer_observation():
    """The int8 rows refuse a value they cannot hold exactly (replay.hip to_i8):
    the fused store sets the same pinned flag and the ring check raises."""
    from dmdqn_amd import _lib
    tr = _trainer(True)
    tr.step()
    tr.obs = tr.obs.clone()
    tr.obs[1, 2, 5] = 0.5  # the next transition's s row
    tr.step()
    with pytest.raises(_lib.DmdqnError):
        tr.agent.ring.check()
