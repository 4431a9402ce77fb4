"""The split learn (dmdqn_learn_grad + dmdqn_adam_agents, agent.set_split_learn)
against the fused kernel: the same Keras-3 Adam on the same 16-bit gradients,
so every parameter, Adam slot, target copy and loss is bit-identical, across
target syncs; and the trainer's "full" schedule that selects it at C2 size
stays bit-identical to the one-stream order."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from dmdqn_amd.agent import AgentConfig, BatchedDQN  # noqa: E402
from dmdqn_amd.env import EnvConfig  # noqa: E402
from dmdqn_amd.trainer import Trainer  # noqa: E402

DEV = "cuda"


def _fill(ag, n, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    for t in range(n):
        s = torch.randint(-1, 24, (ag.E, ag.A, 89), device=DEV, generator=g).float()
        a = torch.randint(0, 4, (ag.E, ag.A), device=DEV, generator=g, dtype=torch.int32)
        r = -torch.rand((ag.E, ag.A), device=DEV, generator=g, dtype=torch.float64) * 100
        ag.remember(s, a, r, s.flip(-1), t % 50 == 49)


@pytest.mark.parametrize("precision", ["fp16", "bf16"])
def test_split_learn_bit_identical_to_fused(precision):
    state = {}
    for split in (False, True):
        cfg = AgentConfig(precision=precision, seed=3, replay_buffer_size=400,
                          target_update_frequency=4)
        ag = BatchedDQN(16, 4, cfg)
        ag.set_split_learn(split)
        assert ag.split_learn == split
        losses = []
        _fill(ag, 130, 1)
        for k in range(12):  # 3 target syncs
            _fill(ag, 1, 100 + k)
            losses.append(ag.learn().clone())
        torch.cuda.synchronize()
        state[split] = [torch.stack(losses)] + [getattr(ag, n).clone() for n in
                                                 ("params", "adam_m", "adam_v", "target", "target_h")]
    for a, b in zip(state[False], state[True]):  # bitwise
        bits = torch.int32 if a.element_size() == 4 else torch.int16
        assert torch.equal(a.view(bits), b.view(bits))


def test_split_learn_rejects_fp32_and_shared():
    with pytest.raises(ValueError):
        BatchedDQN(2, 2, AgentConfig(precision="fp32")).set_split_learn(True)
    with pytest.raises(ValueError):
        BatchedDQN(2, 2, AgentConfig(precision="fp16", shared_params=True)).set_split_learn(True)


def test_c2_full_schedule_with_split_learn_bit_identical():
    """C2's shape (2x2 grid x 256 replicas, bf16; replay 500 to keep it short):
    the one-stream order vs overlap "full" with the split learn -- 140 steps,
    losses, observations and weights bit-identical."""
    res = {}
    for sched in ("none", "full"):
        tr = Trainer(EnvConfig(rows=2, cols=2, num_envs=256, seed=4),
                     AgentConfig(precision="bf16", replay_buffer_size=500, seed=4), overlap=sched,
                     split_learn=sched == "full")
        assert tr.agent.split_learn == (sched == "full")
        losses = []
        for _ in range(140):
            tr.step()
            if tr.last_loss is not None:
                losses.append(tr.last_loss.clone())
        torch.cuda.synchronize()
        res[sched] = (torch.stack(losses).cpu(), tr.agent.params.cpu(), tr.agent.adam_v.cpu(),
                      tr.obs.cpu())
        del tr
        torch.cuda.empty_cache()
    for a, b in zip(res["none"], res["full"]):
        np.testing.assert_array_equal(a.numpy(), b.numpy())


@pytest.mark.parametrize("precision", ["fp16", "bf16"])
def test_adam_is_keras3_adam_bit_exact_on_the_kernel_gradient(precision):
    """Keras-3 Adam (keras/src/optimizers/adam.py update_step) rounds every op
    as TF's separate elementwise kernels: given the gradient the kernel used
    (the split learn exports it), params / m / v after the learn equal the
    f32 numpy update bit for bit -- no fma contraction (common.hpp mul_rn)."""
    import oracle as O
    cfg = AgentConfig(precision=precision, seed=5, replay_buffer_size=300)
    ag = BatchedDQN(8, 4, cfg)
    ag.set_split_learn(True)
    _fill(ag, 160, 2)
    for _ in range(3):  # non-zero Adam slots
        ag.learn()
    p0, m0, v0 = (getattr(ag, n).cpu().numpy().copy() for n in ("params", "adam_m", "adam_v"))
    ag.learn()
    g = ag._split_grad.cpu().numpy()
    alpha, c1, c2, eps = O.keras_adam_consts(ag.learn_step_counter)
    m1 = m0 + (g - m0) * c1
    v1 = v0 + (g * g - v0) * c2
    p1 = p0 - (m1 * alpha) / (np.sqrt(v1) + eps)
    for name, want in (("adam_m", m1), ("adam_v", v1), ("params", p1)):
        got = getattr(ag, name).cpu().numpy()
        assert np.array_equal(got.view(np.int32), want.view(np.int32)), (
            name, int((got != want).sum()))
