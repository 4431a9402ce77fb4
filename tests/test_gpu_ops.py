"""torch.ops.dmdqn.* (TORCH_LIBRARY registration, dmdqn_amd/torch_ext) vs the
same C entry points called through ctypes: bit-identical results, the
current-stream contract and TORCH_CHECK argument errors.  (Every other GPU
test reaches the kernels through these ops, since the Python surfaces use
them.)"""
import ctypes as C

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from dmdqn_amd import _lib, kernels as K, ops  # noqa: E402
from dmdqn_amd._lib import call, ptr, stream_of  # noqa: E402
from dmdqn_amd.agent import AgentConfig, BatchedDQN  # noqa: E402

DEV = "cuda"
D = ops.load()


def test_streams_act_observe_sample_match_c_abi():
    seeds = torch.arange(5, dtype=torch.int64, device=DEV) * 7 + 3
    for kind, fn in (("np", "dmdqn_mt_seed_np"), ("py", "dmdqn_mt_seed_py")):
        a = torch.empty((5, 625), dtype=torch.int32, device=DEV)
        b = torch.empty_like(a)
        D.mt_seed(a, seeds, kind)
        call(fn, ptr(b), ptr(seeds), 5, stream_of())
        assert torch.equal(a, b)
    st1 = K.seed_streams(seeds, "np", DEV)
    st2 = st1.clone()
    out1 = torch.empty((5, 9), dtype=torch.int32, device=DEV)
    out2 = torch.empty_like(out1)
    D.act(st1, 9, 1.0, 4, None, out1)
    call("dmdqn_act", ptr(st2), 5, 9, C.c_double(1.0), 4, None, ptr(out2), stream_of())
    assert torch.equal(out1, out2) and torch.equal(st1, st2)
    halt = torch.randint(0, 20, (5, 9, 12), dtype=torch.int32, device=DEV)
    ph = torch.randint(0, 12, (5, 9), dtype=torch.int32, device=DEV)
    ts = torch.randint(0, 30, (5, 9), dtype=torch.int32, device=DEV)
    prev = torch.randint(0, 9, (5, 9, 17), device=DEV).float()
    bufs = [[torch.empty((5, 9, 17), device=DEV), torch.empty((5, 9, 89), device=DEV),
             torch.empty((5, 9), dtype=torch.float64, device=DEV)] for _ in range(2)]
    D.observe(3, 3, halt, ph, ts, 1, *bufs[0][:2], prev, bufs[0][2])
    call("dmdqn_observe", 3, 3, 5, ptr(halt), ptr(ph), ptr(ts), 1, ptr(bufs[1][0]),
         ptr(bufs[1][1]), ptr(prev), ptr(bufs[1][2]), stream_of())
    for x, y in zip(*bufs):
        assert torch.equal(x, y)
    py1 = K.seed_streams(seeds, "py", DEV)
    py2 = py1.clone()
    i1 = torch.empty((45, 128), dtype=torch.int32, device=DEV)
    i2 = torch.empty_like(i1)
    D.replay_sample(py1, 9, 3000, 128, i1)
    call("dmdqn_replay_sample", ptr(py2), 5, 9, 3000, 128, ptr(i2), stream_of())
    assert torch.equal(i1, i2) and torch.equal(py1, py2)


def test_learn_step_op_matches_c_abi_and_target_sync():
    for precision in ("fp32", "fp16", "bf16"):
        ag = BatchedDQN(2, 2, AgentConfig(replay_buffer_size=200, seed=1, precision=precision))
        rng = np.random.RandomState(0)
        for t in range(150):
            s = torch.from_numpy(rng.randint(-1, 24, size=(2, 2, 89)).astype(np.float32)).to(DEV)
            a = torch.from_numpy(rng.randint(0, 4, size=(2, 2)).astype(np.int32)).to(DEV)
            r = torch.from_numpy(-rng.randint(0, 99, size=(2, 2)).astype(np.float64)).to(DEV)
            ag.remember(s, a, r, s, False)
        keep = {k: getattr(ag, k).clone() for k in ["params", "adam_m", "adam_v", "target"]}
        ag.learn()  # torch.ops.dmdqn.learn_step
        via_op = {k: getattr(ag, k).clone() for k in keep}
        loss_op = ag.loss.clone()
        for k, v in keep.items():
            getattr(ag, k).copy_(v)
        args = ag.c_learn_args()
        call("dmdqn_learn", C.byref(args), stream_of())
        for k in keep:
            assert torch.equal(getattr(ag, k), via_op[k]), (precision, k)
        assert torch.equal(ag.loss, loss_op)
        ag.update_target_network()  # torch.ops.dmdqn.target_sync
        assert torch.equal(ag.target, ag.params)
        if ag.target_h is not None:
            assert torch.equal(ag.target_h[:, :ag.P], ag.params.to(ag.target_h.dtype))


def test_ops_run_on_the_current_stream():
    s = torch.cuda.Stream()
    seeds = torch.arange(3, dtype=torch.int64, device=DEV)
    with torch.cuda.stream(s):
        st = torch.empty((3, 625), dtype=torch.int32, device=DEV)
        D.mt_seed(st, seeds, "np")
        out = torch.empty((3, 4), dtype=torch.int32, device=DEV)
        for _ in range(50):
            D.act(st, 4, 1.0, 4, None, out)
    s.synchronize()
    ref = K.seed_streams(seeds, "np", DEV)
    o2 = torch.empty_like(out)
    for _ in range(50):
        K.act(ref, 4, out=o2)
    assert torch.equal(out, o2)


def test_torch_check_errors():
    st = torch.empty((3, 625), dtype=torch.int64, device=DEV)  # wrong dtype
    with pytest.raises(RuntimeError, match="state must be Int"):
        D.mt_seed(st, torch.arange(3, dtype=torch.int64, device=DEV), "np")
    st = torch.empty((3, 625), dtype=torch.int32, device=DEV)
    out = torch.empty((3, 5), dtype=torch.int32, device=DEV)  # 15 != 3 * 4
    with pytest.raises(RuntimeError, match="actions has 15 elements"):
        D.act(st, 4, 1.0, 4, None, out)
    with pytest.raises(RuntimeError, match="dmdqn_replay_sample failed"):  # C-side check: n < k
        D.replay_sample(st, 4, 100, 128, torch.empty((12, 128), dtype=torch.int32, device=DEV))
    assert isinstance(_lib.load().dmdqn_last_error(), bytes)
