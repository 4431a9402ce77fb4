"""GPU parity: device streams, act, replay sample/store and observe vs the oracle
(bit-exact), called through the C ABI."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import oracle as O  # noqa: E402
from dmdqn_amd import kernels as K  # noqa: E402

DEV = "cuda"


def _u32(t):
    return t.cpu().numpy().view(np.uint32).astype(np.uint64)


@pytest.mark.parametrize("kind", ["np", "py"])
def test_stream_seed_and_draw(kind):
    seeds = [0, 1, 42, 12345, 2**31 - 1, 4000000000, 7, 99]
    st = K.seed_streams(seeds, kind)
    got = _u32(K.draw_u32(st, 1500))
    got2 = _u32(K.draw_u32(st, 700))  # continues the stream across twists
    for e, s in enumerate(seeds):
        ref = O.py_stream(s) if kind == "py" else O.np_stream(s)
        exp = O.u32(ref, 2200)
        np.testing.assert_array_equal(got[e], exp[:1500])
        np.testing.assert_array_equal(got2[e], exp[1500:])


@pytest.mark.parametrize("A", [1, 4, 9, 16, 64])
def test_act_eps1_matches_numpy_stream(A):
    seeds = list(range(100, 100 + 37))
    st = K.seed_streams(seeds, "np")
    for step in range(25):  # several RL steps, crossing MT block boundaries
        a = K.act(st, A).cpu().numpy()
        if step == 0:
            refs = [O.np_stream(s) for s in seeds]
        for e in range(len(seeds)):
            np.testing.assert_array_equal(a[e], O.act(refs[e], A, 1.0))


def test_act_eps_greedy():
    seeds = [3, 4, 5, 6]
    A = 16
    st = K.seed_streams(seeds, "np")
    refs = [O.np_stream(s) for s in seeds]
    g = torch.randint(0, 4, (len(seeds), A), dtype=torch.int32, device=DEV)
    for eps in [0.9, 0.5, 0.05, 0.0]:
        a = K.act(st, A, eps=eps, greedy=g).cpu().numpy()
        gn = g.cpu().numpy()
        for e in range(len(seeds)):
            np.testing.assert_array_equal(a[e], O.act(refs[e], A, eps, gn[e]))


@pytest.mark.parametrize("n", [128, 129, 500, 1045, 1046, 5000, 10000])
def test_replay_sample_matches_cpython(n):
    seeds = [0, 1, 12345, 77]
    A = 9
    st = K.seed_streams(seeds, "py")
    refs = [O.py_stream(s) for s in seeds]
    for rep in range(2):
        idx = K.replay_sample(st, A, n, 128).cpu().numpy().reshape(len(seeds), A, 128)
        for e in range(len(seeds)):
            for j in range(A):
                np.testing.assert_array_equal(idx[e, j], O.py_sample(refs[e], n, 128))


@pytest.mark.parametrize("A,n,k", [(64, 200, 128), (70, 300, 32), (3, 21, 5), (3, 22, 5),
                                   (5, 7, 7), (2, 3000, 1000), (64, 10000, 128), (1, 128, 128),
                                   (4, 20000, 128), (3, 16385, 128), (2, 40000, 256),
                                   (2, 100000, 128)])
def test_replay_sample_shapes(A, n, k):
    """Agent groups beyond one wave (A > 64), small k (setsize 21), k = n and
    large k: every branch and chunk-boundary case of the chunked sampler."""
    seeds = [5, 6, 7]
    st = K.seed_streams(seeds, "py")
    refs = [O.py_stream(s) for s in seeds]
    for rep in range(2):
        idx = K.replay_sample(st, A, n, k).cpu().numpy().reshape(len(seeds), A, k)
        for e in range(len(seeds)):
            for j in range(A):
                np.testing.assert_array_equal(idx[e, j], O.py_sample(refs[e], n, k))


@pytest.mark.parametrize("tlog", [0, 3, 6, 10])
def test_replay_sample_table_collisions(tlog, lib_option):
    """Set branch with the first-lane table capped at 2^tlog entries: values
    sharing a slot (r = r' mod 2^tlog) in almost every chunk resolve in turn."""
    lib_option("sample_tlog", tlog)
    seeds = [8, 9]
    st = K.seed_streams(seeds, "py")
    refs = [O.py_stream(s) for s in seeds]
    for n in (1046, 10000):
        idx = K.replay_sample(st, 16, n, 128).cpu().numpy().reshape(len(seeds), 16, 128)
        for e in range(len(seeds)):
            for j in range(16):
                np.testing.assert_array_equal(idx[e, j], O.py_sample(refs[e], n, 128))


@pytest.mark.parametrize("budget", ["beside_shared_learn", 6400, 14000, 1 << 24])
def test_replay_sample_lds_budget(budget):
    """dmdqn_replay_sample_budget: the sampler block's LDS held to a budget (the
    trainer's "learn" schedule gives it what the shared S' pass leaves of the
    device's CU, dmdqn_device_lds_per_cu: 160 KB on gfx950; 6,400 B leaves the
    set branch a 32-entry table at n = 10,000; a budget beyond the device's
    per-workgroup LDS is clamped to it): the draws are CPython's, whatever the
    table size."""
    from dmdqn_amd import _lib
    assert _lib.device_lds_per_cu() == 160 * 1024  # MI355X (gfx950)
    b = (_lib.device_lds_per_cu() - _lib.learn_shared_lds_bytes()
         if budget == "beside_shared_learn" else budget)
    seeds = [3, 4]
    st = K.seed_streams(seeds, "py")
    refs = [O.py_stream(s) for s in seeds]
    for n in (200, 1046, 10000):
        idx = K.replay_sample(st, 16, n, 128, lds_budget=b).cpu().numpy().reshape(len(seeds), 16, 128)
        for e in range(len(seeds)):
            for j in range(16):
                np.testing.assert_array_equal(idx[e, j], O.py_sample(refs[e], n, 128))


@pytest.mark.parametrize("grid", [(1, 1), (2, 2), (3, 3), (4, 4), (8, 8), (2, 3)])
@pytest.mark.parametrize("mode", [0, 1])
def test_observe_reward(grid, mode):
    R, C = grid
    A = R * C
    E = 33
    g = torch.Generator().manual_seed(R * 10 + C + mode)
    halt = torch.randint(0, 24, (E, A, 12), generator=g, dtype=torch.int32)
    phase = torch.randint(0, 12, (E, A), generator=g, dtype=torch.int32)
    tsp = torch.randint(0, 30, (E, A), generator=g, dtype=torch.int32)
    prev = torch.randint(0, 24, (E, A, 17), generator=g).float()
    loc, obs, rew = K.observe(R, C, halt.to(DEV), phase.to(DEV), tsp.to(DEV), mode,
                              prev_local=prev.to(DEV))
    loc, obs, rew = loc.cpu().numpy(), obs.cpu().numpy(), rew.cpu().numpy()
    for e in range(E):
        L = O.local_state(halt[e].numpy(), phase[e].numpy(), tsp[e].numpy(), mode)
        np.testing.assert_array_equal(loc[e], L)
        np.testing.assert_array_equal(obs[e], O.build_obs(R, C, L))
        np.testing.assert_array_equal(rew[e], O.reward(prev[e].numpy()))


def test_replay_store_roundtrip_and_range_check():
    NA, cap = 40, 7
    ring = K.ReplayRing(NA, cap)
    g = torch.Generator().manual_seed(0)
    rows = []
    for t in range(10):
        s = torch.randint(-1, 24, (NA, 89), generator=g).float()
        n = torch.randint(-1, 24, (NA, 89), generator=g).float()
        a = torch.randint(0, 4, (NA,), generator=g, dtype=torch.int32)
        r = torch.randn(NA, generator=g, dtype=torch.float64)
        d = (torch.rand(NA, generator=g) < 0.3).to(torch.uint8)
        ring.store(s.to(DEV), n.to(DEV), a.to(DEV), r.to(DEV), d.to(DEV))
        rows.append((s, n, a, r, d))
    ring.check()
    # a deque of maxlen cap in cap + SPARE slots: position p -> slot (start + p) % slots
    NS = cap + K.ReplayRing.SPARE
    assert len(ring) == cap and ring.slots == NS and ring.start == (10 - cap) % NS
    S = ring.s.cpu().numpy()
    for p in range(cap):
        t = 10 - cap + p
        slot = int(ring.slots_of(p))
        assert slot == t % NS
        s, n, a, r, d = rows[t]
        np.testing.assert_array_equal(S[:, slot, :89].astype(np.float32), s.numpy())
        np.testing.assert_array_equal(S[:, slot, 89:], 0)
        np.testing.assert_array_equal(ring.n.cpu().numpy()[:, slot, :89].astype(np.float32), n.numpy())
        np.testing.assert_array_equal(ring.a.cpu().numpy()[:, slot], a.numpy())
        np.testing.assert_array_equal(ring.r.cpu().numpy()[:, slot], r.numpy())
        np.testing.assert_array_equal(ring.d.cpu().numpy()[:, slot], d.numpy())
        # the s' row's tail carries the same a, done, r for the learn kernels
        # (include/dmdqn.h DMDQN_ROW_A/_D/_R); everything else past 88 is zero
        N = ring.n.cpu().numpy()[:, slot].view(np.uint8)
        np.testing.assert_array_equal(N[:, 96], a.numpy())
        np.testing.assert_array_equal(N[:, 97], d.numpy())
        np.testing.assert_array_equal(N[:, 104:112].copy().view(np.float64)[:, 0], r.numpy())
        tail = np.delete(np.arange(89, 128), [96 - 89, 97 - 89] + list(range(104 - 89, 112 - 89)))
        np.testing.assert_array_equal(N[:, tail], 0)
    bad = torch.zeros((NA, 89), device=DEV)
    bad[3, 5] = 0.5
    ring.store(bad, bad, torch.zeros(NA, dtype=torch.int32, device=DEV),
               torch.zeros(NA, dtype=torch.float64, device=DEV),
               torch.zeros(NA, dtype=torch.uint8, device=DEV))
    with pytest.raises(Exception):
        ring.check()
