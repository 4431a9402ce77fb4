"""One tiny invocation of the whole hot path on cuda:0, checked against the
CPU oracle (called by __graft_entry__.smoke(); the oracle is test
infrastructure and is passed in by the caller, never imported here).

2x2 grid x 4 env replicas: act (numpy stream) -> sim + observe -> remember,
repeated until the replay holds 128 transitions, then sample (CPython stream)
+ one fused learn step (fp32 MFMA path), each stage compared to the oracle.
"""


def run(TrafficEnv, EnvConfig, BatchedDQN, AgentConfig, K, O, np, torch):
    R, C, E = 2, 2, 4
    A = R * C
    env = TrafficEnv(EnvConfig(rows=R, cols=C, num_envs=E, seed=11), device="cuda:0")
    agent = BatchedDQN(E, A, AgentConfig(precision="fp32", seed=11), device="cuda:0",
                       env_seeds=env.seeds)
    refs = [O.OracleEnv(R, C, int(s)) for s in env.seeds]
    nps = [O.np_stream(int(s)) for s in env.seeds]
    pys = [O.py_stream(int(s)) for s in env.seeds]
    obs = env.reset()
    L = [O.local_state(np.zeros((A, 12)), np.zeros(A), np.zeros(A), 0) for _ in range(E)]
    t = 0
    for step in range(128):
        acts = agent.act(obs)
        a_host = acts.cpu().numpy()
        for e in range(E):
            assert (a_host[e] == O.act(nps[e], A, 1.0)).all(), "act vs numpy stream"
        nobs, rew, done, _ = env.step(acts)
        halt_g = env.halt.cpu().numpy()
        rew_g = rew.cpu().numpy()
        for e in range(E):
            halt, ph, ts, _ = refs[e].step(a_host[e], 3, t, 10, 2400)
            assert (halt_g[e] == halt).all(), "sim halting counts vs oracle"
            assert (rew_g[e] == O.reward(L[e])).all(), "reward vs oracle"
            L[e] = O.local_state(halt, ph, ts, 0)
        t += 10
        agent.remember(obs, acts, rew, nobs, done)
        obs = nobs
    agent.ring.check()
    p0 = agent.keras_params("params").copy()
    loss = agent.replay()
    assert loss is not None, "learn must be active at 128 transitions"
    idx = agent.idx.cpu().numpy()
    lg = loss.cpu().numpy()
    ring = agent.ring
    p_gpu = agent.keras_params("params")
    for j in range(agent.NA):
        e = j // A  # agents of one env draw from that env's stream in junction order
        exp_idx = O.py_sample(pys[e], len(ring), 128)
        assert (idx[j] == exp_idx).all(), "replay indices vs CPython random.sample"
        slots = ring.slots_of(idx[j])
        S = ring.s[j].cpu().numpy()[slots, :89].astype(np.float32)
        S2 = ring.n[j].cpu().numpy()[slots, :89].astype(np.float32)
        Aa = ring.a[j].cpu().numpy()[slots].astype(np.int32)
        Rn = O.zscore(ring.r[j].cpu().numpy()[slots])
        D = ring.d[j].cpu().numpy()[slots].astype(np.float32)
        p = p0[j].copy()
        m = np.zeros_like(p)
        v = np.zeros_like(p)
        l_ref = O.learn(p, p0[j].copy(), m, v, S, Aa, Rn, S2, D, 1)
        assert abs(float(lg[j]) - l_ref) <= 1e-5 * max(1.0, abs(l_ref)), "loss vs oracle"
        assert np.abs(p_gpu[j] - p).max() <= 1e-5, "Adam-updated weights vs oracle"
    torch.cuda.synchronize()
