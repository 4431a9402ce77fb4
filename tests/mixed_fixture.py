"""Replay of tests/golden/learn_mixed.npz (TEST INFRASTRUCTURE).

The fixture is the reference's own DQNAgent (dqn_agent.py:97-434) run under
Keras 3's mixed_float16 / mixed_bfloat16 policy (tests/golden/tf_shim.py,
tests/golden/make_learn_golden.py).  For each run it holds windows of
consecutive learns: the state before the window's first learn and the 16-bit
gradient Keras' Adam received at every learn of the window.  Keras-3 Adam is
elementwise f32 arithmetic, so replaying it on those gradients gives the
reference's exact state before every learn of the window (checked against the
stored w after the window's last learn).

The batches: epsilon stays 1 in these runs, so the deque holds transitions
t = 0..steps-1 of the stored episode in order, and learn k (at loop step t)
draws random.sample(deque, 128) from the CPython stream seeded with `seed`
(dqn_agent.py:63) -- the same indices random.sample(range(len(deque)), 128)
gives, whatever the weights.
"""
import os
import random

import numpy as np

import oracle as O

HERE = os.path.dirname(os.path.abspath(__file__))
PATH = os.path.join(HERE, "golden", "learn_mixed.npz")
RUNS = {"mse_f16": ("fp16", 0), "huber_f16": ("fp16", 1), "mse_bf16": ("bf16", 0)}


def load():
    return np.load(PATH)


def grad_from_bits(bits, precision):
    bits = np.asarray(bits, np.uint16)
    if precision == "fp16":
        return bits.view(np.float16).astype(np.float32)
    return (bits.astype(np.uint32) << 16).view(np.float32)


def cfg(G, tag):
    steps, buf, tuf, seed, init_seed = (int(x) for x in G[f"{tag}_cfg"])
    return dict(steps=steps, buf=buf, tuf=tuf, seed=seed, init_seed=init_seed)


def batches(G, tag):
    """Yield (learn k, loop step t, S, A, Rn, S2, D, deque positions) for every learn."""
    c = cfg(G, tag)
    obs = G[f"{tag}_obs"].astype(np.float32)
    rew, done, act = G[f"{tag}_rew"], G[f"{tag}_done"], G[f"{tag}_actions"]
    rs = random.Random(c["seed"])
    dq, k = [], 0
    for t in range(c["steps"]):
        dq.append(t)
        if len(dq) > c["buf"]:
            dq.pop(0)
        if len(dq) >= 128:
            k += 1
            pos = np.array(rs.sample(range(len(dq)), 128))
            ts = np.array([dq[i] for i in pos])
            yield (k, t, obs[ts], act[ts].astype(np.int32), O.zscore(rew[ts]), obs[ts + 1],
                   done[ts].astype(np.float32), pos)


def window_states(G, tag):
    """{learn k: (w, m, v, target, grad)} -- the reference's state before learn k
    and the gradient of learn k, for every learn inside a window; plus
    {window end k: w after it} for the reconstruction check."""
    prec = RUNS[tag][0]
    tuf = cfg(G, tag)["tuf"]
    grads = G[f"{tag}_grad_bits"]
    out, post, gi = {}, {}, 0
    for i, (a, n) in enumerate(G[f"{tag}_windows"]):
        w, m, v, tg = (G[f"{tag}_win_{x}"][i].copy() for x in ("w", "m", "v", "t"))
        for k in range(int(a), int(a + n)):
            g = grad_from_bits(grads[gi], prec)
            gi += 1
            out[k] = (w.copy(), m.copy(), v.copy(), tg.copy(), g)
            alpha, c1, c2, eps = O.keras_adam_consts(k)
            m = m + (g - m) * c1
            v = v + (g * g - v) * c2
            w = w - (m * alpha) / (np.sqrt(v) + eps)
            if k % tuf == 0:
                tg = w.copy()
        post[int(a + n - 1)] = w
    return out, post
