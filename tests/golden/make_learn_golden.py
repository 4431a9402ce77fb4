"""Golden fixtures for the learn step, made by running the reference's OWN
DQNAgent (src/agents/dqn_agent.py) under the torch-backed TensorFlow shim
(tests/golden/tf_shim.py).  TEST INFRASTRUCTURE ONLY: run in the build
container (needs /root/reference); the GPU box only reads the .npz output.

What executes is the reference code: DQNAgent.__init__ (:97-151),
select_action (:246-274, on the global numpy stream), remember ->
ReplayBuffer.add (:312-326, :31-57), replay -> learn (:428-434, :328-380:
random.sample on the deque, the f64 z-score, Double-DQN target, one-hot,
MSE, GradientTape, Adam.apply_gradients, learn_step_counter and the hard
target sync every target_update_frequency learns) and update_target_network
(:382-387).  The loop mirrors train.py:207-282 for one junction: select_action
-> (env step: synthetic integer observations, train.py-style rewards) ->
remember -> replay.

Runs (all fp32, see tf_shim.py):
  mse    replay_buffer_size 300 (the deque wraps), target_update_frequency 50,
         nn_layers [128, 128] (train.py:120), 520 loop steps = 393 learns;
         epsilon 1 for steps < 400 (A-1), then global_step_count = 40000
         (epsilon = exp(-2): the greedy branch of select_action runs on the
         trained online network).
  huber  the same agent with the loss of src/experimental/agent.py:99
         (tf.keras.losses.Huber(), delta 1) in place of MeanSquaredError,
         360 loop steps = 233 learns, target_update_frequency 40.

Mixed-precision runs (learn_mixed.npz): the policy train.py:61 sets at import,
keras.mixed_precision.set_global_policy("mixed_float16"), is set before the
agent is built, so its Dense layers follow Keras 3's mixed semantics (see
tf_shim.py); "mixed_bfloat16" for the bf16 run (BASELINE config C2's dtype).
Epsilon stays 1 (the reference training path, A-1), so the stored
transitions and the replay draws do not depend on the weights and a GPU run
from the same seeds sees the same batches at every learn.
  mse_f16    460 loop steps = 333 learns, replay 300 (wraps), target sync
             every 50 learns;
  huber_f16  330 steps = 203 learns, replay 200, sync every 40;
  mse_bf16   330 steps = 203 learns, replay 250, sync every 60.
Per learn: the loss, and the smallest gap between the two largest f16 online
Q(S') of the batch in units of the larger one's ulp (tie_ulps: 0 = an exact
tie, which tf.argmax breaks to the first index).  Windows of consecutive
learns: the state before a window's first learn (online w, Adam m, v, target
w; Keras order), the gradient Adam received at each of its learns (16-bit
values, stored as their raw bits: with Keras-3 Adam in f32 they give the
reference's exact state at every learn of the window) and w after its last.

The reference file imported is checked against its SHA-256 first (REF_SHA256);
this script runs only by hand in the build container, never under pytest.

Usage:  python tests/golden/make_learn_golden.py [--out tests/golden] [--only mixed|fp32]
"""
import argparse
import importlib
import os
import random
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
REF_FILE = os.path.join(REF, "src", "agents", "dqn_agent.py")
REF_SHA256 = "04f930e02bc485d2979632a16540936d31a6df8fd695fb3cf9d1f4f314a921f5"
sys.path.insert(0, HERE)
import tf_shim  # noqa: E402


def _import_dqn():
    import hashlib
    with open(REF_FILE, "rb") as f:
        digest = hashlib.sha256(f.read()).hexdigest()
    if digest != REF_SHA256:
        raise SystemExit(f"{REF_FILE}: sha256 {digest} is not the pinned {REF_SHA256}")
    tf_shim.install()
    for name in ["traci", "sumolib", "wandb"]:
        sys.modules.setdefault(name, types.ModuleType(name))
    if REF not in sys.path:
        sys.path.insert(0, REF)
    sys.modules.pop("src.agents.dqn_agent", None)
    return importlib.import_module("src.agents.dqn_agent")


def keras_init(rng, H=128):
    """Keras-order initial weights (HeNormal truncated / GlorotUniform / zeros)."""
    def he(fi, fo):
        std = np.sqrt(2.0 / fi) / 0.87962566103423978
        w = rng.normal(0, std, size=(fi, fo))
        bad = np.abs(w) > 2 * std
        while bad.any():
            w[bad] = rng.normal(0, std, size=int(bad.sum()))
            bad = np.abs(w) > 2 * std
        return w
    lim = np.sqrt(6.0 / (H + 4))
    return [he(89, H).astype(np.float32), np.zeros(H, np.float32), he(H, H).astype(np.float32),
            np.zeros(H, np.float32), rng.uniform(-lim, lim, (H, 4)).astype(np.float32),
            np.zeros(4, np.float32)]


def make_episode(rng, T):
    """Synthetic integer observations (halting counts 0..23, -1 padding), f64
    rewards from the pre-step local state as train.py:159-165,254, done at
    the last step of each 240-step episode (train.py:233-236)."""
    obs = rng.randint(0, 24, size=(T + 1, 89)).astype(np.float32)
    obs[:, 17:21] = rng.randint(0, 2, size=(T + 1, 4))
    pad = rng.rand(T + 1, 4) < 0.3
    for d in range(4):
        obs[pad[:, d], 21 + 17 * d:38 + 17 * d] = -1.0
    loc = -obs[:-1, :12].sum(1).astype(np.float64)
    glob = loc * 9 + rng.randint(-200, 0, size=T)
    rew = 0.3 * loc + 0.7 * glob
    done = (np.arange(T) % 240) == 239
    return obs, rew, done


def run(dq, tag, loss_cls, steps, greedy_from, buf, tuf, seed, init_seed):
    tf_shim.SUMMARIES.clear()
    tfm = sys.modules["tensorflow"]
    tfm.keras.losses.MeanSquaredError = loss_cls  # learn() builds it inline (:352)
    cfg = {"learning_rate": 0.001, "gamma": 0.99, "epsilon_start": 1.0, "epsilon_min": 0.01,
           "epsilon_decay_steps": 200000, "replay_buffer_size": buf, "batch_size": 128,
           "target_update_frequency": tuf, "nn_layers": [128, 128]}
    agent = dq.DQNAgent(89, 4, "J_0_0", cfg)
    rng = np.random.RandomState(init_seed)
    w0 = keras_init(rng)
    agent.online_network.set_weights(w0)
    agent.target_network.set_weights(w0)
    obs, rew, done = make_episode(rng, steps)
    random.seed(seed)
    np.random.seed(seed)
    actions = np.zeros(steps, np.int32)
    losses = np.full(steps, np.nan, np.float64)
    eps = np.zeros(steps, np.float64)
    snaps = {}
    for t in range(steps):
        if t == greedy_from:
            agent.global_step_count = 40000
        s = obs[t][None]
        a = agent.select_action(tfm.convert_to_tensor(s, dtype=tfm.float32))
        actions[t] = int(a)
        eps[t] = agent.get_epsilon()
        agent.remember(s, int(a), float(rew[t]), obs[t + 1][None], bool(done[t]))
        loss = agent.learn()
        if loss is not None:
            losses[t] = float(loss.detach().numpy())
            k = agent.learn_step_counter
            if k in (1, tuf + 1) and (tag == "mse" or k == 1):
                snaps[k] = np.concatenate([w.reshape(-1) for w in agent.online_network.get_weights()])
    flat = lambda ws: np.concatenate([w.reshape(-1) for w in ws])
    summ = {}
    for name in ["q_values_mean", "q_values_std", "action_distribution"]:
        summ[name] = np.stack([v for (n, v, _) in tf_shim.SUMMARIES if n == name])
    return dict(w0=flat(w0), obs=obs.astype(np.int8), rew=rew, done=done.astype(np.uint8),
                actions=actions, losses=losses, eps=eps,
                final_online=flat(agent.online_network.get_weights()),
                final_target=flat(agent.target_network.get_weights()),
                snap_steps=np.array(sorted(snaps)), snaps=np.stack([snaps[k] for k in sorted(snaps)]),
                learn_steps=np.array([agent.learn_step_counter]), **summ,
                cfg=np.array([steps, greedy_from, buf, tuf, seed, init_seed]))


def _flat(ws):
    return np.concatenate([np.asarray(w, np.float32).reshape(-1) for w in ws])


def _adam_slots(agent):
    """Keras-order flat (m, v) of the agent's optimizer (zeros before the first step)."""
    vs = agent.online_network.trainable_variables
    z = [np.zeros(v.t.shape, np.float32) for v in vs]
    sl = [agent.optimizer.slots.get(id(v)) for v in vs]
    m = [z[i] if s is None else s[0].numpy() for i, s in enumerate(sl)]
    v = [z[i] if s is None else s[1].numpy() for i, s in enumerate(sl)]
    return _flat(m), _flat(v)


def _h16_bits(g, policy):
    """A 16-bit gradient (widened to f32 by its cast) as its raw 16 bits."""
    g = np.ascontiguousarray(g, np.float32)
    if policy == "mixed_float16":
        h = g.astype(np.float16)
        assert np.array_equal(h.astype(np.float32), g)
        return h.view(np.uint16)
    u = g.view(np.uint32)
    assert not (u & 0xFFFF).any()
    return (u >> 16).astype(np.uint16)


def run_mixed(dq, tag, policy, loss_cls, steps, buf, tuf, seed, init_seed, windows):
    """windows: [(first learn, number of learns)]: the state before the window's
    first learn, the 16-bit gradient of each of its learns and w after its last."""
    tf_shim.SUMMARIES.clear()
    tfm = sys.modules["tensorflow"]
    tfm.keras.losses.MeanSquaredError = loss_cls
    tfm.keras.mixed_precision.set_global_policy(policy)  # train.py:61
    gaps = []
    argmax0 = tfm.argmax

    def argmax_gap(x, axis=0, output_type=None):
        # the learn's tf.argmax(online(S')) (dqn_agent.py:342): record the
        # batch's smallest top-2 gap in ulps of the 16-bit larger value
        q = x.detach().float().numpy()
        top = np.sort(q, axis=1)
        hi = top[:, -1].astype(np.float64)
        e = np.floor(np.log2(np.maximum(np.abs(hi), 2.0 ** -14)))
        ulp = 2.0 ** (e - (10 if x.dtype == tf_shim.torch.float16 else 7))
        gaps.append(float(((top[:, -1] - top[:, -2]) / ulp).min()))
        return argmax0(x, axis=axis, output_type=output_type)

    starts = {a: i for i, (a, n) in enumerate(windows)}
    ends = {a + n - 1: i for i, (a, n) in enumerate(windows)}
    inside = {k for a, n in windows for k in range(a, a + n)}
    tfm.argmax = argmax_gap
    try:
        cfg = {"learning_rate": 0.001, "gamma": 0.99, "epsilon_start": 1.0, "epsilon_min": 0.01,
               "epsilon_decay_steps": 200000, "replay_buffer_size": buf, "batch_size": 128,
               "target_update_frequency": tuf, "nn_layers": [128, 128]}
        agent = dq.DQNAgent(89, 4, "J_0_0", cfg)
        rng = np.random.RandomState(init_seed)
        w0 = keras_init(rng)
        agent.online_network.set_weights(w0)
        agent.target_network.set_weights(w0)
        obs, rew, done = make_episode(rng, steps)
        random.seed(seed)
        np.random.seed(seed)
        actions = np.zeros(steps, np.int32)
        losses = np.full(steps, np.nan, np.float64)
        win = {k: [None] * len(windows) for k in ["w", "m", "v", "t", "post_w"]}
        grads = []
        for t in range(steps):
            s = obs[t][None]
            a = agent.select_action(tfm.convert_to_tensor(s, dtype=tfm.float32))
            actions[t] = int(a)
            agent.remember(s, int(a), float(rew[t]), obs[t + 1][None], bool(done[t]))
            k = agent.learn_step_counter + 1 if len(agent.replay_buffer) >= 128 else 0
            if k in starts:
                i = starts[k]
                win["m"][i], win["v"][i] = _adam_slots(agent)
                win["w"][i] = _flat(agent.online_network.get_weights())
                win["t"][i] = _flat(agent.target_network.get_weights())
            loss = agent.learn()
            if loss is not None:
                losses[t] = float(loss.detach().numpy())
            if k in inside:
                grads.append(_h16_bits(_flat([g.numpy() for g in agent.optimizer.last_grads]),
                                       policy))
            if k in ends:
                win["post_w"][ends[k]] = _flat(agent.online_network.get_weights())
        assert all(x is not None for v in win.values() for x in v)
    finally:
        tfm.argmax = argmax0
        tfm.keras.mixed_precision.set_global_policy("float32")
    summ = {}
    for name in ["q_values_mean", "q_values_std"]:
        summ[name] = np.stack([v for (n, v, _) in tf_shim.SUMMARIES if n == name])
    res = dict(w0=_flat(w0), obs=obs.astype(np.int8), rew=rew, done=done.astype(np.uint8),
               actions=actions, losses=losses, tie_ulps=np.array(gaps),
               windows=np.array(windows, np.int64), grad_bits=np.stack(grads),
               learn_steps=np.array([agent.learn_step_counter]),
               final_online=_flat(agent.online_network.get_weights()),
               final_target=_flat(agent.target_network.get_weights()),
               cfg=np.array([steps, buf, tuf, seed, init_seed]), **summ)
    res.update({f"win_{k}": np.stack(v) for k, v in win.items()})
    return res


MIXED_RUNS = [
    # tag, policy, loss, loop steps, replay, target sync, seed, init seed,
    # windows (first learn, learns): the replay wraps from learn 173 (mse_f16)
    ("mse_f16", "mixed_float16", "mse", 460, 300, 50, 17, 23, [(1, 64), (181, 32), (333, 1)]),
    ("huber_f16", "mixed_float16", "huber", 330, 200, 40, 13, 29, [(1, 16), (203, 1)]),
    ("mse_bf16", "mixed_bfloat16", "mse", 330, 250, 60, 19, 31, [(1, 16), (203, 1)]),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=HERE)
    ap.add_argument("--only", choices=["mixed", "fp32"], default=None)
    args = ap.parse_args()
    out = os.path.abspath(args.out)
    scratch = "/tmp/dmdqn_golden_scratch"
    os.makedirs(scratch, exist_ok=True)
    os.chdir(scratch)  # log_config.py truncates ./replay_buffer.log
    sys.dont_write_bytecode = True
    import torch
    torch.set_num_threads(1)
    dq = _import_dqn()
    if args.only != "fp32":
        res = {}
        for tag, policy, loss, steps, buf, tuf, seed, init_seed, wins in MIXED_RUNS:
            loss_cls = tf_shim.Huber if loss == "huber" else tf_shim.MeanSquaredError
            r = run_mixed(dq, tag, policy, loss_cls, steps, buf, tuf, seed, init_seed, wins)
            res.update({f"{tag}_{k}": v for k, v in r.items()})
            print(tag, "learns", int(r["learn_steps"][0]), "last loss", r["losses"][-1],
                  "exact ties", int((r["tie_ulps"] == 0).sum()))
        np.savez_compressed(os.path.join(out, "learn_mixed.npz"), **res)
        print("wrote", os.path.join(out, "learn_mixed.npz"))
    if args.only == "mixed":
        return
    res = {}
    for tag, loss_cls, steps, greedy_from, buf, tuf, seed, init_seed in [
            ("mse", tf_shim.MeanSquaredError, 520, 400, 300, 50, 7, 11),
            ("huber", tf_shim.Huber, 360, 300, 200, 40, 3, 5)]:
        r = run(dq, tag, loss_cls, steps, greedy_from, buf, tuf, seed, init_seed)
        res.update({f"{tag}_{k}": v for k, v in r.items()})
        print(tag, "learns", int(r["learn_steps"][0]), "last loss", r["losses"][-1])
    np.savez_compressed(os.path.join(out, "learn.npz"), **res)
    print("wrote", os.path.join(out, "learn.npz"))


if __name__ == "__main__":
    main()
