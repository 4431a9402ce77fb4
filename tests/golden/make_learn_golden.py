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

Usage:  python tests/golden/make_learn_golden.py [--out tests/golden]
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
sys.path.insert(0, HERE)
import tf_shim  # noqa: E402


def _import_dqn():
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=HERE)
    args = ap.parse_args()
    out = os.path.abspath(args.out)
    scratch = "/tmp/dmdqn_golden_scratch"
    os.makedirs(scratch, exist_ok=True)
    os.chdir(scratch)  # log_config.py truncates ./replay_buffer.log
    sys.dont_write_bytecode = True
    import torch
    torch.set_num_threads(1)
    dq = _import_dqn()
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
