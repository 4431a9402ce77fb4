"""Evaluation harness: the reference's src/scripts/test.py on
the GPU path.

Semantics follow test.py:49-150 (run_evaluation_episode) and :153-259
(main_eval), with every evaluation episode of a mode run as one env replica
of a single batched TrafficEnv:
  * episode i of every mode uses seed eval_seed_start + i for the traffic and
    for the numpy stream (set_seeds(episode_seed), test.py:52);
  * modes: 'dqn' -- greedy online-Q action, with eval_epsilon exploration
    drawn as np.random.rand() < eps then randint (test.py:84-87); 'random' --
    np.random.randint(0, 4) alone per agent (test.py:92-93); 'fixed' -- the
    cycle [(action 0, 30 s), (action 2, 30 s)] advanced by step_duration
    before each choice (test.py:93-107, :214-216);
  * per episode: total_reward = sum over steps and agents of the env reward,
    avg_reward_per_agent = total / A, avg_step_queue_sum = mean over agent-steps
    of sum(obs[:12]) of the observation the action was chosen from
    (test.py:124-131, :137-139), steps -- each replica's own, up to its own
    `done` (a replica whose demand drains early stops counting there);
  * summary per mode: mean / std of total_reward and avg_step_queue_sum, mean
    steps, episode count (test.py:237-245).
The reward is the training path's (train.py:254, A-3) -- the reference's
test.py runs the 74-dim SumoTrafficEnvironment whose reward differs; this
harness evaluates the environment the agents are trained in.
"""
from dataclasses import replace

import numpy as np
import torch

from . import kernels as K
from .agent import AgentConfig, BatchedDQN, n_params_keras
from .env import EnvConfig, TrafficEnv

FIXED_CYCLE = ((0, 30.0), (2, 30.0))  # test.py:214-216


def fixed_cycle_actions(n_steps, step_duration, cycle=FIXED_CYCLE):
    """The action at each RL step of test.py's fixed-time state machine."""
    idx, t_in, out = 0, 0.0, []
    for _ in range(n_steps):
        if t_in >= cycle[idx][1]:
            idx = (idx + 1) % len(cycle)
            t_in = 0.0
        out.append(cycle[idx][0])
        t_in += step_duration
    return out


def _policy_weights(weights, A, E):
    """[E*A, P] Keras-order weights: `weights` is a list of A per-junction
    [W1, b1, W2, b2, W3, b3] lists, or a [A, P] / [1, P] array."""
    if isinstance(weights, (list, tuple)):
        flat = np.stack([np.concatenate([np.asarray(w, np.float32).ravel() for w in ws])
                         for ws in weights])
    else:
        flat = np.asarray(weights, np.float32)
    if flat.shape[0] not in (1, A):
        raise ValueError(f"need 1 or {A} policies, got {flat.shape[0]}")
    if flat.shape[0] == 1:
        flat = np.repeat(flat, A, axis=0)
    return np.tile(flat, (E, 1))


def run_mode(env_cfg: EnvConfig, mode, episodes=10, eval_seed_start=10000, eval_epsilon=0.01,
             weights=None, agent_cfg: AgentConfig = None, max_steps=1000, device="cuda"):
    """All `episodes` evaluation episodes of one mode, as env replicas."""
    cfg = replace(env_cfg, num_envs=episodes, seed=eval_seed_start, env_offset=0)
    env = TrafficEnv(cfg, device=device)
    E, A = env.E, env.A
    dev = env.device
    np_state = K.seed_streams(env.seeds, "np", dev)
    agent = None
    if mode == "dqn":
        if weights is None:
            raise ValueError("dqn mode needs trained weights")
        w = _policy_weights(weights, A, E)
        H = next((h for h in (64, 128) if n_params_keras(h) == w.shape[1]), None)
        if H is None:
            raise ValueError(f"policy weights of {w.shape[1]} parameters: need H = 64 or 128")
        acfg = replace(agent_cfg or AgentConfig(), shared_params=False, replay_buffer_size=128,
                       nn_layers=[H, H])
        agent = BatchedDQN(E, A, acfg, device=dev, init_weights=w,
                           streams=(np_state, K.seed_streams(env.seeds, "py", dev)))
    elif mode not in ("random", "fixed"):
        raise ValueError(f"unknown mode {mode!r}")
    n_steps = min(max_steps, cfg.max_sim_time // cfg.step_duration)
    fixed = fixed_cycle_actions(n_steps, cfg.step_duration) if mode == "fixed" else None
    obs = env.reset()
    total = torch.zeros(E, dtype=torch.float64, device=dev)
    qsum = torch.zeros(E, dtype=torch.float64, device=dev)
    # each replica is one evaluation episode: it counts until its own `done`
    # (test.py:75, :115-133); a replica whose demand drained restarts in the
    # env and is masked out from then on
    ended = torch.zeros(E, dtype=torch.bool, device=dev)
    ended_host = np.zeros(E, dtype=bool)
    steps = np.zeros(E, dtype=np.int64)
    step = 0
    while True:
        if mode == "dqn":
            actions = agent.act(obs, eps=eval_epsilon)
        elif mode == "random":
            actions = K.act(np_state, A, uniform=True)  # test.py:92-93: randint only
        else:
            actions = torch.full((E, A), fixed[step], dtype=torch.int32, device=dev)
        live = (~ended).to(torch.float64)
        qsum += live * obs[..., :12].sum(dim=(1, 2), dtype=torch.float64)
        next_obs, reward, done, info = env.step(actions)
        total += live * reward.sum(dim=1)
        steps[~ended_host] += 1
        step += 1
        if "obs_next" in info:
            ended |= info["done"].bool()
            ended_host |= info["restarted"]
            obs = info["obs_next"]
        else:
            obs = next_obs
            if done:
                ended_host[:] = True
        if ended_host.all() or step >= max_steps:  # test.py:133 max_steps_per_episode
            break
    total = total.cpu().numpy()
    qavg = qsum.cpu().numpy() / (steps * A)
    return [{"mode": mode, "seed": int(env.seeds[e]), "total_reward": float(total[e]),
             "avg_reward_per_agent": float(total[e] / A), "avg_step_queue_sum": float(qavg[e]),
             "steps": int(steps[e])} for e in range(E)]


def evaluate(env_cfg: EnvConfig, modes=("dqn", "random"), episodes=10, eval_seed_start=10000,
             eval_epsilon=0.01, weights=None, agent_cfg=None, max_steps=1000, device="cuda"):
    rows = []
    for m in modes:
        rows += run_mode(env_cfg, m, episodes, eval_seed_start, eval_epsilon, weights, agent_cfg,
                         max_steps, device)
    return rows


def summarize(rows):
    """test.py:237-245 groupby('mode') aggregate (pandas DataFrame)."""
    import pandas as pd
    df = pd.DataFrame(rows)
    return df.groupby("mode").agg(
        mean_reward=("total_reward", "mean"), std_reward=("total_reward", "std"),
        mean_avg_queue=("avg_step_queue_sum", "mean"), std_avg_queue=("avg_step_queue_sum", "std"),
        mean_steps=("steps", "mean"), episodes=("seed", "count"))
