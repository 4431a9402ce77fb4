"""The batched reference training loop (src/scripts/train.py:188-316) on the GPU.

One `step()` is one iteration of the loop body for every agent of every env
replica:  act (select_action) -> env step (setPhase, K substeps) -> observe /
reward -> remember -> replay (learn), in the reference's order.  All of it is
kernel launches on one HIP stream; the host keeps only counters.
"""
from dataclasses import dataclass

import torch

from .agent import AgentConfig, BatchedDQN
from .env import EnvConfig, TrafficEnv


@dataclass
class StepStats:
    loss_launched: bool
    done: bool


class Trainer:
    def __init__(self, env_cfg: EnvConfig = None, agent_cfg: AgentConfig = None, device="cuda"):
        self.env = TrafficEnv(env_cfg or EnvConfig(), device=device)
        self.agent = BatchedDQN(self.env.E, self.env.A, agent_cfg or AgentConfig(), device=device,
                                env_seeds=self.env.seeds)
        self.obs = self.env.reset()
        self.episode = 0
        self.step_count = 0
        self.total_steps = 0
        self.last_loss = None
        self.last_reward = None

    def step(self, collect_stats=False):
        """One loop iteration for every replica; collect_stats makes the learn
        also produce the metrics of dqn_agent.py:361-370 (agent.learn_metrics)."""
        env, agent = self.env, self.agent
        actions = agent.act(self.obs)                          # train.py:211-222
        next_obs, reward, done, info = env.step(actions)       # train.py:225-270
        agent.remember(self.obs, actions, reward, next_obs, done)  # train.py:274-282
        loss = agent.learn(collect_stats=collect_stats)
        self.last_loss, self.last_reward = loss, reward
        self.step_count += 1
        self.total_steps += 1
        if done:                                               # train.py:188-190
            self.episode += 1
            self.step_count = 0
            self.obs = env.reset()
        else:
            self.obs = next_obs
        return StepStats(loss is not None, done)

    def agent_env_steps(self, n_steps):
        return n_steps * self.env.E * self.env.A

    def synchronize(self):
        torch.cuda.synchronize(self.env.device)
