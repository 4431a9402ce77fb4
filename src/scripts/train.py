"""src/scripts/train.py -- drop-in training driver on the MI355X kernels.

Same loop as the reference (src/scripts/train.py:182-316): per episode reset,
then while not done: every agent selects an action, the env takes one RL step
(ACTION_MAP phases, STEP_DURATION one-second substeps), rewards are
0.3*local + 0.7*global on the PRE-step state, every agent remembers and
replays (one learn step).  Differences, all outside the hot path:
  * SUMO/TraCI is replaced by the GPU simulator (src/env/traffic_env.py);
  * wandb (network) is replaced by an offline JSONL metrics file;
  * seeds are explicit (--seed), the reference never seeds (A-2).
`--batched` runs the same loop for --envs replicas with one kernel launch per
stage for all agents (dmdqn_amd.trainer.Trainer) -- the throughput path.

  python -m src.scripts.train --episodes 2
  python -m src.scripts.train --batched --envs 1024 --grid 4x4 --episodes 1
"""
import argparse
import json
import logging
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from src.agents import dqn_agent  # noqa: E402
from src.agents.dqn_agent import DQNAgent  # noqa: E402
from src.env.traffic_env import EnvConfig, TrafficEnv  # noqa: E402

EPISODES = 100
MAX_LANES_PER_DIRECTION = 3
STEP_DURATION = 10.0
ACTION_MAP = {0: 0, 1: 3, 2: 6, 3: 9}
MAX_SIM_TIME = 2400

logger = logging.getLogger("dmdqn_logger")

AGENT_CONFIG = {  # train.py:111-121
    "learning_rate": 0.001,
    "gamma": 0.99,
    "epsilon_start": 1.0,
    "epsilon_min": 0.01,
    "epsilon_decay_steps": 200000,
    "replay_buffer_size": 10000,
    "batch_size": 128,
    "target_update_frequency": 500,
    "nn_layers": [128, 128],
}


class SmoothedValue:  # train.py:144-156
    def __init__(self, alpha=0.5):
        self.alpha = alpha
        self.value = None

    def update(self, new_val):
        if self.value is None:
            self.value = new_val
        else:
            self.value = self.alpha * new_val + (1 - self.alpha) * self.value

    def get_value(self):
        return self.value


# SUMO_CFG_PATH of the reference (train.py:50: grid_3x3.sumocfg), derived into the
# simulator's tables by tests/golden/make_scenario.py
DEFAULT_SCENARIO = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__)))), "config", "scenarios", "grid_3x3_p06.npz")


def calculate_local_reward(current_state, next_state):  # train.py:159-160
    return -1.0 * sum(current_state[:12])


def calculate_global_reward(global_state: dict, next_global_state: dict):  # train.py:163-165
    return -1.0 * sum(sum(state[:12]) for state in global_state.values())


def initialize_environment(rows=3, cols=3, seed=0, signal_features="reference", scenario=None):
    env = TrafficEnv(EnvConfig(rows=rows, cols=cols, num_envs=1, seed=seed,
                               step_duration=int(STEP_DURATION), max_sim_time=MAX_SIM_TIME,
                               signal_features=signal_features, scenario=scenario))
    return env, env.get_controlled_intersection_ids()


def create_agents(tl_junctions, config=AGENT_CONFIG):
    return {j: DQNAgent(state_size=89, action_size=4, agent_id=j, config=config) for j in tl_junctions}


def train_agents(episodes=EPISODES, rows=3, cols=3, seed=0, metrics=None, scenario=None,
                 save_dir=None):
    dqn_agent.seed(seed)
    env, tl_junctions = initialize_environment(rows, cols, seed, scenario=scenario)
    agents = create_agents(tl_junctions)
    assert len(agents) == env.R * env.C
    smooth_total = SmoothedValue(alpha=0.3)
    out = open(metrics, "w") if metrics else None
    for episode in range(episodes):
        state_dict = env.reset_dict()
        done, step_count, total_reward = False, 0, 0.0
        while not done:
            actions = {j: agents[j].select_action(state_dict[j][None]) for j in tl_junctions}
            next_state_dict, rewards, done, info = env.step_dict(actions)
            total_reward = sum(rewards.values())
            smooth_total.update(total_reward)
            total_loss = 0.0
            for j in tl_junctions:
                agents[j].remember(state_dict[j][None], actions[j], rewards[j],
                                   next_state_dict[j][None], done)
                total_loss += agents[j].replay()
            if out:
                out.write(json.dumps({"episode": episode, "step": step_count,
                                      "total_reward": total_reward, "total_loss": total_loss,
                                      "smooth_total_reward": smooth_total.get_value()}) + "\n")
            state_dict = next_state_dict
            step_count += 1
        logger.info(f"Episode {episode + 1} complete. Total Reward: {total_reward}")
    if out:
        out.close()
    if save_dir:  # additive: the reference never saves (test.py:195 expects this naming)
        os.makedirs(save_dir, exist_ok=True)
        for j in tl_junctions:
            agents[j].save_model(os.path.join(save_dir, f"agent_{j}.weights.npz"))
    return agents


def train_batched(episodes, rows, cols, envs, precision, seed, metrics=None, scenario=None,
                  shared=False, save_dir=None, resume=None, log_every=20, loss="mse",
                  actuated=False):
    """E env replicas of the loop on the GPU.  The optional JSONL carries the
    reference's learn scalars (dqn_agent.py:361-370: loss, epsilon,
    q_values_mean / _std, action_distribution) and its per-step rewards with
    EMA smoothing (train.py:295-307, SmoothedValue alpha 0.3), averaged over
    replicas, every `log_every` steps (each record syncs)."""
    from dmdqn_amd.agent import AgentConfig
    from dmdqn_amd.trainer import Trainer
    cfg = AgentConfig.from_dict(AGENT_CONFIG)
    cfg.precision, cfg.seed, cfg.shared_params, cfg.loss = precision, seed, shared, loss
    tr = Trainer(EnvConfig(rows=rows, cols=cols, num_envs=envs, seed=seed, scenario=scenario,
                           actuated=actuated), cfg)
    from dmdqn_amd import checkpoint as CK
    if resume:
        CK.load(resume, tr)
    out = open(metrics, "w") if metrics else None
    smooth_global, smooth_total = SmoothedValue(alpha=0.3), SmoothedValue(alpha=0.3)
    t0 = time.perf_counter()
    steps = 0
    while tr.episode < episodes:
        log = out is not None and steps % log_every == 0
        if log:  # global reward of the PRE-step state (train.py:241, A-3)
            glob = -tr.env.local[..., :12].sum(dim=(1, 2), dtype=torch.float64)
        st = tr.step(collect_stats=log)
        steps += 1
        if log:
            total = tr.last_reward.sum(dim=1)                  # train.py:255 per replica
            g, tt = float(glob.mean()), float(total.mean())
            smooth_global.update(g)
            smooth_total.update(tt)
            rec = {"episode": tr.episode, "step": steps, "global_reward": g, "total_reward": tt,
                   "smooth_global_reward": smooth_global.get_value(),
                   "smooth_total_reward": smooth_total.get_value()}
            if st.loss_launched:
                rec.update(tr.agent.learn_metrics())
            out.write(json.dumps(rec) + "\n")
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    print(json.dumps({"agent_env_steps": steps * tr.env.E * tr.env.A, "seconds": round(el, 3),
                      "agent_env_steps_per_s": round(steps * tr.env.E * tr.env.A / el, 1)}))
    if out:
        out.close()
    if save_dir:
        os.makedirs(save_dir, exist_ok=True)
        CK.save(os.path.join(save_dir, "checkpoint.pt"), tr)
        CK.export_keras_weights(tr.agent, save_dir, tr.env.grid.junction_ids, env_index=0)
    return tr


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--episodes", type=int, default=EPISODES)
    ap.add_argument("--grid", default="3x3")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--batched", action="store_true")
    ap.add_argument("--envs", type=int, default=1024)
    ap.add_argument("--precision", default="fp16", choices=["fp32", "fp16", "bf16"])
    ap.add_argument("--metrics", default=None, help="offline JSONL metrics (replaces wandb)")
    ap.add_argument("--scenario", default=None,
                    help="SUMO scenario: a .sumocfg or a .npz from sumo_scenario (default for the "
                         "single-env path: the reference's grid_3x3 + grid_3x3_p06 routes, as "
                         "train.py's SUMO_CONFIG); 'synthetic' = generated demand for --grid")
    ap.add_argument("--shared", action="store_true",
                    help="batched only: one network shared by all agents (C5)")
    ap.add_argument("--save_dir", default=None,
                    help="write agent_<id>.weights.npz (and, batched, checkpoint.pt) at the end")
    ap.add_argument("--resume", default=None, help="batched only: a checkpoint.pt to resume from")
    ap.add_argument("--log_every", type=int, default=20, help="batched metrics interval (steps)")
    ap.add_argument("--loss", default="mse", choices=["mse", "huber"],
                    help="batched only: mse (dqn_agent.py:352) or huber (experimental/agent.py:99)")
    ap.add_argument("--actuated", action="store_true",
                    help="batched only: SUMO's actuated gap-out on phase 0 (default fixed durations)")
    args = ap.parse_args()
    logging.basicConfig(level=logging.INFO)
    rows, cols = (int(x) for x in args.grid.split("x"))
    scenario = args.scenario
    if scenario is None and not args.batched:
        scenario = DEFAULT_SCENARIO
    if scenario == "synthetic":
        scenario = None
    if args.batched:
        train_batched(args.episodes, rows, cols, args.envs, args.precision, args.seed, args.metrics,
                      scenario, args.shared, args.save_dir, args.resume, args.log_every, args.loss,
                      args.actuated)
    else:
        train_agents(args.episodes, rows, cols, args.seed, args.metrics, scenario, args.save_dir)


if __name__ == "__main__":
    main()
