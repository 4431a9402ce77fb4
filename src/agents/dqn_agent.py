"""src/agents/dqn_agent.py -- drop-in DQNAgent / ReplayBuffer on the GPU kernels.

Same constructor and methods as the reference module (src/agents/dqn_agent.py:
ReplayBuffer :27-89, DQNAgent :92-434), same draw order on the process-global
random streams:
  * select_action draws np.random.rand() then (if exploring) np.random.randint
    from the process-global numpy stream (:263-265);
  * replay/learn draws random.sample(buffer, batch) from the process-global
    CPython `random` stream (:63).
Both streams live on the device; seed them with `seed(s)` (the reference's
train.py never seeds -- A-2 -- so an explicit seed is needed for parity runs;
the equivalent reference call is random.seed(s); np.random.seed(s)).

Each DQNAgent is one agent slot run by the fused kernels (act, replay store,
replay sample, learn).  For many agents / many env replicas use
dmdqn_amd.agent.BatchedDQN, which runs all of them in one launch per stage.
"""
import json
import os
import zlib

import numpy as np
import torch

from dmdqn_amd import kernels as K
from dmdqn_amd.agent import AgentConfig, BatchedDQN

_STREAMS = {}


def seed(s, device="cuda"):
    """random.seed(s); np.random.seed(s) for the device-side global streams."""
    _STREAMS[str(device)] = (K.seed_streams([s], "np", device), K.seed_streams([s], "py", device))


def _streams(device):
    if str(device) not in _STREAMS:
        seed(0, device)
    return _STREAMS[str(device)]


def init_seed(seed, agent_id):
    """Initial-weight seed of agent `agent_id` (see DQNAgent.__init__)."""
    return (int(seed) ^ zlib.crc32(str(agent_id).encode())) & 0x7FFFFFFF


def _as_obs(x, device):
    t = torch.as_tensor(np.asarray(x, dtype=np.float32) if not torch.is_tensor(x) else x,
                        dtype=torch.float32)
    return t.reshape(1, 1, 89).to(device)


class ReplayBuffer:
    """Device replay ring of one agent (dqn_agent.py:27-89)."""

    def __init__(self, buffer_size: int, device="cuda"):
        self.device = torch.device(device)
        # float32 rows: any observation value is kept as the reference's
        # buffer keeps it (:39-56); the batched path uses int8 rows
        self.ring = K.ReplayRing(1, buffer_size, device=self.device, row_format="f32")

    def add(self, experience: tuple):
        state, action, reward, next_state, done = experience
        s, n = _as_obs(state, self.device), _as_obs(next_state, self.device)
        self.ring.store(s.reshape(1, 89), n.reshape(1, 89),
                        torch.tensor([int(action)], dtype=torch.int32, device=self.device),
                        torch.tensor([float(reward)], dtype=torch.float64, device=self.device),
                        torch.tensor([int(bool(done))], dtype=torch.uint8, device=self.device))

    def sample(self, batch_size: int):
        """(states, actions, z-scored rewards, next_states, dones) as device tensors,
        or None while fewer than batch_size transitions are stored (:61-62)."""
        n = len(self.ring)
        if n < batch_size:
            return None
        _, py = _streams(self.device)
        idx = K.replay_sample(py, 1, n, batch_size)[0].long()
        slots = self.ring.slots_of(idx)
        # the z-score in float64 numpy on the host, exactly the reference's
        # expression (:66-69: np.mean / np.std use numpy's pairwise summation),
        # so the rewards are bit-identical; the fused learn kernel restates the
        # same order on the device
        r = self.ring.r[0, slots].cpu().numpy()
        rn = ((r - np.mean(r)) / (np.std(r) + 1e-8)).astype(np.float32)
        return (self.ring.s[0, slots, :89].float(), self.ring.a[0, slots].int(),
                torch.from_numpy(rn).to(self.device), self.ring.n[0, slots, :89].float(),
                self.ring.d[0, slots].float())

    def __len__(self):
        return len(self.ring)


class DQNAgent:
    """Double-DQN agent for one intersection (dqn_agent.py:92-434)."""

    def __init__(self, state_size: int, action_size: int, agent_id: str, config: dict,
                 device="cuda"):
        self.agent_id = agent_id
        self.state_size = 89   # hard-coded as in the reference (A-16)
        self.action_size = 4
        cfg = AgentConfig.from_dict(config)
        cfg.nn_layers = list(config.get("nn_layers", [64, 64]))  # reference default :127
        cfg.target_update_frequency = config.get("target_update_frequency", 1000)  # :124-126
        cfg.epsilon_decay_steps = config.get("epsilon_decay_steps", 100000)
        self.learning_rate, self.gamma = cfg.learning_rate, cfg.gamma
        self.epsilon, self.epsilon_min = cfg.epsilon_start, cfg.epsilon_min
        self.batch_size = cfg.batch_size
        self.target_update_frequency = cfg.target_update_frequency
        self.device = torch.device(device)
        # Keras draws every model's initial weights from TF's global generator, so
        # agents start from different weights; here each agent's initial-weight
        # seed is cfg.seed mixed with a hash of its id (TF's stream itself cannot
        # be reproduced)
        cfg.seed = init_seed(cfg.seed, agent_id)
        # float32 replay rows (additive key "replay_rows": "int8" opts back into
        # the batched path's exact-integer rows)
        cfg.replay_rows = config.get("replay_rows", "f32")
        self._core = BatchedDQN(1, 1, cfg, device=self.device, streams=_streams(self.device))
        self.replay_buffer = ReplayBuffer.__new__(ReplayBuffer)
        self.replay_buffer.device, self.replay_buffer.ring = self.device, self._core.ring
        self.global_step_count = 0
        self.learn_step_counter = 0
        # the per-learn scalars the reference writes with tf.summary to
        # logs/<agent_id> (:151, :361-370): kept as last_summary; with the
        # additive config key "summary_dir", also appended as JSON lines to
        # <summary_dir>/<agent_id>/summaries.jsonl (no TensorBoard here)
        self.last_summary = None
        self._summary_path = None
        if config.get("summary_dir"):
            d = os.path.join(config["summary_dir"], str(agent_id))
            os.makedirs(d, exist_ok=True)
            self._summary_path = os.path.join(d, "summaries.jsonl")

    def select_action(self, state_tensor):
        """epsilon-greedy on the global numpy stream (:246-274)."""
        self._core.global_step_count = self.global_step_count
        obs = _as_obs(state_tensor, self.device)
        a = int(self._core.act(obs)[0, 0].item())
        self.epsilon = self._core.epsilon
        return a

    def store_experience(self, experience):
        self.replay_buffer.add(experience)
        self.global_step_count += 1  # :306-310 (the training path never calls it, A-1)

    def remember(self, state, action, reward, next_state, done):
        self.replay_buffer.add((state, action, reward, next_state, done))  # :312-326
        self.replay_buffer.ring.check()  # int8 rows (opt-in): a non-int8 value raises now

    def learn(self):
        """One fused learn step; None while the buffer is underfilled (:333-335)."""
        loss = self._core.learn(collect_stats=True)
        if loss is None:
            return None
        self.learn_step_counter = self._core.learn_step_counter
        m = self._core.learn_metrics()
        self.last_summary = {"step": self.learn_step_counter, "loss": float(loss[0].item()),
                             "epsilon": float(self.epsilon),
                             "q_values_mean": m["q_values_mean"], "q_values_std": m["q_values_std"],
                             "action_distribution": m["action_distribution"]}
        if self._summary_path:
            with open(self._summary_path, "a") as f:
                f.write(json.dumps(self.last_summary) + "\n")
        return self.last_summary["loss"]

    def replay(self) -> float:
        loss = self.learn()
        return 0 if loss is None else loss  # :428-434

    def update_target_network(self):
        self._core.update_target_network()

    def get_epsilon(self) -> float:
        return self.epsilon

    def save_model(self, filepath):
        """Online weights in Keras get_weights order (npz instead of .h5)."""
        np.savez(filepath, *self._core.get_weights(0))

    def load_model(self, filepath):
        try:
            with np.load(filepath) as f:
                self._core.set_weights(0, [f[k] for k in sorted(f.files, key=lambda x: int(x.split("_")[1]))])
            return True
        except Exception:
            return False
