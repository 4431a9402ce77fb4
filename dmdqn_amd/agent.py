"""Batched Double-DQN agents on the GPU (replaces src/agents/dqn_agent.py).

`BatchedDQN` holds NA = E*A independent agents (one per junction per env
replica): online / target Q-networks, Keras-3 Adam slots, replay rings and the
per-env random streams, all resident in HBM.  One call of each method acts,
stores or learns for every agent:

  act(obs)                         DQNAgent.select_action  (dqn_agent.py:246-274)
  remember(s, a, r, s', done)      DQNAgent.remember       (:312-326)
  replay()                         DQNAgent.replay / learn (:328-380, :428-434)
  update_target_network()          (:382-387)

Draw-order contract (bit-exact with the reference when E = 1 and the global
streams are seeded with random.seed(s) / np.random.seed(s)): per env, agents
in junction order draw from that env's numpy stream for act and from its
CPython `random` stream for replay sampling.
"""
import ctypes as C
from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np
import torch

from . import _lib
from . import kernels as K
from .ops import load as _ops

D_IN = 89
N_ACTIONS = 4


class CLearn(C.Structure):
    _fields_ = [(n, C.c_int32) for n in ["NA", "cap", "start", "batch", "hidden", "precision",
                                         "sync_target", "P"]] + [
        (n, C.c_void_p) for n in ["ring_s", "ring_n", "ring_a", "ring_d", "ring_r", "idx",
                                  "params", "adam_m", "adam_v", "target", "target_h",
                                  "loss"]] + [
        (n, C.c_float) for n in ["gamma", "alpha", "c1", "c2", "eps"]] + [
        ("stamps", C.c_void_p), ("qstats", C.c_void_p), ("params_h", C.c_void_p),
        ("loss_kind", C.c_int32), ("rn_out", C.c_void_p), ("row_format", C.c_int32),
        ("xs", C.c_void_p), ("xn", C.c_void_p)]


# ctypes signatures of the learn entry points: the C-ABI tests call them
# directly (c_learn_args); the product path goes through torch.ops.dmdqn
_lib.register({
    "dmdqn_learn": [C.POINTER(CLearn), C.c_void_p],
    "dmdqn_learn_grad": [C.POINTER(CLearn), C.c_void_p, C.c_void_p],
    "dmdqn_adam_agents": [C.POINTER(CLearn), C.c_void_p, C.c_void_p],
    "dmdqn_q_argmax": [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p,
                       C.c_void_p, C.c_void_p],
    "dmdqn_q_argmax_shared": [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p,
                              C.c_void_p, C.c_void_p, C.c_void_p],
    "dmdqn_learn_shared_grad": [C.POINTER(CLearn), C.c_void_p, C.c_int, C.c_void_p, C.c_float,
                                C.c_void_p, C.c_void_p],
    "dmdqn_adam": [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                   C.c_void_p, C.c_int, C.c_float, C.c_float, C.c_float, C.c_float, C.c_float,
                   C.c_int, C.c_void_p],
    "dmdqn_adam_slabs": [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                         C.c_void_p, C.c_int, C.c_void_p, C.c_float, C.c_int, C.c_float, C.c_float,
                         C.c_float, C.c_float, C.c_float, C.c_int, C.c_void_p],
    "dmdqn_target_sync": [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int,
                          C.c_void_p],
})

PRECISIONS = {"fp32": 0, "fp16": 1, "bf16": 2}
# include/dmdqn.h DMDQN_LOSS_*: the reference's MSE (dqn_agent.py:352) and the
# Huber loss of src/experimental/agent.py:99 (delta 1)
LOSSES = {"mse": 0, "huber": 1}
# dtype of the 16-bit operand copies (target shadow, shared online copy)
H16_DTYPES = {"fp16": torch.float16, "bf16": torch.bfloat16}


D_PAD = 96  # feature stride of an observation row in the replay ring (qnet_layout.hpp)
D_TILED = 88  # layer-1 features held in 16x16 tiles; feature 88 is a separate column


def n_params_keras(hidden, n_actions=N_ACTIONS):
    """Parameters of the reference Keras model (dqn_agent.py:153-184)."""
    H = hidden
    return D_IN * H + H + H * H + H + H * n_actions + n_actions


def n_params(hidden, n_actions=N_ACTIONS):
    """Floats per agent in the device layout (qnet_layout.hpp):
    W1T[H][0..87] | W1T[H][88] | W2T[H][H] | W3T[4][H] | b1[H] | b2[H] | b3[4]
    -- the Keras parameter count, no padding."""
    H = hidden
    return H * D_IN + H * H + n_actions * H + 2 * H + n_actions


def tile_wt(WT):
    """[..., N, K] row-major W^T -> [..., N*K] tiled device order (qnet_layout.hpp
    qn_wt): 16 x 16 tiles in row-major tile order, each [K%16 / 8][N%16][K%8]."""
    lead, (N, K) = WT.shape[:-2], WT.shape[-2:]
    t = WT.reshape(lead + (N // 16, 16, K // 16, 2, 8))
    n = len(lead)
    t = np.moveaxis(t, [n + 0, n + 2, n + 3, n + 1, n + 4], list(range(n, n + 5)))
    return t.reshape(lead + (N * K,))


def untile_wt(flat, N, K):
    """Inverse of tile_wt: [..., N*K] tiled -> [..., N, K] row-major."""
    lead = flat.shape[:-1]
    n = len(lead)
    t = flat.reshape(lead + (N // 16, K // 16, 2, 16, 8))
    t = np.moveaxis(t, list(range(n, n + 5)), [n + 0, n + 2, n + 3, n + 1, n + 4])
    return t.reshape(lead + (N, K))


def tile_w1(W1T):
    """[..., H, 89] row-major W1^T -> [..., 89*H] device order (qnet_layout.hpp
    qn_w1): per 16 neurons the tiles of features 0..79 and the first half
    (80..87) of the next, then the column of feature 88."""
    lead, H = W1T.shape[:-2], W1T.shape[-2]
    pad = np.zeros(lead + (H, D_PAD), np.float32)
    pad[..., :D_IN] = W1T
    t = tile_wt(pad).reshape(lead + (H // 16, 6, 2, 16, 8))
    blk = np.concatenate([t[..., :5, :, :, :].reshape(lead + (H // 16, 1280)),
                          t[..., 5, 0, :, :].reshape(lead + (H // 16, 128))], axis=-1)
    return np.concatenate([blk.reshape(lead + (H * D_TILED,)), W1T[..., D_TILED]], axis=-1)


def untile_w1(flat, H):
    """Inverse of tile_w1: [..., 89*H] -> [..., H, 89]."""
    lead = flat.shape[:-1]
    blk = flat[..., :H * D_TILED].reshape(lead + (H // 16, D_TILED * 16))
    t = np.zeros(lead + (H // 16, 6, 2, 16, 8), np.float32)
    t[..., :5, :, :, :] = blk[..., :1280].reshape(lead + (H // 16, 5, 2, 16, 8))
    t[..., 5, 0, :, :] = blk[..., 1280:].reshape(lead + (H // 16, 16, 8))
    W1T = untile_wt(t.reshape(lead + (H * D_PAD,)), H, D_PAD)[..., :D_IN].copy()
    W1T[..., D_TILED] = flat[..., H * D_TILED:H * D_IN]
    return W1T


def keras_to_kernel(flat, hidden):
    """[..., P_keras] Keras get_weights order -> [..., P_kernel] device layout."""
    H = hidden
    flat = np.asarray(flat, dtype=np.float32)
    lead = flat.shape[:-1]
    o = 0
    W1 = flat[..., o:o + D_IN * H].reshape(lead + (D_IN, H)); o += D_IN * H
    b1 = flat[..., o:o + H]; o += H
    W2 = flat[..., o:o + H * H].reshape(lead + (H, H)); o += H * H
    b2 = flat[..., o:o + H]; o += H
    W3 = flat[..., o:o + H * N_ACTIONS].reshape(lead + (H, N_ACTIONS)); o += H * N_ACTIONS
    b3 = flat[..., o:o + N_ACTIONS]
    parts = [tile_w1(np.swapaxes(W1, -1, -2)), tile_wt(np.swapaxes(W2, -1, -2)),
             np.swapaxes(W3, -1, -2).reshape(lead + (-1,)), b1, b2, b3]
    return np.concatenate(parts, axis=-1)


def kernel_to_keras(flat, hidden):
    """Inverse of keras_to_kernel."""
    H = hidden
    flat = np.asarray(flat, dtype=np.float32)
    lead = flat.shape[:-1]
    o = 0
    W1T = untile_w1(flat[..., o:o + H * D_IN], H); o += H * D_IN
    W2T = untile_wt(flat[..., o:o + H * H], H, H); o += H * H
    W3T = flat[..., o:o + N_ACTIONS * H].reshape(lead + (N_ACTIONS, H)); o += N_ACTIONS * H
    b1 = flat[..., o:o + H]; o += H
    b2 = flat[..., o:o + H]; o += H
    b3 = flat[..., o:o + N_ACTIONS]
    parts = [np.swapaxes(W1T, -1, -2).reshape(lead + (-1,)), b1,
             np.swapaxes(W2T, -1, -2).reshape(lead + (-1,)), b2,
             np.swapaxes(W3T, -1, -2).reshape(lead + (-1,)), b3]
    return np.concatenate(parts, axis=-1)


def keras_adam_consts(t, lr, b1=0.9, b2=0.999, eps=1e-7):
    """keras/src/optimizers/adam.py update_step constants for local step t (f32 ops)."""
    f = np.float32
    b1p = np.power(f(b1), f(t), dtype=np.float32)
    b2p = np.power(f(b2), f(t), dtype=np.float32)
    alpha = f(f(lr) * np.sqrt(f(1) - b2p, dtype=np.float32)) / f(f(1) - b1p)
    return float(alpha), float(f(1 - b1)), float(f(1 - b2)), float(f(eps))


def keras_initial_weights(rng, hidden, n_agents):
    """HeNormal (truncated at 2 sigma, stddev sqrt(2/fan_in)/0.8796) for the ReLU
    layers, GlorotUniform for the output layer, zero biases (dqn_agent.py:160-181).
    TF's RNG stream is not reproducible here, so initial weights are an input."""
    H = hidden

    def he(fi, fo):
        std = np.sqrt(2.0 / fi) / 0.87962566103423978
        w = rng.normal(0, std, size=(n_agents, fi, fo))
        bad = np.abs(w) > 2 * std
        while bad.any():
            w[bad] = rng.normal(0, std, size=int(bad.sum()))
            bad = np.abs(w) > 2 * std
        return w.reshape(n_agents, -1)

    lim = np.sqrt(6.0 / (H + N_ACTIONS))
    parts = [he(D_IN, H), np.zeros((n_agents, H)), he(H, H), np.zeros((n_agents, H)),
             rng.uniform(-lim, lim, size=(n_agents, H * N_ACTIONS)), np.zeros((n_agents, N_ACTIONS))]
    return np.concatenate(parts, axis=1).astype(np.float32)


def initial_weights(seed, env_seeds, n_agents, hidden, shared=False):
    """Initial weights [NW, P_keras] for the agents of the replicas whose env
    seeds are `env_seeds` (n_agents per replica).  Each replica's agents draw
    from their own generator, keyed on (seed, env seed), so a rank that owns
    replicas [r*E, (r+1)*E) builds exactly the weights those replicas get in a
    single-process run (shards are independent).  The shared net
    (C5) draws from `seed` alone, identical on every rank."""
    if shared:
        return keras_initial_weights(np.random.RandomState(seed & 0xFFFFFFFF), hidden, 1)
    return np.concatenate([
        keras_initial_weights(np.random.RandomState([seed & 0xFFFFFFFF, int(s) & 0xFFFFFFFF,
                                                     0x5EED]), hidden, n_agents)
        for s in env_seeds])


@dataclass
class AgentConfig:
    """Keys of config/agent_config.yaml; defaults are the values train.py uses
    (train.py:110-121), not the YAML file's (A-17)."""
    learning_rate: float = 0.001
    gamma: float = 0.99
    epsilon_start: float = 1.0
    epsilon_min: float = 0.01
    epsilon_decay_steps: int = 200000
    replay_buffer_size: int = 10000
    batch_size: int = 128
    target_update_frequency: int = 500
    nn_layers: List[int] = field(default_factory=lambda: [128, 128])
    # build-only knobs (additive)
    precision: str = "fp32"          # "fp32" | "fp16" (mixed, the reference's policy) | "bf16"
    loss: str = "mse"                # "mse" (dqn_agent.py:352) | "huber" (experimental/agent.py:99)
    count_env_steps: bool = False    # True fixes A-1 (epsilon decays); False = reference
    seed: int = 0
    # C5 (not in the reference): ONE network shared by every agent,
    # trained on the mean of the per-agent losses; gradients all-reduced over
    # RCCL across ranks.  Requires precision "fp16" and nn_layers [128, 128].
    shared_params: bool = False
    # replay row storage: "int8" (batched path, exact for this env, others
    # raise) | "f32" (any observation value, as dqn_agent.py:39-56 stores it;
    # the per-agent drop-in DQNAgent uses it)
    replay_rows: str = "int8"
    # physical ring slots beyond replay_buffer_size (kernels.ReplayRing): with
    # s spare slots the trainer's "env" schedule lets its side stream run up to
    # s env steps ahead of the learn, which marks every s-th learn for it
    ring_spare: int = 16

    @classmethod
    def from_dict(cls, d):
        known = {k: v for k, v in d.items() if k in cls.__dataclass_fields__}
        return cls(**known)


class BatchedDQN:
    """E*A independent DQN agents (agent index = env * A + junction)."""

    # rotating per-step output buffers (loss, qstats, actions, idx; see
    # __init__): at least 3, and ring_spare + 2 -- under trainer overlap "env"
    # the side stream runs up to ring_spare steps ahead of the learn stream, so
    # it writes the buffers of step t + ring_spare + 1 while the learn of step
    # t and then the caller's reads of step t's outputs may still be queued
    OUT_BUFS = 3

    def __init__(self, num_envs, n_agents, cfg: AgentConfig = None, device="cuda",
                 env_seeds=None, init_weights=None, streams=None):
        self.cfg = cfg = cfg or AgentConfig()
        self._ops = _ops()
        H = cfg.nn_layers[0]
        if len(cfg.nn_layers) != 2 or cfg.nn_layers[1] != H or H not in (64, 128):
            raise ValueError("the fused learn kernel supports nn_layers [64,64] or [128,128]")
        if cfg.batch_size != 128:
            raise ValueError("the fused learn kernel is built for batch_size 128")
        if cfg.precision not in PRECISIONS:
            raise ValueError(f"precision must be one of {list(PRECISIONS)}")
        if cfg.loss not in LOSSES:
            raise ValueError(f"loss must be one of {list(LOSSES)}")
        if cfg.shared_params and (cfg.precision != "fp16" or H != 128):
            raise ValueError("shared_params needs precision 'fp16' and nn_layers [128, 128]")
        self.device = dev = torch.device(device)
        self.E, self.A = num_envs, n_agents
        self.NA = NA = num_envs * n_agents
        self.shared = cfg.shared_params
        self.NW = NW = 1 if self.shared else NA   # parameter sets
        self.H, self.P = H, n_params(H)
        seeds = (np.arange(num_envs, dtype=np.int64) + cfg.seed if env_seeds is None
                 else np.asarray(env_seeds))
        if init_weights is None:
            init_weights = initial_weights(cfg.seed, seeds, n_agents, H, self.shared)
        init = np.asarray(init_weights, dtype=np.float32).reshape(NW, -1)
        if init.shape[1] == n_params_keras(H):
            init = keras_to_kernel(init, H)
        w = torch.as_tensor(init.reshape(NW, self.P))
        self.params = w.to(dev).contiguous()
        self.target = self.params.clone()
        # fp16 / bf16 paths: the target forward reads a 16-bit copy (padded row
        # stride Ph) in the MFMA operand type
        self.Ph = (self.P + 7) // 8 * 8
        self.target_h = self.params_h = None
        h16 = H16_DTYPES.get(cfg.precision)
        if h16 is not None:
            # f16 copies the forwards read (Keras casts the f32 variables to f16);
            # the online copy only for the shared net, whose Adam is a separate
            # pass (fused into the per-agent learn, the extra stores cost more
            # than the halved fragment reads save)
            self.target_h = torch.zeros((NW, self.Ph), dtype=h16, device=dev)
            self._refresh_target_h()
            if self.shared:
                self.params_h = torch.zeros((NW, self.Ph), dtype=h16, device=dev)
                self._refresh_params_h()
        if self.shared:
            # one partial gradient per persistent workgroup (one per CU)
            n_cu = torch.cuda.get_device_properties(dev).multi_processor_count
            self.n_slabs = max(1, min(NA, n_cu))
            self.slab = torch.empty((self.n_slabs, self.P), dtype=torch.float32, device=dev)
            self.grad = torch.zeros(self.P, dtype=torch.float32, device=dev)
            # each batch row's TD target + action between the shared learn's two passes
            self.shared_work = torch.empty(NA * cfg.batch_size * 5, dtype=torch.uint8, device=dev)
        self.adam_m = torch.zeros_like(self.params)
        self.adam_v = torch.zeros_like(self.params)
        if cfg.replay_rows not in ("int8", "f32"):
            raise ValueError("replay_rows must be 'int8' or 'f32'")
        if self.shared and cfg.replay_rows != "int8":
            raise ValueError("the shared-network learn reads int8 replay rows only")
        self.ring = K.ReplayRing(NA, cfg.replay_buffer_size, device=dev, row_format=cfg.replay_rows,
                                 spare=cfg.ring_spare)
        self.OUT_BUFS = max(BatchedDQN.OUT_BUFS, self.ring.spare + 2)
        self._xs = self._xn = None  # float rows: the learn's pre-gathered batch
        if streams is not None:
            # shared (np_state, py_state) device streams, e.g. the process-global
            # ones behind the per-agent DQNAgent surface
            self.np_state, self.py_state = streams
        else:
            self.np_state = K.seed_streams(seeds, "np", dev)
            self.py_state = K.seed_streams(seeds, "py", dev)
        # rotating index buffers: presample() may draw the next learn's batch
        # (on another stream) while the current learn still reads its own, and
        # a caller's read of step t's indices on its stream (queued behind
        # learn t) must not meet the draws of step t+2 (the side stream of
        # trainer overlap "env" waits only for learn t): OUT_BUFS of them
        self._idx_bufs = [torch.empty((NA, cfg.batch_size), dtype=torch.int32, device=dev)
                          for _ in range(self.OUT_BUFS)]
        self._idx_i = 0
        self.idx = self._idx_bufs[0]
        self._presampled = None  # (n, buffer) drawn ahead by presample()
        # per-learn outputs rotate over OUT_BUFS buffers (learn k writes buffer
        # k % OUT_BUFS): under trainer overlap "env" with side_learn, the side
        # stream's learn of step t+1 may run before the caller's main-stream
        # read of step t's loss / stats, and the side stream is ordered only
        # after learn t-1 -- so learn t+1 and t+2 must write other buffers
        # than the one step t's reader holds
        self._loss_bufs = [torch.zeros(NA, dtype=torch.float32, device=dev)
                           for _ in range(self.OUT_BUFS)]
        self._qstats_bufs = [torch.zeros((NA, 6), dtype=torch.float32, device=dev)
                             for _ in range(self.OUT_BUFS)]
        self.loss, self.qstats = self._loss_bufs[0], self._qstats_bufs[0]
        # rotating action buffers: a caller may still read step t's actions on
        # its stream while the trainer's side stream writes steps t+1 and t+2
        # (overlap "env": the side stream waits only for learn t, before which
        # the caller's read of step t is queued) -- OUT_BUFS of them
        self._act_bufs = [torch.empty((num_envs, n_agents), dtype=torch.int32, device=dev)
                          for _ in range(self.OUT_BUFS)]
        self._act_i = 0
        self.actions = self._act_bufs[0]
        self.greedy = torch.empty((num_envs, n_agents), dtype=torch.int32, device=dev)
        self._done_flags = [torch.full((NA,), v, dtype=torch.uint8, device=dev) for v in (0, 1)]
        self.global_step_count = 0
        self.learn_step_counter = 0
        self.epsilon = cfg.epsilon_start
        self.learn_launches = 0
        self.learn_hook = None  # optional callable(before: bool), e.g. HIP event timing
        self.stamps = None      # optional int64 [NA, 16] device tensor: phase timestamps
        self.rn_out = None      # optional f32 [NA, batch] device tensor: the z-scored rewards
        self._split_grad = None  # [NA, P] f32 scratch of the split learn (set_split_learn)
        # the shared net's learns by launch sequence (tests assert which ran):
        # "adam_slabs" = one rank's fused slab reduction + Adam; "allreduce" =
        # k_reduce_slabs -> all-reduce over ranks -> k_adam(gscale = 1/world)
        self.shared_paths = {"adam_slabs": 0, "allreduce": 0}

    def set_split_learn(self, on=True):
        """Run each independent-agent learn as two launches (dmdqn_learn_grad,
        dmdqn_adam_agents): bit-identical to the fused kernel, 4 more bytes of
        HBM traffic per parameter each way, but its bandwidth-bound Adam half
        can share the chip with the next step's act / sim / observe (trainer
        overlap "full"), which the fused kernel's LDS-heavy workgroups leave no
        room for.  fp16 / bf16, independent networks only."""
        if on:
            if self.shared or self.cfg.precision not in H16_DTYPES or self.ring.row_format != "int8":
                raise ValueError("the split learn is for independent fp16 / bf16 networks "
                                 "on int8 replay rows")
            if self._split_grad is None:
                self._split_grad = torch.empty((self.NA, self.P), dtype=torch.float32,
                                               device=self.device)
        else:
            self._split_grad = None

    @property
    def split_learn(self):
        return self._split_grad is not None

    # -------------------------------------------------------------- act
    def current_epsilon(self):
        """dqn_agent.py:258-261 (global_step_count never moves on the reference
        training path, so epsilon stays 1.0 -- A-1)."""
        g = self.global_step_count
        if g < 8000:
            self.epsilon = 1.0
        elif self.epsilon > self.cfg.epsilon_min:
            self.epsilon = max(0.01, 1.0 * float(np.exp(-(g - 8000) / 16000)))
        return self.epsilon

    def act(self, obs, eps=None):
        """obs f32 [E, A, 89] -> actions int32 [E, A] (device).  eps overrides the
        schedule (evaluation, test.py:84-87)."""
        eps, greedy, out = self.act_inputs(obs, eps)
        return K.act(self.np_state, self.A, eps=eps, n_actions=N_ACTIONS, greedy=greedy, out=out)

    def act_inputs(self, obs, eps=None):
        """What a fused env step (TrafficEnv.step_fused) needs to draw act()'s
        actions itself: (eps, greedy or None, the actions buffer to fill).
        The greedy forward (eps < 1) is launched here, as act() does."""
        eps = self.current_epsilon() if eps is None else float(eps)
        greedy = None
        if eps < 1.0:
            self._ops.q_argmax(self.params, self.H, PRECISIONS[self.cfg.precision],
                               obs.reshape(self.NA, D_IN).contiguous(), self.greedy, None,
                               self.shared)
            greedy = self.greedy
        self._act_i = (self._act_i + 1) % self.OUT_BUFS
        self.actions = self._act_bufs[self._act_i]
        return eps, greedy, self.actions

    def remembered(self):
        """The bookkeeping of remember() after a fused env step stored the
        transition into ring slot ring.next_slot."""
        self.ring.advance()
        self.ring.poll()
        if self.cfg.count_env_steps:
            self.global_step_count += 1

    # -------------------------------------------------------------- replay
    def remember(self, obs, actions, rewards, next_obs, done):
        """One transition per agent (ReplayBuffer.add).  obs/next_obs [E,A,89] f32,
        actions [E,A] int32, rewards [E,A] f64, done: bool or uint8 [E]."""
        NA = self.NA
        if isinstance(done, (bool, np.bool_, int)):
            d = self._done_flags[int(bool(done))]  # constant [NA] u8 (no per-step fill)
        else:
            d = done.to(torch.uint8).reshape(self.E, 1).expand(self.E, self.A).reshape(NA).contiguous()
        self.ring.store(obs.reshape(NA, D_IN), next_obs.reshape(NA, D_IN),
                        actions.reshape(NA), rewards.reshape(NA), d)
        self.ring.poll()  # raises (one store late, no stall) on a non-int8 observation
        if self.cfg.count_env_steps:
            self.global_step_count += 1

    def replay(self):
        """DQNAgent.replay for every agent: returns the loss tensor [NA] (device),
        or None while the buffers hold fewer than batch_size transitions."""
        return self.learn()

    def learn(self, collect_stats=False):
        """One fused learn for every agent (None while underfilled).  With
        collect_stats, self.qstats [NA, 6] receives the batch metrics of
        dqn_agent.py:361-363 (see learn_metrics)."""
        if not self.learn_begin(collect_stats):
            return None
        return self.learn_range(0, self.NA)

    def learn_begin(self, collect_stats=False):
        """The host half of learn(): the replay draws (or the presampled ones),
        the learn counter and the Keras Adam constants of this learn.  False
        while underfilled.  The launches follow with learn_range(lo, hi) over
        agent ranges that cover [0, NA) -- independent agents, so ranges may
        run on different streams (trainer overlap "env" with side_learn)."""
        n = len(self.ring)
        if n < self.cfg.batch_size:
            return False
        cfg = self.cfg
        if self._presampled is not None:
            pn, buf = self._presampled
            self._presampled = None
            if pn != n:
                raise RuntimeError(f"presample drew for n={pn}, the ring holds {n}")
            self.idx = buf
        else:
            K.replay_sample(self.py_state, self.A, n, cfg.batch_size, out=self.idx)
        self.learn_step_counter += 1
        alpha, c1, c2, eps = keras_adam_consts(self.learn_step_counter, cfg.learning_rate)
        sync = self.learn_step_counter % cfg.target_update_frequency == 0
        k = self.learn_step_counter % self.OUT_BUFS
        self.loss = self._loss_bufs[k]
        qstats = None
        if collect_stats:
            # zeroed per agent range by learn_range, on the stream that launches
            # the range (the side stream's part must not wait on main)
            self.qstats = qstats = self._qstats_bufs[k]
        self._last_learn = (alpha, c1, c2, eps, sync, qstats)
        self.learn_launches += 1
        return True

    def learn_range(self, lo, hi):
        """Launch the learn begun by learn_begin() for agents [lo, hi) on the
        current stream (the whole range for the shared net).  The timing hook
        brackets the range that starts at agent 0.  Returns self.loss."""
        alpha, c1, c2, eps, sync, qstats = self._last_learn
        cfg, ring = self.cfg, self.ring
        hook = self.learn_hook if lo == 0 else None
        if qstats is not None:
            qstats[lo:hi].zero_()  # the kernels accumulate into it
        if hook:
            hook(True)
        if self.shared:
            if (lo, hi) != (0, self.NA):
                raise ValueError("the shared-net learn runs over every agent at once")
            self._learn_shared(alpha, c1, c2, eps, sync, qstats)
        else:
            xs = xn = None
            if ring.row_format == "f32":  # float rows: the batch gathered in order first
                if (lo, hi) != (0, self.NA):
                    raise ValueError("float-row learns run over every agent at once")
                if self._xs is None:
                    shape = (self.NA, cfg.batch_size, K.ROW_FLOATS)
                    self._xs = torch.empty(shape, dtype=torch.float32, device=self.device)
                    self._xn = torch.empty(shape, dtype=torch.float32, device=self.device)
                ring.gather_f32(self.idx, self._xs, self._xn)
                xs, xn = self._xs, self._xn

            def sl(t):
                return None if t is None else t[lo:hi]
            self._ops.learn_step(sl(ring.s), sl(ring.n), sl(ring.a), sl(ring.d), sl(ring.r),
                                 sl(self.idx), sl(self.params), sl(self.adam_m), sl(self.adam_v),
                                 sl(self.target), sl(self.target_h), sl(self.loss), ring.start,
                                 self.H, PRECISIONS[cfg.precision], sync, cfg.gamma, alpha, c1, c2,
                                 eps, LOSSES[cfg.loss], sl(qstats), sl(self.rn_out),
                                 sl(self.stamps), grad=sl(self._split_grad), xs=xs, xn=xn)
        if hook:
            hook(False)
        return self.loss

    def c_learn_args(self):
        """The dmdqn_learn_args struct of the last learn (ctypes), for tests that
        call the C ABI directly; the tensors it points at belong to self."""
        alpha, c1, c2, eps, sync, qstats = self._last_learn
        cfg = self.cfg
        return CLearn(self.NA, self.ring.slots, self.ring.start, cfg.batch_size, self.H,
                      PRECISIONS[cfg.precision], int(sync), self.P,
                      *[None if t is None else t.data_ptr()
                        for t in [self.ring.s, self.ring.n, self.ring.a, self.ring.d, self.ring.r,
                                  self.idx, self.params, self.adam_m, self.adam_v, self.target,
                                  self.target_h, self.loss]],
                      np.float32(cfg.gamma), alpha, c1, c2, eps,
                      None if self.stamps is None else self.stamps.data_ptr(),
                      None if qstats is None else qstats.data_ptr(),
                      None if self.params_h is None else self.params_h.data_ptr(),
                      LOSSES[cfg.loss], None if self.rn_out is None else self.rn_out.data_ptr(),
                      int(self.ring.row_format == "f32"),
                      None if self._xs is None else self._xs.data_ptr(),
                      None if self._xn is None else self._xn.data_ptr())

    def presample(self, n, lds_budget=0):
        """Draw the next learn's replay indices now (ReplayBuffer.sample,
        dqn_agent.py:59-63) for a ring of n transitions, into the index buffer
        the current learn does not read, on the current stream.  The draws
        depend only on the CPython stream and n, never on the ring contents, so
        they may run before the store that brings the ring to n (trainer
        overlap).  The next learn() must see len(ring) == n.  lds_budget:
        kernels.replay_sample's (the sampler beside the shared learn)."""
        if n < self.cfg.batch_size:
            return False
        if self._presampled is not None:
            raise RuntimeError("presample called twice before a learn")
        self._idx_i = (self._idx_i + 1) % self.OUT_BUFS
        buf = self._idx_bufs[self._idx_i]
        K.replay_sample(self.py_state, self.A, n, self.cfg.batch_size, out=buf,
                        lds_budget=lds_budget)
        self._presampled = (n, buf)
        return True

    def learn_metrics(self):
        """The scalars dqn_agent.py:361-370 logs, from the last learn(collect_stats=True):
        mean over agents of q_values_mean / q_values_std (population std over
        each batch's 128x4 online Q values), the action histogram summed over
        agents, mean loss and epsilon.  Syncs."""
        qs = self.qstats.double()
        n = float(self.cfg.batch_size * N_ACTIONS)
        mean = qs[:, 0] / n
        std = (qs[:, 1] / n - mean * mean).clamp_min(0).sqrt()
        return {"loss": float(self.loss.double().mean()), "epsilon": float(self.epsilon),
                "q_values_mean": float(mean.mean()), "q_values_std": float(std.mean()),
                "action_distribution": qs[:, 2:6].sum(0).round().long().tolist()}

    def _learn_shared(self, alpha, c1, c2, eps, sync, qstats):
        """C5: grad = mean over this rank's agents of the per-agent gradients,
        all-reduced (sum, RCCL) across ranks, then one Adam step with 1/world."""
        import torch.distributed as dist
        ring, cfg = self.ring, self.cfg
        world = 1
        if dist.is_available() and dist.is_initialized():
            world = dist.get_world_size()
        # one rank: the slab reduction and the Adam step as one launch
        # (dmdqn_adam_slabs, the same bits); more ranks: reduce, all-reduce, Adam
        self._ops.learn_shared_grad(ring.s, ring.n, ring.a, ring.d, ring.r, self.idx, self.params,
                                    self.target, self.target_h, self.params_h, self.loss,
                                    ring.start, cfg.gamma, LOSSES[cfg.loss], qstats, self.rn_out,
                                    self.slab, self.grad if world > 1 else None, 1.0 / self.NA,
                                    work=self.shared_work)
        if world == 1:
            self.shared_paths["adam_slabs"] += 1
            self._ops.adam_slabs(self.params, self.adam_m, self.adam_v, self.target, self.target_h,
                                 self.params_h, self.slab, self.grad, 1.0 / self.NA, 1.0, alpha,
                                 c1, c2, eps, sync)
            return
        if world > 1:
            # one flat 114 KB buffer per learn, bounded (dist.BoundedAllReduce:
            # the host runs a few learns ahead; a stalled peer raises DistError)
            from . import dist as D
            if getattr(self, "_allreduce", None) is None:
                self._allreduce = D.BoundedAllReduce()
            if dist.get_backend() == "gloo" and self.grad.is_cuda:
                # gloo (several ranks on one device: the multi-process tests) reduces host memory
                g = self.grad.cpu()
                self._allreduce(g)
                self.grad.copy_(g)
            else:
                self._allreduce(self.grad)
            self.shared_paths["allreduce"] += 1
        self._ops.adam(self.params, self.adam_m, self.adam_v, self.target, self.target_h,
                       self.params_h, self.grad, 1.0 / world, alpha, c1, c2, eps, sync)

    def drain_collectives(self):
        """Wait (bounded, dist.BoundedAllReduce.drain) for the shared net's
        outstanding gradient all-reduces; a no-op without any."""
        ar = getattr(self, "_allreduce", None)
        if ar is not None:
            ar.drain()

    def _refresh_params_h(self):
        if self.params_h is not None:
            self.params_h[:, :self.P].copy_(self.params.to(self.params_h.dtype))

    def _refresh_target_h(self):
        if self.target_h is not None:
            self.target_h[:, :self.P].copy_(self.target.to(self.target_h.dtype))

    def update_target_network(self):
        """dqn_agent.py:382-387: target <- online, and the 16-bit shadow."""
        self._ops.target_sync(self.params, self.target, self.target_h,
                              PRECISIONS[self.cfg.precision])

    # -------------------------------------------------------------- weights
    def keras_params(self, which="params"):
        """[NA, P_keras] copy of params / target / adam_m / adam_v in Keras order."""
        return kernel_to_keras(getattr(self, which).cpu().numpy(), self.H)

    def get_weights(self, agent):
        """Keras get_weights() order for one agent: [W1, b1, W2, b2, W3, b3]."""
        p = kernel_to_keras(self.params[0 if self.shared else agent].cpu().numpy(), self.H)
        H = self.H
        shapes = [(D_IN, H), (H,), (H, H), (H,), (H, N_ACTIONS), (N_ACTIONS,)]
        out, o = [], 0
        for sh in shapes:
            n = int(np.prod(sh))
            out.append(p[o:o + n].reshape(sh).copy())
            o += n
        return out

    def set_weights(self, agent, weights):
        flat = np.concatenate([np.asarray(w, np.float32).reshape(-1) for w in weights])
        agent = 0 if self.shared else agent
        self.params[agent].copy_(torch.from_numpy(keras_to_kernel(flat, self.H)))
        self.target[agent].copy_(self.params[agent])
        self._refresh_params_h()
        self._refresh_target_h()

    def state_dict(self):
        return {"params": self.params.cpu(), "target": self.target.cpu(),
                "adam_m": self.adam_m.cpu(), "adam_v": self.adam_v.cpu(),
                "learn_step_counter": self.learn_step_counter,
                "global_step_count": self.global_step_count}

    def load_state_dict(self, sd):
        for k in ["params", "target", "adam_m", "adam_v"]:
            getattr(self, k).copy_(sd[k].to(self.device))
        self._refresh_params_h()
        self._refresh_target_h()
        self.learn_step_counter = int(sd["learn_step_counter"])
        self.global_step_count = int(sd["global_step_count"])
