"""Checkpoint / resume of the batched training loop.

The reference never checkpoints during training; its only persistence is
DQNAgent.save_model / load_model (dqn_agent.py:401-422), one Keras
``agent_<id>.weights.h5`` per junction, which src/scripts/test.py:195 loads.
This module keeps that naming for the exported weights and adds what a resume
needs, so that load + K steps reproduces an uninterrupted run bit-exactly
(every kernel on the path is deterministic):

  nets      params / target (+ its f16 / bf16 shadow) / Adam m, v, learn counters;
            the shared net's 16-bit online copy is rebuilt from params on load
  replay    the filled part of every ring + the host counter
  streams   both device MT19937 streams per env (numpy act stream, CPython
            sample stream)
  env       lane rings, signal state, origin-queue cursors, stats, the clock,
            the last local state / observation (reward uses the pre-step state)
  trainer   episode / step counters and the current observation

Everything is a tensor or a plain int / float / str, so the file loads with
torch.load(weights_only=True).  Demand tables are NOT stored: they are rebuilt
from the env config (seeds or scenario) and checked against the checkpoint.
"""
import dataclasses
import os

import numpy as np
import torch

FORMAT = "dmdqn-ckpt-4"  # 4: 128-B replay rows (s' rows carry a, done, r); unpadded W1T (qnet_layout.hpp)

_ENV_TENSORS = ["t_x", "t_v", "t_dst", "t_head", "t_cnt", "t_phase_state", "t_ts", "t_qptr",
                "t_stats", "halt", "phase", "tspent", "done_u8"]
_AGENT_TENSORS = ["params", "target", "adam_m", "adam_v", "np_state", "py_state"]


def _cfg_dict(cfg):
    d = dataclasses.asdict(cfg)
    return {k: (v if isinstance(v, (int, float, str, bool, type(None), list)) else str(v))
            for k, v in d.items()}


def trainer_state(tr, include_replay=True):
    """CPU copy of everything a resume needs (see module docstring)."""
    ag, env = tr.agent, tr.env
    st = {"format": FORMAT,
          "env_cfg": _cfg_dict(env.cfg), "agent_cfg": _cfg_dict(ag.cfg),
          "nveh": int(env.nveh),
          "counters": {"learn_step_counter": ag.learn_step_counter,
                       "global_step_count": ag.global_step_count,
                       "epsilon": float(ag.epsilon), "learn_launches": ag.learn_launches,
                       "env_t": env.t, "env_episode": env.episode, "episode": tr.episode,
                       "step_count": tr.step_count, "total_steps": tr.total_steps,
                       "ring_total": ag.ring.total}}
    st["agent"] = {k: getattr(ag, k).cpu() for k in _AGENT_TENSORS}
    if ag.target_h is not None:
        st["agent"]["target_h"] = ag.target_h.cpu()
    st["env"] = {k: getattr(env, k).cpu() for k in _ENV_TENSORS}
    st["env"]["local"] = env.local.cpu()
    st["obs"] = tr.obs.cpu()
    if include_replay:
        n = len(ag.ring)
        st["replay"] = {k: getattr(ag.ring, k)[:, :n].cpu() for k in ["s", "n", "a", "r", "d"]}
    return st


def save(path, tr, include_replay=True):
    torch.cuda.synchronize(tr.env.device)
    torch.save(trainer_state(tr, include_replay), path)


def load(path, tr):
    """Restore a checkpoint into a Trainer built with the same configs."""
    st = torch.load(path, map_location="cpu", weights_only=True)
    if st.get("format") != FORMAT:
        raise ValueError(f"{path}: not a {FORMAT} checkpoint")
    ag, env = tr.agent, tr.env
    if int(st["nveh"]) != int(env.nveh):
        raise ValueError("checkpoint demand does not match this env config (nveh differs)")
    for k, v in st["agent"].items():
        dst = getattr(ag, k)
        if tuple(dst.shape) != tuple(v.shape):
            raise ValueError(f"checkpoint agent.{k} shape {tuple(v.shape)} != {tuple(dst.shape)}")
        dst.copy_(v.to(ag.device))
    for k, v in st["env"].items():
        if k == "local":
            env.local = v.to(env.device)
            continue
        dst = getattr(env, k)
        if tuple(dst.shape) != tuple(v.shape):
            raise ValueError(f"checkpoint env.{k} shape {tuple(v.shape)} != {tuple(dst.shape)}")
        dst.copy_(v.to(env.device))
    c = st["counters"]
    ag.learn_step_counter, ag.global_step_count = c["learn_step_counter"], c["global_step_count"]
    ag.epsilon, ag.learn_launches = c["epsilon"], c["learn_launches"]
    env.t, env.episode = c["env_t"], c["env_episode"]
    tr.episode, tr.step_count, tr.total_steps = c["episode"], c["step_count"], c["total_steps"]
    ag.ring.total = c["ring_total"]
    ag._refresh_params_h()  # the f16 online copy is derived, not stored
    if "replay" in st:
        n = st["replay"]["s"].shape[1]
        for k, v in st["replay"].items():
            getattr(ag.ring, k)[:, :n].copy_(v.to(ag.device))
    tr.obs = st["obs"].to(env.device)
    # the observation the env hands back is a view of its own buffer
    env.obs = tr.obs
    tr.join_streams()  # the restore ran on the caller's stream
    return st


def export_keras_weights(agent, out_dir, junction_ids, env_index=0):
    """One file per junction in the reference's naming (agent_<id>.weights,
    dqn_agent.py:401-410 / test.py:195), as .npz (no HDF5 here): arrays
    arr_0..arr_5 = Keras get_weights() order W1, b1, W2, b2, W3, b3."""
    os.makedirs(out_dir, exist_ok=True)
    A = len(junction_ids)
    paths = []
    for a, jid in enumerate(junction_ids):
        w = agent.get_weights(env_index * A + a)
        p = os.path.join(out_dir, f"agent_{jid}.weights.npz")
        np.savez(p, *w)
        paths.append(p)
    return paths


def load_keras_weights(path):
    """[W1, b1, W2, b2, W3, b3] from an export_keras_weights file."""
    with np.load(path) as f:
        return [f[f"arr_{i}"] for i in range(6)]
