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

# 8: replay rings of cap + ring_spare slots (kernels.ReplayRing, default 16); 7: cap + 1 slots,
# the written slots saved;
# 6: + per-replica clocks and episode counters; 5: + the actuated-mode detector
# times; 4: 128-B replay rows, unpadded W1T
FORMAT = "dmdqn-ckpt-8"

_ENV_TENSORS = ["t_x", "t_v", "t_dst", "t_head", "t_cnt", "t_phase_state", "t_ts", "t_qptr",
                "t_stats", "t_last_det", "t_env", "halt", "phase", "tspent", "done_u8"]
_AGENT_TENSORS = ["params", "target", "adam_m", "adam_v", "np_state", "py_state"]


# Config fields that fix the state layout or its meaning: a resume under a
# different value would restore tensors that mean something else (or leave
# derived state stale), so load() refuses it.
_AGENT_FIXED = ["precision", "shared_params", "nn_layers", "replay_buffer_size", "batch_size",
                "seed", "loss", "target_update_frequency", "count_env_steps", "replay_rows",
                "ring_spare"]
_ENV_FIXED = ["rows", "cols", "num_envs", "env_offset", "seed", "signal_features", "cap_lane",
              "end_ms", "period_ms", "step_duration", "max_sim_time", "action_stride", "scenario",
              "actuated"]
# fields added after format 4 was introduced
_DEFAULTS = {"loss": "mse", "actuated": False, "replay_rows": "int8", "ring_spare": 2}


def _written(total, ring):
    """Ring slots that hold transitions after `total` stores: 0 .. n-1 (once
    the ring has wrapped, every slot; the spare one holds the evicted
    transition, saved with the rest)."""
    return min(int(total), ring.slots)


def _check_cfg(saved, cur, fields, what):
    for k in fields:
        a, b = saved.get(k, _DEFAULTS.get(k)), cur.get(k, _DEFAULTS.get(k))
        if k == "scenario" and a and b:
            a, b = os.path.basename(str(a)), os.path.basename(str(b))
        if a != b:
            raise ValueError(f"checkpoint {what}.{k} = {a!r} but this Trainer has {b!r}: "
                             "build the Trainer with the checkpoint's configuration")


def _cfg_dict(cfg):
    d = dataclasses.asdict(cfg)
    return {k: (v if isinstance(v, (int, float, str, bool, type(None), list)) else str(v))
            for k, v in d.items()}


def trainer_state(tr, include_replay=True):
    """CPU copy of everything a resume needs (see module docstring)."""
    tr.sync_outputs()  # the last side-stream learn's weights (schedule "env")
    ag, env = tr.agent, tr.env
    st = {"format": FORMAT,
          "env_cfg": _cfg_dict(env.cfg), "agent_cfg": _cfg_dict(ag.cfg),
          "nveh": int(env.nveh),
          "counters": {"learn_step_counter": ag.learn_step_counter,
                       "global_step_count": ag.global_step_count,
                       "epsilon": float(ag.epsilon), "learn_launches": ag.learn_launches,
                       "env_t": env.t, "env_episode": env.episode, "episode": tr.episode,
                       "step_count": tr.step_count, "total_steps": tr.total_steps,
                       "ring_total": ag.ring.total,
                       "env_steps": [int(x) for x in env.env_steps],
                       "env_episodes": [int(x) for x in env.env_episodes]}}
    st["agent"] = {k: getattr(ag, k).cpu() for k in _AGENT_TENSORS}
    if ag.target_h is not None:
        st["agent"]["target_h"] = ag.target_h.cpu()
    st["env"] = {k: getattr(env, k).cpu() for k in _ENV_TENSORS}
    st["env"]["local"] = env.local.cpu()
    st["obs"] = tr.obs.cpu()
    if include_replay:
        n = _written(ag.ring.total, ag.ring)
        st["replay"] = {k: getattr(ag.ring, k)[:, :n].cpu() for k in ["s", "n", "a", "r", "d"]}
    return st


def save(path, tr, include_replay=True):
    tr.synchronize()  # every stream, and (C5) the outstanding all-reduces, bounded
    tr.agent.ring.check()  # never persist a replay that holds a refused value
    torch.save(trainer_state(tr, include_replay), path)


def load(path, tr):
    """Restore a checkpoint into a Trainer built with the same configs."""
    st = torch.load(path, map_location="cpu", weights_only=True)
    if st.get("format") != FORMAT:
        raise ValueError(f"{path}: not a {FORMAT} checkpoint")
    ag, env = tr.agent, tr.env
    _check_cfg(st["agent_cfg"], _cfg_dict(ag.cfg), _AGENT_FIXED, "agent_cfg")
    _check_cfg(st["env_cfg"], _cfg_dict(env.cfg), _ENV_FIXED, "env_cfg")
    if int(st["nveh"]) != int(env.nveh):
        raise ValueError("checkpoint demand does not match this env config (nveh differs)")
    if int(st["counters"]["ring_total"]) > 0 and "replay" not in st:
        raise ValueError("checkpoint was saved without its replay (include_replay=False) but its "
                         "rings hold transitions: a resume would train on empty rings")

    # every tensor is checked before the first copy: a mismatch leaves the
    # Trainer untouched instead of half-restored
    copies = []

    def plan(group, dst, v, name):
        if dst is None:
            raise ValueError(f"checkpoint {group}.{name} has no counterpart in this Trainer")
        if tuple(dst.shape) != tuple(v.shape) or dst.dtype != v.dtype:
            raise ValueError(f"checkpoint {group}.{name} {v.dtype}{tuple(v.shape)} != "
                             f"{dst.dtype}{tuple(dst.shape)}")
        copies.append((dst, v))

    for k, v in st["agent"].items():
        plan("agent", getattr(ag, k), v, k)
    for k, v in st["env"].items():
        if k != "local":
            plan("env", getattr(env, k), v, k)
    if tuple(st["env"]["local"].shape) != tuple(env.local.shape):
        raise ValueError(f"checkpoint env.local {tuple(st['env']['local'].shape)} != "
                         f"{tuple(env.local.shape)}")
    if tuple(st["obs"].shape) != tuple(tr.obs.shape):
        raise ValueError(f"checkpoint obs {tuple(st['obs'].shape)} != {tuple(tr.obs.shape)}")
    c = st["counters"]
    if "replay" in st:
        n = st["replay"]["s"].shape[1]
        if n != _written(int(c["ring_total"]), ag.ring):
            raise ValueError(f"checkpoint replay holds {n} slots, its counter says "
                             f"{_written(int(c['ring_total']), ag.ring)}")
        for k, v in st["replay"].items():
            plan("replay", getattr(ag.ring, k)[:, :n], v, k)
    # the restore writes on the caller's stream: order it after everything the
    # trainer queued on its side stream (the "env" schedule's side learn may
    # still be updating its agents' weights and Adam slots -- ADVICE r5)
    tr.quiesce()
    for dst, v in copies:
        dst.copy_(v.to(dst.device))
    env.local = st["env"]["local"].to(env.device)
    ag.learn_step_counter, ag.global_step_count = c["learn_step_counter"], c["global_step_count"]
    ag.epsilon, ag.learn_launches = c["epsilon"], c["learn_launches"]
    env.t, env.episode = c["env_t"], c["env_episode"]
    tr.episode, tr.step_count, tr.total_steps = c["episode"], c["step_count"], c["total_steps"]
    env.env_steps[:] = c["env_steps"]
    env.env_episodes[:] = c["env_episodes"]
    ag.ring.total = c["ring_total"]
    ag._refresh_params_h()  # the 16-bit copies are derived from the f32 nets
    ag._refresh_target_h()
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
