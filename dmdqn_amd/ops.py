"""torch.ops.dmdqn -- the C ABI (include/dmdqn.h) as PyTorch custom operators.

libdmdqn_torch.so registers TORCH_LIBRARY(dmdqn) over the extern "C" entry
points of libdmdqn_hip.so (dmdqn_amd/torch_ext/dmdqn_torch.cpp): each op checks
its tensors with TORCH_CHECK, launches on the current HIP stream of their
device and mutates the arguments its schema marks.  This is the product path
of every Python surface (TrafficEnv, BatchedDQN, Trainer, the drop-in
DQNAgent); the ctypes binding in _lib.py stays for the C-ABI tests, error
strings and the CU-masked stream helper.  Missing libraries raise: there is no
CPU fallback.
"""
import os

import torch

from . import _lib

# which operator wraps which C entry point (include/dmdqn.h)
ENTRY_POINTS = {
    "dmdqn_mt_seed_np": "mt_seed", "dmdqn_mt_seed_py": "mt_seed",
    "dmdqn_mt_draw_u32": "mt_draw_u32", "dmdqn_act": "act", "dmdqn_act_uniform": "act",
    "dmdqn_observe": "observe",
    "dmdqn_replay_store": "replay_store", "dmdqn_replay_sample": "replay_sample",
    "dmdqn_replay_sample_budget": "replay_sample",
    "dmdqn_sim_reset": "sim_reset", "dmdqn_sim_reset_envs": "sim_reset",
    "dmdqn_sim_step": "sim_step", "dmdqn_env_step": "env_step", "dmdqn_learn": "learn_step",
    "dmdqn_learn_grad": "learn_step", "dmdqn_adam_agents": "learn_step",
    "dmdqn_replay_store_f32": "replay_store_f32", "dmdqn_replay_gather_f32": "replay_gather_f32",
    "dmdqn_learn_shared_grad": "learn_shared_grad", "dmdqn_adam": "adam",
    "dmdqn_adam_slabs": "adam_slabs",
    "dmdqn_target_sync": "target_sync", "dmdqn_q_argmax": "q_argmax",
    "dmdqn_q_argmax_shared": "q_argmax",
}

TORCH_LIB_PATH = os.path.join(os.path.dirname(_lib.LIB_PATH), f"libdmdqn_torch{_lib._SUFFIX}.so")
_OPS = None


def load():
    """torch.ops.dmdqn (loads libdmdqn_hip.so, then the operator library)."""
    global _OPS
    if _OPS is None:
        _lib.load()
        if not os.path.exists(TORCH_LIB_PATH):
            raise _lib.DmdqnError(f"{TORCH_LIB_PATH} not found: build it with "
                                  "`python -m dmdqn_amd.build` (no CPU fallback)")
        # the operator library's build-time digest must be the tree's too
        import ctypes
        _lib.verify_digest(ctypes.CDLL(TORCH_LIB_PATH), TORCH_LIB_PATH,
                           symbol="dmdqn_torch_source_digest")
        torch.ops.load_library(TORCH_LIB_PATH)
        _OPS = torch.ops.dmdqn
    return _OPS
