"""src/env/traffic_env.py -- drop-in home of the environment step.

The reference left this module empty and drove SUMO through TraCI directly from
src/scripts/train.py (:99-106, :190, :225-270) with the observation helpers of
src/experimental/order_lanes.py.  Here the whole env step (setPhase, K one-second
substeps, halting counts, 17-dim local states, 89-dim observations, rewards) runs
on the GPU; see dmdqn_amd/env.py for the implementation.

Surfaces:
  TrafficEnv(cfg).reset() / .step(actions[E,A])        batched device tensors
  TrafficEnv(cfg).reset_dict() / .step_dict({id: a})   the same, one replica, dicts
  get_controlled_intersection_ids / get_state_size / get_action_size / close_sumo
The reference's class surface under its own name and constructor is
src/agents/sumo_env.py:SumoTrafficEnvironment.
"""
import yaml

from dmdqn_amd.env import EnvConfig, IDMParams, TrafficEnv  # noqa: F401


def env_config_from_yaml(path="config/env_config.yaml", **overrides):
    """EnvConfig from the reference's env_config.yaml keys (+ additive keys)."""
    with open(path) as f:
        y = yaml.safe_load(f) or {}
    y.update(overrides)
    return EnvConfig(rows=int(y.get("grid_rows", 3)), cols=int(y.get("grid_cols", 3)),
                     num_envs=int(y.get("num_envs", 1)), seed=int(y.get("seed", 0)),
                     step_duration=int(y.get("step_duration", 10)),
                     max_sim_time=int(y.get("max_sim_time", 2400)),
                     signal_features=y.get("signal_features", "reference"))
