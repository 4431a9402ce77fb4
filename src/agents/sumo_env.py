"""src/agents/sumo_env.py -- the reference's SumoTrafficEnvironment class surface
(src/agents/sumo_env.py:48-716) over the GPU simulator, one replica.

A caller written against the reference class switches by changing the import:
the constructor takes the reference's arguments (:58-67), `reset(sumo_seed,
use_gui)` returns {junction_id: observation} (:420-432), `step({id: action})`
returns (observations, rewards, done, info) with info["simulation_time"] and,
on the step that ends the episode, info["termination_reason"] = "sumo_halted"
(no vehicle running or pending, :681-692, checked first) or
"max_time_reached" (:474-487), plus get_controlled_intersection_ids /
get_state_size / get_action_size / start_sumo / close_sumo (:352-432, :694-716).

What runs underneath is the train.py hot path this build replaces
(dmdqn_amd.env.TrafficEnv, one replica): the 89-dim N,S,E,W observation of
order_lanes.build_state_vector and train.py's reward (0.3 local + 0.7 global
from the PRE-step states, train.py:159-165, :254) -- not sumo_env.py's 74-dim
variant and its _calculate_rewards, which no training script of the reference
calls.  Actions follow the class's _apply_actions (:491-530): an id that is
not a controlled junction, an action with no entry in that junction's
action_phases, or a phase string the signal program does not have (the
reference prints a warning) is skipped; setPhase is skipped too when the
junction is already in the requested phase, so its timer runs on; a junction
without an action this step keeps running its program.  Without
"action_phases" a junction's map is empty (:113-117): every action is skipped
and get_action_size() is 0, as in the reference.  Junctions not listed in
controlled_intersections run their programs untouched and are absent from the
observation and reward dicts.  Differences a caller can see, all stated here:
  * action_phases entries may also be phase INDICES (an extension; the
    reference takes state strings, and its `if sumo_phase_string:` would skip
    an index 0 -- here 0 selects phase 0);
  * ids that are not junctions of the network are dropped, as the reference
    drops ids without a traffic light (:116-123); an empty result raises
    ValueError (the reference exits);
  * a step always runs step_duration whole 1-second substeps (step_duration
    must be a whole number of seconds); the reference stops the substep loop
    at the second the network empties (:456-463), so simulation_time on that
    last step can be up to step_duration - 1 s later here;
  * sumo_seed: the simulator is deterministic.  An int seeds the synthetic
    demand (EnvConfig.seed) and rebuilds the replica; "random" keeps the
    current demand.  A scenario's routes are fixed, whatever the seed.
  * use_gui=True raises (there is no GUI); padding_value must be -1.0 and
    max_lanes_per_direction 3 (the observation layout, order_lanes.py:497-555).
"""
import os
from dataclasses import replace

import numpy as np
import torch

from dmdqn_amd import kernels as K
from dmdqn_amd.env import EnvConfig, TrafficEnv

# The signal program every junction of the shipped grid runs
# (grid_3x3.net.xml:893-906; all nine tlLogic elements are identical): the
# state string of each of its 12 phases.  An action_phases entry given as a
# state string selects the FIRST phase with that string, as _apply_actions
# does (sumo_env.py:507-513).
TL_PROGRAM_STATES = [
    "GGGGrgGrrrrrGGGGrgGrrrrr", "yyyyyyyyyyyyyyyyyyyyyyyy", "rrrrrrrrrrrrrrrrrrrrrrrr",
    "GrryGgGrrrrrGrryGgGrrrrr", "yyyyyyyyyyyyyyyyyyyyyyyy", "rrrrrrrrrrrrrrrrrrrrrrrr",
    "GrrrrrGGGGrgGrrrrrGGGGrg", "yyyyyyyyyyyyyyyyyyyyyyyy", "rrrrrrrrrrrrrrrrrrrrrrrr",
    "GrrrrrGrryGgGrrrrrGrryGg", "yyyyyyyyyyyyyyyyyyyyyyyy", "rrrrrrrrrrrrrrrrrrrrrrrr",
]
# train.py:57 ACTION_MAP as SUMO state strings: the action_phases of a caller
# that wants train.py's four green phases (0, 3, 6, 9)
TRAIN_PY_ACTION_PHASES = {a: TL_PROGRAM_STATES[3 * a] for a in range(4)}
DEFAULT_MAX_LANES_PER_DIRECTION = 3
NO_SET_PHASE = -1  # dmdqn_sim_step: no setPhase for this junction this step


def _phase_index(phase):
    """A phase given as a program state string or an index -> the index of
    the FIRST program phase with that string (:510-514); -1 when the program
    has no such phase (the reference warns and skips the action, :519-523)."""
    if isinstance(phase, str):
        return TL_PROGRAM_STATES.index(phase) if phase in TL_PROGRAM_STATES else -1
    p = int(phase)
    if not 0 <= p < len(TL_PROGRAM_STATES):
        raise ValueError(f"phase index {p} outside the 12-phase program")
    return p


class SumoTrafficEnvironment:
    """sumo_env.py:48 SumoTrafficEnvironment on the GPU simulator (one replica).

    sumo_cfg_path: a .sumocfg (its net and route files are loaded, as
    `sumo -c` would) or a scenario .npz (sumo_scenario.Scenario.save); None
    runs the synthetic grid demand of `env_config` (rows, cols, seed, end_ms,
    ...).  net_file_path must exist when given (the reference exits
    otherwise, :94-95); the network itself is the one the .sumocfg names.
    env_config: additive EnvConfig fields (seed, signal_features, actuated,
    demand); num_envs, step_duration, max_sim_time and scenario are set from
    the reference arguments."""

    def __init__(self, sumo_cfg_path, net_file_path, controlled_intersections,
                 max_lanes_per_direction=DEFAULT_MAX_LANES_PER_DIRECTION, step_duration=1.0,
                 max_simulation_time=3600, padding_value=-1.0, *, env_config=None,
                 device="cuda"):
        if net_file_path is not None and not os.path.exists(net_file_path):
            raise FileNotFoundError(f"Network file not found: {net_file_path}")
        if sumo_cfg_path is not None and not os.path.exists(sumo_cfg_path):
            raise FileNotFoundError(f"SUMO configuration not found: {sumo_cfg_path}")
        if sumo_cfg_path is None and env_config is None:
            raise ValueError("sumo_cfg_path=None needs env_config (the synthetic grid)")
        if not controlled_intersections:
            raise ValueError("No controlled intersections defined.")
        if int(max_lanes_per_direction) != DEFAULT_MAX_LANES_PER_DIRECTION:
            raise ValueError("max_lanes_per_direction must be 3 (the 89-dim observation layout)")
        if float(padding_value) != -1.0:
            raise ValueError("padding_value must be -1.0 (the observation's padding)")
        if float(step_duration) != int(step_duration) or int(step_duration) < 1:
            raise ValueError("step_duration must be a whole number of seconds >= 1")
        self.sumo_cfg_path, self.net_file_path = sumo_cfg_path, net_file_path
        self.step_duration = float(step_duration)
        self.max_simulation_time = max_simulation_time
        self.padding_value = float(padding_value)
        self.max_lanes_per_direction = int(max_lanes_per_direction)
        self.device = device
        self._cfg = replace(env_config or EnvConfig(), num_envs=1,
                            step_duration=int(step_duration),
                            max_sim_time=int(np.ceil(float(max_simulation_time))),
                            scenario=sumo_cfg_path, action_stride=1)
        self._build()
        ids = self.env.get_controlled_intersection_ids()  # every signal of the grid
        self.controlled_intersections_config = {c["id"]: c for c in controlled_intersections}
        kept = [j for j in self.controlled_intersections_config if j in ids]
        if not kept:
            raise ValueError("None of the provided 'controlled_intersections' IDs correspond to "
                             "traffic lights found in the network.")
        self.controlled_intersection_ids = kept
        self.traffic_light_ids = {j: j for j in kept}
        # :113-117: the action -> phase map per junction, empty without "action_phases"
        self.action_to_sumo_phase = {
            j: self.controlled_intersections_config[j].get("action_phases", {}) for j in kept}
        self._phase_of = {j: {a: _phase_index(p) for a, p in m.items() if isinstance(p, int) or p}
                          for j, m in self.action_to_sumo_phase.items()}
        self._col = [ids.index(j) for j in kept]  # obs row of each controlled id
        self._signal = {j: ids.index(j) for j in kept}  # signal index in the simulator
        self.state_vector_size = K.OBS_DIM
        self.current_time = 0.0
        self._started = False

    def _build(self):
        self.env = TrafficEnv(self._cfg, device=self.device, auto_restart=False)

    # ------------------------------------------------------------ sumo_env.py:352-432
    def start_sumo(self, use_gui=False, sumo_seed="random", port=None):
        """Load the network and demand at t = 0 (:352-389; `port` is unused)."""
        if use_gui:
            raise ValueError("use_gui: there is no GUI, the simulator runs on the GPU")
        if sumo_seed != "random":
            seed = int(sumo_seed)
            if seed != self._cfg.seed and self._cfg.scenario is None:
                self._cfg = replace(self._cfg, seed=seed)
                self._build()
        self._obs = self.env.reset()
        self.current_time = 0.0
        self._started = True

    def close_sumo(self):
        """:408-418 -- nothing to close; the next step needs reset()."""
        self._started = False

    def reset(self, sumo_seed="random", use_gui=False):
        """:420-432: restart the episode, return {junction_id: obs f32[89]}."""
        self.start_sumo(use_gui=use_gui, sumo_seed=sumo_seed)
        return self._dict(self._obs[0].cpu().numpy())

    def step(self, actions):
        """:434-489: {junction_id: action} -> (observations, rewards, done,
        info), the observation and reward of train.py:238-270."""
        if not self._started:
            raise RuntimeError("call reset() first (the simulation is not running)")
        ph = self._apply_actions(actions)
        obs, rew, done, info = self.env.step(torch.from_numpy(ph).to(self.env.device),
                                             restart=False)
        self.current_time = float(info["simulation_time"])
        out = {"simulation_time": self.current_time}
        if done:
            out["termination_reason"] = self.env.termination_reason(0)
        r = rew[0].cpu().numpy()
        rewards = {j: float(r[c]) for j, c in zip(self.controlled_intersection_ids, self._col)}
        return self._dict(obs[0].cpu().numpy()), rewards, bool(done), out

    def _apply_actions(self, actions):
        """:491-530 -> the simulator's per-signal phase requests [1, A]: the
        phase index to set, or NO_SET_PHASE (unknown id, unmapped action,
        phase string not in the program, or already in that phase)."""
        ph = np.full((1, self.env.A), NO_SET_PHASE, np.int32)
        current = None
        for j, a in actions.items():
            if j not in self.traffic_light_ids:
                continue
            p = self._phase_of[j].get(a, NO_SET_PHASE)
            if p == NO_SET_PHASE:
                s = self.action_to_sumo_phase[j].get(a)
                if s:
                    print(f"Warning: SUMO phase string '{s}' (Action {a}) not found for TL {j}.")
                continue
            if current is None:  # traci.trafficlight.getPhase (:517), one read per step
                current = self.env.phase[0].cpu().numpy()
            c = self._signal[j]
            if int(current[c]) != p:
                ph[0, c] = p
        return ph

    def _dict(self, obs):
        return {j: np.asarray(obs[c], np.float32)
                for j, c in zip(self.controlled_intersection_ids, self._col)}

    # ------------------------------------------------------------ sumo_env.py:694-716
    def get_controlled_intersection_ids(self):
        return list(self.controlled_intersection_ids)

    def get_state_size(self):
        return self.state_vector_size

    def get_action_size(self, intersection_id=None):
        target = (intersection_id if intersection_id in self.action_to_sumo_phase
                  else (self.controlled_intersection_ids[0]
                        if self.controlled_intersection_ids else None))
        return len(self.action_to_sumo_phase.get(target, {})) if target else 0
