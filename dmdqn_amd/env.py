"""Vectorised traffic environment on the GPU (replaces SUMO/TraCI + order_lanes).

`TrafficEnv` keeps E independent replicas of an R x C signalised grid resident
in HBM and steps them all with one simulator launch plus one observe launch
per RL step.  It mirrors two reference surfaces:

* the batched loop body of src/scripts/train.py:207-270 -- `reset()` /
  `step(actions[E, A])` return device tensors (obs [E,A,89] f32, reward [E,A]
  f64, done [E] bool);
* the class API of src/agents/sumo_env.py:SumoTrafficEnvironment -- reset /
  step over {junction_id: ...} dicts for E = 1 (`reset_dict`, `step_dict`),
  get_controlled_intersection_ids / get_state_size / get_action_size /
  close_sumo.

Semantics follow train.py (89-dim N,S,E,W observation, reward on the PRE-step
state, setPhase every RL step with ACTION_MAP {0:0,1:3,2:6,3:9}, K = 10
one-second substeps, done at t >= 2400), not sumo_env.py's 74-dim variant.
"""
from dataclasses import dataclass, field
from typing import Optional

import numpy as np
import torch

from . import kernels as K
from .ops import load as load_ops
from .scenario import Grid, demand_tables

SIGNAL_MODES = {"reference": 0, "intended": 1}


@dataclass
class IDMParams:
    """SUMO passenger-car defaults + grid_3x3 geometry."""
    length: float = 5.0
    min_gap: float = 2.5
    accel: float = 2.6
    decel: float = 4.5
    tau: float = 1.0
    vmax: float = 13.89
    halt_speed: float = 0.1
    len_inner: float = 172.8
    len_outer: float = 86.4
    # actuated mode (EnvConfig.actuated): SUMO's actuated-TLS defaults
    detector_gap_s: float = 2.0   # detector distance upstream = detector_gap_s * vmax
    max_gap: float = 3.0          # gap-out time (s)

    def values(self):
        """The dmdqn_idm constants in struct order (include/dmdqn.h), as float32
        values (two_sqrt_ab = 2 sqrt(a b) computed in float32, as the oracle)."""
        f = np.float32
        two_sqrt_ab = f(2.0) * np.sqrt(f(self.accel) * f(self.decel), dtype=np.float32)
        det = f(self.detector_gap_s) * f(self.vmax)
        return [float(f(x)) for x in (self.length, self.min_gap, self.accel, self.decel, self.tau,
                                      self.vmax, two_sqrt_ab, self.halt_speed, self.len_inner,
                                      self.len_outer, det, self.max_gap)]


@dataclass
class EnvConfig:
    rows: int = 4
    cols: int = 4
    num_envs: int = 1024
    seed: int = 0                # env e uses seed + env_offset + e
    env_offset: int = 0          # global index of this process's first env
    step_duration: int = 10      # STEP_DURATION (train.py:56), 1 s substeps
    max_sim_time: int = 2400     # MAX_SIM_TIME (train.py:58)
    action_stride: int = 3       # ACTION_MAP {a: 3a} (train.py:57)
    signal_features: str = "reference"  # A-5: "reference" (padding) | "intended"
    # A-14: SUMO's actuated gap-out on phase 0 (grid_3x3.net.xml:894, minDur 5,
    # maxDur 50).  Off by default: fixed durations.
    actuated: bool = False
    cap_lane: int = 24           # vehicle slots per lane (172.8 m / 7.5 m + 1)
    end_ms: int = 2_500_000      # last departure (trips_p06.trips.xml:7-9)
    period_ms: Optional[int] = None
    idm: IDMParams = field(default_factory=IDMParams)
    # a real scenario instead of synthetic demand: a .sumocfg (net + routes, as
    # the reference's src/sumo_files/scenarios/grid_3x3.sumocfg) or the .npz
    # sumo_scenario.Scenario.save writes (config/scenarios/grid_3x3_p06.npz).
    # Sets rows / cols / departures (identical in every replica) / lane lengths.
    scenario: Optional[str] = None

    @property
    def n_agents(self):
        return self.rows * self.cols


class TrafficEnv:
    """E replicas of the grid on one device.  All state lives in device memory."""

    def __init__(self, cfg: EnvConfig = None, device="cuda", auto_restart=True):
        """auto_restart (only matters when the demand drains before
        max_sim_time): step() restarts each replica whose episode ended (the
        Trainer's loop); False leaves an ended replica as it ended until the
        caller's reset() (the single-replica SumoTrafficEnvironment surface,
        sumo_env.py:420-489, whose caller reloads)."""
        self.cfg = cfg = cfg or EnvConfig()
        self.auto_restart = auto_restart
        if cfg.signal_features not in SIGNAL_MODES:
            raise ValueError(f"signal_features must be one of {list(SIGNAL_MODES)}")
        self._ops = load_ops()
        self.device = torch.device(device)
        self.scenario = None
        if cfg.scenario:
            from .sumo_scenario import load_scenario, scenario_tables
            sc = self.scenario = load_scenario(cfg.scenario)
            cfg.rows, cfg.cols = sc.rows, sc.cols
            cfg.idm.len_inner, cfg.idm.len_outer = sc.lane_len_inner, sc.lane_len_outer
        self.grid = g = Grid(cfg.rows, cfg.cols)
        self.R, self.C, self.A, self.E = cfg.rows, cfg.cols, g.A, cfg.num_envs
        E, A, NL, cap = self.E, self.A, g.NL, cfg.cap_lane
        self.seeds = np.arange(cfg.num_envs, dtype=np.int64) + cfg.seed + cfg.env_offset
        if self.scenario is not None:
            q_ids, q_off, vdst, nveh, period = scenario_tables(self.scenario, E)
        else:
            q_ids, q_off, vdst, nveh, period = demand_tables(g, self.seeds, cfg.end_ms,
                                                             cfg.period_ms)
        self.nveh, self.period_ms = nveh, period
        # train.py:233-236 ends an episode when t >= MAX_SIM_TIME or no vehicle is
        # running or pending (getMinExpectedNumber() == 0).  While departures are
        # still scheduled at or after max_sim_time (the shipped demand: 2499.6 s
        # > 2400 s) the second condition cannot fire: every replica ends at the
        # same step, and the host clock decides without a device read.
        # Otherwise the replicas end when their own demand has drained, and each
        # restarts on its own `done` as the reference's one env does
        # (train.py:188-207: traci.load, a fresh episode, the replay kept):
        # step() reads the kernel's per-replica flags (one sync per step) and
        # resets those replicas only; each keeps its own clock (t_env).
        self.drains_early = (nveh - 1) * period < cfg.max_sim_time * 1000
        dev = self.device
        z32 = lambda *s: torch.zeros(s, dtype=torch.int32, device=dev)  # noqa: E731
        self.t_x = torch.zeros((E, NL, cap), dtype=torch.float32, device=dev)
        self.t_v = torch.zeros((E, NL, cap), dtype=torch.float32, device=dev)
        self.t_dst = z32(E, NL, cap)
        self.t_head, self.t_cnt, self.t_req, self.t_gfrom = z32(E, NL), z32(E, NL), z32(E, NL), z32(E, NL)
        self.t_fx = torch.zeros((E, NL), dtype=torch.float32, device=dev)
        self.t_fv = torch.zeros((E, NL), dtype=torch.float32, device=dev)
        self.t_phase_state, self.t_ts = z32(E, A), z32(E, A)
        self.t_qptr = z32(E, 4 * A)
        self.t_q_off = torch.from_numpy(q_off).to(dev)
        self.t_q_ids = torch.from_numpy(q_ids.view(np.int16)).to(dev)
        self.t_vdst = torch.from_numpy(vdst.view(np.int16)).to(dev)
        q_dst = np.take_along_axis(vdst, q_ids.astype(np.int64), axis=1)  # queue order
        self.t_q_dst = torch.from_numpy(np.ascontiguousarray(q_dst).view(np.int16)).to(dev)
        self.t_exit_id = torch.from_numpy(g.exit_id.reshape(-1).copy()).to(dev)
        self.t_exit_ao = torch.from_numpy(g.exit_ao.reshape(-1).copy()).to(dev)
        self.t_stats = z32(E, 4)
        self.t_last_det = z32(E, 12 * g.A)
        self.t_env = z32(E)  # each replica's episode clock (s)
        # the dmdqn_sim arrays in the order of the sim ops (dmdqn_torch.cpp make_sim)
        self._sim_state = [self.t_x, self.t_v, self.t_dst, self.t_head, self.t_cnt, self.t_req,
                           self.t_gfrom, self.t_fx, self.t_fv, self.t_phase_state, self.t_ts,
                           self.t_qptr, self.t_stats, self.t_last_det, self.t_env]
        self._sim_tables = [self.t_q_off, self.t_q_ids, self.t_vdst, self.t_exit_id,
                            self.t_exit_ao, self.t_q_dst]
        self._sim_dims = [cfg.rows, cfg.cols, E, cap, period, nveh, int(bool(cfg.actuated))]
        self._idm = cfg.idm.values()
        # observation buffers
        self.halt = z32(E, A, 12)
        self.phase = z32(E, A)
        self.tspent = z32(E, A)
        self.done_u8 = torch.zeros(E, dtype=torch.uint8, device=dev)
        self.mode = SIGNAL_MODES[cfg.signal_features]
        self.local = None
        self.obs = None
        self.t = 0
        self.episode = 0
        # per replica (host): steps into the current episode, episodes completed
        self.env_steps = np.zeros(E, np.int64)
        self.env_episodes = np.zeros(E, np.int64)
        self.sim_hook = None  # callable(before: bool) around the sim launch (bench timing)

    # ------------------------------------------------------------ batched API
    def reset(self):
        """traci.load (train.py:190) for every replica; returns obs [E,A,89]."""
        self._ops.sim_reset(self._sim_state, self._sim_tables, self._sim_dims)
        self.t = 0
        self.env_steps[:] = 0
        self.halt.zero_()
        self.phase.zero_()
        self.tspent.zero_()
        self.local, self.obs, _ = K.observe(self.R, self.C, self.halt, self.phase, self.tspent,
                                            self.mode)
        # the state a replica restarts from (identical for every replica)
        self._local0, self._obs0 = self.local[0].clone(), self.obs[0].clone()
        return self.obs

    def _t0(self):
        """The t0 argument of the sim launches.  Every launch passes t_env, so
        the kernel runs each replica from its own clock and ignores t0; the host
        clock self.t is the shared clock of the lockstep mode only (it stays 0
        when replicas restart on their own, so it cannot outgrow int32)."""
        return 0 if self.drains_early else self.t

    def advance(self):
        """K substeps for every replica with the signals running their program
        (no setPhase, no observation): the sim launch alone.  Diagnostics only
        (bench.py times k_sim_step with it); a training loop calls step()."""
        cfg = self.cfg
        self._ops.sim_step(self._sim_state, self._sim_tables, self._sim_dims, self._idm, None,
                           cfg.action_stride, self._t0(), cfg.step_duration, cfg.max_sim_time,
                           self.halt, self.phase, self.tspent, self.done_u8)
        if not self.drains_early:
            self.t += cfg.step_duration

    def step(self, actions, restart=None):
        """One RL step for all replicas (train.py:225-270).
        actions int32 [E,A] on the device.  Returns (obs', reward, done, info):
        reward [E,A] f64 is computed from the PRE-step local state (A-3).
        restart: overrides auto_restart for this step."""
        if self.local is None:
            raise RuntimeError("call reset() first")
        if actions.dtype != torch.int32 or tuple(actions.shape) != (self.E, self.A):
            raise ValueError(f"actions must be int32 [{self.E},{self.A}]")
        cfg = self.cfg
        if self.sim_hook:
            self.sim_hook(True)
        self._ops.sim_step(self._sim_state, self._sim_tables, self._sim_dims, self._idm, actions,
                           cfg.action_stride, self._t0(), cfg.step_duration, cfg.max_sim_time,
                           self.halt, self.phase, self.tspent, self.done_u8)
        if self.sim_hook:
            self.sim_hook(False)
        prev = self.local
        local, obs, reward = K.observe(self.R, self.C, self.halt, self.phase, self.tspent,
                                       self.mode, prev_local=prev)
        return self._finish_step(local, obs, reward, restart)

    def step_fused(self, np_state, eps, greedy, actions, ring, obs_s, n_actions=4):
        """act + step + remember of one loop iteration in ONE launch per replica
        (dmdqn_env_step, train.py:211-282 up to agent.replay()): select_action's
        draws from np_state (eps; greedy [E,A] when eps < 1) into actions
        [E,A], setPhase + K substeps, the observation / reward, and the
        transition (obs_s, action, reward, obs', the replica's done flag) into
        ring slot ring.next_slot (int8 rows; the caller advances the
        ring).  Bit-identical to act -> step -> ReplayRing.store; returns what
        step() returns."""
        if self.local is None:
            raise RuntimeError("call reset() first")
        if ring.row_format != "int8" or ring.NA != self.E * self.A:
            raise ValueError("step_fused stores int8 rows of E*A agents")
        cfg, E, A, dev = self.cfg, self.E, self.A, self.device
        local = torch.empty((E, A, K.LOCAL_DIM), dtype=torch.float32, device=dev)
        obs = torch.empty((E, A, K.OBS_DIM), dtype=torch.float32, device=dev)
        reward = torch.empty((E, A), dtype=torch.float64, device=dev)
        if self.sim_hook:
            self.sim_hook(True)
        self._ops.env_step(self._sim_state, self._sim_tables, self._sim_dims, self._idm,
                           cfg.action_stride, self._t0(), cfg.step_duration, cfg.max_sim_time,
                           self.halt, self.phase, self.tspent, self.done_u8, np_state, greedy,
                           actions, float(eps), int(n_actions), self.mode, local, obs, self.local,
                           reward, obs_s, ring.next_slot, ring.s, ring.n, ring.a, ring.r,
                           ring.d, ring.err)
        if self.sim_hook:
            self.sim_hook(False)
        return self._finish_step(local, obs, reward)

    def _finish_step(self, local, obs, reward, restart=None):
        cfg = self.cfg
        restart = self.auto_restart if restart is None else restart
        self.local, self.obs = local, obs
        if self.drains_early:
            # the reference rule per replica (done_u8, from the last substep):
            # the transition of replica e carries its own flag, and (restart) a
            # replica whose episode ended restarts now, alone (train.py:188-207);
            # info["obs_next"] is what the next act sees (the restart state for
            # those replicas).  `done` is True when every replica ended at this
            # step -- for E = 1, train.py's `while not done` exactly.  One sync
            # reads the flags and the replicas' clocks together.
            both = torch.cat([self.done_u8.to(torch.int32), self.t_env]).cpu().numpy()
            flags, clock = both[:self.E].astype(bool), both[self.E:]
            info = {"simulation_time": float(clock.max()), "t_env": clock,
                    "done_flags": self.done_u8, "done": self.done_u8.clone()}
            self.env_steps += 1
            done = bool(flags.all())
            obs_next = self.obs
            restarted = flags if restart else np.zeros_like(flags)
            if flags.any():
                # the ended episodes' counters [E,4] (inserted, arrived, running,
                # pending) before any restart clears them
                info["final_stats"] = self.t_stats.clone()
                self.env_episodes[flags] += 1
            if restarted.any():
                self._ops.sim_reset(self._sim_state, self._sim_tables, self._sim_dims,
                                    info["done"])
                m = info["done"].bool().view(self.E, 1, 1)
                self.local = torch.where(m, self._local0, self.local)
                obs_next = torch.where(m, self._obs0, self.obs)
                self.env_steps[flags] = 0
            info["obs_next"] = obs_next
            info["restarted"] = restarted
        else:
            # shared clock and demand horizon: `done` is uniform and known on
            # the host without a device sync
            self.t += cfg.step_duration
            done = self.t >= cfg.max_sim_time
            info = {"simulation_time": float(self.t), "done_flags": self.done_u8, "done": done}
            self.env_steps += 1
            if done:
                self.env_episodes += 1
        return self.obs, reward, done, info

    def termination_reason(self, e=0):
        """sumo_env.py:483-487 for replica e after a step that ended its
        episode: "sumo_halted" when no vehicle is running or pending
        (_is_episode_done_sumo, :681-692; checked first, as there), else
        "max_time_reached".  Reads the replica's counters (syncs)."""
        st = self.t_stats[e].cpu().numpy()
        return "sumo_halted" if int(st[2]) + int(st[3]) == 0 else "max_time_reached"

    def stats(self):
        """[E,4] inserted, arrived, running, pending (syncs)."""
        return self.t_stats.cpu().numpy()

    # ------------------------------------------------------------ reference class API
    def get_controlled_intersection_ids(self):
        return list(self.grid.junction_ids)

    def get_state_size(self):
        return K.OBS_DIM

    def get_action_size(self, intersection_id=None):
        return 4

    def close_sumo(self):
        pass

    def reset_dict(self):
        """SumoTrafficEnvironment.reset (sumo_env.py:420) for E = 1: {id: obs}."""
        if self.E != 1:
            raise ValueError("reset_dict is the single-replica API (num_envs == 1)")
        obs = self.reset()[0].cpu().numpy()
        return {j: obs[a] for a, j in enumerate(self.grid.junction_ids)}

    def step_dict(self, actions):
        """SumoTrafficEnvironment.step (sumo_env.py:434-489) for E = 1 with
        train.py's semantics: {id: action} -> ({id: obs}, {id: reward}, done,
        info).  An ended episode stays ended (no restart) until reset_dict();
        info["termination_reason"] as the reference sets it."""
        if self.E != 1:
            raise ValueError("step_dict is the single-replica API (num_envs == 1)")
        ids = self.grid.junction_ids
        a = torch.tensor([[int(actions[j]) for j in ids]], dtype=torch.int32, device=self.device)
        obs, rew, done, info = self.step(a, restart=False)
        obs, rew = obs[0].cpu().numpy(), rew[0].cpu().numpy()
        out = {"simulation_time": info["simulation_time"]}
        if done:
            out["termination_reason"] = self.termination_reason(0)
        return ({j: obs[a] for a, j in enumerate(ids)}, {j: float(rew[a]) for a, j in enumerate(ids)},
                bool(done), out)
