"""The batched reference training loop (src/scripts/train.py:188-316) on the GPU.

One `step()` is one iteration of the loop body for every agent of every env
replica:  act (select_action) -> env step (setPhase, K substeps) -> observe /
reward -> remember -> replay (learn), in the reference's order.  All of it is
kernel launches; the host keeps only counters.

Schedules (`overlap`).  The reference loop is sequential, but its data flow
is not: the replay draws of a step depend only on the CPython stream and the
ring length (never on the ring contents), and with the reference's epsilon
(1.0 on the training path, A-1) the next act and env step need nothing from
the learn.  Every schedule gives each kernel exactly the inputs of the
sequential order, so results are bit-identical (tests/test_gpu_overlap.py).

  "none"    (default) one stream: act, sim, observe, store, sample, learn.
            With fused=True (default; int8 replay rows) act, sim, observe and
            store are ONE launch per replica (dmdqn_env_step, bit-identical).
  "sample"  the replay draws of step t run on a side stream beside
            act/sim/observe/store of step t (all latency-bound, low occupancy);
            the side stream waits for learn t-1, so nothing shares the GPU
            with a learn.
              side:  [wait learn t-1] sample_t (ev_s)
              main:  act_t sim_t observe_t store_t [wait ev_s] learn_t
            (fused: main runs env_step_t [wait ev_s] learn_t).
  "full"    step t+1's act -> sim -> observe -> sample run on the side stream
            while learn t runs; only remember (which overwrites ring slots
            learn t may read) waits for learn t.  A greedy act (epsilon < 1)
            also waits for the learn, whose weights it reads.  The learn then
            shares the GPU with the sim, so its own duration grows.
              side:  [wait store t-1] act_t sim_t observe_t sample_t (ev_obs)
              main:                  [wait ev_obs] store_t (ev_store) learn_t
            The fused learn's workgroups fill every CU until they end, so the
            side work queued beside it mostly waits; split_learn=True makes the
            learn two launches whose Adam half leaves room beside it.

  "env"     the fused env step of step t+1 (act, sim, observe, remember) and
            the replay draws of learn t+1 run on a side stream beside learn t.
            The ring has s = AgentConfig.ring_spare spare slots (16;
            kernels.ReplayRing: cap + s slots for a deque of maxlen cap), and
            the stores of steps t+1 .. t+s go to slots learn t cannot sample;
            the store of step t+s+1 waits for learn t (its slot is in learn t's
            window) or a later marked learn -- at fixed epsilon 1 the learn
            stream marks every s-th call with an ordering-only event, and the
            side stream runs up to s steps ahead (the agent's per-step output
            buffers rotate over s + 2 copies for it).  A greedy act (epsilon <
            1) waits for learn t's weights.
              side:  [wait the newest marked learn <= t-1] env_step_{t+1} sample_{t+1} (ev_env)
              main:  [wait ev_env of t] learn_t
            With a CU-masked side stream (bench --cu-split) the two split the
            chip.  side_learn=m runs the learn of the last m agents on the side
            stream behind its env step and draws (those CUs idle otherwise):
              side:  ... sample_{t+1} (ev_env) learn_{t+1}[NA-m, NA)
              main:  [wait ev_env] learn_{t+1}[0, NA-m)

  "learn"   the replay draws of step t run on a side stream beside learn t-1
            (everything else on one stream).  For the shared net (C5): its S'
            pass leaves room on every CU for a sampler block, so the draws
            (latency-bound, one block per env) hide behind the learn.
              side:  [wait env_step_{t-1}] sample_t (ev_s)
              main:  env_step_t [wait ev_s] learn_t

What a step returns or exposes per step (obs, reward, loss, agent.actions,
agent.idx) is fresh or double-buffered, so the caller may read it on its own
stream between steps (under "env" with side_learn, read the loss through
last_loss, or call sync_outputs() before reading agent tensors: the side
learn's part is waited for lazily, except on collect_stats steps).  Persistent env/agent state (sim arrays, RNG streams) is
advanced by the next step's side stream without waiting for such reads: read
it host-blocking (.cpu()), and call join_streams() after writing it.
"""
from dataclasses import dataclass

import torch

from . import _lib
from .agent import AgentConfig, BatchedDQN
from .env import EnvConfig, TrafficEnv


SCHEDULES = ("none", "sample", "full", "env", "learn")


@dataclass
class StepStats:
    loss_launched: bool
    done: bool


class Trainer:
    def __init__(self, env_cfg: EnvConfig = None, agent_cfg: AgentConfig = None, device="cuda",
                 overlap="none", side_stream=None, split_learn=False, fused=True,
                 war_events=True, side_learn=0, mark_every_learn=False):
        self.env = TrafficEnv(env_cfg or EnvConfig(), device=device)
        if overlap is True or overlap is False:
            overlap = "full" if overlap else "none"
        if overlap not in SCHEDULES:
            raise ValueError(f"overlap must be one of {SCHEDULES}")
        self.overlap = overlap
        # side_stream: e.g. a CU-masked stream (_lib.cu_masked_stream), so the
        # side work and the learn split the chip instead of sharing CU slots
        self.side = None
        if overlap != "none":
            self.side = side_stream if side_stream is not None else torch.cuda.Stream(self.env.device)
        self._ev_store = self._ev_learn = None
        self._side_pending = None  # overlap "env": the side learn, waited for lazily
        self._ev_env_prev = None  # overlap "learn": the last env step
        self._join = True  # the side stream's first work waits for everything before it
        self.agent = BatchedDQN(self.env.E, self.env.A, agent_cfg or AgentConfig(), device=device,
                                env_seeds=self.env.seeds)
        # overlap "learn": the sampler's LDS is what the shared learn's S' pass
        # leaves of a CU, so one sampler block runs beside each S' workgroup
        # (with the default four-blocks-per-CU budget the two serialise); the
        # CU's LDS is the device's (160 KB on gfx950), and the launcher clamps
        # the budget to what one workgroup may hold
        self._sampler_lds = 0
        if overlap == "learn" and self.agent.shared:
            self._sampler_lds = max(0, _lib.device_lds_per_cu(self.env.device)
                                    - _lib.learn_shared_lds_bytes())
        # split_learn (agent.set_split_learn): the learn as two launches so its
        # Adam half can share the chip with the next step's side-stream work
        # (overlap "full").  Off by default: measured at C2 (round 3), the
        # overlapped sim / act ran 2x / 6x slower beside the bandwidth-bound
        # Adam and the step lost 3 % (3.01 vs 3.09 M steps/s).
        if split_learn:
            self.agent.set_split_learn(True)
        # fused: act + env step + remember as one launch (TrafficEnv.step_fused)
        # on the one-stream schedules; "full" splits them across its streams
        self.fused = bool(fused) and overlap != "full" and self.agent.ring.row_format == "int8"
        if overlap == "env" and not self.fused:
            raise ValueError('overlap "env" runs the fused env step (int8 replay rows, fused=True)')
        # overlap "env": the learn of the last `side_learn` agents runs on the
        # side stream behind the env step and the draws (its CUs idle
        # otherwise while the learn stream works), the rest on the learn
        # stream; independent agents, so the results are the same
        self.side_learn = int(side_learn)
        if self.side_learn:
            if overlap != "env":
                raise ValueError('side_learn runs with overlap "env"')
            if self.agent.shared or not 0 < self.side_learn < self.agent.NA:
                raise ValueError("side_learn: independent nets, 0 < side_learn < E*A")
        # overlap "env" at a fixed epsilon of 1 (A-1: the side stream never reads
        # a learn's output): the learn -> side-stream wait only orders the store
        # of t+2 after learn t's ring reads, so it uses ordering-only events
        # (_lib.OrderEvent, no cache write-back between the learns) from a ring
        # (more events than marks can be alive: a wait never meets a re-record)
        self._war_ring = ([_lib.OrderEvent() for _ in range(max(4, self.agent.ring.spare + 2))]
                          if war_events and overlap == "env" else None)
        self._war_i = 0
        # overlap "env": (call index, event) of the learns the side stream may
        # wait for, newest last.  The store of call k overwrites the slot of
        # store k - slots, which the learns of calls up to k - 1 - spare read
        # (kernels.ReplayRing, spare = AgentConfig.ring_spare), so env step k
        # waits for the newest marked learn of a call <= k - 2 -- never learn
        # k - 1, beside which it runs.  Any learn of calls k - 1 - spare ..
        # k - 2 will do, so under ordering-only events the learn stream marks
        # every spare-th learn, and the side stream runs up to `spare` env
        # steps ahead (C3 / C2 measured faster with 2 than with a mark per
        # learn: profiles/r06/c3_marks, c2_marks).
        self._marks = []
        self._calls = 0
        self.n_marks = 0  # marked calls that learned (tests: every spare-th learn)
        self._mark_every = bool(mark_every_learn)  # A/B: a marker behind every learn
        self.obs = self.env.reset()
        self.episode = 0
        self.step_count = 0
        self.total_steps = 0
        self.last_loss = None
        self.last_reward = None
        self._debug = bool(_lib.load().dmdqn_debug_build())

    def step(self, collect_stats=False):
        """One loop iteration for every replica; collect_stats makes the learn
        also produce the metrics of dqn_agent.py:361-370 (agent.learn_metrics).
        Under the debug-bounds build (DMDQN_VARIANT=debug) every step ends with
        a device sync and the kernels' range checks."""
        if self._debug:
            st = self._step(collect_stats)
            _lib.debug_check()
            return st
        return self._step(collect_stats)

    def _step(self, collect_stats):
        if self.overlap == "full":
            return self._step_overlap(collect_stats)
        if self.overlap == "env":
            return self._step_env_beside_learn(collect_stats)
        if self.overlap == "sample":
            return self._step_side_sample(collect_stats)
        if self.overlap == "learn":
            return self._step_sample_beside_learn(collect_stats)
        env, agent = self.env, self.agent
        next_obs, reward, done, info = self._env_side()
        loss = agent.learn(collect_stats=collect_stats)
        self.last_loss, self.last_reward = loss, reward
        self.obs = self._after_step(done, next_obs, info)
        return StepStats(loss is not None, done)

    def _env_side(self):
        """act -> env step -> remember (train.py:211-282), fused or as three calls."""
        env, agent = self.env, self.agent
        if self.fused:
            eps, greedy, out = agent.act_inputs(self.obs)
            res = env.step_fused(agent.np_state, eps, greedy, out, agent.ring, self.obs)
            agent.remembered()
            return res
        actions = agent.act(self.obs)                          # train.py:211-222
        next_obs, reward, done, info = env.step(actions)       # train.py:225-270
        agent.remember(self.obs, actions, reward, next_obs, info["done"])  # train.py:274-282
        return next_obs, reward, done, info

    def _step_side_sample(self, collect_stats):
        env, agent, side = self.env, self.agent, self.side
        main = torch.cuda.current_stream(env.device)
        if self._join:
            side.wait_stream(main)
            self._join = False
        elif self._ev_learn is not None:
            side.wait_event(self._ev_learn)  # learn t-1 done: nothing beside the next learn
        ev_s = None
        with torch.cuda.stream(side):
            if agent.presample(min(agent.ring.total + 1, agent.ring.cap)):
                ev_s = torch.cuda.Event()
                ev_s.record(side)
        next_obs, reward, done, info = self._env_side()
        if ev_s is not None:
            main.wait_event(ev_s)
        loss = agent.learn(collect_stats=collect_stats)
        self._ev_learn = torch.cuda.Event()
        self._ev_learn.record(main)
        self.last_loss, self.last_reward = loss, reward
        self.obs = self._after_step(done, next_obs, info)
        return StepStats(loss is not None, done)

    def _step_sample_beside_learn(self, collect_stats):
        env, agent, side = self.env, self.agent, self.side
        main = torch.cuda.current_stream(env.device)
        if self._join:
            side.wait_stream(main)
            self._join = False
        elif self._ev_env_prev is not None:
            # env step t-1 done: these draws run beside learn t-1.  They read
            # only the CPython stream and the ring length after this step's
            # store; the index buffer they fill was last read three learns
            # back (agent.OUT_BUFS rotation), before env step t-1
            side.wait_event(self._ev_env_prev)
        ev_s = None
        with torch.cuda.stream(side):
            if agent.presample(min(agent.ring.total + 1, agent.ring.cap),
                               lds_budget=self._sampler_lds):
                ev_s = torch.cuda.Event()
                ev_s.record(side)
        next_obs, reward, done, info = self._env_side()
        self._ev_env_prev = torch.cuda.Event()
        self._ev_env_prev.record(main)
        if ev_s is not None:
            main.wait_event(ev_s)
        loss = agent.learn(collect_stats=collect_stats)
        self.last_loss, self.last_reward = loss, reward
        self.obs = self._after_step(done, next_obs, info)
        return StepStats(loss is not None, done)

    def _step_overlap(self, collect_stats):
        env, agent, side = self.env, self.agent, self.side
        main = torch.cuda.current_stream(env.device)
        if self._join:  # first step, or the caller touched state on its stream
            side.wait_stream(main)
            self._join = False
        elif self._ev_store is not None:
            side.wait_event(self._ev_store)  # remember t-1 has read obs/actions/reward
        if agent.current_epsilon() < 1.0 and self._ev_learn is not None:
            side.wait_event(self._ev_learn)  # greedy act reads the updated weights
        with torch.cuda.stream(side):
            actions = agent.act(self.obs)                          # train.py:211-222
            next_obs, reward, done, info = env.step(actions)       # train.py:225-270
            agent.presample(min(agent.ring.total + 1, agent.ring.cap))
            ev_obs = torch.cuda.Event()
            ev_obs.record(side)
        main.wait_event(ev_obs)
        for t in (self.obs, next_obs, reward, env.local):
            t.record_stream(main)  # side-allocated, read on main
        agent.remember(self.obs, actions, reward, next_obs, info["done"])  # train.py:274-282
        self._ev_store = torch.cuda.Event()
        self._ev_store.record(main)
        loss = agent.learn(collect_stats=collect_stats)
        self._ev_learn = torch.cuda.Event()
        self._ev_learn.record(main)
        self.last_loss, self.last_reward = loss, reward
        self.obs = self._after_step(done, next_obs, info, side=side, main=main)
        return StepStats(loss is not None, done)

    def _step_env_beside_learn(self, collect_stats):
        env, agent, side = self.env, self.agent, self.side
        main = torch.cuda.current_stream(env.device)
        if self._join:  # first step, or the caller touched state on its stream
            side.wait_stream(main)
            self._join = False
        k = self._calls
        self._calls += 1
        spare = agent.ring.slots - agent.ring.cap
        marks = [m for m in self._marks if m[0] <= k - 2]
        if k - 1 - spare >= 0 and not (marks and marks[-1][0] >= k - 1 - spare):
            # (every call k' has a mark in [k' - 1 - spare, k' - 2]: see below)
            raise RuntimeError(f"env schedule: no mark covers call {k - 1 - spare}")
        if marks:
            j, ev = marks[-1]
            # call k - 1 - spare must be covered -- its learn's ring reads and
            # the caller's reads of its outputs, queued on main before the mark
            # of any later call (the main stream is in order: the wait covers
            # every earlier call too)
            if isinstance(ev, _lib.OrderEvent):
                ev.wait(side)
            else:
                side.wait_event(ev)
        self._marks = [m for m in self._marks if m[0] >= k - 1 - spare]
        if agent.current_epsilon() < 1.0 and self._ev_learn is not None:
            # greedy act reads the updated weights (recorded as a full event:
            # an ordering-only one is used only while epsilon is fixed at 1)
            side.wait_event(self._ev_learn)
        with torch.cuda.stream(side):
            next_obs, reward, done, info = self._env_side()
            agent.presample(len(agent.ring))
            self.obs = self._after_step(done, next_obs, info)  # (an episode reset: on side)
            ev_env = torch.cuda.Event()
            ev_env.record(side)
        learned = agent.learn_begin(collect_stats)  # the draws above, the Adam constants
        ev_side = None
        if learned and self.side_learn:
            with torch.cuda.stream(side):
                agent.learn_range(agent.NA - self.side_learn, agent.NA)
                ev_side = torch.cuda.Event()
                ev_side.record(side)
        main.wait_event(ev_env)  # the store learn t reads; what the caller reads after step()
        # side-allocated outputs the caller reads on main: without
        # this the allocator could hand their blocks to step t+2's side work
        # while a main-stream read of them is still queued
        for t in (next_obs, reward, env.local, self.obs):
            t.record_stream(main)
        loss = None
        if learned:
            loss = agent.learn_range(0, agent.NA - self.side_learn)
        war = (self._war_ring is not None and not agent.cfg.count_env_steps
               and agent.current_epsilon() >= 1.0)
        if war and spare >= 2 and not self._mark_every and k % spare:
            # under ordering-only events only every spare-th call is marked
            # (whether or not it learned: the mark also orders the side
            # stream's reuse of the per-step output buffers after the caller's
            # reads of them): any `spare` consecutive calls hold a mark, so
            # the newest mark of a call <= k' - 2 always covers call
            # k' - 1 - spare (checked above)
            pass
        elif war:
            # epsilon cannot fall below 1 later (count_env_steps off): no act
            # will read this learn's weights through the side stream.  What the
            # side stream reads of main's work is then nothing: the side learn
            # (side_learn) reads only its own agents' weights, rings and draws,
            # all written on the side stream -- so an ordering-only event
            # (write after read: the store of t+2 after learn t's ring reads)
            # is enough.  A data hand-over main -> side takes a full event.
            if not self._side_reads_nothing_from_main():  # (not an assert: kept under -O)
                raise RuntimeError("ordering-only learn event with a read-after-write hazard")
            ev = self._war_ring[self._war_i]
            self._war_i = (self._war_i + 1) % len(self._war_ring)
            ev.record(main)
            self._ev_learn = ev
            self._marks.append((k, ev))
            self.n_marks += learned
        else:
            self._ev_learn = torch.cuda.Event()
            self._ev_learn.record(main)
            self._marks.append((k, self._ev_learn))
            self.n_marks += learned
        # the side learn's outputs (its agents' loss, stats and weights) for the
        # caller's stream.  The next learn needs no wait for them: the side
        # stream runs the next env step behind the side learn, and the next
        # learn waits for that.  So a step with stats (their readers follow at
        # once) waits here; otherwise the wait is left to the caller's reads
        # (the last_loss property, sync_outputs()) -- a barrier packet less per
        # step on the learn stream (C2 +2.5 %)
        self._side_pending = None
        if ev_side is not None:
            if collect_stats:
                main.wait_event(ev_side)
            else:
                self._side_pending = ev_side
        self.last_loss, self.last_reward = loss, reward
        return StepStats(loss is not None, done)

    @property
    def last_loss(self):
        """The last learn's per-agent losses (None before the first learn),
        complete on the caller's current stream."""
        self.sync_outputs()
        return self._last_loss

    @last_loss.setter
    def last_loss(self, v):
        self._last_loss = v

    def sync_outputs(self):
        """Make the current stream wait for the last step's side-stream learn
        (schedule "env" with side_learn), so the agent's loss, stats and
        weights read on it are complete.  A no-op otherwise."""
        if getattr(self, "_side_pending", None) is not None:
            torch.cuda.current_stream(self.env.device).wait_event(self._side_pending)

    def _side_reads_nothing_from_main(self):
        """The "env" schedule's invariant for ordering-only learn events: no
        greedy act (its forward reads the learn stream's weights) and the side
        learn's agent range [NA - side_learn, NA) disjoint from the learn
        stream's [0, NA - side_learn) (no side learn for the shared net, whose
        one learn reads every agent)."""
        ag = self.agent
        return (ag.current_epsilon() >= 1.0 and not ag.cfg.count_env_steps
                and 0 <= self.side_learn < ag.NA and not (ag.shared and self.side_learn))

    def _after_step(self, done, next_obs, info, side=None, main=None):
        """Counters and the observation the next act sees (train.py:188-209).
        Replicas that restart on their own `done` (env.drains_early) were reset
        by env.step itself: info["obs_next"] already holds their restart state.
        Otherwise every replica ends together, and the whole batch reloads."""
        env, agent = self.env, self.agent
        self.step_count += 1
        self.total_steps += 1
        if "obs_next" in info:
            if info["restarted"].any():
                agent.ring.check()  # episode boundary: every store so far was exact
                self.episode = int(env.env_episodes.min())
                self.step_count = int(env.env_steps.min())
            return info["obs_next"]
        if not done:
            return next_obs
        agent.ring.check()  # episode boundary: every store so far was exact
        self.episode += 1                                      # train.py:188-190
        self.step_count = 0
        if side is None:
            return env.reset()
        with torch.cuda.stream(side):
            obs = env.reset()
        main.wait_stream(side)
        obs.record_stream(main)
        env.local.record_stream(main)
        return obs

    def join_streams(self):
        """Call after changing trainer state on the caller's stream between
        steps (checkpoint restore, weight loads): the next step's side-stream
        work then waits for it.  Also orders the caller's stream after the
        last side-stream learn (schedule "env" with side_learn), so later
        caller-side writes cannot race it; call quiesce() BEFORE such writes."""
        self.sync_outputs()
        self._side_pending = None
        self._join = True

    def quiesce(self):
        """Order the caller's stream after every piece of trainer work queued
        so far on any stream (the side stream's env step, draws and side
        learn), so the caller may overwrite trainer state on it (checkpoint
        restore).  No host block."""
        self.sync_outputs()
        self._side_pending = None
        if self.side is not None:
            torch.cuda.current_stream(self.env.device).wait_stream(self.side)

    def agent_env_steps(self, n_steps):
        return n_steps * self.env.E * self.env.A

    def synchronize(self):
        """Wait for all device work, and (C5 over RCCL) first for every
        outstanding gradient all-reduce, bounded: a peer that stalled on or
        skipped one raises DistError instead of hanging the synchronize."""
        self.agent.drain_collectives()
        torch.cuda.synchronize(self.env.device)
