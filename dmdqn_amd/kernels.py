"""Thin torch-facing wrappers over the custom operators torch.ops.dmdqn.*
(device tensors in, device tensors out).

PyTorch is used only for device memory and the current HIP stream; every op
below is one (or a few) launches of a hand-written gfx950 kernel in
libdmdqn_hip.so, through the TORCH_LIBRARY(dmdqn) registration (ops.py), on
torch's current stream.
"""
import time

import torch

from . import _lib
from .ops import load as _ops

MT_WORDS = 625
OBS_DIM = 89
LOCAL_DIM = 17
ROW_BYTES = 128  # include/dmdqn.h DMDQN_ROW_BYTES (s' rows carry a, done, r at 96/97/104)
ROW_FLOATS = 96  # DMDQN_ROW_FLOATS: float rows (the drop-in surface)


def _check(t, dtype, shape=None, name="tensor"):
    if not t.is_cuda:
        raise ValueError(f"{name} must be a device tensor")
    if t.dtype != dtype:
        raise TypeError(f"{name} must be {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    if shape is not None and tuple(t.shape) != tuple(shape):
        raise ValueError(f"{name} shape {tuple(t.shape)} != {tuple(shape)}")


# ------------------------------------------------------------------ streams
def seed_streams(seeds, kind, device="cuda"):
    """Device MT19937 streams, one per env.  kind 'np' (numpy RandomState.seed)
    or 'py' (CPython random.seed).  Returns uint32-as-int32 [E, 625]."""
    seeds = torch.as_tensor(seeds, dtype=torch.int64).to(device).contiguous()
    E = seeds.numel()
    st = torch.empty((E, MT_WORDS), dtype=torch.int32, device=device)
    _ops().mt_seed(st, seeds, "np" if kind == "np" else "py")
    return st


def draw_u32(state, count):
    E = state.shape[0]
    out = torch.empty((E, count), dtype=torch.int32, device=state.device)
    _ops().mt_draw_u32(state, count, out)
    return out


# ------------------------------------------------------------------ act
def act(np_state, A, eps=1.0, n_actions=4, greedy=None, out=None, uniform=False):
    """select_action's draws for E envs x A agents (dqn_agent.py:263-265).
    uniform=True: np.random.randint(0, n_actions) alone per agent, the draw of
    the reference evaluation's random mode (src/scripts/test.py:92-93)."""
    E = np_state.shape[0]
    _check(np_state, torch.int32, (E, MT_WORDS), "np_state")
    if out is None:
        out = torch.empty((E, A), dtype=torch.int32, device=np_state.device)
    if greedy is not None:
        _check(greedy, torch.int32, (E, A), "greedy")
    _ops().act(np_state, A, float(eps), n_actions, greedy, out, bool(uniform))
    return out


# ------------------------------------------------------------------ observe
def observe(R, C, halt, phase, tspent, mode, prev_local=None, want_obs=True):
    E = halt.shape[0]
    A = R * C
    _check(halt, torch.int32, (E, A, 12), "halt")
    _check(phase, torch.int32, (E, A), "phase")
    _check(tspent, torch.int32, (E, A), "tspent")
    dev = halt.device
    local = torch.empty((E, A, LOCAL_DIM), dtype=torch.float32, device=dev)
    obs = torch.empty((E, A, OBS_DIM), dtype=torch.float32, device=dev) if want_obs else None
    reward = None
    if prev_local is not None:
        _check(prev_local, torch.float32, (E, A, LOCAL_DIM), "prev_local")
        reward = torch.empty((E, A), dtype=torch.float64, device=dev)
    _ops().observe(R, C, halt, phase, tspent, int(mode), local, obs, prev_local, reward)
    return local, obs, reward


# ------------------------------------------------------------------ replay
class ReplayRing:
    """Device replay rings for NA agents (ReplayBuffer, dqn_agent.py:27-89).

    Each agent keeps the last `cap` transitions (the deque's maxlen) in
    `slots` = cap + SPARE physical ring slots: deque position p (0 = oldest)
    lives in slot (start + p) % slots and the next stores go to the SPARE
    slots no position maps to, total % slots -- so the stores of steps t+1
    and t+2 never touch a slot the learn of step t may read (trainer overlap
    "env": the side stream's env step k waits only for learn k - 1 - SPARE,
    and the learn stream records its ordering event every other learn).  All
    agents add in lockstep, so one host-side counter describes every ring.

    row_format "int8" (the batched path): 128-byte int8 rows, exact for this
    environment's integer features, anything else raises.  "f32" (the
    per-agent drop-in surface): float32 rows of ROW_FLOATS, every value kept
    as the reference's buffer keeps it (dqn_agent.py:39-56)."""

    # default physical slots beyond the deque's maxlen (round 5: 1; round 6: 16
    # -- the env schedule's side stream then runs up to 16 env steps ahead and
    # the learn stream marks every 16th learn: C3 +1.9 %, C2 +1.8 % over 2
    # slots, same box, profiles/r06/ring_spare; the agent's output buffers
    # rotate over ring_spare + 2, BatchedDQN.OUT_BUFS)
    SPARE = 16

    def __init__(self, NA, cap, device="cuda", row_format="int8", spare=None):
        if row_format not in ("int8", "f32"):
            raise ValueError("row_format must be 'int8' or 'f32'")
        spare = self.SPARE if spare is None else int(spare)
        if spare < 1:
            raise ValueError("a replay ring needs at least one spare slot")
        self.NA, self.cap, self.row_format, self.spare = NA, cap, row_format, spare
        self.slots = S = cap + spare
        z = dict(device=device)
        if row_format == "f32":
            self.s = torch.zeros((NA, S, ROW_FLOATS), dtype=torch.float32, **z)
            self.n = torch.zeros((NA, S, ROW_FLOATS), dtype=torch.float32, **z)
        else:
            self.s = torch.zeros((NA, S, ROW_BYTES), dtype=torch.int8, **z)
            self.n = torch.zeros((NA, S, ROW_BYTES), dtype=torch.int8, **z)
        self.a = torch.zeros((NA, S), dtype=torch.uint8, **z)
        self.r = torch.zeros((NA, S), dtype=torch.float64, **z)
        self.d = torch.zeros((NA, S), dtype=torch.uint8, **z)
        # the range flag lives in pinned host memory, written by the store kernel
        # itself (zero-copy; only on an error): polling it needs no copy launch
        if torch.device(device).type == "cuda":
            self.err = torch.zeros(1, dtype=torch.int32, pin_memory=True)
        else:
            self.err = torch.zeros(1, dtype=torch.int32, **z)
        self.device = torch.device(device)
        self.total = 0
        self._err_events = None  # the event recorded behind a store every POLL_LAG polls
        self._poll_i = 0

    def __len__(self):
        return min(self.total, self.cap)

    @property
    def start(self):
        """Slot of deque position 0."""
        return (self.total - len(self)) % self.slots

    @property
    def next_slot(self):
        """The slot the next store writes."""
        return self.total % self.slots

    def slots_of(self, pos):
        """Ring slots of deque positions pos (int or array)."""
        return (self.start + pos) % self.slots

    def store(self, obs_s, obs_n, act, rew, done):
        NA = self.NA
        _check(obs_s, torch.float32, (NA, OBS_DIM), "obs_s")
        _check(obs_n, torch.float32, (NA, OBS_DIM), "obs_n")
        _check(act, torch.int32, (NA,), "act")
        _check(rew, torch.float64, (NA,), "rew")
        _check(done, torch.uint8, (NA,), "done")
        slot = self.next_slot
        if self.row_format == "f32":
            _ops().replay_store_f32(slot, obs_s, obs_n, act, rew, done, self.s, self.n, self.a,
                                    self.r, self.d)
        else:
            _ops().replay_store(slot, obs_s, obs_n, act, rew, done, self.s, self.n, self.a,
                                self.r, self.d, self.err)
        self.advance()

    def advance(self):
        """One transition per agent was written at slot next_slot (store(), or
        a fused env step, env.TrafficEnv.step_fused)."""
        self.total += 1

    def gather_f32(self, idx, xs, xn):
        """Float rows: the batch of deque positions idx [NA, batch] -> xs / xn
        [NA, batch, ROW_FLOATS] in batch order (the learn reads them there)."""
        _ops().replay_gather_f32(self.s, self.n, idx, self.start, xs, xn)

    def check(self):
        """Raise if a stored value was not exactly representable (syncs the
        current stream, behind every store issued on it).  Float rows hold any
        value: nothing to check."""
        if self.row_format == "f32":
            return
        if self.err.is_pinned():
            torch.cuda.current_stream(self.device).synchronize()
        if int(self.err[0]) != 0:
            raise _lib.DmdqnError(_RANGE_MSG)

    def poll(self):
        """Deferred check without stalling the stream.  The store kernels write
        the (sticky) flag straight into pinned host memory.  Every POLL_LAG-th
        poll waits for the event recorded POLL_LAG polls earlier (behind that
        poll's store), reads the flag, raises if it is set, and records a new
        event: a bad store raises at most 2 POLL_LAG - 1 polls later (the
        product path polls after every store), the host keeps up to ~POLL_LAG
        steps of work queued ahead of the GPU, and the queue carries one event
        marker per POLL_LAG steps (each costs the GPU a few microseconds).
        Episode ends and checkpoint saves call check(), which waits.  The
        reference stores float32 rows (dqn_agent.py:39-56), and this build's
        int8 rows must never silently hold a rounded value."""
        if self.row_format == "f32":
            return
        if not self.err.is_pinned():  # a CPU-device ring: nothing in flight
            self.check()
            return
        self._poll_i += 1
        if self._poll_i % POLL_LAG:
            return
        if self._err_events is None:
            self._err_events = torch.cuda.Event()
            self._err_live = False
        stream = torch.cuda.current_stream(self.device)  # the ring's device, not the current one
        ev = self._err_events
        if self._err_live:
            t0 = time.perf_counter()
            ev.synchronize()  # recorded POLL_LAG polls ago: complete unless the host is ahead
            POLL_WAIT_S[0] += time.perf_counter() - t0
            if int(self.err[0]) != 0:
                raise _lib.DmdqnError(_RANGE_MSG)
        ev.record(stream)
        self._err_live = True


POLL_LAG = 4  # steps the host may run ahead of the replay range check
# host seconds spent blocked in poll() (bench.py: the host's own issue cost is
# the issue time minus this -- a host POLL_LAG steps ahead of the GPU waits here)
POLL_WAIT_S = [0.0]


_RANGE_MSG = ("replay_store: an observation value is not an integer in [-128, 127]; the int8 "
              "replay rows store this env's features exactly and refuse anything else")


def replay_sample(py_state, A, n, k=128, out=None, lds_budget=0):
    """ReplayBuffer.sample for E x A agents (dmdqn_replay_sample); lds_budget
    (bytes, 0 = default) bounds the sampler block's LDS, e.g. to run beside
    the shared learn (trainer schedule "learn"); the draws do not depend on it."""
    E = py_state.shape[0]
    _check(py_state, torch.int32, (E, MT_WORDS), "py_state")
    if out is None:
        out = torch.empty((E * A, k), dtype=torch.int32, device=py_state.device)
    _ops().replay_sample(py_state, A, int(n), int(k), out, int(lds_budget))
    return out
