/* dmdqn.h -- C ABI of the MI355X-native dmdqn hot path (libdmdqn_hip.so).
 *
 * Every entry point takes plain device pointers + sizes and a hipStream_t
 * (passed as void*; NULL = default stream), launches asynchronously on that
 * stream and returns 0 on success or a negative DMDQN_E* code.  Argument
 * errors are detected on the host before any launch; the message is then
 * available from dmdqn_last_error().  No torch types cross this boundary.
 *
 * Units: E envs (replicas) per process, A agents (junctions, row-major J_r_c)
 * per env, NA = E*A agent slots.  One "agent-env step" = one agent in one env
 * completing one iteration of the reference loop (src/scripts/train.py:207-310).
 *
 * Which reference interface each entry point replaces is cited per function.
 * The reference itself has no FFI (it is pure Python over TraCI/Keras); the
 * ctypes binding a maintainer would add is shown in INTEGRATION.md.
 */
#ifndef DMDQN_H
#define DMDQN_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DMDQN_OK 0
#define DMDQN_EINVAL -1   /* bad argument (shape / size / null pointer)        */
#define DMDQN_EHIP -2     /* HIP runtime error at launch                       */
#define DMDQN_ERANGE -3   /* value not representable in the chosen storage    */

/* Number of 32-bit words of one MT19937 stream on the device: 624 state words
 * followed by the position word (mti). */
#define DMDQN_MT_WORDS 625
/* Observation / local-state sizes (order_lanes.py:497, :554). */
#define DMDQN_OBS_DIM 89
#define DMDQN_LOCAL_DIM 17
/* Replay rows: one 128-byte line per stored observation (int8 features 0..88,
 * zero to byte 95).  The s' row of a transition also carries the transition's
 * action (byte DMDQN_ROW_A), done flag (DMDQN_ROW_D) and f64 reward (bytes
 * DMDQN_ROW_R..+7), so a sampled transition is one aligned line of s' plus one
 * of s -- no scattered reads of the per-slot arrays in the learn kernels. */
#define DMDQN_ROW_BYTES 128
#define DMDQN_ROW_A 96
#define DMDQN_ROW_D 97
#define DMDQN_ROW_R 104
/* Float replay rows (the per-agent drop-in surface, any observation value, as
 * ReplayBuffer.add stores it, dqn_agent.py:39-56): DMDQN_ROW_FLOATS f32 per
 * row (features 0..88, zero to 95); a, done and r live in the per-slot arrays
 * only.  dmdqn_learn_args.row_format selects them. */
#define DMDQN_ROW_FLOATS 96
#define DMDQN_ROWS_I8 0
#define DMDQN_ROWS_F32 1

const char *dmdqn_last_error(void);
/* ABI version.  4 (round 6): version 3 plus dmdqn_source_digest and
 * dmdqn_device_lds_per_cu; dmdqn_replay_sample_budget clamps lds_budget to the
 * device's per-workgroup LDS.  3 (round 5): dmdqn_adam_slabs (the slab reduction and the
 * Adam step of the shared net in one launch), dmdqn_learn_shared_grad with
 * grad == NULL (the slabs left for it), dmdqn_replay_sample_budget and
 * dmdqn_learn_shared_lds_bytes.  2 (round 4/5): the replay ring arguments `cap` of the learn,
 * gather and store entry points are the PHYSICAL slot count of the ring -- a
 * deque of maxlen N lives in N + k slots, k >= 1 (position p at slot (start +
 * p) % (N + k), the next stores in the k slots no position maps to; the Python
 * ring uses k = 2 since round 6, k = 1 before), so a caller passes N + k; dmdqn_learn_shared_grad requires `work`; dmdqn_sim_step takes
 * action < 0 as "no setPhase".  1: cap = maxlen, work optional. */
int dmdqn_version(void);

/* The digest of the sources this library was built from (16 hex chars:
 * dmdqn_amd/build.py tree_digest over csrc/, the include/ headers and the operator
 * library's source, plus the common compile flags), generated at build time.
 * The Python loader refuses a library whose digest is not the tree's, so a
 * stale prebuilt .so cannot run as current code. */
const char *dmdqn_source_digest(void);

/* The LDS of one CU of `device` (hipDeviceAttributeMaxSharedMemoryPerMultiprocessor):
 * the trainer sizes a sampler block to run beside the shared learn's S' pass
 * with it.  0 or DMDQN_EINVAL / DMDQN_EHIP. */
int dmdqn_device_lds_per_cu(int device, size_t *out);

/* Debug-bounds build (libdmdqn_hip_debug.so, -DDMDQN_DEBUG_BOUNDS): kernels
 * check the ring slots, edges, replay indices and stored actions they derive,
 * clamp a bad one and record it.  dmdqn_debug_status() returns the OR of the
 * recorded DBG_* bits (dmdqn_amd/csrc/common.hpp: 1 sim ring, 2 sim edge,
 * 4 sample index, 8 learn index, 16 learn action) and clears them; it waits
 * for the device (hipMemcpyFromSymbol) and returns -1 on a HIP error.  Always
 * 0 in the normal build; dmdqn_debug_build() says which build this is. */
int dmdqn_debug_status(void);
int dmdqn_debug_build(void);

/* Run-time options: the test / A-B hooks of the launchers.  Each is read from
 * the environment ONCE, when the library loads, and changes afterwards only
 * through dmdqn_set_option (no launch reads the environment):
 *   DMDQN_OPT_SIM_PATH (env DMDQN_SIM_PATH = reg | lds | global): force the
 *     simulator's kernel path; 0 = auto (the launcher's choice by grid size),
 *     1 = register lanes, 2 = LDS image, 3 = global memory.
 *   DMDQN_OPT_SAMPLE_TLOG (env DMDQN_SAMPLE_TLOG = n): cap the replay
 *     sampler's first-lane table at 2^n entries, 0 <= n <= 20 (forces
 *     collisions); 32 = no cap (default).
 * dmdqn_set_option returns 0 or DMDQN_EINVAL (unknown option or value);
 * dmdqn_get_option returns the current value (DMDQN_EINVAL for an unknown
 * option).  Neither is synchronised with launches issued by other host
 * threads. */
#define DMDQN_OPT_SIM_PATH 0
#define DMDQN_OPT_SAMPLE_TLOG 1
int dmdqn_set_option(int option, int value);
int dmdqn_get_option(int option);

/* A HIP stream (returned in *stream as hipStream_t) whose kernels run only on
 * the CUs set in mask[n_words] (CU i = bit i % 32 of word i / 32).  The
 * trainer's optional split schedule runs the next step's act / sim / observe /
 * sample on such a stream beside the learn on the complementary one.  No
 * reference counterpart (SUMO stepped in its own process). */
int dmdqn_stream_create_cumask(uint32_t n_words, const uint32_t *mask, void **stream);
int dmdqn_stream_destroy(void *stream);

/* Timing events for bench.py's per-launch kernel timing: a HIP event (in
 * *event, hipEvent_t) created with hipEventDisableSystemFence, so recording it
 * between two kernels adds no cache write-back / invalidate (a default timing
 * event's system-scope release cost C2's step ~11 us per learn).  Only for
 * timing: not for ordering streams or for host visibility.  elapsed: the time
 * between two recorded events in ms (both complete: synchronize first).  No
 * reference counterpart. */
int dmdqn_timing_event_create(void **event);
/* An ordering-only event (no timing, hipEventDisableSystemFence): a stream
 * waiting on it (dmdqn_stream_wait_event) starts after the work recorded
 * before it has COMPLETED, with no release of that work's writes -- for
 * write-after-read ordering (the trainer's env step of t+2 may overwrite ring
 * slots only after learn t has read them), never for handing data over. */
int dmdqn_order_event_create(void **event);
int dmdqn_stream_wait_event(void *stream, void *event);
int dmdqn_event_record(void *event, void *stream);
int dmdqn_event_synchronize(void *event);
int dmdqn_event_elapsed_ms(void *start, void *end, float *ms);
int dmdqn_event_destroy(void *event);

/* HBM streaming probe (round 5): bench.py times it once, outside the timed
 * region, on the learn's stream, and reports the learn's bandwidth as a
 * fraction of what this box streams in the same process.  mode 0: copy,
 * dst[i] = src[i] over n_bytes (n_bytes read, n_bytes written); mode 1:
 * triad, dst[i] = src[i] + src[n_bytes/4 + i] in f32 (src holds 2 * n_bytes:
 * 2 n_bytes read, n_bytes written); mode 2: read, n_bytes of src read, one
 * 16-B sum per thread written to dst (8 MiB per 256 CUs); modes 3..5: the
 * same with non-temporal loads and stores.  16-B aligned, n_bytes a multiple
 * of 16.  No reference counterpart. */
int dmdqn_stream_probe(void *dst, const void *src, size_t n_bytes, int mode, void *stream);

/* ------------------------------------------------------------------ streams
 * Seed E MT19937 streams on the device.
 *  _np: numpy legacy RandomState.seed(int) (init_genrand); replaces the global
 *       np.random stream drawn at src/agents/dqn_agent.py:263-265.
 *  _py: CPython random.seed(int) (init_by_array of the 32-bit words); replaces
 *       the global `random` stream drawn at src/agents/dqn_agent.py:63.
 * state: uint32 [E][DMDQN_MT_WORDS];  seeds: uint64 [E] (device memory). */
int dmdqn_mt_seed_np(uint32_t *state, const uint64_t *seeds, int E, void *stream);
int dmdqn_mt_seed_py(uint32_t *state, const uint64_t *seeds, int E, void *stream);

/* Draw `count` raw tempered uint32 outputs per stream (test hook). out [E][count]. */
int dmdqn_mt_draw_u32(uint32_t *state, int E, int count, uint32_t *out, void *stream);

/* ------------------------------------------------------------------ act
 * Replaces DQNAgent.select_action (src/agents/dqn_agent.py:246-274) for all
 * agents of all envs: per env, agents in junction order draw rand() then, if
 * rand() < eps, randint(0, n_actions) from the env's numpy stream; otherwise
 * take greedy[e*A+j] (argmax of the online Q, see dmdqn_q_argmax).
 * greedy may be NULL only when eps >= 1.  actions: int32 [E*A]. */
int dmdqn_act(uint32_t *np_state, int E, int A, double eps, int n_actions,
              const int32_t *greedy, int32_t *actions, void *stream);

/* A uniform action per agent drawn as np.random.randint(0, n_actions) alone
 * (no rand() first): the 'random' mode of the reference's evaluation script
 * (src/scripts/test.py:92-93).  Per env, agents in junction order. */
int dmdqn_act_uniform(uint32_t *np_state, int E, int A, int n_actions, int32_t *actions,
                      void *stream);

/* ------------------------------------------------------------------ observe
 * Replaces order_lanes.get_own_state (:430-499), build_state_vector (:502-555)
 * and the reward lines of train.py (:159-165, :254).
 *   halt   int32 [E][A][12]  halting vehicles per incoming lane (n,s,e,w x lane)
 *   phase  int32 [E][A]      current TL phase index
 *   tspent int32 [E][A]      seconds since the phase started
 *   mode   0 = reference (traci.junction.getType absent: [0,0,0,0], -1.0)
 *          1 = intended (PHASE_ENCODING one-hot, time spent)
 * Outputs (any may be NULL): local f32 [E][A][17], obs f32 [E][A][89].
 * reward f64 [E][A] is computed from prev_local (the PRE-step state, A-3);
 * pass prev_local = NULL to skip it. */
int dmdqn_observe(int R, int C, int E, const int32_t *halt, const int32_t *phase,
                  const int32_t *tspent, int mode, float *local, float *obs,
                  const float *prev_local, double *reward, void *stream);

/* ------------------------------------------------------------------ replay
 * Replaces ReplayBuffer.add (src/agents/dqn_agent.py:31-57): one transition
 * per agent into ring slot `slot` (capacity `cap`).  Observations are stored
 * as int8 rows of DMDQN_ROW_BYTES (exact for this env's integer features; a
 * non-representable value sets *err to DMDQN_ERANGE with a plain store, so
 * err may be device memory or pinned host memory the host polls without a
 * copy).  done: uint8 [NA].
 * ring_s / ring_n int8 [NA][cap][DMDQN_ROW_BYTES] (ring_n rows also receive
 * a, done and r at DMDQN_ROW_A / _D / _R); ring_a uint8 [NA][cap];
 * ring_r f64 [NA][cap]; ring_d uint8 [NA][cap] (the same values, per slot, for
 * the fp32 learn kernel and the host); err int32 [1] (device). */
int dmdqn_replay_store(int NA, int cap, int slot, const float *obs_s,
                       const float *obs_n, const int32_t *act, const double *rew,
                       const uint8_t *done, int8_t *ring_s, int8_t *ring_n,
                       uint8_t *ring_a, double *ring_r, uint8_t *ring_d,
                       int32_t *err, void *stream);

/* dmdqn_replay_store for float rows (DMDQN_ROWS_F32): rows_s / rows_n f32
 * [NA][cap][DMDQN_ROW_FLOATS], every value stored as given (the reference's
 * float32 buffer, dqn_agent.py:39-56); ring_a / ring_r / ring_d as above. */
int dmdqn_replay_store_f32(int NA, int cap, int slot, const float *obs_s, const float *obs_n,
                           const int32_t *act, const double *rew, const uint8_t *done,
                           float *rows_s, float *rows_n, uint8_t *ring_a, double *ring_r,
                           uint8_t *ring_d, void *stream);

/* The float-row learn's gather (ReplayBuffer.sample :63-64 on float rows):
 * xs / xn f32 [NA][batch][DMDQN_ROW_FLOATS] <- the rows of deque positions
 * idx [NA][batch] (slot = (start + pos) % cap), in batch order.  The learn
 * kernels then read X(S) / X(S') from xs / xn (dmdqn_learn_args.xs / .xn). */
int dmdqn_replay_gather_f32(const float *rows_s, const float *rows_n, const int32_t *idx,
                            int NA, int cap, int start, int batch, float *xs, float *xn,
                            void *stream);

/* Replaces random.sample(self.buffer, k) (dqn_agent.py:63): per env, agents
 * j = 0..A-1 in order draw k deque positions (0 = oldest) from a deque of
 * length n with CPython's algorithm on the env's `random` stream.
 * idx: int32 [E*A][k]. */
int dmdqn_replay_sample(uint32_t *py_state, int E, int A, int n, int k,
                        int32_t *idx, void *stream);
/* dmdqn_replay_sample with the sampler block's LDS held within lds_budget
 * bytes (0: the default, four blocks per CU) in the set branch (n > setsize,
 * the steady state): its first-lane table shrinks to fit -- slower on
 * collisions, the same draws.  The pool branch (n <= setsize, while a ring
 * fills) ignores the budget.  E.g. 160 KB less
 * dmdqn_learn_shared_lds_bytes() lets one sampler block per CU run beside the
 * shared learn's S' pass (trainer schedule "learn"). */
int dmdqn_replay_sample_budget(uint32_t *py_state, int E, int A, int n, int k, size_t lds_budget,
                               int32_t *idx, void *stream);

/* ------------------------------------------------------------------ simulator
 * Vectorised grid microsimulation that replaces SUMO behind train.py:225-236
 * (traci.trafficlight.setPhase x A, simulationStep x K, getTime,
 * getMinExpectedNumber) and the lane reads of order_lanes.py:449-482
 * (getLastStepHaltingNumber, getPhase, getNextSwitch, getPhaseDuration).
 *
 * Network: R x C grid of junctions J_r_c (row-major index a = r*C + c).
 * Edges: 4*A incoming approaches (edge id a*4+d, d = 0 n, 1 s, 2 e, 3 w: the
 * side the vehicle comes FROM) then X = 2R+2C exit edges (id 4A+x).  Each
 * edge has 3 lanes (lane id = edge*3 + k); NL = 3*(4A+X).  Per lane a ring of
 * cap_lane vehicle slots (front = head).  All arrays are device memory; the
 * layout is [E][...] with the per-env block contiguous. */
typedef struct dmdqn_sim {
    int32_t R, C, E, cap_lane;   /* grid, envs, slots per lane                 */
    int32_t period_ms, nveh;     /* demand: vehicle i departs at i*period_ms   */
    float *x, *v;                /* [E][NL][cap_lane] front position, speed     */
    int32_t *dst;                /* [E][NL][cap_lane] destination edge id       */
    int32_t *head, *cnt;         /* [E][NL] ring head / occupancy              */
    int32_t *req, *gfrom;        /* [E][NL] scratch: requested lane, granted src */
    float *fx, *fv;              /* [E][NL] scratch: front vehicle tentative    */
    int32_t *tl_phase, *tl_ts;   /* [E][A] TL phase index, phase start time     */
    int32_t *qptr;               /* [E][4A] next vehicle of each origin queue   */
    const int32_t *q_off;        /* [E][4A+1] origin-queue offsets into q_ids   */
    const uint16_t *q_ids;       /* [E][nveh] vehicle ids sorted (origin, id)  */
    const uint16_t *vdst;        /* [E][nveh] destination edge of vehicle i    */
    const int32_t *exit_id;      /* [A*4] exit id of (a, out-dir) or -1        */
    const int32_t *exit_ao;      /* [X][2] (a, out-dir) of exit x              */
    int32_t *stats;              /* [E][4] inserted, arrived, running, pending */
    const uint16_t *q_dst;       /* [E][nveh] vdst[q_ids[i]]: destination of the
                                    vehicle at queue position i                */
    int32_t actuated;            /* 1: SUMO's actuated gap-out on phase 0
                                    (grid_3x3.net.xml:894, minDur 5 maxDur 50;
                                    SURVEY A-14); 0: fixed durations (default) */
    int32_t *last_det;           /* [E][12A] substep of the last detection on each
                                    observed lane's detector (actuated mode; the
                                    reset writes -1000)                        */
    int32_t *t_env;              /* [E] each replica's episode clock (s), or NULL:
                                    every replica runs at the step's t0.  With it
                                    a replica restarts on its own `done`
                                    (dmdqn_sim_reset_envs) as the reference's one
                                    env does (train.py:188-207, 233-236); the
                                    step reads t0 from it and advances it by K */
} dmdqn_sim;

/* Car-following / geometry constants (SUMO passenger defaults + grid_3x3
 * geometry: grid_3x3.net.xml:652-891). */
typedef struct dmdqn_idm {
    float length, min_gap, accel, decel, tau, vmax, two_sqrt_ab, halt_speed;
    float len_inner, len_outer;  /* J->J lanes 172.8 m; END->J and J->END 86.4 m */
    float det_dist, max_gap;     /* actuated mode: detector distance upstream of
                                    the stop line (SUMO detector-gap 2 s x 13.89
                                    m/s) and the gap-out time (max-gap 3 s)    */
} dmdqn_idm;

/* Reset every env to t = 0: empty lanes, all TLs in phase 0 (started at 0),
 * origin queues rewound (replaces traci.load, train.py:190). */
int dmdqn_sim_reset(const dmdqn_sim *sim, void *stream);

/* dmdqn_sim_reset for the envs e with mask[e] != 0 only (uint8 [E], device):
 * the replicas whose episode ended restart while the others run on. */
int dmdqn_sim_reset_envs(const dmdqn_sim *sim, const uint8_t *mask, void *stream);

/* One RL step for every env (train.py:225-236): if actions != NULL set
 * phase = action_stride*action (ACTION_MAP {0:0,1:3,2:6,3:9}) with the phase
 * timer restarted at t0 -- except where action < 0: no setPhase for that
 * junction, its program runs on with its timer (the reference class skips
 * unmapped actions and an unchanged phase, sumo_env.py:491-530) -- then run K
 * one-second substeps from time t0 (with
 * sim->t_env: t0 = t_env[e] per replica, and t_env[e] += K).
 * With sim->actuated, phase 0 is SUMO's actuated phase (grid_3x3.net.xml:894):
 * it ends once it has run minDur = 5 s and no vehicle has been over a detector
 * of its green lanes for more than max_gap, or at maxDur = 50 s; the other
 * phases keep their fixed durations.
 * Outputs after the last substep (time t0+K):
 *   halt   int32 [E][A][12] vehicles with v < halt_speed per incoming lane
 *   phase  int32 [E][A], tspent int32 [E][A] (= t - phase start)
 *   done   uint8 [E] = (t0+K >= max_time) || no vehicle running or pending. */
int dmdqn_sim_step(const dmdqn_sim *sim, const dmdqn_idm *idm, const int32_t *actions,
                   int action_stride, int t0, int K, int max_time, int32_t *halt,
                   int32_t *phase, int32_t *tspent, uint8_t *done, void *stream);

/* The env side of one loop iteration in ONE launch (one block per env):
 * select_action's draws, setPhase + K substeps, the observation / reward and
 * ReplayBuffer.add -- train.py:211-282 up to agent.replay() -- with the same
 * results as dmdqn_act, dmdqn_sim_step, dmdqn_observe and dmdqn_replay_store
 * issued in that order (int8 rows), bit for bit.  The block keeps the halting
 * counts, signals and observation in LDS between them instead of four kernels
 * passing them through HBM (three fewer launches per step). */
typedef struct dmdqn_env_fuse {
    /* act (dmdqn_act): np_state [E][DMDQN_MT_WORDS]; greedy [E*A] (NULL when
     * eps >= 1); actions [E*A] out */
    uint32_t *np_state;
    const int32_t *greedy;
    int32_t *actions;
    double eps;
    int32_t n_actions;
    /* observe (dmdqn_observe): mode 0 / 1; local [E][A][17], obs [E][A][89],
     * reward [E][A] out; prev_local [E][A][17] the pre-step local state */
    int32_t mode;
    float *local, *obs;
    const float *prev_local;
    double *reward;
    /* remember (dmdqn_replay_store, done = the step's done flag of the env):
     * obs_s [E][A][89] the observation the act saw; rings of NA = E*A agents */
    const float *obs_s;
    int32_t cap, slot;
    int8_t *ring_s, *ring_n;
    uint8_t *ring_a;
    double *ring_r;
    uint8_t *ring_d;
    int32_t *err;
} dmdqn_env_fuse;

int dmdqn_env_step(const dmdqn_sim *sim, const dmdqn_idm *idm, const dmdqn_env_fuse *fuse,
                   int action_stride, int t0, int K, int max_time, int32_t *halt,
                   int32_t *phase, int32_t *tspent, uint8_t *done, void *stream);

/* ------------------------------------------------------------------ learn
 * Replaces DQNAgent.learn (src/agents/dqn_agent.py:328-380) + the target sync
 * (:376-377, :382-387) for NA independent agents in ONE launch (one workgroup
 * per agent): replay gather (ReplayBuffer.sample :64-84, z-scored rewards),
 * Double-DQN target, MSE loss, backward and Keras-3 Adam, fused.
 * Parameters (and target, Adam m, v) use the device layout of qnet_layout.hpp
 * per agent: W1T[H][0..87] (tiled) W1T[H][88] W2T[H][H] (tiled) W3T[4][H] b1[H]
 * b2[H] b3[4] -- the Keras kernels transposed, exactly the Keras parameter count
 * (P floats, row stride P; the host converts to / from the Keras get_weights()
 * order).
 * precision: 0 = fp32 MFMA (exact f32 products), 1 = fp16 MFMA with fp32
 * accumulation and fp32 master weights (the reference's mixed_float16),
 * 2 = the same with bf16 MFMA operands (mixed_bfloat16; BASELINE config C2). */
/* Loss of the learn step: MSE is the reference's (dqn_agent.py:141, :352);
 * Huber (delta 1, Keras mean reduction) is the loss of
 * src/experimental/agent.py:99 that BASELINE.json's north_star names. */
#define DMDQN_LOSS_MSE 0
#define DMDQN_LOSS_HUBER 1

/* cap: the ring's physical slot count (replay_buffer_size + 1, see
 * dmdqn_version); start: the slot of deque position 0. */
typedef struct dmdqn_learn_args {
    int32_t NA, cap, start, batch, hidden, precision, sync_target, P;
    const int8_t *ring_s, *ring_n;   /* [NA][cap][DMDQN_ROW_BYTES]; the 16-bit
                                        kernels read a, done, r from the s'
                                        row, the fp32 kernel from the arrays */
    const uint8_t *ring_a, *ring_d;  /* [NA][cap]                            */
    const double *ring_r;            /* [NA][cap]                            */
    const int32_t *idx;              /* [NA][batch] deque positions          */
    float *params, *adam_m, *adam_v; /* [NA][P] online weights + Adam slots  */
    float *target;                   /* [NA][P] target network               */
    uint16_t *target_h;              /* precision 1 / 2: [NA][Ph] f16 / bf16 copy of the
                                        target (Ph = P rounded up to 8) used by
                                        the target forward -- Keras casts the
                                        f32 target to f16 for its matmuls, so
                                        this is the exact operand; written on
                                        target syncs.  NULL: use `target`.     */
    float *loss;                     /* [NA] loss of this learn (or NULL)     */
    float gamma, alpha, c1, c2, eps; /* alpha = lr*sqrt(1-b2^t)/(1-b1^t),
                                        c1 = 1-b1, c2 = 1-b2 (float32)       */
    uint64_t *stamps;                /* diagnostics: NULL, or [NA][16] phase
                                        end times (s_memrealtime, 100 MHz)   */
    float *qstats;                   /* metrics: NULL, or [NA][6] += sum Q(S),
                                        sum Q(S)^2 over the batch's 128x4
                                        online values, counts of actions 0..3
                                        (dqn_agent.py:361-363); zero it first */
    uint16_t *params_h;              /* shared net only (dmdqn_learn_shared_grad,
                                        required there): [Ph] f16 copy of the
                                        online net (Keras' f16 cast of the f32
                                        variables) the forwards read; dmdqn_adam
                                        rewrites it.  Ignored by dmdqn_learn. */
    int32_t loss_kind;               /* DMDQN_LOSS_MSE (default) | DMDQN_LOSS_HUBER */
    float *rn_out;                   /* diagnostics: NULL, or [NA][batch] the
                                        z-scored rewards the learn used
                                        (ReplayBuffer.sample :66-69, f32)     */
    int32_t row_format;              /* DMDQN_ROWS_I8 (0, default): ring_s /
                                        ring_n int8 rows; DMDQN_ROWS_F32: the
                                        batch's rows pre-gathered into xs / xn
                                        (dmdqn_replay_gather_f32), a / done / r
                                        from ring_a / ring_d / ring_r; the
                                        16-bit kernels cast them to 16 bits as
                                        Keras' mixed policy does, the fp32
                                        kernel reads them as f32.  Independent
                                        nets only (not the shared C5 learn).  */
    const float *xs, *xn;            /* DMDQN_ROWS_F32: [NA][batch][DMDQN_ROW_FLOATS] */
} dmdqn_learn_args;

int dmdqn_learn(const dmdqn_learn_args *args, void *stream);

/* dmdqn_learn split in two launches (precision 1 / 2 only; same arithmetic,
 * bit-identical results -- the same DQNAgent.replay, dqn_agent.py:328-380):
 * dmdqn_learn_grad runs the forward/backward and writes each agent's 16-bit
 * gradient (the values Keras's Adam receives, as f32) to grad [NA][P] (device
 * layout); dmdqn_adam_agents then applies the Keras-3 Adam step of the same
 * args (alpha, c1, c2, eps, sync_target) to params / adam_m / adam_v (and
 * target / target_h on a sync).  The second launch is bandwidth-bound and
 * small-footprint, so the next env step's work can share the chip with it
 * (trainer.py, overlap "full").  grad is scratch owned by the caller. */
int dmdqn_learn_grad(const dmdqn_learn_args *args, float *grad, void *stream);
int dmdqn_adam_agents(const dmdqn_learn_args *args, const float *grad, void *stream);

/* Hard target sync outside a learn (DQNAgent.update_target_network,
 * dqn_agent.py:382-387): target[NW][P] <- params[NW][P]; when target_h is not
 * NULL (precision 1 = f16, 2 = bf16) also its 16-bit shadow [NW][Ph], RNE. */
int dmdqn_target_sync(const float *params, float *target, uint16_t *target_h, int NW, int P,
                      int Ph, int precision, void *stream);

/* Greedy actions argmax_a Q_online(obs) for NA agents (dqn_agent.py:268-273,
 * first max on ties); obs f32 [NA][89]; out int32 [NA]; q_out (optional)
 * f32 [NA][4].  precision as dmdqn_learn: 0 f32; 1 / 2 the forward Keras runs
 * under mixed_float16 / mixed_bfloat16 (16-bit weights and activations, f32
 * sums, 16-bit Q).  Used by dmdqn_act when eps < 1. */
int dmdqn_q_argmax(const float *params, int NA, int P, int hidden, int precision,
                   const float *obs, int32_t *out, float *q_out, void *stream);

/* dmdqn_q_argmax with ONE parameter set shared by all NA agents (C5). */
int dmdqn_q_argmax_shared(const float *params, int NA, int P, int hidden, int precision,
                          const float *obs, int32_t *out, float *q_out, void *stream);

/* ------------------------------------------------------------------ shared-parameter DQN
 * Configuration C5 (NOT in the reference, which trains one network
 * per junction): ONE online / target network for all agents of all envs (and
 * all ranks).  Every agent keeps its own replay ring and draws its own batch
 * indices exactly as in the independent configuration; its batch runs the same
 * Double-DQN forward/backward as dmdqn_learn, and the gradients are summed:
 *     grad[P] = scale * sum_agents dL_agent / dtheta     (device layout, f32)
 * With scale = 1 / (agents on all ranks) and an all-reduce(sum) of grad across
 * ranks in between, the following dmdqn_adam step is the Adam step of the mean
 * per-agent loss, identical on every rank.
 * args: params / target / target_h point at ONE network ([P], [Ph]); adam_m /
 * adam_v are not used here; loss [NA] receives each agent's loss.
 * slab: f32 [n_slabs][P] scratch, one partial sum per persistent workgroup
 * (one workgroup per CU: n_slabs = 256 on MI355X).  precision must be 1.
 * work: device scratch of dmdqn_learn_shared_work_bytes(NA) bytes (each batch
 * row's TD target and action between the kernel's two passes: the S' pass
 * with both nets resident in LDS, then the gradient pass); required.
 * grad == NULL: the slabs are left unreduced for dmdqn_adam_slabs (one rank). */
int dmdqn_learn_shared_grad(const dmdqn_learn_args *args, float *slab, int n_slabs, float *grad,
                            float scale, void *work, void *stream);
size_t dmdqn_learn_shared_work_bytes(int NA);
/* The LDS of one workgroup of the shared learn's S' pass (one per CU). */
size_t dmdqn_learn_shared_lds_bytes(void);

/* Keras-3 Adam (dqn_agent.py:357, A-11) on n flat parameters with gradient
 * gscale * grad[i]; params_h (when not NULL) receives the f16 copy of every
 * updated parameter; sync != 0 also copies params to target (and its f16
 * shadow target_h, when not NULL) -- the hard target sync of dqn_agent.py:376-387. */
int dmdqn_adam(float *params, float *adam_m, float *adam_v, float *target, uint16_t *target_h,
               uint16_t *params_h, const float *grad, int n, float gscale, float alpha, float c1,
               float c2, float eps, int sync, void *stream);

/* The slab reduction of dmdqn_learn_shared_grad (grad = scale * sum of the
 * n_slabs slabs, same order, written to grad) followed by dmdqn_adam on it, in
 * one launch: for one rank, where no all-reduce comes between the two.  n must
 * be the shared net's parameter count; results bit-identical to
 * dmdqn_learn_shared_grad(grad) + dmdqn_adam. */
int dmdqn_adam_slabs(float *params, float *adam_m, float *adam_v, float *target,
                     uint16_t *target_h, uint16_t *params_h, const float *slab, int n_slabs,
                     float *grad, float scale, int n, float gscale, float alpha, float c1,
                     float c2, float eps, int sync, void *stream);

#ifdef __cplusplus
}
#endif
#endif
