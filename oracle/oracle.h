/* oracle.h -- CPU restatement of the dmdqn hot path (TEST INFRASTRUCTURE).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * link or load this code; the product path (dmdqn_amd) never does.
 */
#ifndef DMDQN_ORACLE_H
#define DMDQN_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    uint32_t mt[624];
    int32_t mti;
} orc_mt;

/* ---- random streams (oracle_rng.c) ---- */
void orc_mt_init_genrand(orc_mt *s, uint32_t seed);
void orc_mt_init_by_array(orc_mt *s, const uint32_t *key, int len);
void orc_py_seed(orc_mt *s, uint64_t seed);
void orc_np_seed(orc_mt *s, uint32_t seed);
uint32_t orc_mt_u32(orc_mt *s);
uint32_t orc_py_randbelow(orc_mt *s, uint32_t n);
int orc_py_sample(orc_mt *s, uint32_t n, uint32_t k, int32_t *out);
double orc_np_rand(orc_mt *s);
uint32_t orc_np_randint(orc_mt *s, uint32_t hi);
double orc_np_sum(const double *a, long n);
void orc_zscore(const double *r, long n, float *out);
void orc_act(orc_mt *s, int nagents, double eps, const int32_t *greedy, int32_t *out);

/* ---- observation / reward (oracle_obs.c) ---- */
void orc_neighbors(int R, int C, int32_t *nbr);
void orc_local_state(int A, const int32_t *halt, const int32_t *phase,
                     const int32_t *tspent, int mode, float *local);
void orc_build_obs(int R, int C, const float *local, float *obs);
void orc_reward(int A, const float *local, double *rew);

/* ---- grid microsimulation (oracle_sim.c) ---- */
typedef struct {
    float length, min_gap, accel, decel, tau, vmax, two_sqrt_ab, halt_speed;
    float len_inner, len_outer;
    float det_dist, max_gap; /* actuated mode: detector distance, gap-out time */
} orc_idm;
typedef struct orc_env orc_env;
orc_env *orc_env_create(int R, int C, int cap, uint64_t seed, long end_ms, int period_ms,
                        const orc_idm *P);
void orc_env_free(orc_env *g);
void orc_env_set_demand(orc_env *g, int nveh, int period_ms, const uint16_t *q_ids,
                        const int32_t *q_off, const uint16_t *vdst);
void orc_env_reset(orc_env *g);
void orc_env_step(orc_env *g, const int32_t *actions, int stride, int t0, int K, int max_time,
                  int32_t *halt, int32_t *phase, int32_t *tspent, uint8_t *done);
int orc_env_info(const orc_env *g, int32_t *out);
void orc_env_lanes(const orc_env *g, float *x, float *v, int32_t *dst, int32_t *head, int32_t *cnt);
void orc_env_demand(const orc_env *g, uint16_t *q_ids, int32_t *q_off, uint16_t *vdst);
void orc_env_enable_trace(orc_env *g, int max_events);
void orc_env_set_actuated(orc_env *g, int on);
int orc_env_trace(const orc_env *g, int32_t *out);

/* ---- learn step (oracle_learn.c) ---- */
long orc_qnet_nparams(int H1, int H2, int NA);
void orc_qnet_forward(const float *p, int H1, int H2, int NA, const float *x, int B, float *q,
                      float *z1c, float *z2c);
float orc_learn(float *p, const float *target, float *m, float *v, int H1, int H2, int NA,
                int B, const float *S, const int32_t *A, const float *Rn, const float *S2,
                const float *Dn, const float *hyper, float *grad_out, int loss_kind);

/* ---- the whole training loop, OpenMP over replicas (oracle_loop.c; bench CPU baseline) ---- */
double orc_train_loop(int R, int C, int E, int fill, int steps, uint64_t seed, int threads,
                      long *agent_steps);

#ifdef __cplusplus
}
#endif
#endif
