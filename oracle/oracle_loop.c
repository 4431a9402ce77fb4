/* oracle_loop.c -- the reference training loop body (src/scripts/train.py:207-310)
 * for E independent env replicas on the CPU, OpenMP over replicas.
 *
 * TEST INFRASTRUCTURE: only bench.py's cpu_baseline leg calls it.  It chains
 * the same restated pieces the parity tests pin (orc_act, orc_env_step,
 * orc_local_state / orc_build_obs / orc_reward, orc_py_sample, orc_zscore,
 * orc_learn), with the replay kept as plain f32 rows, so the baseline is the
 * reference's semantics on the host -- 1 thread, or one replica per core.
 *
 * Per replica and step: act (eps = 1, A-1), setPhase + 10 substeps, observe,
 * pre-step reward (A-3), remember, and once the ring holds 128 transitions,
 * for each agent: random.sample(128) -> batch -> z-score -> Double-DQN learn
 * with Keras Adam (hard target copy every 500 learns).
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <omp.h>

#include "oracle.h"

#define OBS 89
#define BATCH 128

typedef struct {
    int R, C, A, cap, n, t, learn_steps;
    long P;
    orc_env *env;
    orc_mt np, py;
    float *params, *target, *m, *v;  /* [A][P] */
    float *S, *S2, *Dn;              /* [A][cap][89], [A][cap][89], [A][cap] */
    int32_t *Aa;                     /* [A][cap] */
    double *Rr;                      /* [A][cap] */
    float *L, *obs, *L2, *obs2;      /* [A][17], [A][89] */
    /* scratch */
    int32_t *acts, *halt, *ph, *ts, *idx, *Ab;
    double *rew, *rb;
    float *Sb, *S2b, *Db, *Rn;
} loop_env;

static uint64_t splitmix(uint64_t *s) {
    uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static loop_env *loop_env_new(int R, int C, int cap, uint64_t seed) {
    loop_env *e = (loop_env *)calloc(1, sizeof(loop_env));
    const int A = R * C;
    e->R = R; e->C = C; e->A = A; e->cap = cap;
    orc_idm P = {5.0f, 2.5f, 2.6f, 4.5f, 1.0f, 13.89f, 0.0f, 0.1f, 172.8f, 86.4f};
    P.two_sqrt_ab = 2.0f * sqrtf(P.accel * P.decel);
    e->env = orc_env_create(R, C, 24, seed, 2500000, 0, &P);
    orc_np_seed(&e->np, (uint32_t)seed);
    orc_py_seed(&e->py, seed);
    e->P = orc_qnet_nparams(128, 128, 4);
    size_t np_ = (size_t)A * e->P;
    e->params = (float *)malloc(np_ * sizeof(float));
    e->target = (float *)malloc(np_ * sizeof(float));
    e->m = (float *)calloc(np_, sizeof(float));
    e->v = (float *)calloc(np_, sizeof(float));
    uint64_t st = seed * 7919u + 1;
    for (size_t i = 0; i < np_; i++)  /* uniform +-0.05: the baseline times, it does not train */
        e->params[i] = (float)((double)(splitmix(&st) >> 11) / 9007199254740992.0 - 0.5) * 0.1f;
    memcpy(e->target, e->params, np_ * sizeof(float));
    size_t rows = (size_t)A * cap;
    e->S = (float *)calloc(rows * OBS, sizeof(float));
    e->S2 = (float *)calloc(rows * OBS, sizeof(float));
    e->Dn = (float *)calloc(rows, sizeof(float));
    e->Aa = (int32_t *)calloc(rows, sizeof(int32_t));
    e->Rr = (double *)calloc(rows, sizeof(double));
    e->L = (float *)calloc((size_t)A * 17, sizeof(float));
    e->L2 = (float *)calloc((size_t)A * 17, sizeof(float));
    e->obs = (float *)calloc((size_t)A * OBS, sizeof(float));
    e->obs2 = (float *)calloc((size_t)A * OBS, sizeof(float));
    e->acts = (int32_t *)calloc(A, sizeof(int32_t));
    e->halt = (int32_t *)calloc((size_t)A * 12, sizeof(int32_t));
    e->ph = (int32_t *)calloc(A, sizeof(int32_t));
    e->ts = (int32_t *)calloc(A, sizeof(int32_t));
    e->idx = (int32_t *)calloc(BATCH, sizeof(int32_t));
    e->Ab = (int32_t *)calloc(BATCH, sizeof(int32_t));
    e->rew = (double *)calloc(A, sizeof(double));
    e->rb = (double *)calloc(BATCH, sizeof(double));
    e->Sb = (float *)calloc((size_t)BATCH * OBS, sizeof(float));
    e->S2b = (float *)calloc((size_t)BATCH * OBS, sizeof(float));
    e->Db = (float *)calloc(BATCH, sizeof(float));
    e->Rn = (float *)calloc(BATCH, sizeof(float));
    orc_local_state(A, e->halt, e->ph, e->ts, 0, e->L);
    orc_build_obs(R, C, e->L, e->obs);
    return e;
}

static void loop_env_free(loop_env *e) {
    orc_env_free(e->env);
    free(e->params); free(e->target); free(e->m); free(e->v);
    free(e->S); free(e->S2); free(e->Dn); free(e->Aa); free(e->Rr);
    free(e->L); free(e->L2); free(e->obs); free(e->obs2);
    free(e->acts); free(e->halt); free(e->ph); free(e->ts); free(e->idx); free(e->Ab);
    free(e->rew); free(e->rb); free(e->Sb); free(e->S2b); free(e->Db); free(e->Rn);
    free(e);
}

/* One loop iteration for every agent of the replica. */
static void loop_step(loop_env *e, int learn) {
    const int A = e->A;
    uint8_t done = 0;
    orc_act(&e->np, A, 1.0, NULL, e->acts);
    orc_env_step(e->env, e->acts, 3, e->t, 10, 2400, e->halt, e->ph, e->ts, &done);
    e->t += 10;
    orc_local_state(A, e->halt, e->ph, e->ts, 0, e->L2);
    orc_build_obs(e->R, e->C, e->L2, e->obs2);
    orc_reward(A, e->L, e->rew);
    const int slot = e->n % e->cap;
    for (int a = 0; a < A; a++) {
        size_t r = (size_t)a * e->cap + slot;
        memcpy(e->S + r * OBS, e->obs + (size_t)a * OBS, OBS * sizeof(float));
        memcpy(e->S2 + r * OBS, e->obs2 + (size_t)a * OBS, OBS * sizeof(float));
        e->Aa[r] = e->acts[a];
        e->Rr[r] = e->rew[a];
        e->Dn[r] = e->t >= 2400 ? 1.0f : 0.0f;
    }
    e->n++;
    const int size = e->n < e->cap ? e->n : e->cap;
    if (learn && size >= BATCH) {
        e->learn_steps++;
        const float b1p = powf(0.9f, (float)e->learn_steps), b2p = powf(0.999f, (float)e->learn_steps);
        const float hyper[5] = {0.99f, 0.001f * sqrtf(1.0f - b2p) / (1.0f - b1p), 0.1f, 0.001f,
                                1e-7f};
        const int start = e->n <= e->cap ? 0 : e->n % e->cap;
        for (int a = 0; a < A; a++) {
            orc_py_sample(&e->py, (uint32_t)size, BATCH, e->idx);
            for (int i = 0; i < BATCH; i++) {
                size_t r = (size_t)a * e->cap + (size_t)((start + e->idx[i]) % e->cap);
                memcpy(e->Sb + (size_t)i * OBS, e->S + r * OBS, OBS * sizeof(float));
                memcpy(e->S2b + (size_t)i * OBS, e->S2 + r * OBS, OBS * sizeof(float));
                e->Ab[i] = e->Aa[r];
                e->rb[i] = e->Rr[r];
                e->Db[i] = e->Dn[r];
            }
            orc_zscore(e->rb, BATCH, e->Rn);
            size_t o = (size_t)a * e->P;
            orc_learn(e->params + o, e->target + o, e->m + o, e->v + o, 128, 128, 4, BATCH, e->Sb,
                      e->Ab, e->Rn, e->S2b, e->Db, hyper, NULL, 0);
        }
        if (e->learn_steps % 500 == 0)
            memcpy(e->target, e->params, (size_t)A * e->P * sizeof(float));
    }
    float *tl = e->L; e->L = e->L2; e->L2 = tl;
    float *to = e->obs; e->obs = e->obs2; e->obs2 = to;
    if (e->t >= 2400) {
        orc_env_reset(e->env);
        e->t = 0;
    }
}

/* E replicas x (fill untimed steps + `steps` timed steps), OpenMP over replicas
 * with `threads` threads.  Returns the timed wall seconds; *agent_steps gets
 * the agent-env steps of the timed region. */
double orc_train_loop(int R, int C, int E, int fill, int steps, uint64_t seed, int threads,
                      long *agent_steps) {
    loop_env **envs = (loop_env **)calloc((size_t)E, sizeof(loop_env *));
    const int cap = fill + steps + 1 < 10000 ? fill + steps + 1 : 10000;
    omp_set_num_threads(threads);
#pragma omp parallel for schedule(static)
    for (int e = 0; e < E; e++) {
        envs[e] = loop_env_new(R, C, cap, seed + (uint64_t)e);
        for (int k = 0; k < fill; k++) loop_step(envs[e], 0);
    }
    const double t0 = omp_get_wtime();
#pragma omp parallel for schedule(dynamic, 1)
    for (int e = 0; e < E; e++)
        for (int k = 0; k < steps; k++) loop_step(envs[e], 1);
    const double el = omp_get_wtime() - t0;
    if (agent_steps) *agent_steps = (long)E * steps * R * C;
    for (int e = 0; e < E; e++) loop_env_free(envs[e]);
    free(envs);
    return el;
}
