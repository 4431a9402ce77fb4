/* oracle_rng.c -- CPU restatement of the reference's random streams.
 *
 * TEST INFRASTRUCTURE ONLY (the checker, never the product): only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 * Parity: pinned by tests/golden/rng.npz and tests/golden/replay_sample.npz,
 * which were produced by CPython 3.10 `random` and numpy 2.2 RandomState
 * (the reference pins Python 3.11 / numpy 2.1.3; both algorithms are frozen).
 *
 * Reference call sites restated here:
 *   dqn_agent.py:63     random.sample(self.buffer, batch_size)  (CPython random)
 *   dqn_agent.py:66-69  reward z-score (numpy mean/std, f64, +1e-8)
 *   dqn_agent.py:263    np.random.rand()                        (numpy legacy)
 *   dqn_agent.py:265    np.random.randint(0, self.action_size)  (numpy legacy)
 */
#include "oracle.h"

#include <math.h>
#include <string.h>

#define MT_N 624
#define MT_M 397

void orc_mt_init_genrand(orc_mt *s, uint32_t seed) {
    /* numpy legacy RandomState.seed(int) -> init_genrand */
    s->mt[0] = seed;
    for (int i = 1; i < MT_N; i++)
        s->mt[i] = 1812433253u * (s->mt[i - 1] ^ (s->mt[i - 1] >> 30)) + (uint32_t)i;
    s->mti = MT_N;
}

void orc_mt_init_by_array(orc_mt *s, const uint32_t *key, int len) {
    /* CPython random.seed(int) -> init_by_array(abs(int) as 32-bit words) */
    orc_mt_init_genrand(s, 19650218u);
    int i = 1, j = 0, k = (MT_N > len ? MT_N : len);
    for (; k; k--) {
        s->mt[i] = (s->mt[i] ^ ((s->mt[i - 1] ^ (s->mt[i - 1] >> 30)) * 1664525u)) + key[j] + (uint32_t)j;
        i++; j++;
        if (i >= MT_N) { s->mt[0] = s->mt[MT_N - 1]; i = 1; }
        if (j >= len) j = 0;
    }
    for (k = MT_N - 1; k; k--) {
        s->mt[i] = (s->mt[i] ^ ((s->mt[i - 1] ^ (s->mt[i - 1] >> 30)) * 1566083941u)) - (uint32_t)i;
        i++;
        if (i >= MT_N) { s->mt[0] = s->mt[MT_N - 1]; i = 1; }
    }
    s->mt[0] = 0x80000000u;
    s->mti = MT_N;
}

void orc_py_seed(orc_mt *s, uint64_t seed) {
    uint32_t key[2];
    int len = 0;
    key[len++] = (uint32_t)(seed & 0xffffffffu);
    if (seed >> 32) key[len++] = (uint32_t)(seed >> 32);
    orc_mt_init_by_array(s, key, len);
}

void orc_np_seed(orc_mt *s, uint32_t seed) { orc_mt_init_genrand(s, seed); }

static void mt_twist(orc_mt *s) {
    static const uint32_t mag01[2] = {0u, 0x9908b0dfu};
    int kk;
    uint32_t y;
    for (kk = 0; kk < MT_N - MT_M; kk++) {
        y = (s->mt[kk] & 0x80000000u) | (s->mt[kk + 1] & 0x7fffffffu);
        s->mt[kk] = s->mt[kk + MT_M] ^ (y >> 1) ^ mag01[y & 1u];
    }
    for (; kk < MT_N - 1; kk++) {
        y = (s->mt[kk] & 0x80000000u) | (s->mt[kk + 1] & 0x7fffffffu);
        s->mt[kk] = s->mt[kk + (MT_M - MT_N)] ^ (y >> 1) ^ mag01[y & 1u];
    }
    y = (s->mt[MT_N - 1] & 0x80000000u) | (s->mt[0] & 0x7fffffffu);
    s->mt[MT_N - 1] = s->mt[MT_M - 1] ^ (y >> 1) ^ mag01[y & 1u];
    s->mti = 0;
}

uint32_t orc_mt_u32(orc_mt *s) {
    if (s->mti >= MT_N) mt_twist(s);
    uint32_t y = s->mt[s->mti++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}

/* CPython Lib/random.py  Random._randbelow_with_getrandbits */
uint32_t orc_py_randbelow(orc_mt *s, uint32_t n) {
    int k = 0;
    while ((n >> k) != 0 && k < 32) k++; /* n.bit_length() */
    uint32_t r = orc_mt_u32(s) >> (32 - k);
    while (r >= n) r = orc_mt_u32(s) >> (32 - k);
    return r;
}

/* CPython Lib/random.py  Random.sample(population, k)  (3.10/3.11 body) */
int orc_py_sample(orc_mt *s, uint32_t n, uint32_t k, int32_t *out) {
    if (k > n) return -1;
    uint32_t setsize = 21;
    if (k > 5) {
        /* 4 ** _ceil(_log(k * 3, 4)) ; float log as CPython does */
        double e = ceil(log((double)k * 3.0) / log(4.0));
        setsize += (uint32_t)pow(4.0, e);
    }
    if (n <= setsize) {
        int32_t pool[4200];
        if (n > 4200) return -2;
        for (uint32_t i = 0; i < n; i++) pool[i] = (int32_t)i;
        for (uint32_t i = 0; i < k; i++) {
            uint32_t j = orc_py_randbelow(s, n - i);
            out[i] = pool[j];
            pool[j] = pool[n - i - 1];
        }
    } else {
        static uint8_t selected[1u << 20];
        if (n > (1u << 20)) return -3;
        memset(selected, 0, n);
        for (uint32_t i = 0; i < k; i++) {
            uint32_t j = orc_py_randbelow(s, n);
            while (selected[j]) j = orc_py_randbelow(s, n);
            selected[j] = 1;
            out[i] = (int32_t)j;
        }
    }
    return 0;
}

/* numpy legacy random_sample / rk_double */
double orc_np_rand(orc_mt *s) {
    int32_t a = (int32_t)(orc_mt_u32(s) >> 5), b = (int32_t)(orc_mt_u32(s) >> 6);
    return (a * 67108864.0 + b) / 9007199254740992.0;
}

/* numpy legacy randint(0, hi) for hi-1 <= 0xffffffff: masked rejection */
uint32_t orc_np_randint(orc_mt *s, uint32_t hi) {
    uint32_t rng = hi - 1, mask = rng;
    if (rng == 0) return 0;
    mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4;
    mask |= mask >> 8; mask |= mask >> 16;
    uint32_t v;
    while ((v = (orc_mt_u32(s) & mask)) > rng) {}
    return v;
}

/* numpy pairwise summation (numpy/_core/src/umath/loops_utils.h.src) */
static double pairwise_sum(const double *a, long n) {
    if (n < 8) {
        double res = 0.;
        for (long i = 0; i < n; i++) res += a[i];
        return res;
    } else if (n <= 128) {
        double r[8], res;
        long i;
        for (int j = 0; j < 8; j++) r[j] = a[j];
        for (i = 8; i < n - (n % 8); i += 8)
            for (int j = 0; j < 8; j++) r[j] += a[i + j];
        res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; i++) res += a[i];
        return res;
    } else {
        long n2 = n / 2;
        n2 -= n2 % 8;
        return pairwise_sum(a, n2) + pairwise_sum(a + n2, n - n2);
    }
}

/* np.add.reduce over a contiguous f64 vector (identity 0 then pairwise) */
double orc_np_sum(const double *a, long n) { return 0.0 + pairwise_sum(a, n); }

/* dqn_agent.py:66-69 then the f32 cast at :82 */
void orc_zscore(const double *r, long n, float *out) {
    double mean = orc_np_sum(r, n) / (double)n;
    double dev[4096];
    for (long i = 0; i < n; i++) {
        double d = r[i] - mean;
        dev[i] = d * d;
    }
    double var = orc_np_sum(dev, n) / (double)n;
    double sd = sqrt(var);
    for (long i = 0; i < n; i++) out[i] = (float)((r[i] - mean) / (sd + 1e-8));
}

/* dqn_agent.py:246-274 with the reference's epsilon (A-1). greedy[j] is the
 * argmax action for agent j (used only when rand() >= eps). */
void orc_act(orc_mt *s, int nagents, double eps, const int32_t *greedy, int32_t *out) {
    for (int j = 0; j < nagents; j++) {
        if (orc_np_rand(s) < eps)
            out[j] = (int32_t)orc_np_randint(s, 4);
        else
            out[j] = greedy ? greedy[j] : 0;
    }
}
