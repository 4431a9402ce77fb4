// rng.hip -- device MT19937 streams: seeding, act (numpy legacy stream) and
// replay sampling (CPython `random` stream), one wave per env stream.
//
// Reference behaviour restated (and pinned bit-exactly by tests/golden):
//   src/agents/dqn_agent.py:258-265  epsilon-greedy: np.random.rand(),
//                                    np.random.randint(0, action_size)
//   src/agents/dqn_agent.py:63       random.sample(self.buffer, batch_size)
// Draw order contract: per env, agents j = 0..A-1 in junction (J_r_c,
// row-major) order, exactly as train.py:211-222 / :274-282 iterate them.
#include <math.h>

#include "common.hpp"

namespace dmdqn {

// ------------------------------------------------------------------ seeding
__global__ void k_seed_np(uint32_t *state, const uint64_t *seeds, int E) {
    int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= E) return;
    uint32_t *mt = state + (size_t)e * DMDQN_MT_WORDS;
    uint32_t prev = (uint32_t)(seeds[e] & 0xffffffffu);
    mt[0] = prev;
    for (int i = 1; i < MT_N; i++) {
        prev = 1812433253u * (prev ^ (prev >> 30)) + (uint32_t)i;
        mt[i] = prev;
    }
    mt[MT_N] = MT_N;
}

// CPython init_by_array; one wave per stream, lane 0 runs the recurrence in LDS.
__global__ void __launch_bounds__(64) k_seed_py(uint32_t *state, const uint64_t *seeds, int E) {
    __shared__ uint32_t mt[MT_N];
    int e = blockIdx.x;
    if (threadIdx.x == 0) {
        uint64_t s = seeds[e];
        uint32_t key[2];
        int len = 0;
        key[len++] = (uint32_t)(s & 0xffffffffu);
        if (s >> 32) key[len++] = (uint32_t)(s >> 32);
        mt[0] = 19650218u;
        for (int i = 1; i < MT_N; i++)
            mt[i] = 1812433253u * (mt[i - 1] ^ (mt[i - 1] >> 30)) + (uint32_t)i;
        int i = 1, j = 0;
        for (int k = (MT_N > len ? MT_N : len); k; k--) {
            mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1664525u)) + key[j] + (uint32_t)j;
            i++; j++;
            if (i >= MT_N) { mt[0] = mt[MT_N - 1]; i = 1; }
            if (j >= len) j = 0;
        }
        for (int k = MT_N - 1; k; k--) {
            mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1566083941u)) - (uint32_t)i;
            i++;
            if (i >= MT_N) { mt[0] = mt[MT_N - 1]; i = 1; }
        }
        mt[0] = 0x80000000u;
    }
    __syncthreads();
    uint32_t *g = state + (size_t)e * DMDQN_MT_WORDS;
    for (int i = threadIdx.x; i < MT_N; i += 64) g[i] = mt[i];
    if (threadIdx.x == 0) g[MT_N] = MT_N;
}

// ------------------------------------------------------------------ raw draws
__global__ void __launch_bounds__(64) k_draw_u32(uint32_t *state, int count, uint32_t *out) {
    __shared__ uint32_t mt[MT_N], tmp[MT_N];
    MTWave w{mt, tmp, 0};
    uint32_t *g = state + (size_t)blockIdx.x * DMDQN_MT_WORDS;
    w.load(g);
    for (int i = 0; i < count; i++) {
        uint32_t v = w.next();
        if (threadIdx.x == 0) out[(size_t)blockIdx.x * count + i] = v;
    }
    __syncthreads();
    w.store(g);
}

// ------------------------------------------------------------------ act
// numpy legacy random_sample: ((u>>5) * 2^26 + (u>>6)) / 2^53 (exact in f64).
__device__ __forceinline__ double np_double(MTWave &w) {
    int32_t a = (int32_t)(w.next() >> 5);
    int32_t b = (int32_t)(w.next() >> 6);
    return ((double)a * 67108864.0 + (double)b) / 9007199254740992.0;
}

__global__ void __launch_bounds__(64) k_act(uint32_t *np_state, int A, double eps, uint32_t rng,
                                            uint32_t mask, const int32_t *greedy,
                                            int32_t *actions) {
    __shared__ uint32_t mt[MT_N], tmp[MT_N];
    MTWave w{mt, tmp, 0};
    const int e = blockIdx.x;
    uint32_t *g = np_state + (size_t)e * DMDQN_MT_WORDS;
    w.load(g);
    for (int j = 0; j < A; j++) {
        double r = np_double(w);
        int32_t a;
        if (r < eps) {  // dqn_agent.py:263-265
            uint32_t v;
            do { v = w.next() & mask; } while (v > rng);
            a = (int32_t)v;
        } else {
            a = greedy[(size_t)e * A + j];
        }
        if (threadIdx.x == 0) actions[(size_t)e * A + j] = a;
    }
    __syncthreads();
    w.store(g);
}

// ------------------------------------------------------------------ sample
// CPython Random._randbelow_with_getrandbits: k = n.bit_length(),
// r = getrandbits(k) = u32 >> (32-k), redraw while r >= n.
__device__ __forceinline__ uint32_t py_randbelow(MTWave &w, uint32_t n) {
    const int k = 32 - __clz(n);
    uint32_t r = w.next() >> (32 - k);
    while (r >= n) r = w.next() >> (32 - k);
    return r;
}

// CPython Random.sample (3.10/3.11), population = deque of length n.
// Pool branch (n <= setsize): partial Fisher-Yates over a u32 pool in LDS.
// Set branch: rejection against an n-bit "selected" bitmap in LDS.
// All lanes execute the same loop and perform the same (identical-value)
// LDS updates, so each lane's reads are ordered after its own writes.
__global__ void __launch_bounds__(64) k_sample(uint32_t *py_state, int A, uint32_t n, int k,
                                               uint32_t setsize, int32_t *idx) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    uint32_t *mt = smem, *tmp = smem + MT_N, *aux = smem + 2 * MT_N;
    MTWave w{mt, tmp, 0};
    const int e = blockIdx.x;
    uint32_t *g = py_state + (size_t)e * DMDQN_MT_WORDS;
    w.load(g);
    const bool pool_branch = n <= setsize;
    for (int j = 0; j < A; j++) {
        int32_t *out = idx + ((size_t)e * A + j) * k;
        if (pool_branch) {
            for (uint32_t i = threadIdx.x; i < n; i += 64) aux[i] = i;
            __syncthreads();
            for (int i = 0; i < k; i++) {
                uint32_t m = n - (uint32_t)i;
                uint32_t jj = py_randbelow(w, m);
                uint32_t v = aux[jj];
                if (threadIdx.x == 0) out[i] = (int32_t)v;
                aux[jj] = aux[m - 1];
            }
        } else {
            const uint32_t words = (n + 31u) >> 5;
            for (uint32_t i = threadIdx.x; i < words; i += 64) aux[i] = 0u;
            __syncthreads();
            for (int i = 0; i < k; i++) {
                uint32_t jj = py_randbelow(w, n);
                while (aux[jj >> 5] & (1u << (jj & 31))) jj = py_randbelow(w, n);
                aux[jj >> 5] |= (1u << (jj & 31));
                if (threadIdx.x == 0) out[i] = (int32_t)jj;
            }
        }
        __syncthreads();
    }
    w.store(g);
}

}  // namespace dmdqn

using namespace dmdqn;

extern "C" int dmdqn_mt_seed_np(uint32_t *state, const uint64_t *seeds, int E, void *stream) {
    DMDQN_REQUIRE(state && seeds && E > 0, "dmdqn_mt_seed_np: null pointer or E<=0");
    hipLaunchKernelGGL(k_seed_np, dim3((E + 63) / 64), dim3(64), 0, as_stream(stream), state, seeds, E);
    DMDQN_LAUNCH_CHECK("k_seed_np");
    return DMDQN_OK;
}

extern "C" int dmdqn_mt_seed_py(uint32_t *state, const uint64_t *seeds, int E, void *stream) {
    DMDQN_REQUIRE(state && seeds && E > 0, "dmdqn_mt_seed_py: null pointer or E<=0");
    hipLaunchKernelGGL(k_seed_py, dim3(E), dim3(64), 0, as_stream(stream), state, seeds, E);
    DMDQN_LAUNCH_CHECK("k_seed_py");
    return DMDQN_OK;
}

extern "C" int dmdqn_mt_draw_u32(uint32_t *state, int E, int count, uint32_t *out, void *stream) {
    DMDQN_REQUIRE(state && out && E > 0 && count >= 0, "dmdqn_mt_draw_u32: bad args");
    hipLaunchKernelGGL(k_draw_u32, dim3(E), dim3(64), 0, as_stream(stream), state, count, out);
    DMDQN_LAUNCH_CHECK("k_draw_u32");
    return DMDQN_OK;
}

extern "C" int dmdqn_act(uint32_t *np_state, int E, int A, double eps, int n_actions,
                         const int32_t *greedy, int32_t *actions, void *stream) {
    DMDQN_REQUIRE(np_state && actions && E > 0 && A > 0, "dmdqn_act: bad args");
    DMDQN_REQUIRE(n_actions >= 1, "dmdqn_act: n_actions must be >= 1");
    DMDQN_REQUIRE(greedy || eps >= 1.0, "dmdqn_act: greedy actions required when eps < 1");
    uint32_t rng = (uint32_t)(n_actions - 1), mask = rng;
    mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4; mask |= mask >> 8; mask |= mask >> 16;
    hipLaunchKernelGGL(k_act, dim3(E), dim3(64), 0, as_stream(stream), np_state, A, eps, rng, mask,
                       greedy, actions);
    DMDQN_LAUNCH_CHECK("k_act");
    return DMDQN_OK;
}

extern "C" int dmdqn_replay_sample(uint32_t *py_state, int E, int A, int n, int k,
                                   int32_t *idx, void *stream) {
    DMDQN_REQUIRE(py_state && idx && E > 0 && A > 0, "dmdqn_replay_sample: bad args");
    DMDQN_REQUIRE(k >= 1 && n >= k, "dmdqn_replay_sample: need 1 <= k <= n (k=%d n=%d)", k, n);
    uint32_t setsize = 21;
    if (k > 5) setsize += (uint32_t)pow(4.0, ceil(log((double)k * 3.0) / log(4.0)));
    size_t aux_words = ((uint32_t)n <= setsize) ? (size_t)n : (size_t)((n + 31) / 32);
    size_t lds = (2 * MT_N + aux_words) * sizeof(uint32_t);
    DMDQN_REQUIRE(lds <= 160 * 1024, "dmdqn_replay_sample: n=%d too large for LDS", n);
    hipLaunchKernelGGL(k_sample, dim3(E), dim3(64), lds, as_stream(stream), py_state, A,
                       (uint32_t)n, k, setsize, idx);
    DMDQN_LAUNCH_CHECK("k_sample");
    return DMDQN_OK;
}
