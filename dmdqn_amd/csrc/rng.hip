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
#include <stdlib.h>

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
// draw_rand 0: no rand() draw, every action is randint (test.py:92 random mode)
__global__ void __launch_bounds__(64) k_act(uint32_t *np_state, int A, double eps, uint32_t rng,
                                            uint32_t mask, const int32_t *greedy,
                                            int32_t *actions, int draw_rand) {
    __shared__ uint32_t mt[MT_N], tmp[MT_N];
    MTWave w{mt, tmp, 0};
    const int e = blockIdx.x;
    uint32_t *g = np_state + (size_t)e * DMDQN_MT_WORDS;
    const int per = draw_rand ? 3 : 1, mti0 = (int)g[MT_N];
    if (act_fast_ok(mti0, A, per, eps, rng, mask, draw_rand)) {  // one wave: reads before the write
        for (int j = threadIdx.x; j < A; j += 64)
            actions[(size_t)e * A + j] = act_fast(g, mti0, j, per, mask);
        if (threadIdx.x == 0) g[MT_N] = (uint32_t)(mti0 + A * per);
        return;
    }
    w.load(g);
    for (int j = 0; j < A; j++) {
        const double r = draw_rand ? np_double(w) : 0.0;
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

// CPython Random.sample (3.10/3.11), population = deque of length n:
//   pool branch (n <= setsize): pool = list(range(n)); for i < k:
//       j = randbelow(n - i); result[i] = pool[j]; pool[j] = pool[n - i - 1]
//   set branch: for i < k: j = randbelow(n), redrawn while j in selected.
// randbelow(m) = getrandbits(bit_length(m)), redrawn while >= m.
//
// Pool branch (k_sample): one wave per env consumes the env's stream 64
// tempered words at a time ("chunk", lane l <-> word mti + l) and decides every
// word of the chunk at once instead of one dependent LDS round trip per draw.
// Phase 1: whether a word is accepted depends only on the word and on
// m = n - i, never on the pool.  Lane l is accepted iff
// getrandbits(bit_length(m - c_l)) < m - c_l, where c_l counts the accepted
// lanes below l.  That recurrence is solved by iterating
// c <- exclusive popcount(ballot(accepted(c))) from c = 0: each pass makes at
// least one more lane exact (lane 0 always is), and a fixed point is the
// sequential answer.  Accepted positions j go to LDS, per agent.  Phase 2:
// every agent's k pool swaps run in parallel, lane = agent, each on its own
// u16 pool in LDS (only the swap chain is sequential).
// The set branch is k_sample_set below.  In both, the agent whose k-th pick
// falls inside a chunk consumes the chunk only up to that word; the next agent
// starts at the word after.
__device__ __forceinline__ uint32_t bitlen(uint32_t m) { return 32u - (uint32_t)__clz(m); }
__device__ __forceinline__ uint32_t getbits(uint32_t u, uint32_t kb) {
    return u >> (32u - kb);  // kb in 1..32
}
__device__ __forceinline__ uint64_t lanes_below() {
    const int l = threadIdx.x;
    return l ? (~0ull >> (64 - l)) : 0ull;
}

__global__ void __launch_bounds__(64) k_sample(uint32_t *py_state, int A, uint32_t n, int k,
                                               int32_t *idx) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    uint32_t *mt = smem, *tmp = smem + MT_N, *aux = smem + 2 * MT_N;
    MTWave w{mt, tmp, 0};
    const int e = blockIdx.x, l = threadIdx.x;
    uint32_t *g = py_state + (size_t)e * DMDQN_MT_WORDS;
    w.load(g);
    {
        uint16_t *sel = reinterpret_cast<uint16_t *>(aux);           // [A][k]
        uint16_t *pool = sel + (((size_t)A * k + 1) & ~(size_t)1);  // [min(A,64)][n]
        // ---- phase 1: the stream -> accepted j per (agent, i)
        int j = 0, i = 0;
        while (j < A) {
            if (w.mti >= MT_N) w.refill();
            const int cnt = min(64, MT_N - w.mti);
            const bool live = l < cnt;
            const uint32_t u = tmp[w.mti + (live ? l : 0)];
            const uint32_t m0 = n - (uint32_t)i;
            uint64_t acc = 0;
            int c = 0;
            uint32_t r = 0;
            bool a = false;
            for (;;) {
                const uint32_t mm = (uint32_t)c < m0 ? m0 - (uint32_t)c : 1u;
                r = getbits(u, bitlen(mm));
                a = live && r < mm;
                const uint64_t nacc = __ballot(a);
                if (nacc == acc) break;
                acc = nacc;
                c = __popcll(acc & lanes_below());
            }
            const int total = __popcll(acc), need = k - i;
            int taken = total, consumed = cnt;
            if (total >= need) {
                const uint64_t last = __ballot(a && c == need - 1);
                consumed = __ffsll((unsigned long long)last);  // lane + 1
                taken = need;
            }
            if (a && c < taken) sel[(size_t)j * k + i + c] = (uint16_t)r;
            w.mti += consumed;
            i += taken;
            if (i == k) { j++; i = 0; }
        }
        __syncthreads();
        // ---- phase 2: pool swaps, lane = agent (groups of 64 agents)
        for (int j0 = 0; j0 < A; j0 += 64) {
            const int G = min(64, A - j0);
            for (uint32_t q = l; q < n; q += 64)  // pool[g][q] = q (no runtime modulo)
                for (int g = 0; g < G; g++) pool[(size_t)g * n + q] = (uint16_t)q;
            __syncthreads();
            if (l < G) {
                uint16_t *P = pool + (size_t)l * n;
                const uint16_t *Sj = sel + (size_t)(j0 + l) * k;
                int32_t *o = idx + ((size_t)e * A + j0 + l) * k;
                for (int q = 0; q < k; q++) {
                    const uint32_t x = Sj[q];
                    const uint16_t v = P[x], last = P[n - 1 - (uint32_t)q];
                    DMDQN_DBG(x < n - (uint32_t)q && v < n, DBG_SAMPLE);
                    o[q] = (int32_t)v;
                    P[x] = last;
                }
            }
            __syncthreads();
        }
    }
    __syncthreads();
    w.store(g);
}

// Set branch with NW waves on one env stream (dmdqn_replay_sample picks it
// for n > setsize): each iteration decides a chunk of 64*NW consecutive
// words -- one per thread -- instead of 128 per wave, so an agent's ~210
// words (n = 10000: acceptance n / 2^14) usually take one iteration instead
// of two, and the per-word instruction stream is spread over NW SIMDs (one
// wave on one stream is issue-bound: ~250 instructions per 128 words).  Same
// decisions as k_sample's set branch word for word: out-of-range and
// already-selected words (LDS bitmap) are rejected, a repeat within the chunk
// is rejected by the first-lane table (block-wide, pending lanes only:
// atomicMax, barrier, read, barrier), positions come from the block prefix of the accepted
// flags, and the agent whose k-th pick falls inside the chunk consumes it up
// to that word.
template <int NW>
__global__ void __launch_bounds__(64 * NW) k_sample_set(uint32_t *py_state, int A, uint32_t n, int k,
                                                       int tlog, int32_t *idx) {
    constexpr int NT = 64 * NW;
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    __shared__ int s_cnt[NW];
    __shared__ int s_cons;
    // two raw 624-word blocks of the stream: the current one and, once a chunk
    // reaches past it, the next (twisted ahead out of place); words are
    // tempered as they are read, so a chunk is always 64*NW words long
    uint32_t *cur = smem, *nxt = smem + MT_N, *bm = smem + 2 * MT_N;
    const uint32_t words = (n + 31u) >> 5, kb = bitlen(n);
    uint32_t *first = bm + words;  // [T + 1]: entry T, the dummy slot of non-candidates, is never touched
    const uint32_t tmask = (1u << tlog) - 1u, dummy = tmask + 1u;
    // first-lane table entries: (round << ib) | (imask - ((r >> tlog) << 9 | tid)),
    // taken with atomicMax: the current round's entries beat every older one
    // and, among themselves, the smallest (r >> tlog, word) wins -- the table
    // never needs resetting between rounds
    const uint32_t ib = 9u + (kb > (uint32_t)tlog ? kb - (uint32_t)tlog : 0u);
    const uint32_t imask = (1u << ib) - 1u, emax = (uint32_t)(((uint64_t)1 << (32 - ib)) - 1u);
    uint32_t ep = 1;  // round number (0 = empty)
    const int tid = threadIdx.x, wv = tid >> 6, e = blockIdx.x;
    uint32_t *g = py_state + (size_t)e * DMDQN_MT_WORDS;
    for (int t = tid; t < MT_N; t += NT) cur[t] = g[t];
    int mti = (int)g[MT_N];
    bool ahead = false;  // nxt holds the block after cur
    for (uint32_t t = tid; t < words; t += NT) bm[t] = 0u;
    for (uint32_t t = tid; t <= dummy; t += NT) first[t] = 0u;
    __syncthreads();
    int j = 0, i = 0;
    int32_t *out = idx + (size_t)e * A * k;  // agent j's i-th pick
    while (j < A) {
        if (mti >= MT_N) {  // block-uniform: enter the next block
            if (!ahead) mt_twist_into<NT>(cur, nxt);
            uint32_t *t2 = cur; cur = nxt; nxt = t2;
            mti -= MT_N;
            ahead = false;
        }
        if (!ahead && mti + NT > MT_N) {
            mt_twist_into<NT>(cur, nxt);
            ahead = true;
        }
        const int cnt = NT;
        const int w = mti + tid;
        const uint32_t r = getbits(mt_temper(w < MT_N ? cur[w] : nxt[w - MT_N]), kb);
        const bool inr = r < n;
        const uint32_t bw = bm[inr ? r >> 5 : 0u];
        const bool cand = inr && !((bw >> (r & 31)) & 1u);
        const uint32_t slot = cand ? (r & tmask) : dummy;
        const uint32_t inner = ((r >> tlog) << 9) | (uint32_t)tid;
        bool pend = cand, dup = false;
        uint64_t b;
        do {  // the read of a round sees its every write, the next round's writes wait for it
            if (ep >= emax) {  // block-uniform, after the last round's reads: restart the rounds
                for (uint32_t t = tid; t <= dummy; t += NT) first[t] = 0u;
                __syncthreads();
                ep = 1;
            }
            // only the pending lanes touch the table (round 4's form sent every
            // other lane's max of 0 to the dummy entry: a same-address atomic
            // serialised over up to 256 lanes in every round)
            if (pend) atomicMax(&first[slot], (ep << ib) | (imask - inner));
            __syncthreads();
            if (pend) {
                const uint32_t wi = imask - (first[slot] & imask);  // the winner's (r >> tlog, word)
                if ((wi >> 9) == (inner >> 9)) {  // same r: decided
                    dup = wi != inner;
                    pend = false;
                }
            }
            ep++;
            // the accepted count per wave, final in the round that leaves no lane
            // pending (the loop's barrier publishes it)
            b = __ballot(cand && !dup && !pend);
            if ((tid & 63) == 0) s_cnt[wv] = __popcll(b);
        } while (__syncthreads_or(pend));
        const bool acc = cand && !dup;
        int before = 0, total = 0;
#pragma unroll
        for (int w2 = 0; w2 < NW; w2++) {
            const int c2 = s_cnt[w2];
            before += w2 < wv ? c2 : 0;
            total += c2;
        }
        const int ln = tid & 63;
        const uint64_t below = ln ? (~0ull >> (64 - ln)) : 0ull;
        const int c = before + __popcll(b & below), need = k - i;
        if (total >= need) {  // block-uniform: agent j's last chunk (no bitmap update needed)
            if (acc && c == need - 1) s_cons = tid + 1;
            if (acc && c < need) {
                DMDQN_DBG(r < n, DBG_SAMPLE);
                out[i + c] = (int32_t)r;
            }
            __syncthreads();
            mti += s_cons;
            j++;
            i = 0;
            out += k;
            for (uint32_t t = tid; t < words; t += NT) bm[t] = 0u;
        } else {
            if (acc) {
                DMDQN_DBG(r < n, DBG_SAMPLE);
                out[i + c] = (int32_t)r;
                atomicOr(&bm[r >> 5], 1u << (r & 31));
            }
            mti += cnt;
            i += total;
        }
        __syncthreads();
    }
    if (mti > MT_N) {  // the last pick ended in the next block (at exactly 624 the
                       // stored state stays (cur, 624), as CPython's would)
        uint32_t *t2 = cur; cur = nxt; nxt = t2;
        mti -= MT_N;
    }
    for (int t = tid; t < MT_N; t += NT) g[t] = cur[t];
    if (tid == 0) g[MT_N] = (uint32_t)mti;
}

DMDQN_DBG_READER(dbg_flags_rng)

}  // namespace dmdqn

using namespace dmdqn;

namespace dmdqn {
size_t device_lds_per_block();  // capi.cpp: the current device's per-workgroup LDS
}

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
                       greedy, actions, 1);
    DMDQN_LAUNCH_CHECK("k_act");
    return DMDQN_OK;
}

extern "C" int dmdqn_act_uniform(uint32_t *np_state, int E, int A, int n_actions,
                                 int32_t *actions, void *stream) {
    DMDQN_REQUIRE(np_state && actions && E > 0 && A > 0, "dmdqn_act_uniform: bad args");
    DMDQN_REQUIRE(n_actions >= 1, "dmdqn_act_uniform: n_actions must be >= 1");
    uint32_t rng = (uint32_t)(n_actions - 1), mask = rng;
    mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4; mask |= mask >> 8; mask |= mask >> 16;
    hipLaunchKernelGGL(k_act, dim3(E), dim3(64), 0, as_stream(stream), np_state, A, 1.0, rng, mask,
                       nullptr, actions, 0);
    DMDQN_LAUNCH_CHECK("k_act");
    return DMDQN_OK;
}

extern "C" int dmdqn_replay_sample_budget(uint32_t *py_state, int E, int A, int n, int k,
                                          size_t lds_budget, int32_t *idx, void *stream) {
    DMDQN_REQUIRE(py_state && idx && E > 0 && A > 0, "dmdqn_replay_sample: bad args");
    DMDQN_REQUIRE(k >= 1 && n >= k, "dmdqn_replay_sample: need 1 <= k <= n (k=%d n=%d)", k, n);
    uint32_t setsize = 21;
    if (k > 5) setsize += (uint32_t)pow(4.0, ceil(log((double)k * 3.0) / log(4.0)));
    const bool pool = (uint32_t)n <= setsize;
    DMDQN_REQUIRE(!pool || n <= 65535, "dmdqn_replay_sample: pool branch needs n <= 65535");
    // pool branch: u16 sel [A][k] + u16 pools [min(A,64)][n]; set branch: n-bit bitmap
    size_t aux_bytes = pool ? (((size_t)A * k + 1) & ~(size_t)1) * 2 + (size_t)(A < 64 ? A : 64) * n * 2
                            : (size_t)((n + 31) / 32) * 4;
    size_t lds = 2 * MT_N * sizeof(uint32_t) + aux_bytes;
    // set branch: the first-lane table, 2^tlog u32 entries: no more than n
    // needs, within 39 KB per block in all (four blocks per CU) when that
    // leaves at least 4 KB for it, else up to 32 KB; with lds_budget, within
    // that (e.g. beside the shared learn's S' pass: the trainer's "learn"
    // schedule); DMDQN_OPT_SAMPLE_TLOG caps it (tests: collisions in every
    // chunk).  The table size changes only the speed, never the draws.
    int tlog = 0;
    const size_t lds_max = device_lds_per_block();
    if (lds_budget > lds_max) lds_budget = lds_max;  // never more than a workgroup may hold
    if (!pool) {
        const size_t quad = lds_budget ? lds_budget : 39 * 1024;
        DMDQN_REQUIRE(!lds_budget || quad >= lds + 16 + 4,
                      "dmdqn_replay_sample: lds_budget %zu below the %zu B the set branch needs",
                      lds_budget, lds + 20);
        const size_t room = (quad >= lds + 4096 + 4 || lds_budget) ? quad - lds - 4 : 32 * 1024;
        while (tlog < 20 && ((size_t)4 << (tlog + 1)) <= room && (1u << tlog) < (uint32_t)n) tlog++;
        const int cap = option(DMDQN_OPT_SAMPLE_TLOG);
        if (cap < tlog) tlog = cap;
        lds += ((size_t)4 << tlog) + 4;  // + the dummy entry first[T]
    }
    DMDQN_REQUIRE(lds <= lds_max, "dmdqn_replay_sample: n=%d too large for LDS (%zu > %zu B)", n,
                  lds, lds_max);
    if (!pool) {  // set branch: four waves per stream
        hipLaunchKernelGGL(k_sample_set<4>, dim3(E), dim3(256), lds, as_stream(stream), py_state, A,
                           (uint32_t)n, k, tlog, idx);
        DMDQN_LAUNCH_CHECK("k_sample_set");
        return DMDQN_OK;
    }
    hipLaunchKernelGGL(k_sample, dim3(E), dim3(64), lds, as_stream(stream), py_state, A,
                       (uint32_t)n, k, idx);
    DMDQN_LAUNCH_CHECK("k_sample");
    return DMDQN_OK;
}

extern "C" int dmdqn_replay_sample(uint32_t *py_state, int E, int A, int n, int k, int32_t *idx,
                                   void *stream) {
    return dmdqn_replay_sample_budget(py_state, E, A, n, k, 0, idx, stream);
}
