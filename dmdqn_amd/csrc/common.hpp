// common.hpp -- shared host/device helpers for the dmdqn HIP kernels (gfx950).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string>

#include "../../include/dmdqn.h"

namespace dmdqn {

// ---------------------------------------------------------------- host side
void set_error(const char *fmt, ...);

#define DMDQN_REQUIRE(cond, ...)          \
    do {                                  \
        if (!(cond)) {                    \
            ::dmdqn::set_error(__VA_ARGS__); \
            return DMDQN_EINVAL;          \
        }                                 \
    } while (0)

#define DMDQN_LAUNCH_CHECK(what)                                              \
    do {                                                                      \
        hipError_t e_ = hipGetLastError();                                    \
        if (e_ != hipSuccess) {                                               \
            ::dmdqn::set_error("%s: %s", what, hipGetErrorString(e_));        \
            return DMDQN_EHIP;                                                \
        }                                                                     \
    } while (0)

inline hipStream_t as_stream(void *s) { return reinterpret_cast<hipStream_t>(s); }

// Run-time options (include/dmdqn.h DMDQN_OPT_*): read from the environment
// once, when the library loads (capi.cpp), then only through dmdqn_set_option.
int option(int which);

// ---------------------------------------------------------------- debug-bounds build
// Built with -DDMDQN_DEBUG_BOUNDS (python -m dmdqn_amd.build --debug ->
// libdmdqn_hip_debug.so): kernels check the indices they derive and
// OR a bit into a per-source-file device flag (the bad index is clamped, so
// nothing is touched out of range); dmdqn_debug_status() returns and clears
// the flags of every file.  The normal build compiles the checks to nothing.
enum : int {
    DBG_SIM_RING = 1,     // lane head / count / append slot outside its ring
    DBG_SIM_EDGE = 2,     // a route leaves the grid where there is no exit edge
    DBG_SAMPLE = 4,       // a replay index outside [0, n)
    DBG_LEARN_IDX = 8,    // a deque position outside [0, cap)
    DBG_LEARN_ACT = 16,   // a stored action outside [0, 4)
};
#ifdef DMDQN_DEBUG_BOUNDS
static __device__ int g_dbg_flags;
#define DMDQN_DBG(cond, bit)                                                   \
    do {                                                                       \
        if (!(cond)) atomicOr(&::dmdqn::g_dbg_flags, (int)(bit));             \
    } while (0)
#define DMDQN_DBG_READER(fn)                                                   \
    int fn() {                                                                 \
        int v = 0, z = 0;                                                      \
        if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(::dmdqn::g_dbg_flags), sizeof(int)) != hipSuccess) \
            return -1;                                                         \
        if (hipMemcpyToSymbol(HIP_SYMBOL(::dmdqn::g_dbg_flags), &z, sizeof(int)) != hipSuccess) \
            return -1;                                                         \
        return v;                                                              \
    }
#else
#define DMDQN_DBG(cond, bit) do { } while (0)
#define DMDQN_DBG_READER(fn) \
    int fn() { return 0; }
#endif

// ---------------------------------------------------------------- MT19937
// One stream = 624 state words + position.  Device kernels that consume a
// stream run ONE wave (64 lanes) per stream: the state lives in LDS, the twist
// is done cooperatively, and the (data-dependent) consumption loop is executed
// wave-uniformly so every lane sees the same draw.
constexpr int MT_N = 624;
constexpr int MT_M = 397;

__device__ __forceinline__ uint32_t mt_temper(uint32_t y) {
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}

__device__ __forceinline__ uint32_t mt_mix(uint32_t hi_word, uint32_t lo_word, uint32_t far) {
    uint32_t y = (hi_word & 0x80000000u) | (lo_word & 0x7fffffffu);
    return far ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
}

// Cooperative twist of mt[624] in LDS by the 64 lanes of a one-wave block.
// Sequential semantics (CPython _randommodule.c genrand_uint32) are kept by
// splitting the index range where the recurrence reads freshly written words:
//   [0,227) reads old mt[k+397]; [227,454) reads new mt[k-227] from [0,227);
//   [454,623) reads new mt[k-227] from [227,396); 623 reads new mt[0], mt[396].
__device__ inline void mt_twist_wave(uint32_t *mt) {
    const int l = threadIdx.x;
    uint32_t nv[4];
    // phase 1
#pragma unroll
    for (int c = 0; c < 4; c++) {
        int k = c * 64 + l;
        if (k < 227) nv[c] = mt_mix(mt[k], mt[k + 1], mt[k + MT_M]);
    }
    __syncthreads();
#pragma unroll
    for (int c = 0; c < 4; c++) {
        int k = c * 64 + l;
        if (k < 227) mt[k] = nv[c];
    }
    __syncthreads();
    // phase 2a: k in [227,454)
#pragma unroll
    for (int c = 0; c < 4; c++) {
        int k = 227 + c * 64 + l;
        if (k < 454) nv[c] = mt_mix(mt[k], mt[k + 1], mt[k - 227]);
    }
    __syncthreads();
#pragma unroll
    for (int c = 0; c < 4; c++) {
        int k = 227 + c * 64 + l;
        if (k < 454) mt[k] = nv[c];
    }
    __syncthreads();
    // phase 2b: k in [454,623)
#pragma unroll
    for (int c = 0; c < 3; c++) {
        int k = 454 + c * 64 + l;
        if (k < 623) nv[c] = mt_mix(mt[k], mt[k + 1], mt[k - 227]);
    }
    __syncthreads();
#pragma unroll
    for (int c = 0; c < 3; c++) {
        int k = 454 + c * 64 + l;
        if (k < 623) mt[k] = nv[c];
    }
    __syncthreads();
    if (l == 0) mt[623] = mt_mix(mt[623], mt[0], mt[MT_M - 1]);
    __syncthreads();
}

// The same twist by a block of NT >= 256 threads: one word per thread per
// phase instead of four chunks of 64 lanes (every lane past the first wave
// would redo them).
template <int NT>
__device__ inline void mt_twist_block(uint32_t *mt) {
    static_assert(NT >= 256, "one word per thread per phase");
    const int k = threadIdx.x;
    uint32_t nv = 0;
    if (k < 227) nv = mt_mix(mt[k], mt[k + 1], mt[k + MT_M]);
    __syncthreads();
    if (k < 227) mt[k] = nv;
    __syncthreads();
    if (k < 227) nv = mt_mix(mt[227 + k], mt[228 + k], mt[k]);
    __syncthreads();
    if (k < 227) mt[227 + k] = nv;
    __syncthreads();
    if (k < 169) nv = mt_mix(mt[454 + k], mt[455 + k], mt[227 + k]);
    __syncthreads();
    if (k < 169) mt[454 + k] = nv;
    __syncthreads();
    if (k == 0) mt[623] = mt_mix(mt[623], mt[0], mt[MT_M - 1]);
    __syncthreads();
}

// The next 624-word block of the stream whose current raw block is cur,
// written to nxt (cur unchanged): the same recurrence as mt_twist_wave with
// the freshly written words read from nxt, so the phases need no read/write
// split.  A block of NT >= 256 threads, one word per thread per phase.
template <int NT>
__device__ inline void mt_twist_into(const uint32_t *cur, uint32_t *nxt) {
    static_assert(NT >= 256, "one word per thread per phase");
    const int k = threadIdx.x;
    if (k < 227) nxt[k] = mt_mix(cur[k], cur[k + 1], cur[k + MT_M]);
    __syncthreads();
    if (k < 227) nxt[227 + k] = mt_mix(cur[227 + k], cur[228 + k], nxt[k]);
    __syncthreads();
    if (k < 169) nxt[454 + k] = mt_mix(cur[454 + k], cur[455 + k], nxt[227 + k]);
    __syncthreads();
    if (k == 0) nxt[623] = mt_mix(cur[623], nxt[0], nxt[MT_M - 1]);
    __syncthreads();
}

// Wave-resident stream: raw state words in LDS plus a tempered copy of the
// current block (tempered in parallel right after each twist) so the
// sequential consumer does one LDS read per draw.
struct MTWave {
    uint32_t *mt;    // [624] LDS
    uint32_t *out;   // [624] LDS, tempered outputs of the current block
    int mti;         // wave-uniform position

    __device__ void load(const uint32_t *g) {
        for (int i = threadIdx.x; i < MT_N; i += 64) mt[i] = g[i];
        mti = (int)g[MT_N];
        __syncthreads();
        for (int i = threadIdx.x; i < MT_N; i += 64) out[i] = mt_temper(mt[i]);
        __syncthreads();
    }
    __device__ void store(uint32_t *g) const {
        for (int i = threadIdx.x; i < MT_N; i += 64) g[i] = mt[i];
        if (threadIdx.x == 0) g[MT_N] = (uint32_t)mti;
    }
    __device__ void refill() {
        mt_twist_wave(mt);
        for (int i = threadIdx.x; i < MT_N; i += 64) out[i] = mt_temper(mt[i]);
        __syncthreads();
        mti = 0;
    }
    // Wave-uniform: every lane calls it with the same control flow.
    __device__ __forceinline__ uint32_t next() {
        if (mti >= MT_N) refill();
        return out[mti++];
    }
};

// numpy legacy random_sample: ((u>>5) * 2^26 + (u>>6)) / 2^53 (exact in f64).
__device__ __forceinline__ double np_double(MTWave &w) {
    int32_t a = (int32_t)(w.next() >> 5);
    int32_t b = (int32_t)(w.next() >> 6);
    return ((double)a * 67108864.0 + (double)b) / 9007199254740992.0;
}

// select_action's draws without staging the stream, when every agent's draw
// count is fixed: eps >= 1 (the reference's training path keeps epsilon at
// 1.0, A-1) and a power-of-two action count (randint never redraws).  Then
// rand() always passes (r < 1 <= eps) and agent j consumes the `per` words
// per*j .. per*j + per-1 of the stream (per = 3: two for rand(), one for
// randint; per = 1: randint alone, test.py:92-93) and its action is the last
// one & mask: one load of the raw state per agent.  Valid while the A*per
// words lie inside the current 624-word block (mti + A*per <= 624), i.e. no
// twist is due; the caller checks act_fast_ok and writes the new position
// mti + A*per after every thread has read the old one.
__device__ __forceinline__ bool act_fast_ok(int mti, int A, int per, double eps, uint32_t rng,
                                           uint32_t mask, int draw_rand) {
    return (!draw_rand || eps >= 1.0) && rng == mask && mti + A * per <= MT_N;
}
__device__ __forceinline__ int32_t act_fast(const uint32_t *g, int mti, int j, int per,
                                            uint32_t mask) {
    return (int32_t)(mt_temper(g[mti + per * j + per - 1]) & mask);
}

// An observation value as an exact int8 replay byte (ReplayBuffer.add's float32
// row, dqn_agent.py:39-56, holds this env's small integers exactly); anything
// else sets *err = DMDQN_ERANGE and stores 0.
__device__ __forceinline__ int8_t to_i8(float v, int32_t *err) {
    float r = rintf(v);
    if (!(r == v) || r < -128.0f || r > 127.0f) {
        // every writer stores the same code: a plain store (err may be pinned
        // host memory, where device atomics are not available)
        *reinterpret_cast<volatile int32_t *>(err) = DMDQN_ERANGE;
        return 0;
    }
    return (int8_t)(int)r;
}

// Learn metrics of dqn_agent.py:361-363 for one agent's batch: sum and sum of
// squares of the online Q(S) values [128][4] (q_values_mean / _std) and the
// histogram of the batch actions (action_distribution), added into
// qstats[agent][6].  Called by every thread after Q(S) is in z3; waves 0-1
// (batch rows 0..127) contribute, no barrier inside.
__device__ inline void learn_qstats(float *qstats, int agent, const float *z3, const int *act) {
    const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
    if (w >= 2) return;
    const float4 q = *reinterpret_cast<const float4 *>(z3 + tid * 4);
    float s1 = (q.x + q.y) + (q.z + q.w);
    float s2 = (q.x * q.x + q.y * q.y) + (q.z * q.z + q.w * q.w);
    for (int off = 32; off > 0; off >>= 1) {
        s1 += __shfl_xor(s1, off);
        s2 += __shfl_xor(s2, off);
    }
    const int ac = act[tid];
    float cnt[4];
#pragma unroll
    for (int k = 0; k < 4; k++) cnt[k] = (float)__popcll(__ballot(ac == k));
    if (l == 0) {
        float *o = qstats + (size_t)agent * 6;
        atomicAdd(o + 0, s1);
        atomicAdd(o + 1, s2);
#pragma unroll
        for (int k = 0; k < 4; k++) atomicAdd(o + 2 + k, cnt[k]);
    }
}

// Per-row loss term and dL/dq for a batch of B rows, diff = q - y:
//   DMDQN_LOSS_MSE    (dqn_agent.py:352, MeanSquaredError): diff^2, 2 diff / B
//   DMDQN_LOSS_HUBER  (src/experimental/agent.py:99, keras Huber, delta 1):
//                     |d| <= 1 ? d^2 / 2 : |d| - 1/2,  clip(d, -1, 1) / B
// The loss is the mean of the terms.  kind is uniform over the block, so the
// select costs two VALU ops per row.
// An f32 product the compiler may not fuse into an fma with the add that
// consumes it, whatever the file's -ffp-contract (clang's "fast", which the
// learn files use for their MFMA epilogues, fuses across statements and
// disregards `#pragma clang fp contract(off)`): the empty asm makes the
// rounded product opaque.  For the arithmetic that must round every op as
// TF's separate elementwise kernels do -- Keras-3 Adam, the TD target, the
// squared error.
__device__ __forceinline__ float mul_rn(float a, float b) {
    float p = a * b;
    asm("" : "+v"(p));
    return p;
}

__device__ __forceinline__ void loss_term(int kind, float diff, float inv_b, float &term,
                                          float &dq) {
    if (kind == DMDQN_LOSS_HUBER) {
        const float ae = fabsf(diff);
        term = ae <= 1.0f ? mul_rn(0.5f * diff, diff) : ae - 0.5f;
        dq = (ae <= 1.0f ? diff : copysignf(1.0f, diff)) * inv_b;
    } else {
        term = mul_rn(diff, diff);
        dq = 2.0f * diff * inv_b;
    }
}

}  // namespace dmdqn
