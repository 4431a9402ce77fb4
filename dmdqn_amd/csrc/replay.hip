// replay.hip -- replay ring store (ReplayBuffer.add, src/agents/dqn_agent.py:31-57).
//
// Layout (per agent slot, capacity cap, ring position = total_adds % cap):
//   ring_s, ring_n : int8  [NA][cap][128]  s and s' rows: features 0..88, zero
//                                          to byte 95; the s' row also holds a
//                                          (byte 96), done (97) and r (f64,
//                                          104..111) -- the learn kernels' copy
//   ring_a         : uint8 [NA][cap]
//   ring_r         : f64   [NA][cap]       Python-float reward, kept in f64 so
//                                          the batch z-score is numpy-exact
//   ring_d         : uint8 [NA][cap]
// Observations of this env are small integers (queue counts <= 23, one-hot,
// time spent, -1 padding), so int8 storage is exact; any value that is not an
// integer in [-128,127] sets *err = DMDQN_ERANGE instead of being rounded.
#include "common.hpp"

namespace dmdqn {

// One thread per (agent, 4-byte group): 32 groups of 4 bytes per row.
__global__ void k_replay_store(int NA, int cap, int slot, const float *obs_s, const float *obs_n,
                               const int32_t *act, const double *rew, const uint8_t *done,
                               int8_t *ring_s, int8_t *ring_n, uint8_t *ring_a, double *ring_r,
                               uint8_t *ring_d, int32_t *err) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    constexpr int G = DMDQN_ROW_BYTES / 4;
    const int agent = t / G, grp = t - agent * G;
    if (agent >= NA) return;
    const size_t row = ((size_t)agent * cap + slot);
    uint32_t ws = 0, wn = 0;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int i = grp * 4 + q;
        if (i < DMDQN_OBS_DIM) {
            ws |= (uint32_t)(uint8_t)to_i8(obs_s[(size_t)agent * DMDQN_OBS_DIM + i], err) << (8 * q);
            wn |= (uint32_t)(uint8_t)to_i8(obs_n[(size_t)agent * DMDQN_OBS_DIM + i], err) << (8 * q);
        }
    }
    if (4 * grp == DMDQN_ROW_A) {
        static_assert(DMDQN_ROW_D == DMDQN_ROW_A + 1, "a and done share a word");
        wn = (uint32_t)(uint8_t)act[agent] | (done[agent] ? 1u : 0u) << 8;
    } else if (4 * grp == DMDQN_ROW_R || 4 * grp == DMDQN_ROW_R + 4) {
        const unsigned long long rb = __double_as_longlong(rew[agent]);
        wn = (uint32_t)(4 * grp == DMDQN_ROW_R ? rb : rb >> 32);
    }
    reinterpret_cast<uint32_t *>(ring_s + row * DMDQN_ROW_BYTES)[grp] = ws;
    reinterpret_cast<uint32_t *>(ring_n + row * DMDQN_ROW_BYTES)[grp] = wn;
    if (grp == 0) {
        ring_a[row] = (uint8_t)act[agent];
        ring_r[row] = rew[agent];
        ring_d[row] = done[agent] ? 1 : 0;
    }
}

// Float rows (DMDQN_ROWS_F32): one thread per (agent, feature group of 4).
__global__ void k_replay_store_f32(int NA, int cap, int slot, const float *obs_s, const float *obs_n,
                                   const int32_t *act, const double *rew, const uint8_t *done,
                                   float *rows_s, float *rows_n, uint8_t *ring_a, double *ring_r,
                                   uint8_t *ring_d) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    constexpr int G = DMDQN_ROW_FLOATS / 4;
    const int agent = t / G, grp = t - agent * G;
    if (agent >= NA) return;
    const size_t row = (size_t)agent * cap + slot;
    float4 vs = make_float4(0.f, 0.f, 0.f, 0.f), vn = vs;
    float *ps = &vs.x, *pn = &vn.x;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int i = grp * 4 + q;
        if (i < DMDQN_OBS_DIM) {
            ps[q] = obs_s[(size_t)agent * DMDQN_OBS_DIM + i];
            pn[q] = obs_n[(size_t)agent * DMDQN_OBS_DIM + i];
        }
    }
    reinterpret_cast<float4 *>(rows_s + row * DMDQN_ROW_FLOATS)[grp] = vs;
    reinterpret_cast<float4 *>(rows_n + row * DMDQN_ROW_FLOATS)[grp] = vn;
    if (grp == 0) {
        ring_a[row] = (uint8_t)act[agent];
        ring_r[row] = rew[agent];
        ring_d[row] = done[agent] ? 1 : 0;
    }
}

// xs / xn [NA][batch][96] <- the sampled rows, in batch order.
__global__ void k_replay_gather_f32(const float *rows_s, const float *rows_n, const int32_t *idx,
                                    int NA, int cap, int start, int batch, float *xs, float *xn) {
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    constexpr int G = DMDQN_ROW_FLOATS / 4;
    const size_t rowi = t / G;
    const int grp = (int)(t - rowi * G);
    if (rowi >= (size_t)NA * batch) return;
    const int agent = (int)(rowi / batch);
    int pos = idx[rowi];
    DMDQN_DBG(pos >= 0 && pos < cap, DBG_LEARN_IDX);  // as the int8 learn's gather
#ifdef DMDQN_DEBUG_BOUNDS
    if (pos < 0 || pos >= cap) pos = 0;
#endif
    int s = start + pos;
    if (s >= cap) s -= cap;
    const size_t src = ((size_t)agent * cap + s) * DMDQN_ROW_FLOATS;
    reinterpret_cast<float4 *>(xs + rowi * DMDQN_ROW_FLOATS)[grp] =
        reinterpret_cast<const float4 *>(rows_s + src)[grp];
    reinterpret_cast<float4 *>(xn + rowi * DMDQN_ROW_FLOATS)[grp] =
        reinterpret_cast<const float4 *>(rows_n + src)[grp];
}

DMDQN_DBG_READER(dbg_flags_replay)

}  // namespace dmdqn

using namespace dmdqn;

extern "C" int dmdqn_replay_store_f32(int NA, int cap, int slot, const float *obs_s,
                                      const float *obs_n, const int32_t *act, const double *rew,
                                      const uint8_t *done, float *rows_s, float *rows_n,
                                      uint8_t *ring_a, double *ring_r, uint8_t *ring_d,
                                      void *stream) {
    DMDQN_REQUIRE(NA > 0 && cap > 0 && slot >= 0 && slot < cap,
                  "dmdqn_replay_store_f32: NA=%d cap=%d slot=%d", NA, cap, slot);
    DMDQN_REQUIRE(obs_s && obs_n && act && rew && done && rows_s && rows_n && ring_a && ring_r &&
                      ring_d,
                  "dmdqn_replay_store_f32: null pointer");
    const int threads = NA * (DMDQN_ROW_FLOATS / 4);
    hipLaunchKernelGGL(k_replay_store_f32, dim3((threads + 255) / 256), dim3(256), 0,
                       as_stream(stream), NA, cap, slot, obs_s, obs_n, act, rew, done, rows_s,
                       rows_n, ring_a, ring_r, ring_d);
    DMDQN_LAUNCH_CHECK("k_replay_store_f32");
    return DMDQN_OK;
}

extern "C" int dmdqn_replay_gather_f32(const float *rows_s, const float *rows_n,
                                       const int32_t *idx, int NA, int cap, int start, int batch,
                                       float *xs, float *xn, void *stream) {
    DMDQN_REQUIRE(rows_s && rows_n && idx && xs && xn, "dmdqn_replay_gather_f32: null pointer");
    DMDQN_REQUIRE(NA > 0 && cap > 0 && batch > 0 && start >= 0 && start < cap,
                  "dmdqn_replay_gather_f32: NA=%d cap=%d start=%d batch=%d", NA, cap, start, batch);
    const size_t threads = (size_t)NA * batch * (DMDQN_ROW_FLOATS / 4);
    hipLaunchKernelGGL(k_replay_gather_f32, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0,
                       as_stream(stream), rows_s, rows_n, idx, NA, cap, start, batch, xs, xn);
    DMDQN_LAUNCH_CHECK("k_replay_gather_f32");
    return DMDQN_OK;
}

extern "C" int dmdqn_replay_store(int NA, int cap, int slot, const float *obs_s,
                                  const float *obs_n, const int32_t *act, const double *rew,
                                  const uint8_t *done, int8_t *ring_s, int8_t *ring_n,
                                  uint8_t *ring_a, double *ring_r, uint8_t *ring_d,
                                  int32_t *err, void *stream) {
    DMDQN_REQUIRE(NA > 0 && cap > 0 && slot >= 0 && slot < cap,
                  "dmdqn_replay_store: NA=%d cap=%d slot=%d", NA, cap, slot);
    DMDQN_REQUIRE(obs_s && obs_n && act && rew && done && ring_s && ring_n && ring_a && ring_r &&
                      ring_d && err,
                  "dmdqn_replay_store: null pointer");
    const int threads = NA * (DMDQN_ROW_BYTES / 4);
    hipLaunchKernelGGL(k_replay_store, dim3((threads + 255) / 256), dim3(256), 0,
                       as_stream(stream), NA, cap, slot, obs_s, obs_n, act, rew, done, ring_s,
                       ring_n, ring_a, ring_r, ring_d, err);
    DMDQN_LAUNCH_CHECK("k_replay_store");
    return DMDQN_OK;
}
