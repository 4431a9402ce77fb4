// observe.hpp -- device functions shared by the observe and sim kernels.
#pragma once
#include "common.hpp"

namespace dmdqn {

// Neighbour of junction a=(r,c) in direction d (0 n, 1 s, 2 e, 3 w) or -1
// (order_lanes.py:399-405: n=(r-1,c), s=(r+1,c), e=(r,c+1), w=(r,c-1)).
__device__ __forceinline__ int neighbor(int R, int C, int a, int d) {
    int r = a / C, c = a - r * C;
    switch (d) {
        case 0: return r > 0 ? a - C : -1;
        case 1: return r < R - 1 ? a + C : -1;
        case 2: return c < C - 1 ? a + 1 : -1;
        default: return c > 0 ? a - 1 : -1;
    }
}

// Feature f (0..16) of get_own_state (order_lanes.py:430-499).
__device__ __forceinline__ float local_feature(int f, const int32_t *halt12, int phase,
                                               int tspent, int mode) {
    if (f < 12) return (float)halt12[f];
    if (f < 16) return (mode == 1 && phase == f - 12) ? 1.0f : 0.0f;  // PHASE_ENCODING
    return mode == 1 ? (float)tspent : -1.0f;
}

// Element i (0..88) of build_state_vector for agent a, from loc[A][17].
__device__ __forceinline__ float obs_feature(int R, int C, int a, int i, const float *loc) {
    if (i < 17) return loc[a * 17 + i];
    if (i < 21) return neighbor(R, C, a, i - 17) >= 0 ? 1.0f : 0.0f;
    int d = (i - 21) / 17, f = (i - 21) - d * 17;
    int b = neighbor(R, C, a, d);
    return b >= 0 ? loc[b * 17 + f] : -1.0f;
}

// train.py:254  0.3 * local_reward + 0.7 * global_reward  (Python floats).
__device__ __forceinline__ double combine_reward(double local_r, double global_r) {
    double x = __dmul_rn(0.3, local_r);
    double y = __dmul_rn(0.7, global_r);
    return __dadd_rn(x, y);
}

}  // namespace dmdqn
