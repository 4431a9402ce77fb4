// sim.hpp -- grid geometry, routing, signal program and IDM for sim.hip.
#pragma once
#include "common.hpp"

namespace dmdqn {

// 12-phase program of every tlLogic in grid_3x3.net.xml:893-906 (actuated
// min/max of phase 0 ignored: fixed 25 s).
__constant__ int kPhaseDur[12] = {25, 6, 2, 20, 6, 2, 25, 6, 2, 20, 6, 2};
// Green movements per phase: bit (d*4 + m), approach d = 0 n,1 s,2 e,3 w
// (side the vehicle comes from), movement m = 0 right,1 straight,2 left,
// 3 U-turn.  'G' and 'g' are green, 'y' and 'r' stop.  Derived from the
// phase strings with the link layout of grid_3x3.net.xml:1375-1461
// (per approach: r, s, s, -, l, t).
__constant__ uint32_t kGreen[12] = {0x11BB, 0, 0, 0x11DD, 0, 0, 0xBB11, 0, 0, 0xDD11, 0, 0};

constexpr int kArrive = -2;
enum { DIR_N = 0, DIR_S = 1, DIR_E = 2, DIR_W = 3 };
enum { MV_R = 0, MV_S = 1, MV_L = 2, MV_U = 3 };

__device__ __forceinline__ int opp(int d) { return d ^ 1; }
__device__ __forceinline__ int right_of(int h) {  // n->e, s->w, e->s, w->n
    return h == DIR_N ? DIR_E : h == DIR_S ? DIR_W : h == DIR_E ? DIR_S : DIR_N;
}
__device__ __forceinline__ int movement(int h, int o) {
    if (o == h) return MV_S;
    if (o == opp(h)) return MV_U;
    if (o == right_of(h)) return MV_R;
    return MV_L;
}

__device__ __forceinline__ int nbr(int a, int d, int R, int C) {
    int r = a / C, c = a - r * C;
    switch (d) {
        case DIR_N: return r > 0 ? a - C : -1;
        case DIR_S: return r < R - 1 ? a + C : -1;
        case DIR_E: return c < C - 1 ? a + 1 : -1;
        default: return c > 0 ? a - 1 : -1;
    }
}

__device__ __forceinline__ float lane_length(int e, int A, int R, int C, const dmdqn_idm &P) {
    if (e >= 4 * A) return P.len_outer;
    return nbr(e >> 2, e & 3, R, C) >= 0 ? P.len_inner : P.len_outer;
}

// Out-direction at junction a for a vehicle heading h toward destination edge
// dst: move toward the junction the destination edge leaves from, keeping
// straight when that reduces the distance, vertical before horizontal, a
// U-turn only when it is the only reducing move; at that junction take the
// destination's direction.
__device__ __forceinline__ int route_out(int a, int h, int dst, int R, int C,
                                         const int32_t *exit_ao) {
    const int A = R * C;
    int tj, to;
    if (dst >= 4 * A) {
        int x = dst - 4 * A;
        tj = exit_ao[2 * x];
        to = exit_ao[2 * x + 1];
    } else {
        int b = dst >> 2, db = dst & 3;
        tj = nbr(b, db, R, C);
        to = opp(db);
    }
    if (a == tj) return to;
    int r = a / C, c = a - r * C, rt = tj / C, ct = tj - rt * C;
    int dv = rt < r ? DIR_N : (rt > r ? DIR_S : -1);
    int dh = ct > c ? DIR_E : (ct < c ? DIR_W : -1);
    if (h == dv || h == dh) return h;
    if (dv >= 0 && dv != opp(h)) return dv;
    if (dh >= 0 && dh != opp(h)) return dh;
    return dv >= 0 ? dv : dh;
}

__device__ __forceinline__ int next_edge(int a, int o, int R, int C, const int32_t *exit_id) {
    int nb = nbr(a, o, R, C);
    return nb >= 0 ? nb * 4 + opp(o) : 4 * R * C + exit_id[a * 4 + o];
}

// Lane index for movement m on incoming edge e: right -> 0, left/U -> 2,
// straight -> the emptier of lanes 0/1 (ties -> 1).
__device__ __forceinline__ int lane_for_move(int m, int e, const int32_t *cnt) {
    if (m == MV_R) return 0;
    if (m != MV_S) return 2;
    return cnt[e * 3 + 1] <= cnt[e * 3 + 0] ? 1 : 0;
}

// Lane a vehicle takes when entering edge e2 from lane index kf.
__device__ __forceinline__ int lane_for(int e2, int kf, int dst, const int32_t *cnt, int A,
                                        int R, int C, const int32_t *exit_ao) {
    if (e2 >= 4 * A || e2 == dst) return kf;  // connections keep the lane index
    int h2 = opp(e2 & 3);
    int o2 = route_out(e2 >> 2, h2, dst, R, C, exit_ao);
    return lane_for_move(movement(h2, o2), e2, cnt);
}

// The 5 lanes that can feed edge e2 (in approach order n,s,e,w, lane order).
// Returns false for fringe-in edges (nothing upstream).
__device__ __forceinline__ bool feeders(int e2, int A, int R, int C, const int32_t *exit_ao,
                                        int fl[5]) {
    int as, o;
    if (e2 < 4 * A) {
        as = nbr(e2 >> 2, e2 & 3, R, C);
        if (as < 0) return false;
        o = opp(e2 & 3);
    } else {
        int x = e2 - 4 * A;
        as = exit_ao[2 * x];
        o = exit_ao[2 * x + 1];
    }
    int n = 0;
    for (int d = 0; d < 4; d++) {
        int m = movement(opp(d), o), base = (as * 4 + d) * 3;
        if (m == MV_S) {
            fl[n++] = base;
            fl[n++] = base + 1;
        } else if (m == MV_R) {
            fl[n++] = base;
        } else {
            fl[n++] = base + 2;
        }
    }
    return true;
}

// IDM (Treiber): a [1 - (v/v0)^4 - (s*/s)^2], s* = s0 + max(0, vT + v dv/(2 sqrt(ab))).
// Fixed evaluation order (mirrored by oracle/oracle_sim.c).
__device__ __forceinline__ float idm_free(float v, const dmdqn_idm &P) {
    float r = v / P.vmax;
    float r2 = r * r;
    float r4 = r2 * r2;
    return P.accel * (1.0f - r4);
}

__device__ __forceinline__ float idm_acc(float v, float s, float dv, const dmdqn_idm &P) {
    float r = v / P.vmax;
    float r2 = r * r;
    float r4 = r2 * r2;
    float ss = v * P.tau + (v * dv) / P.two_sqrt_ab;
    if (ss < 0.0f) ss = 0.0f;
    float sstar = P.min_gap + ss;
    if (s < 0.01f) s = 0.01f;
    float q = sstar / s;
    float t1 = 1.0f - r4;
    return P.accel * (t1 - q * q);
}

__device__ __forceinline__ float clamp_speed(float v, const dmdqn_idm &P) {
    if (v < 0.0f) return 0.0f;
    if (v > P.vmax) return P.vmax;
    return v;
}

}  // namespace dmdqn
