// sim.hpp -- grid geometry, routing, signal program and IDM for sim.hip.
#pragma once
#include "common.hpp"

namespace dmdqn {

// 12-phase program of every tlLogic in grid_3x3.net.xml:893-906 (actuated
// min/max of phase 0 ignored: fixed 25 s): 25, 6, 2, 20, 6, 2, 25, 6, 2, 20,
// 6, 2.  Computed with selects instead of a table: a per-lane index into a
// __constant__ array is a vector memory load (L2 latency inside every pass).
__device__ __forceinline__ int phase_dur(int p) {
    const int r = p - 3 * (p / 3);
    return r == 1 ? 6 : r == 2 ? 2 : (p == 3 || p == 9) ? 20 : 25;
}
// Green movements per phase: bit (d*4 + m), approach d = 0 n,1 s,2 e,3 w
// (side the vehicle comes from), movement m = 0 right,1 straight,2 left,
// 3 U-turn.  'G' and 'g' are green, 'y' and 'r' stop.  Derived from the
// phase strings with the link layout of grid_3x3.net.xml:1375-1461
// (per approach: r, s, s, -, l, t): phases 0, 3, 6, 9 -> 0x11BB, 0x11DD,
// 0xBB11, 0xDD11, the rest none.
__device__ __forceinline__ uint32_t green_mask(int p) {
    uint32_t g = p == 0 ? 0x11BBu : 0u;
    g = p == 3 ? 0x11DDu : g;
    g = p == 6 ? 0xBB11u : g;
    return p == 9 ? 0xDD11u : g;
}
// Actuated mode (dmdqn_sim.actuated): phase 0 carries minDur 5 / maxDur 50
// (grid_3x3.net.xml:894); the others have no actuation range.
constexpr int kActMin = 5, kActMax = 50;
constexpr int kNoDetection = -1000;

// Observed lanes (lane k of approach d) with a green link in phase p: lane 0
// carries right + straight, lane 1 straight, lane 2 left + U-turn.  Bit d*3+k.
__host__ __device__ constexpr uint32_t green_lanes(uint32_t g) {
    uint32_t out = 0;
    for (int d = 0; d < 4; d++) {
        const uint32_t m = (g >> (4 * d)) & 15u;
        out |= (m & 3u ? 1u : 0u) << (3 * d);
        out |= (m & 2u ? 1u : 0u) << (3 * d + 1);
        out |= (m & 12u ? 1u : 0u) << (3 * d + 2);
    }
    return out;
}

// threadIdx.x behind an empty asm (the value the compiler cannot see through):
// expressions of it are recomputed where they are used instead of being
// hoisted out of a loop and held in (or spilled from) registers.
__device__ __forceinline__ int opaque_tid() {
    int t = threadIdx.x;
    asm volatile("" : "+v"(t));
    return t;
}

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

// Static grid topology as LDS tables, built once per launch (k_sim_step), so
// that no pass divides by the runtime grid width:
//   jrc[a]    = r * 16 + c of junction a = r*C + c
//   dinfo[e]  = tj * 4 + to for destination edge e: the junction tj to steer
//               toward and the out-direction `to` taken there (approach edge
//               b*4+db: tj = nbr(b, db), to = opp(db); exit x: exit_ao[x])
struct Topo {
    int R, C, A;
    const int32_t *jrc, *dinfo, *exit_id, *exit_ao;
    const float *elen;  // [4A + X] lane length of each edge

    __device__ __forceinline__ int row(int a) const { return jrc[a] >> 4; }
    __device__ __forceinline__ int col(int a) const { return jrc[a] & 15; }
    __device__ __forceinline__ int nbr(int a, int d) const {
        const int rc = jrc[a], r = rc >> 4, c = rc & 15;
        switch (d) {
            case DIR_N: return r > 0 ? a - C : -1;
            case DIR_S: return r < R - 1 ? a + C : -1;
            case DIR_E: return c < C - 1 ? a + 1 : -1;
            default: return c > 0 ? a - 1 : -1;
        }
    }
};

// Bytes of the tables for an R x C grid (dynamic LDS, 4-byte entries).
__host__ __device__ inline size_t topo_bytes(int R, int C) {
    const int A = R * C, X = 2 * R + 2 * C;
    return (size_t)(A + (4 * A + X) + 4 * A + 2 * X + (4 * A + X)) * 4;
}

// Fill the tables at `mem` (all threads; caller syncs) and return the view.
__device__ __forceinline__ Topo build_topo(int32_t *mem, int R, int C, const int32_t *g_exit_id,
                                           const int32_t *g_exit_ao, float len_inner,
                                           float len_outer) {
    const int A = R * C, X = 2 * R + 2 * C, NE = 4 * A + X, tid = threadIdx.x,
              nt = blockDim.x;
    int32_t *jrc = mem, *dinfo = jrc + A, *xid = dinfo + NE, *xao = xid + 4 * A;
    float *elen = reinterpret_cast<float *>(xao + 2 * X);
    if (nt >= NE && nt >= 4 * A && nt >= 2 * X) {
        // one entry of each table per thread: every load issued before the
        // first store (one memory round trip; the loops below wait per table)
        const int i = tid, ex = i - 4 * A;
        const bool isx = ex >= 0 && i < NE;
        const int vid = g_exit_id[i < 4 * A ? i : 0], vao = g_exit_ao[i < 2 * X ? i : 0];
        const int xtj = g_exit_ao[isx ? 2 * ex : 0], xto = g_exit_ao[isx ? 2 * ex + 1 : 0];
        if (i < A) jrc[i] = (i / C) * 16 + (i % C);
        if (i < 4 * A) xid[i] = vid;
        if (i < 2 * X) xao[i] = vao;
        if (i < NE) {
            int tj = xtj, to = xto;
            bool inner = false;
            if (!isx) {
                const int b = i >> 2, db = i & 3, r = b / C, c = b % C;
                tj = db == DIR_N ? (r > 0 ? b - C : -1) : db == DIR_S ? (r < R - 1 ? b + C : -1)
                   : db == DIR_E ? (c < C - 1 ? b + 1 : -1) : (c > 0 ? b - 1 : -1);
                inner = tj >= 0;
                if (tj < 0) tj = 0;
                to = opp(db);
            }
            dinfo[i] = tj * 4 + to;
            elen[i] = inner ? len_inner : len_outer;
        }
        return Topo{R, C, A, jrc, dinfo, xid, xao, elen};
    }
    for (int a = tid; a < A; a += nt) jrc[a] = (a / C) * 16 + (a % C);
    for (int i = tid; i < 4 * A; i += nt) xid[i] = g_exit_id[i];
    for (int i = tid; i < 2 * X; i += nt) xao[i] = g_exit_ao[i];
    for (int e = tid; e < NE; e += nt) {
        int tj, to;
        bool inner = false;
        if (e >= 4 * A) {
            tj = g_exit_ao[2 * (e - 4 * A)];
            to = g_exit_ao[2 * (e - 4 * A) + 1];
        } else {  // upstream junction of approach edge e (none for fringe edges: never a
                  // routing target -- a vehicle on its destination edge drives free)
            const int b = e >> 2, db = e & 3, r = b / C, c = b % C;
            tj = db == DIR_N ? (r > 0 ? b - C : -1) : db == DIR_S ? (r < R - 1 ? b + C : -1)
               : db == DIR_E ? (c < C - 1 ? b + 1 : -1) : (c > 0 ? b - 1 : -1);
            inner = tj >= 0;
            if (tj < 0) tj = 0;
            to = opp(db);
        }
        dinfo[e] = tj * 4 + to;
        elen[e] = inner ? len_inner : len_outer;
    }
    return Topo{R, C, A, jrc, dinfo, xid, xao, elen};
}

__device__ __forceinline__ float lane_length(const Topo &T, int e) { return T.elen[e]; }

// Out-direction at junction a for a vehicle heading h toward destination edge
// dst: move toward the junction the destination edge leaves from, keeping
// straight when that reduces the distance, vertical before horizontal, a
// U-turn only when it is the only reducing move; at that junction take the
// destination's direction.
__device__ __forceinline__ int route_out(const Topo &T, int a, int h, int dst) {
    const int tt = T.dinfo[dst], tj = tt >> 2, to = tt & 3;
    if (a == tj) return to;
    const int r = T.row(a), c = T.col(a), rt = T.row(tj), ct = T.col(tj);
    int dv = rt < r ? DIR_N : (rt > r ? DIR_S : -1);
    int dh = ct > c ? DIR_E : (ct < c ? DIR_W : -1);
    if (h == dv || h == dh) return h;
    if (dv >= 0 && dv != opp(h)) return dv;
    if (dh >= 0 && dh != opp(h)) return dh;
    return dv >= 0 ? dv : dh;
}

// Route words (the per-vehicle u16 carried in the lane rings, dmdqn_sim.vdst):
//   < 0x8000  the destination edge; the vehicle is routed on the fly (route_out)
//   >= 0x8000 an explicit route (a loaded SUMO scenario, grid_3x3_p06.rou.xml):
//             c = w & 0x7fff holds the out-directions still to take, 2 bits per
//             junction from the lowest, above a sentinel 1 -- c == 1 means the
//             vehicle is on the last edge of its route.
constexpr int kRouted = 0x8000;

__device__ __forceinline__ bool on_final_edge(int w, int e) {
    return w < kRouted ? w == e : (w & 0x7fff) == 1;
}

__device__ __forceinline__ int out_dir(const Topo &T, int a, int h, int w) {
    return w < kRouted ? route_out(T, a, h, w) : (w & 3);
}

// The route word once the vehicle has crossed the junction at the end of its edge.
__device__ __forceinline__ int route_advance(int w) {
    return w < kRouted ? w : (kRouted | ((w & 0x7fff) >> 2));
}

__device__ __forceinline__ int next_edge(const Topo &T, int a, int o) {
    int nb = T.nbr(a, o);
    return nb >= 0 ? nb * 4 + opp(o) : 4 * T.A + T.exit_id[a * 4 + o];
}

// Lane index for movement m on incoming edge e: right -> 0, left/U -> 2,
// straight -> the emptier of lanes 0/1 (ties -> 1).
__device__ __forceinline__ int lane_for_move(int m, int e, const int32_t *cnt) {
    if (m == MV_R) return 0;
    if (m != MV_S) return 2;
    return cnt[e * 3 + 1] <= cnt[e * 3 + 0] ? 1 : 0;
}

// Lane a vehicle takes when entering edge e2 from lane index kf; w2 is its
// route word on e2 (route_advance of the word it has now).
__device__ __forceinline__ int lane_for(const Topo &T, int e2, int kf, int w2,
                                        const int32_t *cnt) {
    if (e2 >= 4 * T.A || on_final_edge(w2, e2)) return kf;  // connections keep the lane index
    int h2 = opp(e2 & 3);
    int o2 = out_dir(T, e2 >> 2, h2, w2);
    return lane_for_move(movement(h2, o2), e2, cnt);
}

// Upstream junction `as` and out-direction `o` of the movements that feed edge
// e2; false for fringe-in edges (nothing upstream).
__device__ __forceinline__ bool feed_src(const Topo &T, int e2, int &as, int &o) {
    if (e2 < 4 * T.A) {
        as = T.nbr(e2 >> 2, e2 & 3);
        o = opp(e2 & 3);
        return as >= 0;
    }
    const int x = e2 - 4 * T.A;
    as = T.exit_ao[2 * x];
    o = T.exit_ao[2 * x + 1];
    return true;
}

// The i-th of the 5 lanes that feed edge e2 (approach order n,s,e,w, lane
// order within an approach): the straight approach d = opp(o) contributes
// lanes 0 and 1, right turns lane 0, left / U-turns lane 2.  A function of a
// compile-time i (callers unroll), so no per-thread array is indexed.
__device__ __forceinline__ int feeder(int as, int o, int i) {
    int pos = 0, out = 0;
#pragma unroll
    for (int d = 0; d < 4; d++) {
        const int m = movement(opp(d), o), base = (as * 4 + d) * 3;
        if (m == MV_S) {
            if (pos == i) out = base;
            if (pos + 1 == i) out = base + 1;
            pos += 2;
        } else {
            if (pos == i) out = base + (m == MV_R ? 0 : 2);
            pos += 1;
        }
    }
    return out;
}

// IDM (Treiber): a [1 - (v/v0)^4 - (s*/s)^2], s* = s0 + max(0, vT + v dv/(2 sqrt(ab))).
// Fixed evaluation order (mirrored by oracle/oracle_sim.c).
// dmdqn_idm plus the f32 reciprocals of its two constant divisors, computed
// once per launch (oracle_sim.c does the same divisions: bit-identical).
struct IdmK : dmdqn_idm {
    float inv_vmax, inv_two_sqrt_ab;
    __device__ explicit IdmK(const dmdqn_idm &p)
        : dmdqn_idm(p), inv_vmax(1.0f / p.vmax), inv_two_sqrt_ab(1.0f / p.two_sqrt_ab) {}
};

// sstar / s rounded as IEEE f32 division: the compiler's expansion of `/`
// (v_rcp_f32 refined by Newton-Raphson, then two residual corrections of the
// quotient) without its v_div_scale / v_div_fmas scaling and v_div_fixup
// special-case steps, which are the identity for the operands the IDM passes
// -- finite and normal, the numerator in [min_gap, ~10^3], the denominator
// clamped to >= 0.01 and below ~10^4: the same roundings in the same order,
// so the same quotient bits, in 8 instructions instead of 12 (pass C's
// per-vehicle chain; test_gpu_sim.py holds it to the oracle's `/`).
__device__ __forceinline__ float idm_div(float a, float b) {
    float y = __builtin_amdgcn_rcpf(b);
    const float e = __builtin_fmaf(-b, y, 1.0f);
    y = __builtin_fmaf(e, y, y);
    float q = a * y;
    const float r = __builtin_fmaf(-b, q, a);
    q = __builtin_fmaf(r, y, q);
    const float r2 = __builtin_fmaf(-b, q, a);
    return __builtin_fmaf(r2, y, q);
}

__device__ __forceinline__ float idm_free(float v, const IdmK &P) {
    float r = v * P.inv_vmax;
    float r2 = r * r;
    float r4 = r2 * r2;
    return P.accel * (1.0f - r4);
}

__device__ __forceinline__ float idm_acc(float v, float s, float dv, const IdmK &P) {
    float r = v * P.inv_vmax;
    float r2 = r * r;
    float r4 = r2 * r2;
    float ss = v * P.tau + (v * dv) * P.inv_two_sqrt_ab;
    ss = __builtin_fmaxf(ss, 0.0f);  // (clamps: see clamp_speed)
    float sstar = P.min_gap + ss;
    s = __builtin_fmaxf(s, 0.01f);
    float q = idm_div(sstar, s);
    float t1 = 1.0f - r4;
    return P.accel * (t1 - q * q);
}

// idm_acc, or idm_free when nofront, from one evaluation: free road is the
// same expression without the interaction term, accel * ((1 - r^4) - 0) ==
// accel * (1 - r^4) exactly; red is idm_acc(v, s, v) = dv of v - 0.
__device__ __forceinline__ float idm_sel(float v, float s, float dv, bool nofront,
                                         const IdmK &P) {
    float r = v * P.inv_vmax;
    float r2 = r * r;
    float r4 = r2 * r2;
    float ss = v * P.tau + (v * dv) * P.inv_two_sqrt_ab;
    ss = __builtin_fmaxf(ss, 0.0f);
    float sstar = P.min_gap + ss;
    s = __builtin_fmaxf(s, 0.01f);
    float q = idm_div(sstar, s);
    float t1 = 1.0f - r4;
    return P.accel * (t1 - (nofront ? 0.0f : q * q));
}

// v < 0 -> 0, v > vmax -> vmax, else v (oracle_sim.c's compares) as one
// v_med3_f32; the IDM clamps above as v_max_f32.  The same bits for every
// value these see: no NaN, and never -0.0 (speeds, gaps and the IDM terms are
// sums of a +0 / positive speed term and products that round to +0 at worst,
// x - x is +0 in round-to-nearest), where max / med3 could pick the other
// zero.  Each select was a compare plus a cndmask in pass C's per-vehicle
// chain, the longest lane's walk that bounds the pass.
__device__ __forceinline__ float clamp_speed(float v, const IdmK &P) {
    return __builtin_amdgcn_fmed3f(v, 0.0f, P.vmax);
}

}  // namespace dmdqn
