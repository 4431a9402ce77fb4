// sim.hip -- vectorised grid microsimulation replacing SUMO/TraCI (one block per env).
//
// What it replaces (src/scripts/train.py:225-236 and the TraCI reads of
// src/experimental/order_lanes.py:449-482):
//   traci.trafficlight.setPhase(j, ACTION_MAP[a])   -> phase = 3a, timer restart
//   traci.simulationStep() x K                       -> K one-second substeps
//   traci.lane.getLastStepHaltingNumber(lane)        -> halt[a][12] (v < 0.1 m/s)
//   getPhase / getNextSwitch / getPhaseDuration      -> phase, tspent
//   getMinExpectedNumber() == 0 or t >= MAX_SIM_TIME -> done
// The car-following model is IDM over per-lane vehicle rings (a NEW simulator,
// not SUMO's Krauss: parity is against the C restatement in oracle/oracle_sim.c,
// bit-exact, which needs -ffp-contract=off and the fixed operation order below).
//
// One substep (time t -> t+1), each pass data-parallel over lanes, passes
// separated by block barriers:
//   TL    phase advance when t - start >= duration (12-phase program of
//         grid_3x3.net.xml:893-906, actuation ignored)
//   A     front vehicle of each lane: route, target lane, IDM vs the target
//         lane's last vehicle (green) or the stop line (red/yellow); request
//   B     each target lane grants at most one request (feeder priority rotates
//         with t) if it has room
//   C     every lane advances its vehicles front-to-back (IDM, no overlap);
//         granted fronts leave, arrivals are removed
//   D     target lanes append the vehicle they granted (its route word
//         advanced past the junction: sim.hpp route words)
//   E     origin queues insert one departed vehicle per edge if there is room
#include <stdlib.h>
#include <string.h>
#include <type_traits>

#include "common.hpp"
#include "observe.hpp"
#include "sim.hpp"

namespace dmdqn {

__device__ __forceinline__ int last_slot(int head, int cnt, int cap) {
    int s = head + cnt - 1;
    return s >= cap ? s - cap : s;
}

// Positions of each lane held in the LDS image (kImg view); positions past it
// stay in the HBM arrays.  4x4 at 12: a 38 KB image, four env blocks per CU.
#ifndef DMDQN_LDS_POS
#define DMDQN_LDS_POS 12
#endif
constexpr int kLdsPos = DMDQN_LDS_POS;
constexpr int kOvPre = 8;  // HBM positions pass C loads ahead

// DT: element type of the destination rings -- int32 in HBM (dmdqn_sim.dst),
// u16 in the LDS image (edge ids < 440: grids up to 10 x 10).
//
// HBM view: per-lane rings [cap] addressed from head (a pop advances head).
// LDS image (kImg): a lane's first C1 (= min(cap, kLdsPos)) positions are a
// ring of C1 LDS slots from head[l] -- an interleaved (x, v) pair and a u16
// route word per slot; positions >= C1 (long queues only) sit compacted in the
// HBM arrays at their lane position.  A pop advances the LDS head and moves the
// first HBM vehicle into the freed slot (the HBM tail shifts down one).  Each
// lane's last vehicle is kept in lastx / lastv, and pdst holds the route word
// of a front that left during this substep (pass D reads it).
template <typename DT>
struct EnvViewT {
    static constexpr bool kImg = std::is_same<DT, uint16_t>::value;
    const dmdqn_sim &S;
    int e, A, X, NL, cap, C1;
    float *x, *v;
    float2 *xv;
    float *lastx, *lastv;
    DT *dst;
    int32_t *gdst;
    uint16_t *pdst;
    int32_t *head, *cnt, *req, *gfrom;
    float *fx, *fv;
    int32_t *phase, *ts, *qptr, *stats, *last_det;
    const int32_t *q_off;
    const uint16_t *q_ids, *vdst, *q_dst;

    __device__ EnvViewT(const dmdqn_sim &s, int env) : S(s), e(env) {
        A = s.R * s.C;
        X = 2 * s.R + 2 * s.C;
        NL = 3 * (4 * A + X);
        cap = s.cap_lane;
        C1 = cap < kLdsPos ? cap : kLdsPos;
        size_t ls = (size_t)env * NL;
        x = s.x + ls * cap;
        v = s.v + ls * cap;
        gdst = s.dst + ls * cap;
        xv = nullptr;
        lastx = lastv = nullptr;
        pdst = nullptr;
        if constexpr (std::is_same<DT, int32_t>::value) dst = gdst;
        else dst = nullptr;  // the LDS image: set up by k_sim_step
        head = s.head + ls;
        cnt = s.cnt + ls;
        req = s.req + ls;
        gfrom = s.gfrom + ls;
        fx = s.fx + ls;
        fv = s.fv + ls;
        phase = s.tl_phase + (size_t)env * A;
        ts = s.tl_ts + (size_t)env * A;
        qptr = s.qptr + (size_t)env * 4 * A;
        q_off = s.q_off + (size_t)env * (4 * A + 1);
        q_ids = s.q_ids + (size_t)env * s.nveh;
        vdst = s.vdst + (size_t)env * s.nveh;
        q_dst = s.q_dst + (size_t)env * s.nveh;
        stats = s.stats + (size_t)env * 4;
        last_det = s.last_det + (size_t)env * 12 * A;
    }
    // HBM rings: slot i of the lane block
    __device__ __forceinline__ float2 ld(size_t i) const { return make_float2(x[i], v[i]); }
    __device__ __forceinline__ void st(size_t i, float2 a) const { x[i] = a.x; v[i] = a.y; }
    // LDS image: position i of lane l (i < C1: LDS ring slot, else HBM)
    __device__ __forceinline__ int lslot(int l, int i) const {
        const int s = head[l] + i;
        return l * C1 + (s >= C1 ? s - C1 : s);
    }
    __device__ __forceinline__ float2 getp(int l, int i) const {
        if (i < C1) return xv[lslot(l, i)];
        const size_t k = (size_t)l * cap + i;
        return make_float2(x[k], v[k]);
    }
    __device__ __forceinline__ void putp(int l, int i, float2 a) const {
        if (i < C1) {
            xv[lslot(l, i)] = a;
        } else {
            const size_t k = (size_t)l * cap + i;
            x[k] = a.x;
            v[k] = a.y;
        }
    }
    __device__ __forceinline__ int dstp(int l, int i) const {
        return i < C1 ? (int)dst[lslot(l, i)] : gdst[(size_t)l * cap + i];
    }
    __device__ __forceinline__ void set_dstp(int l, int i, int d) const {
        if (i < C1) dst[lslot(l, i)] = (DT)d;
        else gdst[(size_t)l * cap + i] = d;
    }
    // the last vehicle of lane l holding nc > 0 vehicles
    __device__ __forceinline__ float2 last(int l, int nc) const {
        if constexpr (kImg) return make_float2(lastx[l], lastv[l]);
        else return ld((size_t)l * cap + last_slot(head[l], nc, cap));
    }
    __device__ __forceinline__ void set_last(int l, float2 a) const {
        if constexpr (kImg) { lastx[l] = a.x; lastv[l] = a.y; }
    }
};
using EnvView = EnvViewT<int32_t>;

// ---------------------------------------------------------------- substep
// Next vehicle of an origin queue: queue position p -> (id, destination).
struct QNext {
    int id, dst;
};
constexpr int QSLOTS = 2;  // queues per thread: 4A <= 2 * blockDim (grids up to 128 junctions)

template <typename View>
__device__ __forceinline__ QNext next_vehicle(const View &V, int p) {
    return QNext{(int)V.q_ids[p], (int)V.q_dst[p]};
}

#ifndef SIM_LANE_STRIDE_NT
#define SIM_LANE_STRIDE_NT 1  // 0: the lane arrays NL apart, as before round 4 (A/B)
#endif
#ifdef DMDQN_SIM_PROFILE  // diagnostic build: per-pass ticks of thread 0 -> halt[env][0][0..7]
#define SIM_PROF(i)                                                          \
    do {                                                                     \
        if (threadIdx.x == 0) {                                              \
            const uint64_t _n = __builtin_amdgcn_s_memrealtime();           \
            prof[i] += _n - prof_t;                                          \
            prof_t = _n;                                                     \
        }                                                                    \
    } while (0)
#else
#define SIM_PROF(i) do { } while (0)
#endif

// The routing decision of a lane's front is a function of the lane and the
// front's route word only (static topology): the movement m at the junction
// ahead, the next edge e2 and the movement there (mv2 < 0: keep the lane
// index).  Each thread keeps it for its first lane (l = tid) across substeps
// and recomputes it only when the front's route word changes -- a front
// waits at the stop line for many substeps.
struct RouteCache {
    int d0, m, e2, mv2;
};

template <bool kAct, typename View>
__device__ __forceinline__ void substep(View &V, const Topo &T, const IdmK &P, int t,
                                        QNext qn[QSLOTS], RouteCache &rc, uint64_t *prof,
                                        uint64_t &prof_t) {
    const dmdqn_sim &S = V.S;
    const int A = V.A, NL = V.NL, cap = V.cap;
    const int tid = threadIdx.x, nt = blockDim.x;

    // ---- TL: natural phase advance (fixed durations; actuated gap-out of
    // phase 0 in actuated mode: after minDur, once no vehicle has been over a
    // detector of the phase's green lanes for more than max_gap, or at maxDur)
    for (int a = tid; a < A; a += nt) {
        const int p = V.phase[a], el = t - V.ts[a];
        bool sw;
        if (S.actuated && p == 0) {
            constexpr uint32_t gl = green_lanes(0x11BB);  // green_mask(0)
            int last = kNoDetection;
#pragma unroll
            for (int k = 0; k < 12; k++)
                if ((gl >> k) & 1u) last = max(last, V.last_det[a * 12 + k]);
            sw = el >= kActMax || (el >= kActMin && (float)(t - last) > P.max_gap);
        } else {
            sw = el >= phase_dur(p);
        }
        if (sw) {
            V.phase[a] = (p + 1) % 12;
            V.ts[a] = t;
        }
    }
    __syncthreads();
    SIM_PROF(0);

    // ---- A: front vehicles decide.  One IDM evaluation per front (free
    // road: no interaction term; green with a vehicle on the target lane: that
    // vehicle; red/yellow: the stop line), its inputs chosen by selects.
    for (int l = tid; l < NL; l += nt) {
        V.gfrom[l] = -1;
        int n = V.cnt[l];
        if (n == 0) {
            V.req[l] = -1;
            continue;
        }
        const int e = l / 3, kf = l - 3 * e;
        float2 f0;
        int d0;
        if constexpr (View::kImg) {
            const int k0 = l * V.C1 + V.head[l];
            f0 = V.xv[k0];
            d0 = V.dst[k0];
        } else {
            const int h0 = V.head[l];
            const size_t base = (size_t)l * cap;
            f0 = V.ld(base + h0);
            d0 = V.dst[base + h0];
        }
        const float x0 = f0.x, v0 = f0.y;
        const float len = lane_length(T, e);
        // exit edge or last edge: free road
        const bool free_road = e >= 4 * A || on_final_edge(d0, e);
        bool green = false, lead = false;
        int tl = -1;
        float xl = 0.0f, vl = 0.0f;
        if (!free_road) {
            const int aj = e >> 2, d = e & 3, h = opp(d);
            int m, e2, mv2;
            if (l == tid && rc.d0 == d0) {
                m = rc.m;
                e2 = rc.e2;
                mv2 = rc.mv2;
            } else {
                const int o = out_dir(T, aj, h, d0);
                m = movement(h, o);
                DMDQN_DBG(T.nbr(aj, o) >= 0 || T.exit_id[aj * 4 + o] >= 0, DBG_SIM_EDGE);
                e2 = next_edge(T, aj, o);
                // lane_for: connections keep the lane index onto exit / final edges
                const int w2 = route_advance(d0);
                mv2 = -1;
                if (!(e2 >= 4 * A || on_final_edge(w2, e2))) {
                    const int h2 = opp(e2 & 3);
                    mv2 = movement(h2, out_dir(T, e2 >> 2, h2, w2));
                }
                if (l == tid) rc = RouteCache{d0, m, e2, mv2};
            }
            const int k2 = mv2 < 0 ? kf : lane_for_move(mv2, e2, V.cnt);
            tl = e2 * 3 + k2;
            green = (green_mask(V.phase[aj]) >> (d * 4 + m)) & 1;
            const int nc = V.cnt[tl];
            lead = green && nc > 0;
            if constexpr (View::kImg) {  // per-lane last-vehicle arrays: always readable
                xl = V.lastx[tl];
                vl = V.lastv[tl];
            } else if (lead) {
                const float2 lt = V.last(tl, nc);
                xl = lt.x;
                vl = lt.y;
            }
        }
        const bool nofront = free_road || (green && !lead);
        const float gap = (len - x0) + (green ? (xl - P.length) : P.min_gap);
        const float acc = idm_sel(v0, gap, v0 - (lead ? vl : 0.0f), nofront, P);
        float vn = clamp_speed(v0 + acc, P);
        float xn = x0 + vn;
        const bool over = xn > len;
        V.req[l] = free_road ? kArrive : (over && green ? tl : -1);
        const bool stop = !free_road && over && !green;
        V.fx[l] = stop ? len : xn;
        V.fv[l] = stop ? 0.0f : vn;
    }
    __syncthreads();
    SIM_PROF(1);

    // ---- B: target lanes grant one request
    // All 5 request slots are read at once; the first requester in the order
    // rotated by t % 5 is the only one considered (granted if there is room).
    for (int tl = tid; tl < NL; tl += nt) {
        int as, o;
        if (!feed_src(T, tl / 3, as, o)) continue;
        int f[5];
        uint32_t mask = 0;
#pragma unroll
        for (int i = 0; i < 5; i++) {
            f[i] = feeder(as, o, i);
            mask |= (V.req[f[i]] == tl ? 1u : 0u) << i;
        }
        if (!mask) continue;
        const int start = t % 5;
        const uint32_t rot = ((mask >> start) | (mask << (5 - start))) & 31u;
        int k = start + __ffs(rot) - 1;
        if (k >= 5) k -= 5;
        int fsel = f[0];
#pragma unroll
        for (int i = 1; i < 5; i++) fsel = k == i ? f[i] : fsel;
        int nc = V.cnt[tl];
        bool room = nc < cap;
        if (room && nc > 0) room = (V.last(tl, nc).x - P.length) >= P.min_gap;
        if (room) V.gfrom[tl] = fsel;
    }
    __syncthreads();
    SIM_PROF(2);

    // ---- C: advance every lane; fronts leave (granted) or arrive
    for (int l = tid; l < NL; l += nt) {
        int n = V.cnt[l];
        if (n == 0) continue;
        const int e = l / 3;
        const float len = lane_length(T, e);
        const size_t base = (size_t)l * cap;
        const int hd = V.head[l];  // HBM ring head, or the LDS ring head (image)
        // LDS image, long queue: the HBM positions' (x, v) are loaded together
        // here, so their latency overlaps the front and the LDS walk instead of
        // one L2 round trip per vehicle
        float2 ov[kOvPre];
        const int no = View::kImg ? n - V.C1 : 0;
        if (View::kImg && no > 0) {
#pragma unroll
            for (int j = 0; j < kOvPre; j++)
                if (j < no) ov[j] = make_float2(V.x[base + V.C1 + j], V.v[base + V.C1 + j]);
        }
        // front
        const float2 f0 = View::kImg ? V.xv[l * V.C1 + hd] : V.ld(base + hd);
        float lead_x_old = f0.x, lead_v_old = f0.y;
        float lead_x_new = V.fx[l];
        float fvn = V.fv[l];
        const int rq = V.req[l];
        bool pop = false;
        if (rq == kArrive) {
            pop = lead_x_new >= len;
            if (pop) atomicAdd(&V.stats[1], 1);
        } else if (rq >= 0) {
            // granted? the target lane recorded the source lane in gfrom
            pop = V.gfrom[rq] == l;
            if (!pop) {
                lead_x_new = len;
                fvn = 0.0f;
            }
        }
        if constexpr (View::kImg) {
            if (!pop) V.xv[l * V.C1 + hd] = make_float2(lead_x_new, fvn);
            else V.pdst[l] = V.dst[l * V.C1 + hd];  // the leaving front's route word, for pass D
        } else {
            if (!pop) V.st(base + hd, make_float2(lead_x_new, fvn));
        }
        // actuated mode: a vehicle's body over the detector point dp during
        // the substep (old front < dp + length, new front >= dp)
        const float dp = len - P.det_dist, dpl = dp + P.length;
        bool det = lead_x_new >= dp && lead_x_old < dpl;
        float2 lastv2 = make_float2(lead_x_new, fvn);
        // one follower: IDM against the old leader state, no overlap with the
        // leader's new position
        // (selects, no branches: the LDS walk below runs it for every lane of
        // the wave up to the wave's longest lane, `act` false past a lane's end)
        auto follow = [&](float xi, float vi, bool act = true) -> float2 {
            const float gap = (lead_x_old - P.length) - xi;
            const float acc = idm_acc(vi, gap, vi - lead_v_old, P);
            const float vc = clamp_speed(vi + acc, P);
            const float xc = xi + vc;
            const float lim = lead_x_new - P.length, dl = lim - xi;
            const bool over = xc > lim, back = lim < xi;
            const float xn = over ? (back ? xi : lim) : xc;
            const float vn = over ? (back ? 0.0f : dl) : vc;
            if (kAct) det = det || (act && xn >= dp && xi < dpl);
            const float2 r = make_float2(xn, vn);
            lastv2 = act ? r : lastv2;
            lead_x_old = act ? xi : lead_x_old;
            lead_v_old = act ? vi : lead_v_old;
            lead_x_new = act ? xn : lead_x_new;
            return r;
        };
        if constexpr (View::kImg) {
            // positions 1 .. m-1: the LDS ring, updated in place; then the HBM
            // positions of a long queue (after a pop the first of them moves
            // into the slot the front left, the rest shift down one)
            const int C1 = V.C1, m = n < C1 ? n : C1, sh = pop ? 1 : 0;
            float2 *xl = V.xv + l * C1;
            uint16_t *dl = V.dst + l * C1;
            // wave-uniform trip count (ballot): a lane past its end keeps its
            // state and writes into its own unoccupied ring slots (i < C1)
            int sl = hd + 1 == C1 ? 0 : hd + 1;
            float2 nxt = xl[sl];
            for (int i = 1; __ballot(i < m); i++) {
                const float2 cur = nxt;
                const int sc = sl;
                sl = sl + 1 == C1 ? 0 : sl + 1;
                if (i + 1 < C1) nxt = xl[sl];
                xl[sc] = follow(cur.x, cur.y, i < m);
            }
            if (no > 0) {
                int od[kOvPre];
                if (sh) {
#pragma unroll
                    for (int j = 0; j < kOvPre; j++)
                        if (j < no) od[j] = V.gdst[base + C1 + j];
                }
#pragma unroll
                for (int j = 0; j < kOvPre; j++) {
                    if (j < no) {
                        const float2 r = follow(ov[j].x, ov[j].y);
                        const size_t k = base + C1 + j - sh;
                        if (sh && j == 0) {
                            xl[hd] = r;
                            dl[hd] = (uint16_t)od[0];
                        } else {
                            V.x[k] = r.x;
                            V.v[k] = r.y;
                            if (sh) V.gdst[k] = od[j];
                        }
                    }
                }
                for (int i = C1 + kOvPre; i < n; i++) {  // cap > C1 + kOvPre only
                    const size_t k = base + i;
                    const float2 r = follow(V.x[k], V.v[k]);
                    V.x[k - sh] = r.x;
                    V.v[k - sh] = r.y;
                    if (sh) V.gdst[k - 1] = V.gdst[k];
                }
            }
        } else {
            // the next follower's (x, v) is loaded before this one is computed
            // and stored.  (Computing a chunk of 4 followers' IDMs together --
            // they depend only on old values -- measured 9 % slower.)
            int s = hd;
            int sn = (s + 1 == cap) ? 0 : s + 1;
            float2 nxt = n > 1 ? V.ld(base + sn) : make_float2(0.0f, 0.0f);
            for (int i = 1; i < n; i++) {
                s = sn;
                const float2 cur = nxt;
                sn = (s + 1 == cap) ? 0 : s + 1;
                if (i + 1 < n) nxt = V.ld(base + sn);
                V.st(base + s, follow(cur.x, cur.y));
            }
        }
        if (pop) {
            const int ring = View::kImg ? V.C1 : cap;
            V.head[l] = (hd + 1 == ring) ? 0 : hd + 1;
            V.cnt[l] = n - 1;
        }
        if (n - (pop ? 1 : 0) > 0) V.set_last(l, lastv2);
        if (kAct && det && l < 12 * A) V.last_det[l] = t + 1;
    }
    __syncthreads();
    SIM_PROF(3);

    // ---- D: append granted vehicles
    for (int tl = tid; tl < NL; tl += nt) {
        const int f = V.gfrom[tl];
        if (f < 0) continue;
        const int e2 = tl / 3;
        (void)e2;
        const float over = V.fx[f] - lane_length(T, f / 3);
        const float vin = V.fv[f];
        // the source lane already popped its front; read its (old) destination
        // from the slot it vacated (LDS image: from pdst)
        int dv;
        if constexpr (View::kImg) {
            dv = route_advance(V.pdst[f]);
        } else {
            const int fh = V.head[f] == 0 ? cap - 1 : V.head[f] - 1;
            dv = route_advance(V.dst[(size_t)f * cap + fh]);
        }
        int nc = V.cnt[tl];
        float xe = over;
        if (nc > 0) {
            float lim = V.last(tl, nc).x - P.length - P.min_gap;
            if (lim < xe) xe = lim;
        }
        if (xe < 0.0f) xe = 0.0f;
        DMDQN_DBG(nc < cap, DBG_SIM_RING);  // pass B granted only with room
        if constexpr (View::kImg) {
            V.putp(tl, nc, make_float2(xe, vin));
            V.set_dstp(tl, nc, dv);
        } else {
            int slot = V.head[tl] + nc;
            if (slot >= cap) slot -= cap;
            V.st((size_t)tl * cap + slot, make_float2(xe, vin));
            V.dst[(size_t)tl * cap + slot] = dv;
        }
        V.set_last(tl, make_float2(xe, vin));
        V.cnt[tl] = nc + 1;
    }
    __syncthreads();
    SIM_PROF(4);

    // ---- E: insertion from the origin queues (vehicles with depart <= t).
    // Queue e is always handled by thread e % nt (slot q = e / nt), which keeps
    // the queue's next vehicle (id, destination) in registers: after an
    // insertion it issues the loads of the following one, consumed a substep
    // later, so the HBM/L2 latency of the departure table is off the chain.
#pragma unroll
    for (int q = 0; q < QSLOTS; q++) {
        const int e = tid + q * nt;
        if (e >= 4 * A) continue;
        int p = V.qptr[e];
        if (p >= V.q_off[e + 1]) continue;
        const int id = qn[q].id;
        if ((long long)id * S.period_ms > (long long)t * 1000) continue;
        const int d0 = qn[q].dst;
        const int aj = e >> 2, d = e & 3, h = opp(d);
        // a one-edge route departs on the straight lanes (its origin is its end)
        const int m = on_final_edge(d0, e) ? (int)MV_S : movement(h, out_dir(T, aj, h, d0));
        const int k = lane_for_move(m, e, V.cnt);
        const int l = e * 3 + k;
        const int nc = V.cnt[l];
        if (nc >= cap) continue;
        if (nc > 0 && V.last(l, nc).x < 2.0f * P.length + P.min_gap) continue;
        if constexpr (View::kImg) {
            V.putp(l, nc, make_float2(P.length, 0.0f));
            V.set_dstp(l, nc, d0);
        } else {
            int slot = V.head[l] + nc;
            if (slot >= cap) slot -= cap;
            V.st((size_t)l * cap + slot, make_float2(P.length, 0.0f));
            V.dst[(size_t)l * cap + slot] = d0;
        }
        V.set_last(l, make_float2(P.length, 0.0f));
        V.cnt[l] = nc + 1;
        V.qptr[e] = p + 1;
        atomicAdd(&V.stats[0], 1);
        if (p + 1 < V.q_off[e + 1]) qn[q] = next_vehicle(V, p + 1);
    }
    __syncthreads();
    SIM_PROF(5);
}

// ================================================================ fused env step
// dmdqn_env_step: the act draws before the substeps (prologue) and the
// observation, reward and replay store after them (epilogue) run inside the
// sim block, with the same arithmetic as k_act (rng.hip), k_observe
// (observe.hip) and k_replay_store (replay.hip): bit-identical results, three
// fewer launches per step, and the halting counts / signals / observation
// read from LDS instead of passed between kernels through HBM.
constexpr size_t kMtBytes = 2 * MT_N * sizeof(uint32_t);

// fused_tail's scratch: loc f32 [A][17], act i32 [A], nbr i32 [A][4], then
// (16-byte aligned) the observation rows f32 [A][92] and sums f64 [A + 1]
__host__ __device__ inline size_t tail_bytes(int A) {
    return (((size_t)A * 22 * 4 + 15) & ~(size_t)15) + (size_t)A * 92 * 4 + (size_t)(A + 1) * 8;
}

// Where the prologue's MT stream and the epilogue's scratch go in the dynamic
// LDS of a block whose own layout takes `base` bytes: at offset 0 when the
// block's first bytes are dead there (free_start: before staging, free_end:
// after the write-back), else past `base`.
struct FuseLayout {
    size_t mt_off, tail_off, bytes;
};
__host__ __device__ inline FuseLayout fuse_layout(size_t base, size_t free_start, size_t free_end,
                                                  int A) {
    FuseLayout f;
    const size_t extra = (base + 15) & ~(size_t)15;
    f.bytes = base;
    f.mt_off = free_start >= kMtBytes ? 0 : extra;
    if (f.mt_off && extra + kMtBytes > f.bytes) f.bytes = extra + kMtBytes;
    f.tail_off = free_end >= tail_bytes(A) ? 0 : extra;
    if (f.tail_off && extra + tail_bytes(A) > f.bytes) f.bytes = extra + tail_bytes(A);
    return f;
}

// select_action for the env's A agents (k_act with draw_rand): every thread of
// the block consumes the stream in lockstep (the draws are wave-uniform; the
// MTWave loops and barriers are correct for a block of several waves, whose
// extra lanes write identical values); thread j returns agent j's action.
// The fixed-count case (act_fast: the training path) reads each agent's word
// straight from the raw state -- no LDS, no barrier -- and leaves the stream
// position to fused_act_done; the general case stages the stream in mtbuf.
__device__ int fused_act(const dmdqn_env_fuse &F, int A, uint32_t *mtbuf, bool &fast) {
    const int e = blockIdx.x;
    const uint32_t rng = (uint32_t)(F.n_actions - 1);
    uint32_t mask = rng;
    mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4; mask |= mask >> 8; mask |= mask >> 16;
    uint32_t *g = F.np_state + (size_t)e * DMDQN_MT_WORDS;
    const int mti0 = (int)g[MT_N];
    fast = act_fast_ok(mti0, A, 3, F.eps, rng, mask, 1);
    if (fast)  // stored by fused_act_done: the load's latency hides behind the staging
        return (int)threadIdx.x < A ? act_fast(g, mti0, threadIdx.x, 3, mask) : 0;
    MTWave w{mtbuf, mtbuf + MT_N, 0};
    w.load(g);
    int mine = 0;
    for (int j = 0; j < A; j++) {
        const double r = np_double(w);
        int a;
        if (r < F.eps) {  // dqn_agent.py:263-265
            uint32_t v;
            do { v = w.next() & mask; } while (v > rng);
            a = (int)v;
        } else {
            a = F.greedy[(size_t)e * A + j];
        }
        if ((int)threadIdx.x == j) mine = a;
    }
    __syncthreads();
    if (threadIdx.x < 64) w.store(g);
    if ((int)threadIdx.x < A) F.actions[(size_t)e * A + threadIdx.x] = mine;
    __syncthreads();  // the stream's LDS may be reused from here on (the LDS image)
    return mine;
}

// After a barrier that follows every thread's read of the old position.
__device__ __forceinline__ void fused_act_done(const dmdqn_env_fuse &F, int A, bool fast,
                                               int my_act) {
    if (!fast) return;
    if ((int)threadIdx.x < A) F.actions[(size_t)blockIdx.x * A + threadIdx.x] = my_act;
    if (threadIdx.x == 0) {
        uint32_t *g = F.np_state + (size_t)blockIdx.x * DMDQN_MT_WORDS;
        g[MT_N] = g[MT_N] + (uint32_t)(3 * A);
    }
}

// The epilogue's inputs that do not depend on the substeps, loaded before
// them (their latency hides behind the staging): the packed int8 s-row words
// of this thread's first two (agent, 4-byte group) store slots, and the
// reward's pre-step sum of agent `tid` (train.py:159-165).
constexpr int kPreWords = 2;
#ifndef DMDQN_FUSE_PREFETCH
#define DMDQN_FUSE_PREFETCH 1
#endif
constexpr bool kFusePre = DMDQN_FUSE_PREFETCH;  // LDS path (A/B switch)
struct TailPre {
    uint32_t ws[kPreWords];
    double sum;
};
__device__ __forceinline__ uint32_t s_row_word(const dmdqn_env_fuse &F, size_t agent, int grp) {
    const float *os = F.obs_s + agent * DMDQN_OBS_DIM;
    uint32_t ws = 0;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int k = grp * 4 + q;
        if (k < DMDQN_OBS_DIM) ws |= (uint32_t)(uint8_t)to_i8(os[k], F.err) << (8 * q);
    }
    return ws;
}
__device__ TailPre fused_prefetch(const dmdqn_env_fuse &F, int A) {
    constexpr int G = DMDQN_ROW_BYTES / 4;
    const int tid = threadIdx.x, nt = blockDim.x;
    const size_t eo = (size_t)blockIdx.x * A;
    TailPre p;
#pragma unroll
    for (int it = 0; it < kPreWords; it++) {
        const int i = tid + it * nt;
        p.ws[it] = i < A * G ? s_row_word(F, eo + i / G, i % G) : 0u;
    }
    p.sum = 0.0;
    if (tid < A) {
        const float *pl = F.prev_local + (eo + tid) * 17;
        for (int k = 0; k < 12; k++) p.sum += (double)pl[k];
    }
    return p;
}

// k_observe + k_replay_store of this env from LDS: s_halt [A][12], s_phase /
// s_ts [A] (phase start times, tspent = t - ts); my_act is thread a's action.
// Every thread calls it after a barrier that completed those arrays.  The
// observation rows are built once, into LDS (stride kObsLd: 16-byte aligned
// rows) and HBM; the s'-row bytes are packed from the LDS rows.
constexpr int kObsLd = 92;
__host__ __device__ inline size_t tail_obs_off(int A) {
    return (((size_t)A * (17 + 1 + 4) * 4 + 15) & ~(size_t)15);
}
template <bool kPre = true>
__device__ void fused_tail(const dmdqn_env_fuse &F, int R, int C, int t, bool done_e, int my_act,
                           const TailPre &pre, const int32_t *s_halt, const int32_t *s_phase,
                           const int32_t *s_ts, char *scratch) {
    const int A = R * C, e = blockIdx.x, tid = threadIdx.x, nt = blockDim.x;
    float *loc = reinterpret_cast<float *>(scratch);          // [A][17]
    int32_t *act = reinterpret_cast<int32_t *>(loc + A * 17);  // [A]
    int32_t *nbr = act + A;                                   // [A][4]
    float *img = reinterpret_cast<float *>(scratch + tail_obs_off(A));  // [A][kObsLd]
    double *sums = reinterpret_cast<double *>(img + (size_t)A * kObsLd);  // [A + 1]
    const size_t eo = (size_t)e * A;
    if (tid < A) {
        act[tid] = my_act;
        if constexpr (kPre) {
            sums[tid] = pre.sum;
        } else {
            const float *pl = F.prev_local + (eo + tid) * 17;
            double sm = 0.0;
            for (int q = 0; q < 12; q++) sm += (double)pl[q];
            sums[tid] = sm;
        }
    }
    for (int i = tid; i < 4 * A; i += nt) nbr[i] = neighbor(R, C, i >> 2, i & 3);
    for (int i = tid; i < A * 17; i += nt) {  // get_own_state (order_lanes.py:430-499)
        const int a = i / 17, f = i - a * 17;
        const float v = local_feature(f, s_halt + a * 12, s_phase[a], t - s_ts[a], F.mode);
        loc[i] = v;
        F.local[eo * 17 + i] = v;
    }
    __syncthreads();
    if (tid == 0) {
        double g = 0.0;
        for (int a = 0; a < A; a++) g += sums[a];
        sums[A] = -1.0 * g;
    }
    for (int i = tid; i < A * DMDQN_OBS_DIM; i += nt) {  // build_state_vector (:502-555)
        const int a = i / DMDQN_OBS_DIM, k = i - a * DMDQN_OBS_DIM;
        float v;
        if (k < 17) {
            v = loc[a * 17 + k];
        } else if (k < 21) {
            v = nbr[a * 4 + k - 17] >= 0 ? 1.0f : 0.0f;
        } else {
            const int d = (k - 21) / 17, f = (k - 21) - d * 17, b = nbr[a * 4 + d];
            v = b >= 0 ? loc[b * 17 + f] : -1.0f;
        }
        img[a * kObsLd + k] = v;
        F.obs[eo * DMDQN_OBS_DIM + i] = v;
    }
    if (tid < A)
        for (int k = DMDQN_OBS_DIM; k < kObsLd; k++) img[tid * kObsLd + k] = 0.0f;
    __syncthreads();
    // ReplayBuffer.add: one thread per (agent, 4-byte group), as k_replay_store;
    // the reward (train.py:159-165, :254) by the threads that store it
    constexpr int G = DMDQN_ROW_BYTES / 4;
    const double gsum = sums[A];
    for (int it = 0, i = tid; i < A * G; it++, i += nt) {
        const int a = i / G, grp = i - a * G;
        const size_t row = (eo + a) * (size_t)F.cap + F.slot;
        const uint32_t ws = kPre && it < kPreWords ? pre.ws[it < kPreWords ? it : 0]
                                                   : s_row_word(F, eo + a, grp);
        uint32_t wn = 0;
        if (4 * grp < DMDQN_OBS_DIM) {  // (row floats 89..91 are zero: bytes 89..95 stay 0)
            const float4 o = *reinterpret_cast<const float4 *>(img + a * kObsLd + 4 * grp);
            wn = (uint32_t)(uint8_t)to_i8(o.x, F.err) | (uint32_t)(uint8_t)to_i8(o.y, F.err) << 8 |
                 (uint32_t)(uint8_t)to_i8(o.z, F.err) << 16 | (uint32_t)(uint8_t)to_i8(o.w, F.err) << 24;
        }
        const bool rw = grp == 0 || 4 * grp == DMDQN_ROW_R || 4 * grp == DMDQN_ROW_R + 4;
        const double r = rw ? combine_reward(-1.0 * sums[a], gsum) : 0.0;
        if (4 * grp == DMDQN_ROW_A) {
            wn = (uint32_t)(uint8_t)act[a] | (done_e ? 1u : 0u) << 8;
        } else if (4 * grp == DMDQN_ROW_R || 4 * grp == DMDQN_ROW_R + 4) {
            const unsigned long long rb = __double_as_longlong(r);
            wn = (uint32_t)(4 * grp == DMDQN_ROW_R ? rb : rb >> 32);
        }
        reinterpret_cast<uint32_t *>(F.ring_s + row * DMDQN_ROW_BYTES)[grp] = ws;
        reinterpret_cast<uint32_t *>(F.ring_n + row * DMDQN_ROW_BYTES)[grp] = wn;
        if (grp == 0) {
            F.ring_a[row] = (uint8_t)act[a];
            F.ring_r[row] = r;
            F.ring_d[row] = done_e ? 1 : 0;
            F.reward[eo + a] = r;
        }
    }
}

// LDS image of one env's mutable state (kLDS path): compacted lanes' first C1
// positions as (x, v) f32 pairs [NL][C1], their u16 route words [NL][C1] and
// pdst [NL], then head, cnt, req, gfrom, fx, fv, lastx, lastv [NL], phase, ts
// [A], qptr [4A], stats [4], q_off [4A+1], last_det [12A].  4x4 grid: 38.4 KB
// (+1.1 KB of topology) -> four env blocks per CU, all 1024 envs of C3 resident
// at once (the full-ring image was 65 KB: two per CU, two rounds).
__host__ __device__ inline size_t sim_lds_bytes(int R, int C, int cap) {
    const int A = R * C, NL = 3 * (4 * A + 2 * R + 2 * C);
    const int C1 = cap < kLdsPos ? cap : kLdsPos;
    return (size_t)NL * C1 * 8 + (size_t)NL * (C1 + 1) * 2 + (size_t)NL * 8 * 4 + (size_t)A * 8 +
           (size_t)A * 16 + 16 + (size_t)(4 * A + 1) * 4 + (size_t)A * 48;  // q_off, last_det
}

// Sum over the wave (integer: exact in any order); the block totals below take
// one LDS atomic per wave instead of one per thread at a single address, which
// the LDS serialises lane by lane (up to 1024-way in the 8x8 register path).
__device__ __forceinline__ int wave_sum(int x) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off);
    return x;
}

// One RL step per env (block).  kLDS: the env's state is staged into LDS for
// the K substeps (every pass is then an LDS-latency loop instead of an L2 one:
// pass C walks each lane's vehicles front to back); only occupied positions
// move between HBM and LDS, and the lanes are written back compacted (head 0).
// !kLDS: the same passes on global memory rings.
template <bool kLDS, bool kAct, bool kFuse>
__global__ void __launch_bounds__(256, 4) k_sim_step(dmdqn_sim S, dmdqn_idm Pa, const int32_t *actions,
                                                  int stride, int t0_arg, int K, int max_time,
                                                  int32_t *halt, int32_t *phase_out,
                                                  int32_t *tspent, uint8_t *done,
                                                  dmdqn_env_fuse F) {
    extern __shared__ __attribute__((aligned(16))) char dyn[];
    const int t0 = S.t_env ? S.t_env[blockIdx.x] : t0_arg;  // the replica's own clock
    const uint64_t prof_t0 = __builtin_amdgcn_s_memrealtime();
    const IdmK P(Pa);
    // topology tables after the state image (kLDS) or alone (global path)
    const size_t topo_off = kLDS ? sim_lds_bytes(S.R, S.C, S.cap_lane) : 0;
    const Topo T = build_topo(reinterpret_cast<int32_t *>(dyn + topo_off), S.R, S.C, S.exit_id,
                              S.exit_ao, P.len_inner, P.len_outer);  // synced below
    EnvView G(S, blockIdx.x);
    EnvViewT<typename std::conditional<kLDS, uint16_t, int32_t>::type> V(S, blockIdx.x);
    const int A = V.A, NL = V.NL, cap = V.cap;
    const int tid = threadIdx.x, nt = blockDim.x;
    // fused step: the act draws first (the MT stream lives in the image's dead
    // position slots until staging), the halting counts later in the topology
    // tables' place (dead after the substeps)
    const size_t xv_bytes = kLDS ? (size_t)NL * V.C1 * 8 : 0;
    const FuseLayout fl = fuse_layout(topo_off + topo_bytes(S.R, S.C), xv_bytes, xv_bytes, A);
    int32_t *const s_halt = reinterpret_cast<int32_t *>(dyn + topo_off);
    int my_act = 0;
    bool act_fast = false;
    TailPre pre{};
    if constexpr (kFuse) {
        my_act = fused_act(F, A, reinterpret_cast<uint32_t *>(dyn + fl.mt_off), act_fast);
        if constexpr (kFusePre) pre = fused_prefetch(F, A);
    }
    if constexpr (kLDS) {
        const int C1 = V.C1;
        const size_t NS = (size_t)NL * C1;
        V.xv = reinterpret_cast<float2 *>(dyn);
        V.dst = reinterpret_cast<uint16_t *>(V.xv + NS);
        V.pdst = V.dst + NS;
        V.head = reinterpret_cast<int32_t *>(V.pdst + NL);  // NL(C1 + 1) u16: NL = 6 * ... is even
        V.cnt = V.head + NL;
        V.req = V.cnt + NL;
        V.gfrom = V.req + NL;
        V.fx = reinterpret_cast<float *>(V.gfrom + NL);
        V.fv = V.fx + NL;
        V.lastx = V.fv + NL;
        V.lastv = V.lastx + NL;
        V.phase = reinterpret_cast<int32_t *>(V.lastv + NL);
        V.ts = V.phase + A;
        V.qptr = V.ts + A;
        V.stats = V.qptr + 4 * A;
        int32_t *qoff = V.stats + 4;
        for (int i = tid; i <= 4 * A; i += nt) qoff[i] = G.q_off[i];
        V.q_off = qoff;
        V.last_det = qoff + 4 * A + 1;
        if (S.actuated)
            for (int i = tid; i < 12 * A; i += nt) V.last_det[i] = G.last_det[i];
        // each thread stages its lanes' occupied positions < C1 (~8 % of the
        // rings).  A lane whose ring does not start at slot 0 (written by the
        // HBM path, or a checkpoint of it) is first rotated in place in HBM
        // (cycle-leader rotation by head: scalar temporaries only).
        for (int l = tid; l < NL; l += nt) {
            int h = G.head[l], n = G.cnt[l];
            DMDQN_DBG(h >= 0 && h < cap && n >= 0 && n <= cap, DBG_SIM_RING);
#ifdef DMDQN_DEBUG_BOUNDS
            if (!(h >= 0 && h < cap && n >= 0 && n <= cap)) h = n = 0;
#endif
            V.cnt[l] = n;
            V.head[l] = 0;
            const size_t base = (size_t)l * cap;
            if (h != 0 && n > 0) {
                int g = cap, b = h;  // gcd(cap, h) cycles
                while (b) { const int r = g % b; g = b; b = r; }
                for (int c = 0; c < g; c++) {
                    const float tx = G.x[base + c], tv = G.v[base + c];
                    const int td = G.dst[base + c];
                    int j = c;
                    for (;;) {
                        int k = j + h;
                        if (k >= cap) k -= cap;
                        if (k == c) break;
                        G.x[base + j] = G.x[base + k];
                        G.v[base + j] = G.v[base + k];
                        G.dst[base + j] = G.dst[base + k];
                        j = k;
                    }
                    G.x[base + j] = tx;
                    G.v[base + j] = tv;
                    G.dst[base + j] = td;
                }
            }
            float2 lt = make_float2(0.0f, 0.0f);
            for (int i = 0; i < n && i < C1; i++) {
                lt = make_float2(G.x[base + i], G.v[base + i]);
                V.xv[l * C1 + i] = lt;
                V.dst[l * C1 + i] = (uint16_t)G.dst[base + i];
            }
            if (n > C1) lt = make_float2(G.x[base + n - 1], G.v[base + n - 1]);
            V.lastx[l] = lt.x;
            V.lastv[l] = lt.y;
        }
        for (int a = tid; a < A; a += nt) {
            V.phase[a] = G.phase[a];
            V.ts[a] = G.ts[a];
        }
        for (int e = tid; e < 4 * A; e += nt) V.qptr[e] = G.qptr[e];
        if (tid < 4) V.stats[tid] = G.stats[tid];
    }
    if constexpr (kFuse) {
        if (tid < A) {  // A <= blockDim (dmdqn_env_step)
            V.phase[tid] = stride * my_act;
            V.ts[tid] = t0;
        }
    } else if (actions) {
        for (int a = tid; a < A; a += nt) {
            // a negative action: no setPhase, the junction's program runs on
            // with its timer (the reference class's skipped actions)
            const int act = actions[(size_t)blockIdx.x * A + a];
            if (act >= 0) {
                V.phase[a] = stride * act;
                V.ts[a] = t0;
            }
        }
    }
    __syncthreads();
    if constexpr (kFuse) fused_act_done(F, A, act_fast, my_act);
    QNext qn[QSLOTS];
#pragma unroll
    for (int q = 0; q < QSLOTS; q++) {
        const int e = tid + q * nt;
        qn[q] = QNext{0, 0};
        if (e < 4 * A && V.qptr[e] < V.q_off[e + 1]) qn[q] = next_vehicle(V, V.qptr[e]);
    }
    uint64_t prof[8] = {0, 0, 0, 0, 0, 0, 0, 0}, prof_t = __builtin_amdgcn_s_memrealtime();
    prof[6] = prof_t - prof_t0;  // staging
    RouteCache rc{-1, 0, 0, 0};
    for (int k = 0; k < K; k++) substep<kAct>(V, T, P, t0 + k, qn, rc, prof, prof_t);
    const int t = t0 + K;
    // halting counts on the observed (incoming) lanes + bookkeeping
    __shared__ int s_running, s_pending;
    if (tid == 0) { s_running = 0; s_pending = 0; }
    __syncthreads();
    int run = 0, pend = 0;
    for (int l = tid; l < NL; l += nt) {
        const int n = V.cnt[l];
        run += n;
        if (l < 12 * A) {
            int h = 0;
            if constexpr (kLDS) {
                for (int i = 0; i < n; i++) h += V.getp(l, i).y < P.halt_speed ? 1 : 0;
            } else {
                int s = V.head[l];
                const size_t base = (size_t)l * cap;
                for (int i = 0; i < n; i++) {
                    h += V.ld(base + s).y < P.halt_speed ? 1 : 0;
                    s = (s + 1 == cap) ? 0 : s + 1;
                }
            }
            halt[(size_t)blockIdx.x * 12 * A + l] = h;
            if constexpr (kFuse) s_halt[l] = h;
        }
    }
    for (int e = tid; e < 4 * A; e += nt) pend += V.q_off[e + 1] - V.qptr[e];
    run = wave_sum(run);
    pend = wave_sum(pend);
    if ((tid & 63) == 0) {
        atomicAdd(&s_running, run);
        atomicAdd(&s_pending, pend);
    }
    for (int a = tid; a < A; a += nt) {
        phase_out[(size_t)blockIdx.x * A + a] = V.phase[a];
        tspent[(size_t)blockIdx.x * A + a] = t - V.ts[a];
    }
    __syncthreads();
    if (tid == 0) {
        G.stats[0] = V.stats[0];
        G.stats[1] = V.stats[1];
        G.stats[2] = s_running;
        G.stats[3] = s_pending;
        done[blockIdx.x] = (t >= max_time || (s_running + s_pending) == 0) ? 1 : 0;
        if (S.t_env) S.t_env[blockIdx.x] = t;
    }
    if constexpr (kLDS) {
        // write back: occupied LDS positions (the rest are in HBM already),
        // lane counts (head 0), signals, queues
        for (int l = tid; l < NL; l += nt) {
            const int n = V.cnt[l], C1 = V.C1;
            G.head[l] = 0;
            G.cnt[l] = n;
            const size_t base = (size_t)l * cap;
            for (int i = 0, sl = V.head[l]; i < n && i < C1; i++, sl = sl + 1 == C1 ? 0 : sl + 1) {
                const float2 a = V.xv[l * C1 + sl];
                G.x[base + i] = a.x;
                G.v[base + i] = a.y;
                G.dst[base + i] = V.dst[l * C1 + sl];
            }
        }
        for (int a = tid; a < A; a += nt) {
            G.phase[a] = V.phase[a];
            G.ts[a] = V.ts[a];
        }
        for (int e = tid; e < 4 * A; e += nt) G.qptr[e] = V.qptr[e];
        if (S.actuated)
            for (int i = tid; i < 12 * A; i += nt) G.last_det[i] = V.last_det[i];
    }
    if constexpr (kFuse) {
        __syncthreads();  // the write-back has read the image: its slots are scratch now
        const bool done_e = t >= max_time || (s_running + s_pending) == 0;
        fused_tail<kFusePre>(F, S.R, S.C, t, done_e, my_act, pre, s_halt, V.phase, V.ts,
                             dyn + fl.tail_off);
    }
#ifdef DMDQN_SIM_PROFILE
    __syncthreads();
    if (tid == 0) {
        prof[7] = __builtin_amdgcn_s_memrealtime() - prof_t;  // halting + write-back
        for (int i = 0; i < 8; i++) halt[(size_t)blockIdx.x * 12 * A + i] = (int32_t)prof[i];
    }
#endif
}

// ================================================================ register path
// One thread per lane (NL <= NT): the lane's vehicles live in that thread's
// registers, compacted (front at index 0, up to RCAP), for all K substeps;
// LDS holds only what other lanes read -- per lane the vehicle count, the last
// vehicle (x, v), the front's request and tentative move, the grant, the
// route word of a vehicle that left, a pending insertion -- about 37 B per
// lane instead of the ring image's 240 (4x4: 11 KB instead of 65 KB), so every
// env of a 1024-replica launch is resident at once (4 per CU; 8x8: one
// 1024-thread block per CU), and pass C walks registers instead of LDS.
// Same passes, same IEEE operation order as the LDS path / oracle_sim.c
// (bit-exact); the rings are written back compacted (head 0).
constexpr int RCAP = 24;

__device__ __forceinline__ int wave_max_uniform(int x) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) x = max(x, __shfl_xor(x, off));
    return __builtin_amdgcn_readfirstlane(x);
}

// A lane's vehicle speeds.  In registers for blocks of up to 512 threads.
// A 1024-thread block (8x8: 128 VGPRs per thread) cannot hold three RCAP
// arrays, and the compiler then demotes one dynamically indexed array to
// scratch memory (every access a vector-memory round trip; ~130 MB of scratch
// write-back per C5 launch): there the speeds live in an LDS column
// [RCAP][NT] (thread-contiguous, conflict-free) as a ring from head h, so a
// pop moves the head instead of 23 values.
struct VColL {
    float *p;  // this thread's column, stride nt
    int h, nt;
    __device__ __forceinline__ float &at(int i) const {
        const int s = h + i;
        return p[(s >= RCAP ? s - RCAP : s) * nt];
    }
};
// V_ accessors: the register array, or (kL) the LDS column
template <bool kL>
__device__ __forceinline__ float vget(const float (&V_)[RCAP], const VColL &c, int i) {
    if constexpr (kL) return c.at(i);
    else return V_[i];
}
template <bool kL>
__device__ __forceinline__ void vset(float (&V_)[RCAP], const VColL &c, int i, float x) {
    if constexpr (kL) c.at(i) = x;
    else V_[i] = x;
}
template <bool kL>
__device__ __forceinline__ void vpop(float (&V_)[RCAP], VColL &c) {
    if constexpr (kL) {
        c.h = c.h + 1 == RCAP ? 0 : c.h + 1;
    } else {
#pragma unroll
        for (int i = 0; i < RCAP - 1; i++) V_[i] = V_[i + 1];
    }
}

// Route words (16 bits, sim.hpp) of a register lane, two per VGPR: vehicle i
// in half i & 1 of D2_[i >> 1].  Packing halves the array (12 VGPRs instead of
// 24): the 1024-thread kernel runs at 128 VGPRs per thread and spilled.
constexpr int RCAP2 = RCAP / 2;
static_assert(RCAP % 2 == 0, "route words in pairs");
__device__ __forceinline__ int dget(const uint32_t (&D2_)[RCAP2], int i) {
    return (int)((D2_[i >> 1] >> (16 * (i & 1))) & 0xffffu);
}
__device__ __forceinline__ void dset(uint32_t (&D2_)[RCAP2], int i, int w) {
    const uint32_t sh = 16 * (i & 1), x = D2_[i >> 1];
    D2_[i >> 1] = (x & ~(0xffffu << sh)) | ((uint32_t)w << sh);
}
// the front leaves: every word moves down one position (a funnel shift per pair)
__device__ __forceinline__ void dpop(uint32_t (&D2_)[RCAP2]) {
#pragma unroll
    for (int p = 0; p < RCAP2 - 1; p++) D2_[p] = __builtin_amdgcn_alignbit(D2_[p + 1], D2_[p], 16);
    D2_[RCAP2 - 1] >>= 16;
}

// append a vehicle at the back of a register lane (constant indices only; the
// words past the lane's count are never read)
template <bool kL>
__device__ __forceinline__ void lane_append(float (&X_)[RCAP], float (&V_)[RCAP], const VColL &c,
                                            uint32_t (&D2_)[RCAP2], int &n, float &lx, float &lv,
                                            float xv, float vv, int dv) {
#pragma unroll
    for (int i = 0; i < RCAP; i++) {
        const bool here = i == n;
        X_[i] = here ? xv : X_[i];
        if constexpr (!kL) V_[i] = here ? vv : V_[i];
    }
#pragma unroll
    for (int p = 0; p < RCAP2; p++) {
        D2_[p] = 2 * p == n ? (uint32_t)dv : D2_[p];
        D2_[p] = 2 * p + 1 == n ? (D2_[p] & 0xffffu) | ((uint32_t)dv << 16) : D2_[p];
    }
    if constexpr (kL) c.at(n) = vv;
    n++;
    lx = xv;
    lv = vv;
}

// The nine per-lane arrays are `ls` entries apart (ls = the block's thread
// count, a compile-time constant in the kernel): every lane array is then the
// thread's one LDS address plus an immediate offset, instead of a VGPR per
// array held across the substep loop (the 1024-thread kernel spilled them).
__host__ __device__ inline size_t sim_reg_lds_bytes(int R, int C, int ls) {
    const int A = R * C;
    return (size_t)ls * 9 * 4 + (size_t)A * 8 + (size_t)A * 48 + 16 + topo_bytes(R, C);
}

// Offset of the speed columns (1024-thread blocks) past the block's own LDS
// (and the fused step's MT stream / epilogue scratch).
__host__ __device__ inline size_t reg_vcol_off(int R, int C, bool fused, int ls) {
    const int A = R * C;
    size_t b = sim_reg_lds_bytes(R, C, ls);
    if (fused) b = fuse_layout(b, 0, (size_t)ls * 9 * 4, A).bytes;
    return (b + 15) & ~(size_t)15;
}

// Total LDS of the register path (what the launcher passes) and, in
// *perm_off, where the lane order lives: the block's own arrays (and the fused
// step's), the speed columns of a 1024-thread block, then the lane order
// (u16 per thread) and its 32 bin counters.
__host__ __device__ inline size_t reg_lds_total(int R, int C, bool fused, int ls, int nt,
                                                size_t *perm_off) {
    const int A = R * C;
    size_t b = sim_reg_lds_bytes(R, C, ls);
    if (fused) b = fuse_layout(b, 0, (size_t)ls * 9 * 4, A).bytes;
    if (nt > 512) b = reg_vcol_off(R, C, fused, ls) + (size_t)RCAP * nt * 4;
    const size_t p = (b + 15) & ~(size_t)15;
    if (perm_off) *perm_off = p;
    return p + (size_t)nt * 2 + 32 * 4;
}

// Which lane each thread owns for this launch: the lanes in DESCENDING order
// of their vehicle counts at the launch's start (s_lane[tid] = lane).  Every
// pass that walks a lane's vehicles runs to the longest lane of the wave
// (wave-uniform loops over register arrays); with lanes in launch order the
// 16 waves' longest lanes summed to ~5.7x the vehicles / 64 of an 8x8 replica
// (oracle, steady state), sorted ~2.7x.  Per-lane results do not depend on
// which thread computes them (lanes meet only through lane-indexed LDS
// arrays and integer counters), so the order changes no bit -- nor does the
// order of the lanes of equal count, which the LDS atomics below leave to
// the hardware.  Counting sort: one LDS atomic per lane (its rank within its
// count's bin), one wave's prefix scan over the RCAP + 1 bins, one store.
// (Round 6's first form, a ballot and a wave-reduced atomic per wave and
// key, took ~4.5 us of an 8x8 launch.)
// Lane tid's count c and head h (loaded by the caller at the kernel's start)
// are left in s_n / s_h (lane-indexed LDS) for the thread that takes the lane.
template <int NT>
__device__ void lane_order(int c, int h, int NL, uint16_t *s_lane, int32_t *s_bin, int32_t *s_n,
                           int32_t *s_h) {
    const int tid = threadIdx.x;
    if (tid < 32) s_bin[tid] = 0;
    int key = 0;
    if (tid < NL) {
        s_n[tid] = c;
        s_h[tid] = h;
        key = RCAP - (c < 0 ? 0 : c > RCAP ? RCAP : c);
    }
    __syncthreads();
    int r = 0;
    if (tid < NL) r = atomicAdd(&s_bin[key], 1);
    __syncthreads();
    if (tid < 64) {  // exclusive prefix of the bins (wave 0)
        const int v = tid <= RCAP ? s_bin[tid] : 0;
        int x = v;
#pragma unroll
        for (int off = 1; off < 32; off <<= 1) {
            const int y = __shfl_up(x, off);
            x += tid >= off ? y : 0;
        }
        if (tid <= RCAP) s_bin[tid] = x - v;
    }
    __syncthreads();
    if (tid < NL) s_lane[s_bin[key] + r] = (uint16_t)tid;
    __syncthreads();
}

template <int NT, bool kFuse>
__global__ void __launch_bounds__(NT, NT <= 256 ? 2 : 1)
k_sim_step_reg(dmdqn_sim S, dmdqn_idm Pa, const int32_t *actions, int stride, int t0_arg, int K,
               int max_time, int32_t *halt, int32_t *phase_out, int32_t *tspent, uint8_t *done,
               dmdqn_env_fuse F) {
    extern __shared__ __attribute__((aligned(16))) char dyn[];
#ifdef DMDQN_SIM_PROFILE
    const uint64_t prof_t0 = __builtin_amdgcn_s_memrealtime();
#endif
    const int t0 = S.t_env ? S.t_env[blockIdx.x] : t0_arg;  // the replica's own clock
    const IdmK P(Pa);
    EnvView G(S, blockIdx.x);
    const int A = G.A, NL = G.NL, cap = G.cap;
    const int tid = threadIdx.x;
    // The prologue's loads are issued as early as their addresses allow, so
    // that their memory round trips overlap (one wait covers several): this
    // thread's origin queue position and end, and the counters (each wait
    // below otherwise exposed one more round trip of the launch's start).
    const bool leader = tid < 4 * A;  // origin queue q = tid
    int qp = 0, qend = 0, qid = 0, qdst = 0;
    if (leader) {
        qp = G.qptr[tid];
        qend = G.q_off[tid + 1];
    }
    const int st0 = tid < 2 ? G.stats[tid] : 0;
    int cnt0 = 0, head0 = 0;  // lane tid's (lane_order)
    if (tid < NL) {
        cnt0 = G.cnt[tid];
        head0 = G.head[tid];
    }
    // ---- LDS: published per-lane values, signals, detector times, stats, topology
    // lane arrays LS entries apart (sim_reg_lds_bytes)
    constexpr int LS_ = SIM_LANE_STRIDE_NT ? NT : 0;
    const int LS = LS_ ? LS_ : NL;
    int32_t *s_cnt = reinterpret_cast<int32_t *>(dyn);
    float *s_lx = reinterpret_cast<float *>(s_cnt + LS), *s_lv = s_lx + LS;
    int32_t *s_req = reinterpret_cast<int32_t *>(s_lv + LS), *s_gfrom = s_req + LS;
    float *s_fx = reinterpret_cast<float *>(s_gfrom + LS), *s_fv = s_fx + LS;
    int32_t *s_mdst = reinterpret_cast<int32_t *>(s_fv + LS), *s_ins = s_mdst + LS;
    int32_t *s_phase = s_ins + LS, *s_ts = s_phase + A, *s_ldet = s_ts + A;
    int32_t *s_stats = s_ldet + 12 * A;  // inserted, arrived, running, pending
    // fused step: the MT stream past the block's own LDS; the halting counts
    // later in the topology tables' place, the epilogue's scratch in the
    // published-lane arrays (both dead by then).  The actions are drawn
    // first: their two dependent loads (the stream position, then its words)
    // overlap the topology's and the lanes' loads below.
    const FuseLayout fl = fuse_layout(sim_reg_lds_bytes(S.R, S.C, LS), 0, (size_t)LS * 9 * 4, A);
    int32_t *const s_halt = s_stats + 4;
    int my_act = 0;
    bool act_fast = false;
    if constexpr (kFuse) my_act = fused_act(F, A, reinterpret_cast<uint32_t *>(dyn + fl.mt_off), act_fast);
    const Topo T = build_topo(s_stats + 4, S.R, S.C, S.exit_id, S.exit_ao, P.len_inner,
                              P.len_outer);  // synced below

    // ---- this thread's lane (registers) and origin queue
    // the lanes by descending vehicle count (lane_order): s_lane[tid] = lane
#ifdef DMDQN_SIM_PROFILE
    const uint64_t prof_topo = __builtin_amdgcn_s_memrealtime();  // after the act draw + topology
#endif
    size_t perm_off = 0;
    (void)reg_lds_total(S.R, S.C, kFuse, LS, NT, &perm_off);
    uint16_t *const s_lane = reinterpret_cast<uint16_t *>(dyn + perm_off);
    lane_order<NT>(cnt0, head0, NL, s_lane, reinterpret_cast<int32_t *>(dyn + perm_off + (size_t)NT * 2),
                   s_cnt, s_gfrom);  // (s_gfrom: the heads until pass B)
#ifdef DMDQN_SIM_PROFILE
    const uint64_t prof_lo = __builtin_amdgcn_s_memrealtime();  // after lane_order
#endif
    if (leader && qp < qend) {  // in flight beside the vehicle staging
        qid = G.q_ids[qp];
        qdst = G.q_dst[qp];
    }
    const bool own = tid < NL;
    const int l = own ? (int)s_lane[tid] : tid;  // (e = l / 3, kf = l % 3: inside the substep loop)
    constexpr bool kL = NT > 512;  // speeds in the LDS column (VColL)
    float X_[RCAP], V_[RCAP];
    VColL Vc{nullptr, 0, NT};
    if constexpr (kL) Vc.p = reinterpret_cast<float *>(dyn + reg_vcol_off(S.R, S.C, kFuse, LS)) + tid;
    uint32_t D2_[RCAP2];
    int n = 0;
    float lx = 0.0f, lv = 0.0f;
    if (own) {
        const int h = s_gfrom[l];
        n = s_cnt[l];
        DMDQN_DBG(h >= 0 && h < cap && n >= 0 && n <= RCAP && n <= cap, DBG_SIM_RING);
        const size_t base = (size_t)l * cap;
        const int nm = wave_max_uniform(n);
        // Every load of the lane in flight at once: chunks of 8 vehicles
        // (chunk count wave-uniform, bounded by the wave's longest lane; all
        // chunks issued before the first is consumed) with constant register
        // indices -- a rolled loop, indexing the arrays
        // with a scalar (s_set_gpr_idx), waited out a memory round trip per
        // vehicle.  Buffer loads: a vehicle past the lane's count gets an
        // offset beyond the buffer's range, which makes no memory request
        // and returns 0 (the array entries past the count are never read).
        // The last vehicle (x, v) is picked from the loaded values.
        const uint32_t nb = (uint32_t)NL * (uint32_t)cap * 4u;
        const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(G.x, 0, nb, 0x00020000);
        const __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc(G.v, 0, nb, 0x00020000);
        const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(G.dst, 0, nb, 0x00020000);
        float tv[RCAP] = {};
        uint32_t td[RCAP] = {};
#pragma unroll
        for (int c = 0; c < RCAP / 8; c++) {
            if (8 * c < nm) {
#pragma unroll
                for (int j = 0; j < 8; j++) {
                    const int i = 8 * c + j;
                    const int s0 = h + i, sl = s0 >= cap ? s0 - cap : s0;
                    const uint32_t off = i < n ? (uint32_t)(base + sl) * 4u : 0x80000000u;
                    X_[i] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rx, off, 0, 0));
                    tv[i] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rv, off, 0, 0));
                    td[i] = __builtin_amdgcn_raw_buffer_load_b32(rd, off, 0, 0);
                }
            }
        }
        // (consumed unconditionally -- the same chunk conditions here let the
        // compiler merge each chunk's loads with its consumption again, one
        // wait per chunk; entries past the count are never read)
#pragma unroll
        for (int i = 0; i < RCAP; i++) {
            vset<kL>(V_, Vc, i, tv[i]);
            if (i & 1) {
                // (an empty asm pins the packing here: hoisted into the chunk's
                // load branch, it waited on each chunk's loads in turn)
                uint32_t lo = td[i - 1], hi = td[i];
                asm volatile("" : "+v"(lo), "+v"(hi));
                D2_[i >> 1] = __builtin_amdgcn_perm(hi, lo, 0x05040100u);  // lo.b0 lo.b1 hi.b0 hi.b1
            }
            lx = i == n - 1 ? X_[i] : lx;
            lv = i == n - 1 ? tv[i] : lv;
        }
        s_cnt[l] = n;
        s_lx[l] = lx;
        s_lv[l] = lv;
        s_ins[l] = -1;
    } else {
        const int nm = wave_max_uniform(0);
        (void)nm;
    }
#ifdef DMDQN_SIM_PROFILE
    const uint64_t prof_veh = __builtin_amdgcn_s_memrealtime();  // prologue to the staged vehicles
#endif
    TailPre pre{};
    if constexpr (kFuse) {
        // (1024-thread blocks have no VGPRs to hold the prefetch across the substeps)
        if constexpr (!kL) pre = fused_prefetch(F, A);
        if (tid < A) {  // A <= NT (dmdqn_env_step)
            s_phase[tid] = stride * my_act;
            s_ts[tid] = t0;
        }
    } else {
        for (int a = tid; a < A; a += NT) {
            const int act = actions ? actions[(size_t)blockIdx.x * A + a] : -1;  // < 0: keep
            s_phase[a] = act >= 0 ? stride * act : G.phase[a];
            s_ts[a] = act >= 0 ? t0 : G.ts[a];
        }
    }
    if (S.actuated)
        for (int i = tid; i < 12 * A; i += NT) s_ldet[i] = G.last_det[i];
    if (tid < 2) s_stats[tid] = st0;
    if (tid == 2 || tid == 3) s_stats[tid] = 0;
    __syncthreads();
    if constexpr (kFuse) {
        fused_act_done(F, A, act_fast, my_act);
        // parked in the MT stream's LDS (dead from here on) instead of a VGPR
        // held across the substeps (this kernel is at its register limit)
        if (tid < A) reinterpret_cast<int32_t *>(dyn + fl.mt_off)[tid] = my_act;
    }
    // the lane's length: re-read from the topology table each substep (an LDS
    // read) rather than held in a VGPR across the substeps (register limit)
#define LANE_LEN() (own ? lane_length(T, e) : 0.0f)

    // TL at time t: natural phase advance (and the actuated gap-out of phase 0)
    auto tl_pass = [&](int t) {
        for (int a = tid; a < A; a += NT) {
            const int p = s_phase[a], el = t - s_ts[a];
            bool sw;
            if (S.actuated && p == 0) {
                constexpr uint32_t gl = green_lanes(0x11BB);  // green_mask(0)
                int last = kNoDetection;
#pragma unroll
                for (int k = 0; k < 12; k++)
                    if ((gl >> k) & 1u) last = max(last, s_ldet[a * 12 + k]);
                sw = el >= kActMax || (el >= kActMin && (float)(t - last) > P.max_gap);
            } else {
                sw = el >= phase_dur(p);
            }
            if (sw) {
                s_phase[a] = (p + 1) % 12;
                s_ts[a] = t;
            }
        }
    };
    // an insertion the lane's origin queue ordered in the previous pass E
#define TAKE_INSERT()                                                   \
    do {                                                                \
        if (own) {                                                      \
            const int d_ = s_ins[l];                                    \
            if (d_ != -1) {                                             \
                DMDQN_DBG(n < RCAP, DBG_SIM_RING);                      \
                lane_append<kL>(X_, V_, Vc, D2_, n, lx, lv, P.length, 0.0f, d_); \
                s_ins[l] = -1;                                          \
            }                                                           \
        }                                                               \
    } while (0)

    tl_pass(t0);
    __syncthreads();
    int rc_d0 = -1, rc_pk = 0;  // pass A's route cache (route words are >= 0)
    // Pass B's five feeder lanes of this thread's lane (static: computed once
    // here, 10 bits each, bit 20 of fd_pk1 = the lane has feeders) instead of
    // per substep
    int fd_pk0 = 0, fd_pk1 = 0;
    if (own) {
        int as, o;
        if (feed_src(T, l / 3, as, o)) {
            fd_pk0 = feeder(as, o, 0) | (feeder(as, o, 1) << 10) | (feeder(as, o, 2) << 20);
            fd_pk1 = feeder(as, o, 3) | (feeder(as, o, 4) << 10) | (1 << 20);
        }
    }
#ifdef DMDQN_SIM_PROFILE
    uint64_t prof[8] = {0, 0, 0, 0, 0, 0, 0, 0}, prof_t = __builtin_amdgcn_s_memrealtime();
    prof[6] = prof_t - prof_t0;  // staging
    prof[0] = prof_veh - prof_t0;  // (register path: slot 0 = the part up to the staged vehicles)
#endif
    for (int k = 0; k < K; k++) {
        const int t = t0 + k;
        // the lane ids again from an opaque thread id: expressions of them are
        // then computed in the loop instead of hoisted above it and held --
        // the 1024-thread fused kernel spilled 16 such invariants to scratch
        const int tq = opaque_tid();
        const int l = tq < NL ? (int)s_lane[tq] : tq, e = l / 3, kf = l - 3 * (l / 3);
        const float len = LANE_LEN();
        TAKE_INSERT();
        // ---- A: the front vehicle decides (route, target lane, IDM, request).
        // One IDM evaluation, its inputs chosen by selects (free road: no
        // interaction term; green with a vehicle on the target lane: that
        // vehicle; red / yellow: the stop line), as the LDS path's pass A --
        // separate evaluations per branch ran every one a divergent wave
        // took.  The route decisions of the front (its out-direction,
        // movement, next edge and the movement it will take there) depend
        // only on the lane and the front's route word: cached per thread
        // (rc_d0; packed e2 | m << 12 | (mv2 + 1) << 16) and recomputed when
        // the front changes.
        int rq = -1;
        float fx = 0.0f, fv = 0.0f;
        if (own && n > 0) {
            const float x0 = X_[0], v0 = vget<kL>(V_, Vc, 0);
            const int d0 = dget(D2_, 0);
            const bool free_road = e >= 4 * A || on_final_edge(d0, e);
            bool green = false, lead = false;
            int tl = -1;
            float xl = 0.0f, vl = 0.0f;
            if (!free_road) {
                const int aj = e >> 2, d = e & 3, h = opp(d);
                if (rc_d0 != d0) {
                    const int o = out_dir(T, aj, h, d0);
                    const int m = movement(h, o);
                    DMDQN_DBG(T.nbr(aj, o) >= 0 || T.exit_id[aj * 4 + o] >= 0, DBG_SIM_EDGE);
                    const int e2 = next_edge(T, aj, o);
                    const int w2 = route_advance(d0);
                    int mv2 = -1;
                    if (!(e2 >= 4 * A || on_final_edge(w2, e2))) {
                        const int h2 = opp(e2 & 3);
                        mv2 = movement(h2, out_dir(T, e2 >> 2, h2, w2));
                    }
                    rc_pk = e2 | (m << 12) | ((mv2 + 1) << 16);
                    rc_d0 = d0;
                }
                const int e2 = rc_pk & 0xfff, m = (rc_pk >> 12) & 0xf, mv2 = (rc_pk >> 16) - 1;
                const int k2 = mv2 < 0 ? kf : lane_for_move(mv2, e2, s_cnt);
                tl = e2 * 3 + k2;
                green = (green_mask(s_phase[aj]) >> (d * 4 + m)) & 1;
                lead = green && s_cnt[tl] > 0;
                xl = s_lx[tl];
                vl = s_lv[tl];
            }
            const bool nofront = free_road || (green && !lead);
            const float gap = (len - x0) + (green ? (xl - P.length) : P.min_gap);
            const float acc = idm_sel(v0, gap, v0 - (lead ? vl : 0.0f), nofront, P);
            fv = clamp_speed(v0 + acc, P);
            fx = x0 + fv;
            const bool over = fx > len;
            rq = free_road ? kArrive : (over && green ? tl : -1);
            const bool stop = !free_road && over && !green;
            fx = stop ? len : fx;
            fv = stop ? 0.0f : fv;
            s_fx[l] = fx;
            s_fv[l] = fv;
        }
        if (own) s_req[l] = rq;
        __syncthreads();
        SIM_PROF(1);

        // ---- B: this lane, as a target, grants one request if it has room
        if (own) {
            int g = -1;
            if (fd_pk1 >> 20) {  // the lane has feeders (fd_pk0 / fd_pk1, above the loop)
                int f[5];
                f[0] = fd_pk0 & 1023;
                f[1] = (fd_pk0 >> 10) & 1023;
                f[2] = (fd_pk0 >> 20) & 1023;
                f[3] = fd_pk1 & 1023;
                f[4] = (fd_pk1 >> 10) & 1023;
                uint32_t mask = 0;
#pragma unroll
                for (int i = 0; i < 5; i++) mask |= (s_req[f[i]] == l ? 1u : 0u) << i;
                if (mask) {
                    const int start = t % 5;
                    const uint32_t rot = ((mask >> start) | (mask << (5 - start))) & 31u;
                    int kk = start + __ffs(rot) - 1;
                    if (kk >= 5) kk -= 5;
                    int fsel = f[0];
#pragma unroll
                    for (int i = 1; i < 5; i++) fsel = kk == i ? f[i] : fsel;
                    bool room = n < cap;
                    if (room && n > 0) room = (lx - P.length) >= P.min_gap;
                    if (room) g = fsel;
                }
            }
            s_gfrom[l] = g;
        }
        __syncthreads();
        SIM_PROF(2);

        // ---- C: advance this lane front to back; the front leaves or arrives
        {
            const int nm = wave_max_uniform(own ? n : 0);
            if (own && n > 0) {
                const float lead_x_old0 = X_[0], lead_v_old0 = vget<kL>(V_, Vc, 0);
                float lead_x_new = fx, fvn = fv;
                bool pop = false;
                if (rq == kArrive) {
                    pop = lead_x_new >= len;
                    if (pop) atomicAdd(&s_stats[1], 1);
                } else if (rq >= 0) {
                    pop = s_gfrom[rq] == l;
                    if (!pop) {
                        lead_x_new = len;
                        fvn = 0.0f;
                    } else {
                        s_mdst[l] = route_advance(dget(D2_, 0));
                    }
                }
                if (!pop) {
                    X_[0] = lead_x_new;
                    vset<kL>(V_, Vc, 0, fvn);
                }
                const float dp = len - P.det_dist, dpl = dp + P.length;
                bool det = lead_x_new >= dp && lead_x_old0 < dpl;
                float lead_x_old = lead_x_old0, lead_v_old = lead_v_old0;
                float last_x = X_[0], last_v = vget<kL>(V_, Vc, 0);
                // (LDS speeds: vehicle i + 1's speed is read while vehicle i is
                // computed -- the walk of the wave's longest lane otherwise
                // waits out one LDS round trip per vehicle -- and its column
                // slot is stepped from vehicle i's, which vehicle i's store
                // then reuses; slot i + 1 <= RCAP stays in the column)
                float vnx = 0.0f, *pn = nullptr;
                int sn = 0;
                if constexpr (kL) {
                    sn = Vc.h + 1 == RCAP ? 0 : Vc.h + 1;
                    pn = Vc.p + sn * NT;
                    vnx = *pn;
                }
                for (int i = 1; i < nm; i++) {
                    if (i < n) {
                        const float xi = X_[i];
                        float vi, *pc = pn;
                        if constexpr (kL) {
                            vi = vnx;
                            sn = sn + 1 == RCAP ? 0 : sn + 1;
                            pn = sn == 0 ? Vc.p : pn + NT;
                            vnx = *pn;
                        } else {
                            vi = V_[i];
                        }
                        const float gap = (lead_x_old - P.length) - xi;
                        const float acc = idm_acc(vi, gap, vi - lead_v_old, P);
                        float vn = clamp_speed(vi + acc, P);
                        float xn = xi + vn;
                        const float lim = lead_x_new - P.length;
                        // no overlap with the leader's new position: stop at
                        // lim, or stand if lim is behind (selects, not branches)
                        const bool over = xn > lim, stand = lim < xi;
                        const float xc = stand ? xi : lim, vc = stand ? 0.0f : lim - xi;
                        xn = over ? xc : xn;
                        vn = over ? vc : vn;
                        X_[i] = xn;
                        if constexpr (kL) *pc = vn;
                        else V_[i] = vn;
                        det = det || (xn >= dp && xi < dpl);
                        lead_x_old = xi;
                        lead_v_old = vi;
                        lead_x_new = xn;
                        last_x = xn;
                        last_v = vn;
                    }
                }
                if (pop) {
#pragma unroll
                    for (int i = 0; i < RCAP - 1; i++) X_[i] = X_[i + 1];
                    dpop(D2_);
                    vpop<kL>(V_, Vc);
                    n--;
                }
                lx = last_x;
                lv = last_v;
                s_cnt[l] = n;
                s_lx[l] = lx;
                s_lv[l] = lv;
                if (S.actuated && det && l < 12 * A) s_ldet[l] = t + 1;
            }
        }
        __syncthreads();
        SIM_PROF(3);

        // ---- D: this lane appends the vehicle it granted
        if (own) {
            const int f = s_gfrom[l];
            if (f >= 0) {
                const float over = s_fx[f] - lane_length(T, f / 3);
                const float vin = s_fv[f];
                const int dv = s_mdst[f];
                float xe = over;
                if (n > 0) {
                    const float lim = lx - P.length - P.min_gap;
                    if (lim < xe) xe = lim;
                }
                if (xe < 0.0f) xe = 0.0f;
                DMDQN_DBG(n < cap && n < RCAP, DBG_SIM_RING);  // pass B granted only with room
                lane_append<kL>(X_, V_, Vc, D2_, n, lx, lv, xe, vin, dv);
                s_cnt[l] = n;
                s_lx[l] = lx;
                s_lv[l] = lv;
            }
        }
        __syncthreads();
        SIM_PROF(4);

        // ---- E: each origin queue inserts its next departed vehicle if there is
        // room (the lane's owner takes it into its registers at the next pass);
        // then the signals advance to t + 1
        if (leader && qp < qend && (long long)qid * S.period_ms <= (long long)t * 1000) {
            const int q = tid, d0 = qdst;
            const int aj = q >> 2, h = opp(q & 3);
            // a one-edge route departs on the straight lanes (its origin is its end)
            const int m = on_final_edge(d0, q) ? (int)MV_S : movement(h, out_dir(T, aj, h, d0));
            const int li = q * 3 + lane_for_move(m, q, s_cnt);
            const int nc = s_cnt[li];
            bool room = nc < cap;
            if (room && nc > 0) room = s_lx[li] >= 2.0f * P.length + P.min_gap;
            if (room) {
                s_cnt[li] = nc + 1;
                s_lx[li] = P.length;
                s_lv[li] = 0.0f;
                s_ins[li] = d0;
                atomicAdd(&s_stats[0], 1);
                qp++;
                if (qp < qend) { qid = G.q_ids[qp]; qdst = G.q_dst[qp]; }
            }
        }
        if (k + 1 < K) tl_pass(t + 1);
        __syncthreads();
        SIM_PROF(5);  // E + the signals (pass "TL" stays 0 here)
    }
    TAKE_INSERT();
#undef TAKE_INSERT
#undef LANE_LEN
    const int t = t0 + K;
    // ---- outputs: halting counts, signals, running / pending, done
    int run = own ? n : 0, pend = leader ? qend - qp : 0;
    // ... and the write-back of this lane's vehicles, compacted (head 0): as
    // the staging, chunks of 8 with constant register indices (each chunk's
    // LDS speed reads in flight together), buffer stores whose offset is out
    // of range past the lane's count (dropped)
    {
        const int nm = wave_max_uniform(own ? n : 0);
        if (own) {
            const size_t base = (size_t)l * cap;
            const uint32_t nb = (uint32_t)NL * (uint32_t)cap * 4u;
            const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(G.x, 0, nb, 0x00020000);
            const __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc(G.v, 0, nb, 0x00020000);
            const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(G.dst, 0, nb, 0x00020000);
            int hc = 0;
#pragma unroll
            for (int c = 0; c < RCAP / 8; c++) {
                if (8 * c < nm) {
                    float tv[8];
#pragma unroll
                    for (int j = 0; j < 8; j++) tv[j] = vget<kL>(V_, Vc, 8 * c + j);
#pragma unroll
                    for (int j = 0; j < 8; j++) {
                        const int i = 8 * c + j;
                        const bool in = i < n;
                        const uint32_t off = in ? (uint32_t)(base + i) * 4u : 0x80000000u;
                        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(X_[i]), rx, off, 0, 0);
                        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(tv[j]), rv, off, 0, 0);
                        __builtin_amdgcn_raw_buffer_store_b32((uint32_t)dget(D2_, i), rd, off, 0, 0);
                        hc += in && tv[j] < P.halt_speed ? 1 : 0;
                    }
                }
            }
            if (l < 12 * A) {
                halt[(size_t)blockIdx.x * 12 * A + l] = hc;
                if constexpr (kFuse) s_halt[l] = hc;
            }
            G.head[l] = 0;
            G.cnt[l] = n;
        }
    }
    run = wave_sum(run);
    pend = wave_sum(pend);
    if ((tid & 63) == 0) {
        atomicAdd(&s_stats[2], run);
        atomicAdd(&s_stats[3], pend);
    }
    for (int a = tid; a < A; a += NT) {
        phase_out[(size_t)blockIdx.x * A + a] = s_phase[a];
        tspent[(size_t)blockIdx.x * A + a] = t - s_ts[a];
        G.phase[a] = s_phase[a];
        G.ts[a] = s_ts[a];
    }
    if (S.actuated)
        for (int i = tid; i < 12 * A; i += NT) G.last_det[i] = s_ldet[i];
    if (leader) G.qptr[tid] = qp;
    __syncthreads();
    if (tid == 0) {
        G.stats[0] = s_stats[0];
        G.stats[1] = s_stats[1];
        G.stats[2] = s_stats[2];
        G.stats[3] = s_stats[3];
        done[blockIdx.x] = (t >= max_time || (s_stats[2] + s_stats[3]) == 0) ? 1 : 0;
        if (S.t_env) S.t_env[blockIdx.x] = t;
    }
    if constexpr (kFuse) {
        const bool done_e = t >= max_time || (s_stats[2] + s_stats[3]) == 0;
        const int act_back = tid < A ? reinterpret_cast<const int32_t *>(dyn + fl.mt_off)[tid] : 0;
        fused_tail<!kL>(F, S.R, S.C, t, done_e, act_back, pre, s_halt, s_phase, s_ts,
                        dyn + fl.tail_off);
    }
#ifdef DMDQN_SIM_PROFILE
    __syncthreads();
    if (tid == 0) {
        prof[7] = __builtin_amdgcn_s_memrealtime() - prof_t;  // halting + write-back
        for (int i = 0; i < 8; i++) halt[(size_t)blockIdx.x * 12 * A + i] = (int32_t)prof[i];
        halt[(size_t)blockIdx.x * 12 * A + 8] = (int32_t)(prof_topo - prof_t0);
        halt[(size_t)blockIdx.x * 12 * A + 9] = (int32_t)(prof_lo - prof_t0);
    }
#endif
}

__global__ void k_sim_reset(dmdqn_sim S, const uint8_t *mask) {
    if (mask && !mask[blockIdx.x]) return;  // only the replicas whose episode ended
    EnvView V(S, blockIdx.x);
    if (S.t_env && threadIdx.x == 0) S.t_env[blockIdx.x] = 0;
    for (int l = threadIdx.x; l < V.NL; l += blockDim.x) {
        V.head[l] = 0;
        V.cnt[l] = 0;
        V.req[l] = -1;
        V.gfrom[l] = -1;
    }
    for (int a = threadIdx.x; a < V.A; a += blockDim.x) {
        V.phase[a] = 0;
        V.ts[a] = 0;
    }
    for (int e = threadIdx.x; e < 4 * V.A; e += blockDim.x) V.qptr[e] = V.q_off[e];
    for (int i = threadIdx.x; i < 12 * V.A; i += blockDim.x) V.last_det[i] = kNoDetection;
    if (threadIdx.x < 4) V.stats[threadIdx.x] = 0;
}

DMDQN_DBG_READER(dbg_flags_sim)

}  // namespace dmdqn

using namespace dmdqn;

static int check_sim(const dmdqn_sim *s) {
    DMDQN_REQUIRE(s, "dmdqn_sim: null");
    DMDQN_REQUIRE(s->R >= 1 && s->C >= 1 && s->R <= 10 && s->C <= 10, "dmdqn_sim: grid %dx%d",
                  s->R, s->C);
    DMDQN_REQUIRE(s->E >= 1 && s->cap_lane >= 2 && s->cap_lane <= 64, "dmdqn_sim: E/cap_lane");
    DMDQN_REQUIRE(s->nveh >= 0 && s->nveh <= 65535 && s->period_ms > 0, "dmdqn_sim: demand");
    DMDQN_REQUIRE(s->actuated == 0 || s->actuated == 1, "dmdqn_sim: actuated must be 0 or 1");
    DMDQN_REQUIRE(4 * s->R * s->C <= 2 * 256, "dmdqn_sim: at most 128 junctions (queue slots)");
    DMDQN_REQUIRE(s->x && s->v && s->dst && s->head && s->cnt && s->req && s->gfrom && s->fx &&
                      s->fv && s->tl_phase && s->tl_ts && s->qptr && s->q_off && s->exit_id &&
                      s->exit_ao && s->stats && s->last_det &&
                      (s->nveh == 0 || (s->q_ids && s->vdst && s->q_dst)),
                  "dmdqn_sim: null array");
    return DMDQN_OK;
}

extern "C" int dmdqn_sim_reset(const dmdqn_sim *sim, void *stream) {
    return dmdqn_sim_reset_envs(sim, nullptr, stream);
}

extern "C" int dmdqn_sim_reset_envs(const dmdqn_sim *sim, const uint8_t *mask, void *stream) {
    int rc = check_sim(sim);
    if (rc) return rc;
    hipLaunchKernelGGL(k_sim_reset, dim3(sim->E), dim3(256), 0, as_stream(stream), *sim, mask);
    DMDQN_LAUNCH_CHECK("k_sim_reset");
    return DMDQN_OK;
}

// One launcher for dmdqn_sim_step (F == nullptr) and dmdqn_env_step.
static int launch_sim(const dmdqn_sim *sim, const dmdqn_idm *idm, const int32_t *actions,
                      const dmdqn_env_fuse *F, int action_stride, int t0, int K, int max_time,
                      int32_t *halt, int32_t *phase, int32_t *tspent, uint8_t *done,
                      void *stream) {
    int rc = check_sim(sim);
    if (rc) return rc;
    DMDQN_REQUIRE(idm && halt && phase && tspent && done, "dmdqn_sim_step: null output");
    DMDQN_REQUIRE(K >= 0 && t0 >= 0 && action_stride >= 0, "dmdqn_sim_step: K/t0");
    DMDQN_REQUIRE(action_stride * 3 < 12, "dmdqn_sim_step: action_stride*3 must be < 12");
    const int A = sim->R * sim->C, NL = 3 * (4 * A + 2 * sim->R + 2 * sim->C);
    const size_t lds = sim_lds_bytes(sim->R, sim->C, sim->cap_lane);
    const size_t topo = topo_bytes(sim->R, sim->C);
    const bool fits_lds = lds + topo <= 160 * 1024 - 64;
    const bool lds_2cu = 2 * (lds + topo + 16) <= 160 * 1024;
    // Path: the LDS image when at least two env blocks fit per CU (4x4: 38.5 KB,
    // four per CU), else the register path when a block can own every lane
    // (8x8: 0.22 ms vs 0.45 ms on global memory; its 139 KB image would run one
    // block per CU), else the LDS image if it fits at all, else global memory.
    // DMDQN_OPT_SIM_PATH (1 reg, 2 lds, 3 global) forces one (A/B, tests).
    const int force = option(DMDQN_OPT_SIM_PATH);
    const bool reg_ok = NL <= 1024 && sim->cap_lane <= RCAP;
    bool use_reg = !lds_2cu && reg_ok;
    bool use_lds = fits_lds && !use_reg;
    if (force == 1) { use_reg = reg_ok; use_lds = !reg_ok && fits_lds; }
    if (force == 2) { use_reg = false; use_lds = fits_lds; }
    if (force == 3) { use_reg = false; use_lds = false; }
    const dmdqn_env_fuse f = F ? *F : dmdqn_env_fuse{};
    if (use_reg) {
        const int nt = NL <= 256 ? 256 : NL <= 512 ? 512 : 1024;
        const int ls = SIM_LANE_STRIDE_NT ? nt : NL;  // the kernel's lane-array stride
        const size_t rlds = reg_lds_total(sim->R, sim->C, F != nullptr, ls, nt, nullptr);
        DMDQN_REQUIRE(rlds <= 160 * 1024, "dmdqn_sim_step: register path needs %zu bytes of LDS", rlds);
        auto go = [&](auto kern) {
            hipLaunchKernelGGL(kern, dim3(sim->E), dim3(nt), rlds, as_stream(stream), *sim, *idm,
                               actions, action_stride, t0, K, max_time, halt, phase, tspent, done,
                               f);
        };
        if (nt == 256) F ? go(k_sim_step_reg<256, true>) : go(k_sim_step_reg<256, false>);
        else if (nt == 512) F ? go(k_sim_step_reg<512, true>) : go(k_sim_step_reg<512, false>);
        else F ? go(k_sim_step_reg<1024, true>) : go(k_sim_step_reg<1024, false>);
        DMDQN_LAUNCH_CHECK("k_sim_step_reg");
        return DMDQN_OK;
    }
    // kAct: the actuated-mode detector bookkeeping is compiled in only when used
    const size_t base = use_lds ? lds + topo : topo;
    const size_t xvb = use_lds ? (size_t)NL * (sim->cap_lane < kLdsPos ? sim->cap_lane : kLdsPos) * 8 : 0;
    const size_t bytes = F ? fuse_layout(base, xvb, xvb, A).bytes : base;
    DMDQN_REQUIRE(bytes <= 160 * 1024 - 64, "dmdqn_env_step: %zu bytes of LDS", bytes);
    auto launch = [&](auto kern) {
        hipLaunchKernelGGL(kern, dim3(sim->E), dim3(256), bytes, as_stream(stream), *sim, *idm,
                           actions, action_stride, t0, K, max_time, halt, phase, tspent, done, f);
    };
    if (use_lds) {
        if (sim->actuated) F ? launch(k_sim_step<true, true, true>) : launch(k_sim_step<true, true, false>);
        else F ? launch(k_sim_step<true, false, true>) : launch(k_sim_step<true, false, false>);
    } else {
        if (sim->actuated) F ? launch(k_sim_step<false, true, true>) : launch(k_sim_step<false, true, false>);
        else F ? launch(k_sim_step<false, false, true>) : launch(k_sim_step<false, false, false>);
    }
    DMDQN_LAUNCH_CHECK("k_sim_step");
    return DMDQN_OK;
}

extern "C" int dmdqn_sim_step(const dmdqn_sim *sim, const dmdqn_idm *idm, const int32_t *actions,
                              int action_stride, int t0, int K, int max_time, int32_t *halt,
                              int32_t *phase, int32_t *tspent, uint8_t *done, void *stream) {
    return launch_sim(sim, idm, actions, nullptr, action_stride, t0, K, max_time, halt, phase,
                      tspent, done, stream);
}

extern "C" int dmdqn_env_step(const dmdqn_sim *sim, const dmdqn_idm *idm, const dmdqn_env_fuse *F,
                              int action_stride, int t0, int K, int max_time, int32_t *halt,
                              int32_t *phase, int32_t *tspent, uint8_t *done, void *stream) {
    DMDQN_REQUIRE(F, "dmdqn_env_step: null fuse");
    DMDQN_REQUIRE(sim && sim->R * sim->C <= 100, "dmdqn_env_step: at most 100 junctions");
    DMDQN_REQUIRE(F->np_state && F->actions && F->n_actions >= 1, "dmdqn_env_step: act arguments");
    DMDQN_REQUIRE(F->greedy || F->eps >= 1.0, "dmdqn_env_step: greedy actions required when eps < 1");
    DMDQN_REQUIRE(F->mode == 0 || F->mode == 1, "dmdqn_env_step: mode must be 0 or 1");
    DMDQN_REQUIRE(F->local && F->obs && F->prev_local && F->reward, "dmdqn_env_step: observe arrays");
    DMDQN_REQUIRE(F->obs_s && F->ring_s && F->ring_n && F->ring_a && F->ring_r && F->ring_d && F->err,
                  "dmdqn_env_step: replay arrays");
    DMDQN_REQUIRE(F->cap > 0 && F->slot >= 0 && F->slot < F->cap, "dmdqn_env_step: cap=%d slot=%d",
                  F->cap, F->slot);
    return launch_sim(sim, idm, nullptr, F, action_stride, t0, K, max_time, halt, phase, tspent,
                      done, stream);
}
