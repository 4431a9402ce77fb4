/* oracle_sim.c -- CPU restatement of the grid microsimulation (TEST INFRASTRUCTURE).
 *
 * The reference's env step is SUMO 1.22 over TraCI (src/scripts/train.py:225-236,
 * order_lanes.py:449-482).  SUMO is an un-vendored C++ binary, absent here; its
 * Krauss dynamics cannot be reproduced bit-for-bit, so the build replaces it
 * with a new IDM simulator: parity of the HIP simulator is pinned to THIS
 * restatement (bit-exact, same IEEE operation order, -ffp-contract=off).
 * What is pinned to the reference itself: the TL program and link layout
 * (grid_3x3.net.xml:893-906, :1375-1461), ACTION_MAP (train.py:57), the
 * setPhase-every-step timer restart, K = STEP_DURATION substeps, done rule
 * (train.py:231-236), the halting threshold 0.1 m/s, and the demand process
 * (randomTrips period/fringe-factor, trips_p06.trips.xml:7-9).
 *
 * Processing per substep follows the passes TL, A, B, C, D, E described in
 * dmdqn_amd/csrc/sim.hip; lanes are visited in index order, which is
 * equivalent because no pass reads what the same pass writes for another lane.
 */
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

static const int PDUR[12] = {25, 6, 2, 20, 6, 2, 25, 6, 2, 20, 6, 2};
static const unsigned GREEN[12] = {0x11BB, 0, 0, 0x11DD, 0, 0, 0xBB11, 0, 0, 0xDD11, 0, 0};
/* actuated mode (SURVEY A-14): phase 0 minDur 5 / maxDur 50, grid_3x3.net.xml:894 */
#define ACT_MIN 5
#define ACT_MAX 50
#define NO_DET (-1000)
enum { N_ = 0, S_ = 1, E_ = 2, W_ = 3 };
enum { MR = 0, MS = 1, ML = 2, MU = 3 };
#define ARRIVE (-2)

struct orc_env {
    int R, C, A, X, NL, cap, period_ms, nveh;
    float *x, *v;
    int *dst, *head, *cnt, *req, *gfrom;
    float *fx, *fv;
    int *phase, *ts, *qptr, *q_off;
    uint16_t *q_ids, *vdst;
    int *exit_id, *exit_ao;
    int stats[4];
    orc_idm P;
    /* optional trace (tests): vehicle id per ring slot and the (vehicle, edge)
     * of every edge entry (insertion or junction crossing) */
    int *vid, *trace, ntrace, max_trace;
    int actuated, *last_det; /* [12A] */
};

static int opp(int d) { return d ^ 1; }
static int right_of(int h) { return h == N_ ? E_ : h == S_ ? W_ : h == E_ ? S_ : N_; }
static int movement(int h, int o) {
    if (o == h) return MS;
    if (o == opp(h)) return MU;
    if (o == right_of(h)) return MR;
    return ML;
}
static int nbr(const orc_env *g, int a, int d) {
    int r = a / g->C, c = a % g->C;
    if (d == N_) return r > 0 ? a - g->C : -1;
    if (d == S_) return r < g->R - 1 ? a + g->C : -1;
    if (d == E_) return c < g->C - 1 ? a + 1 : -1;
    return c > 0 ? a - 1 : -1;
}
static float lane_len(const orc_env *g, int e) {
    if (e >= 4 * g->A) return g->P.len_outer;
    return nbr(g, e >> 2, e & 3) >= 0 ? g->P.len_inner : g->P.len_outer;
}
static int route_out(const orc_env *g, int a, int h, int dst) {
    int tj, to;
    if (dst >= 4 * g->A) {
        int x = dst - 4 * g->A;
        tj = g->exit_ao[2 * x];
        to = g->exit_ao[2 * x + 1];
    } else {
        tj = nbr(g, dst >> 2, dst & 3);
        to = opp(dst & 3);
    }
    if (a == tj) return to;
    int r = a / g->C, c = a % g->C, rt = tj / g->C, ct = tj % g->C;
    int dv = rt < r ? N_ : (rt > r ? S_ : -1);
    int dh = ct > c ? E_ : (ct < c ? W_ : -1);
    if (h == dv || h == dh) return h;
    if (dv >= 0 && dv != opp(h)) return dv;
    if (dh >= 0 && dh != opp(h)) return dh;
    return dv >= 0 ? dv : dh;
}
/* route words (sim.hpp): < 0x8000 destination edge (routed on the fly);
 * >= 0x8000 explicit route, 2-bit out-directions above a sentinel 1 */
#define ROUTED 0x8000
static int on_final(int w, int e) { return w < ROUTED ? w == e : (w & 0x7fff) == 1; }
static int out_dir(const orc_env *g, int a, int h, int w) {
    return w < ROUTED ? route_out(g, a, h, w) : (w & 3);
}
static int advance(int w) { return w < ROUTED ? w : (ROUTED | ((w & 0x7fff) >> 2)); }

static int next_edge(const orc_env *g, int a, int o) {
    int nb = nbr(g, a, o);
    return nb >= 0 ? nb * 4 + opp(o) : 4 * g->A + g->exit_id[a * 4 + o];
}
static int lane_for_move(const orc_env *g, const int *cnt, int m, int e) {
    (void)g;
    if (m == MR) return 0;
    if (m != MS) return 2;
    return cnt[e * 3 + 1] <= cnt[e * 3 + 0] ? 1 : 0;
}
static int lane_for(const orc_env *g, const int *cnt, int e2, int kf, int w2) {
    if (e2 >= 4 * g->A || on_final(w2, e2)) return kf;
    int h2 = opp(e2 & 3);
    int o2 = out_dir(g, e2 >> 2, h2, w2);
    return lane_for_move(g, cnt, movement(h2, o2), e2);
}
static int feeders(const orc_env *g, int e2, int fl[5]) {
    int as, o;
    if (e2 < 4 * g->A) {
        as = nbr(g, e2 >> 2, e2 & 3);
        if (as < 0) return 0;
        o = opp(e2 & 3);
    } else {
        int x = e2 - 4 * g->A;
        as = g->exit_ao[2 * x];
        o = g->exit_ao[2 * x + 1];
    }
    int n = 0;
    for (int d = 0; d < 4; d++) {
        int m = movement(opp(d), o), base = (as * 4 + d) * 3;
        if (m == MS) { fl[n++] = base; fl[n++] = base + 1; }
        else if (m == MR) fl[n++] = base;
        else fl[n++] = base + 2;
    }
    return 1;
}

/* IDM, same operation order as sim.hpp */
/* The IDM divides by the constants vmax and 2 sqrt(ab) through their f32
 * reciprocals (one rounding each, as the HIP kernel does: sim.hpp IdmK). */
static float idm_free(const orc_idm *P, float v) {
    float r = v * (1.0f / P->vmax);
    float r2 = r * r;
    float r4 = r2 * r2;
    return P->accel * (1.0f - r4);
}
static float idm_acc(const orc_idm *P, float v, float s, float dv) {
    float r = v * (1.0f / P->vmax);
    float r2 = r * r;
    float r4 = r2 * r2;
    float ss = v * P->tau + (v * dv) * (1.0f / P->two_sqrt_ab);
    if (ss < 0.0f) ss = 0.0f;
    float sstar = P->min_gap + ss;
    if (s < 0.01f) s = 0.01f;
    float q = sstar / s;
    float t1 = 1.0f - r4;
    return P->accel * (t1 - q * q);
}
static float clampv(const orc_idm *P, float v) {
    if (v < 0.0f) return 0.0f;
    if (v > P->vmax) return P->vmax;
    return v;
}

/* ------------------------------------------------------------ demand */
static uint64_t splitmix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static int pick(const uint64_t *cum, int n, uint64_t u) { /* searchsorted side=right */
    for (int i = 0; i < n; i++)
        if (cum[i] > u) return i;
    return n - 1;
}

static void make_demand(orc_env *g, uint64_t seed, long end_ms) {
    int A = g->A;
    int N = (int)((end_ms + g->period_ms - 1) / g->period_ms);
    g->nveh = N;
    int no = 4 * A, nd = 0;
    uint64_t ocum[400], dcum[400];
    int dedge[400];
    uint64_t acc = 0;
    for (int e = 0; e < no; e++) {
        acc += nbr(g, e >> 2, e & 3) < 0 ? 5 : 1;
        ocum[e] = acc;
    }
    acc = 0;
    for (int e = 0; e < no; e++)
        if (nbr(g, e >> 2, e & 3) >= 0) { acc += 1; dcum[nd] = acc; dedge[nd++] = e; }
    for (int x = 0; x < g->X; x++) { acc += 5; dcum[nd] = acc; dedge[nd++] = 4 * A + x; }
    int *origin = (int *)malloc(sizeof(int) * N);
    g->q_ids = (uint16_t *)malloc(sizeof(uint16_t) * (N ? N : 1));
    g->vdst = (uint16_t *)malloc(sizeof(uint16_t) * (N ? N : 1));
    g->q_off = (int *)calloc((size_t)(no > 0 ? no + 1 : 1), sizeof(int));
    for (int i = 0; i < N; i++) {
        uint64_t z = splitmix64(seed ^ ((uint64_t)i * 0xD1B54A32D192ED03ull));
        int o = pick(ocum, no, z % ocum[no - 1]);
        uint64_t z2 = splitmix64(z);
        int d = dedge[pick(dcum, nd, z2 % dcum[nd - 1])];
        while (d == o) {
            z2 = splitmix64(z2);
            d = dedge[pick(dcum, nd, z2 % dcum[nd - 1])];
        }
        origin[i] = o;
        g->vdst[i] = (uint16_t)d;
        g->q_off[o + 1]++;
    }
    for (int e = 0; e < no; e++) g->q_off[e + 1] += g->q_off[e];
    int *fill = (int *)calloc((size_t)(no > 0 ? no : 1), sizeof(int));
    for (int i = 0; i < N; i++) { /* stable: ids ascending within an origin */
        int o = origin[i];
        g->q_ids[g->q_off[o] + fill[o]++] = (uint16_t)i;
    }
    free(fill);
    free(origin);
}

/* ------------------------------------------------------------ lifecycle */
orc_env *orc_env_create(int R, int C, int cap, uint64_t seed, long end_ms, int period_ms,
                        const orc_idm *P) {
    orc_env *g = (orc_env *)calloc(1, sizeof(orc_env));
    g->R = R; g->C = C; g->A = R * C; g->cap = cap;
    g->P = *P;
    g->exit_id = (int *)malloc(sizeof(int) * 4 * g->A);
    g->exit_ao = (int *)malloc(sizeof(int) * 2 * (2 * R + 2 * C));
    int X = 0;
    for (int a = 0; a < g->A; a++)
        for (int o = 0; o < 4; o++) {
            if (nbr(g, a, o) < 0) {
                g->exit_id[a * 4 + o] = X;
                g->exit_ao[2 * X] = a;
                g->exit_ao[2 * X + 1] = o;
                X++;
            } else {
                g->exit_id[a * 4 + o] = -1;
            }
        }
    g->X = X;
    g->NL = 3 * (4 * g->A + X);
    int fringe = 0;
    for (int e = 0; e < 4 * g->A; e++) fringe += nbr(g, e >> 2, e & 3) < 0;
    g->period_ms = period_ms > 0 ? period_ms : 7200 / fringe;
    size_t ns = (size_t)g->NL * cap;
    g->x = (float *)calloc(ns, sizeof(float));
    g->v = (float *)calloc(ns, sizeof(float));
    g->dst = (int *)calloc(ns, sizeof(int));
    g->head = (int *)calloc(g->NL, sizeof(int));
    g->cnt = (int *)calloc(g->NL, sizeof(int));
    g->req = (int *)calloc(g->NL, sizeof(int));
    g->gfrom = (int *)calloc(g->NL, sizeof(int));
    g->fx = (float *)calloc(g->NL, sizeof(float));
    g->fv = (float *)calloc(g->NL, sizeof(float));
    g->phase = (int *)calloc(g->A, sizeof(int));
    g->ts = (int *)calloc(g->A, sizeof(int));
    g->qptr = (int *)calloc(4 * g->A, sizeof(int));
    g->last_det = (int *)calloc(12 * g->A, sizeof(int));
    make_demand(g, seed, end_ms);
    orc_env_reset(g);
    return g;
}

/* Replace the generated demand with explicit tables (a loaded SUMO scenario,
 * dmdqn_amd/sumo_scenario.py): vehicle i departs at i * period_ms from origin
 * queue q (ids q_ids[q_off[q] .. q_off[q+1])) toward edge vdst[i]. Resets. */
void orc_env_set_demand(orc_env *g, int nveh, int period_ms, const uint16_t *q_ids,
                        const int32_t *q_off, const uint16_t *vdst) {
    free(g->q_ids); free(g->vdst); free(g->q_off);
    g->nveh = nveh;
    g->period_ms = period_ms;
    g->q_ids = (uint16_t *)malloc(sizeof(uint16_t) * (size_t)(nveh > 0 ? nveh : 1));
    g->vdst = (uint16_t *)malloc(sizeof(uint16_t) * (size_t)(nveh > 0 ? nveh : 1));
    g->q_off = (int *)malloc(sizeof(int) * (size_t)(4 * g->A + 1));
    memcpy(g->q_ids, q_ids, sizeof(uint16_t) * (size_t)nveh);
    memcpy(g->vdst, vdst, sizeof(uint16_t) * (size_t)nveh);
    for (int i = 0; i <= 4 * g->A; i++) g->q_off[i] = q_off[i];
    orc_env_reset(g);
}

/* Trace every edge entry (vehicle id, simulator edge) into trace[2 * max_events]
 * from now on; orc_env_trace_count returns the number of entries (may exceed
 * max_events: the excess is dropped). */
void orc_env_enable_trace(orc_env *g, int max_events) {
    free(g->vid); free(g->trace);
    g->vid = (int *)calloc((size_t)g->NL * g->cap, sizeof(int));
    g->trace = (int *)malloc(sizeof(int) * 2 * (size_t)(max_events > 0 ? max_events : 1));
    g->ntrace = 0;
    g->max_trace = max_events;
}

int orc_env_trace(const orc_env *g, int32_t *out) {
    int n = g->ntrace < g->max_trace ? g->ntrace : g->max_trace;
    if (out) memcpy(out, g->trace, sizeof(int) * 2 * (size_t)n);
    return g->ntrace;
}

/* SUMO's actuated gap-out on phase 0 (0 = fixed durations, the default). */
void orc_env_set_actuated(orc_env *g, int on) { g->actuated = on ? 1 : 0; }

void orc_env_free(orc_env *g) {
    if (!g) return;
    free(g->vid); free(g->trace);
    free(g->x); free(g->v); free(g->dst); free(g->head); free(g->cnt); free(g->req);
    free(g->gfrom); free(g->fx); free(g->fv); free(g->phase); free(g->ts); free(g->qptr);
    free(g->q_off); free(g->q_ids); free(g->vdst); free(g->exit_id); free(g->exit_ao);
    free(g->last_det);
    free(g);
}

void orc_env_reset(orc_env *g) {
    memset(g->head, 0, sizeof(int) * g->NL);
    memset(g->cnt, 0, sizeof(int) * g->NL);
    for (int l = 0; l < g->NL; l++) { g->req[l] = -1; g->gfrom[l] = -1; }
    memset(g->phase, 0, sizeof(int) * g->A);
    memset(g->ts, 0, sizeof(int) * g->A);
    for (int e = 0; e < 4 * g->A; e++) g->qptr[e] = g->q_off[e];
    for (int i = 0; i < 12 * g->A; i++) g->last_det[i] = NO_DET;
    memset(g->stats, 0, sizeof(g->stats));
}

static int last_slot(int head, int cnt, int cap) {
    int s = head + cnt - 1;
    return s >= cap ? s - cap : s;
}

static void substep(orc_env *g, int t) {
    const orc_idm *P = &g->P;
    const int A = g->A, cap = g->cap;
    for (int a = 0; a < A; a++) {
        int p = g->phase[a], el = t - g->ts[a], sw;
        if (g->actuated && p == 0) {
            /* lanes with a green link in phase 0: lane 0 right+straight, 1
             * straight, 2 left+U; the last detection over them */
            int last = NO_DET;
            for (int d = 0; d < 4; d++)
                for (int k = 0; k < 3; k++) {
                    unsigned m = (GREEN[0] >> (4 * d)) & 15u;
                    int green = k == 0 ? (m & 3u) != 0 : k == 1 ? (m & 2u) != 0 : (m & 12u) != 0;
                    if (green && g->last_det[a * 12 + d * 3 + k] > last)
                        last = g->last_det[a * 12 + d * 3 + k];
                }
            sw = el >= ACT_MAX || (el >= ACT_MIN && (float)(t - last) > P->max_gap);
        } else {
            sw = el >= PDUR[p];
        }
        if (sw) { g->phase[a] = (p + 1) % 12; g->ts[a] = t; }
    }
    /* A */
    for (int l = 0; l < g->NL; l++) {
        g->req[l] = -1;
        g->gfrom[l] = -1;
        if (g->cnt[l] == 0) continue;
        int e = l / 3, kf = l % 3, h0 = g->head[l];
        size_t base = (size_t)l * cap;
        float x0 = g->x[base + h0], v0 = g->v[base + h0];
        int d0 = g->dst[base + h0];
        float len = lane_len(g, e), acc, vn, xn;
        if (e >= 4 * A || on_final(d0, e)) {
            acc = idm_free(P, v0);
            vn = clampv(P, v0 + acc);
            xn = x0 + vn;
            g->req[l] = ARRIVE;
        } else {
            int aj = e >> 2, d = e & 3, h = opp(d);
            int o = out_dir(g, aj, h, d0);
            int m = movement(h, o);
            int e2 = next_edge(g, aj, o);
            int tl = e2 * 3 + lane_for(g, g->cnt, e2, kf, advance(d0));
            int green = (GREEN[g->phase[aj]] >> (d * 4 + m)) & 1;
            if (green) {
                int nc = g->cnt[tl];
                if (nc > 0) {
                    int ls = last_slot(g->head[tl], nc, cap);
                    float xl = g->x[(size_t)tl * cap + ls], vl = g->v[(size_t)tl * cap + ls];
                    float gap = (len - x0) + (xl - P->length);
                    acc = idm_acc(P, v0, gap, v0 - vl);
                } else {
                    acc = idm_free(P, v0);
                }
            } else {
                float gap = (len - x0) + P->min_gap;
                acc = idm_acc(P, v0, gap, v0);
            }
            vn = clampv(P, v0 + acc);
            xn = x0 + vn;
            if (xn > len) {
                if (green) g->req[l] = tl;
                else { xn = len; vn = 0.0f; }
            }
        }
        g->fx[l] = xn;
        g->fv[l] = vn;
    }
    /* B */
    for (int tl = 0; tl < g->NL; tl++) {
        int fl[5];
        if (!feeders(g, tl / 3, fl)) continue;
        int start = t % 5;
        for (int i = 0; i < 5; i++) {
            int f = fl[(start + i) % 5];
            if (g->req[f] != tl) continue;
            int nc = g->cnt[tl], room = nc < cap;
            if (room && nc > 0) {
                int ls = last_slot(g->head[tl], nc, cap);
                room = (g->x[(size_t)tl * cap + ls] - P->length) >= P->min_gap;
            }
            if (room) g->gfrom[tl] = f;
            break;
        }
    }
    /* C */
    for (int l = 0; l < g->NL; l++) {
        int n = g->cnt[l];
        if (n == 0) continue;
        float len = lane_len(g, l / 3);
        size_t base = (size_t)l * cap;
        int hd = g->head[l];
        float lxo = g->x[base + hd], lvo = g->v[base + hd], lxn = g->fx[l], fvn = g->fv[l];
        int rq = g->req[l], pop = 0;
        if (rq == ARRIVE) {
            pop = lxn >= len;
            if (pop) g->stats[1]++;
        } else if (rq >= 0) {
            pop = g->gfrom[rq] == l;
            if (!pop) { lxn = len; fvn = 0.0f; }
        }
        if (!pop) { g->x[base + hd] = lxn; g->v[base + hd] = fvn; }
        float dp = len - P->det_dist, dpl = dp + P->length;
        int det = lxn >= dp && lxo < dpl;
        int s = hd;
        for (int i = 1; i < n; i++) {
            s = (s + 1 == cap) ? 0 : s + 1;
            float xi = g->x[base + s], vi = g->v[base + s];
            float gap = (lxo - P->length) - xi;
            float acc = idm_acc(P, vi, gap, vi - lvo);
            float vn = clampv(P, vi + acc), xn = xi + vn;
            float lim = lxn - P->length;
            if (xn > lim) {
                if (lim < xi) { xn = xi; vn = 0.0f; }
                else { xn = lim; vn = lim - xi; }
            }
            g->x[base + s] = xn;
            g->v[base + s] = vn;
            det = det || (xn >= dp && xi < dpl);
            lxo = xi; lvo = vi; lxn = xn;
        }
        if (pop) { g->head[l] = (hd + 1 == cap) ? 0 : hd + 1; g->cnt[l] = n - 1; }
        if (g->actuated && det && l < 12 * A) g->last_det[l] = t + 1;
    }
    /* D */
    for (int tl = 0; tl < g->NL; tl++) {
        int f = g->gfrom[tl];
        if (f < 0) continue;
        float over = g->fx[f] - lane_len(g, f / 3), vin = g->fv[f];
        int fh = g->head[f] == 0 ? cap - 1 : g->head[f] - 1;
        int dv = advance(g->dst[(size_t)f * cap + fh]);
        int nc = g->cnt[tl];
        float xe = over;
        if (nc > 0) {
            int ls = last_slot(g->head[tl], nc, cap);
            float lim = g->x[(size_t)tl * cap + ls] - P->length - P->min_gap;
            if (lim < xe) xe = lim;
        }
        if (xe < 0.0f) xe = 0.0f;
        int slot = g->head[tl] + nc;
        if (slot >= cap) slot -= cap;
        g->x[(size_t)tl * cap + slot] = xe;
        g->v[(size_t)tl * cap + slot] = vin;
        g->dst[(size_t)tl * cap + slot] = dv;
        g->cnt[tl] = nc + 1;
        if (g->vid) {
            int id = g->vid[(size_t)f * cap + fh];
            g->vid[(size_t)tl * cap + slot] = id;
            if (g->ntrace < g->max_trace) {
                g->trace[2 * g->ntrace] = id;
                g->trace[2 * g->ntrace + 1] = tl / 3;
            }
            g->ntrace++;
        }
    }
    /* E */
    for (int e = 0; e < 4 * A; e++) {
        int p = g->qptr[e];
        if (p >= g->q_off[e + 1]) continue;
        int id = g->q_ids[p];
        if ((long long)id * g->period_ms > (long long)t * 1000) continue;
        int d0 = g->vdst[id], h = opp(e & 3);
        int m = on_final(d0, e) ? MS : movement(h, out_dir(g, e >> 2, h, d0));
        int l = e * 3 + lane_for_move(g, g->cnt, m, e);
        int nc = g->cnt[l];
        if (nc >= cap) continue;
        if (nc > 0) {
            int ls = last_slot(g->head[l], nc, cap);
            if (g->x[(size_t)l * cap + ls] < 2.0f * P->length + P->min_gap) continue;
        }
        int slot = g->head[l] + nc;
        if (slot >= cap) slot -= cap;
        g->x[(size_t)l * cap + slot] = P->length;
        g->v[(size_t)l * cap + slot] = 0.0f;
        g->dst[(size_t)l * cap + slot] = d0;
        g->cnt[l] = nc + 1;
        g->qptr[e] = p + 1;
        if (g->vid) {
            g->vid[(size_t)l * cap + slot] = id;
            if (g->ntrace < g->max_trace) {
                g->trace[2 * g->ntrace] = id;
                g->trace[2 * g->ntrace + 1] = e;
            }
            g->ntrace++;
        }
        g->stats[0]++;
    }
}

void orc_env_step(orc_env *g, const int32_t *actions, int stride, int t0, int K, int max_time,
                  int32_t *halt, int32_t *phase, int32_t *tspent, uint8_t *done) {
    if (actions)  /* a negative action: no setPhase (the program runs on, timer kept) */
        for (int a = 0; a < g->A; a++)
            if (actions[a] >= 0) { g->phase[a] = stride * actions[a]; g->ts[a] = t0; }
    for (int k = 0; k < K; k++) substep(g, t0 + k);
    int t = t0 + K, run = 0, pend = 0;
    for (int l = 0; l < g->NL; l++) {
        int n = g->cnt[l];
        run += n;
        if (l < 12 * g->A) {
            int h = 0, s = g->head[l];
            for (int i = 0; i < n; i++) {
                h += g->v[(size_t)l * g->cap + s] < g->P.halt_speed;
                s = (s + 1 == g->cap) ? 0 : s + 1;
            }
            halt[l] = h;
        }
    }
    for (int e = 0; e < 4 * g->A; e++) pend += g->q_off[e + 1] - g->qptr[e];
    for (int a = 0; a < g->A; a++) { phase[a] = g->phase[a]; tspent[a] = t - g->ts[a]; }
    g->stats[2] = run;
    g->stats[3] = pend;
    *done = (t >= max_time || run + pend == 0) ? 1 : 0;
}

int orc_env_info(const orc_env *g, int32_t *out /*[8]*/) {
    out[0] = g->NL; out[1] = g->nveh; out[2] = g->period_ms; out[3] = g->X;
    for (int i = 0; i < 4; i++) out[4 + i] = g->stats[i];
    return 0;
}

void orc_env_lanes(const orc_env *g, float *x, float *v, int32_t *dst, int32_t *head, int32_t *cnt) {
    size_t ns = (size_t)g->NL * g->cap;
    memcpy(x, g->x, ns * sizeof(float));
    memcpy(v, g->v, ns * sizeof(float));
    for (size_t i = 0; i < ns; i++) dst[i] = g->dst[i];
    memcpy(head, g->head, sizeof(int) * g->NL);
    memcpy(cnt, g->cnt, sizeof(int) * g->NL);
}

void orc_env_demand(const orc_env *g, uint16_t *q_ids, int32_t *q_off, uint16_t *vdst) {
    memcpy(q_ids, g->q_ids, sizeof(uint16_t) * g->nveh);
    memcpy(q_off, g->q_off, sizeof(int) * (4 * g->A + 1));
    memcpy(vdst, g->vdst, sizeof(uint16_t) * g->nveh);
}
