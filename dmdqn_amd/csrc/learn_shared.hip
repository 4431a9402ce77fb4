// learn_shared.hip -- the shared-parameter learn of configuration C5 (SURVEY
// 8e; not in the reference, which trains one network per junction) as two
// batched passes over every agent's 128-row batch (f16, the reference's
// mixed_float16 rounding points: learn_h16.hpp).
//
//   k_shared_next   per agent: z-score (dqn_agent.py:66-69), X(S') from the
//                   s' rows, target and online forwards of S', first-max
//                   argmax, y = r^ + (gamma (1 - d)) Q_t(S')[a*] (:342-347);
//                   writes y and the batch actions.  Both nets in LDS.
//   k_shared_grad4  per agent: X(S), online forward, MSE / Huber dL/dQ, and
//                   the backward; the weight gradients of all the agents a
//                   workgroup walks accumulate in registers and are written
//                   once per workgroup as a partial slab (k_reduce_slabs,
//                   RCCL all-reduce and k_adam follow).
//
// The S' pass runs "wave owns rows": a wave takes a 16-row tile through all
// three layers in registers.  The transposed GEMMs Z^T = W^T X^T leave each
// lane with 4 consecutive neurons of one row (MFMA C layout), and two such
// tiles are exactly the 8 K-values the next layer's B operand needs when the
// next layer's weights are stored with that K order (kperm below) -- so the
// activations never go through LDS in the forward, and no barrier is needed.
// The weight fragments come from LDS (one 16-byte read per lane per MFMA,
// conflict-free).  The gradient pass runs "wave owns neurons" (below): each
// wave keeps its weight slice in registers and the layers exchange
// activations through LDS images.
#include <math.h>

#include "common.hpp"
#include "qnet_layout.hpp"

namespace dmdqn {
namespace shk {

typedef _Float16 h16;
typedef h16 half8 __attribute__((ext_vector_type(8)));
typedef h16 half4v __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short v4s __attribute__((vector_size(8)));
typedef __attribute__((address_space(3))) v4s lds_v4s;

constexpr int B_ = 128, H = 128, NACT = QN_NA, DP = QN_DP;
using L = QL<H>;

__device__ __forceinline__ f32x4 mfma(half8 a, half8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ float r16(float x) { return (float)(h16)x; }
__device__ __forceinline__ half8 zero8() {
    half8 r;
#pragma unroll
    for (int e = 0; e < 8; e++) r[e] = (h16)0.0f;
    return r;
}

// K order of layers 2 and 3: slot 8g + e of K-step s holds neuron kperm(s, g, e)
// -- the neurons lane group g of a row holds after the previous layer's two
// output tiles 2s (e < 4) and 2s + 1 (e >= 4).
__device__ __forceinline__ int kperm(int s, int g, int e) {
    return 32 * s + 16 * (e >> 2) + 4 * g + (e & 3);
}

// ---------------------------------------------------------------- LDS images
// The blocked, XOR-permuted activation images of learn_h16.hpp (hoff): 8-row x
// 32-column blocks, conflict-free row-fragment and transposed reads.
template <int LD = H>
__device__ __forceinline__ int hoff(int r, int c) {
    const int ch = c >> 3;
    return 8 * LD * (r >> 3) + 256 * (ch >> 2) + 32 * (r & 7) +
           8 * ((ch & 3) ^ (((r >> 1) & 1) | ((r >> 2) & 2))) + (c & 7);
}

// hoff(r, c) = hoff(r & 15, c & 31) + 16 LD (r >> 4) + 256 (c >> 5) (the XOR
// takes row bits 1 and 3): the callers pass that split (rlo = r & 15, clo =
// c & 31, rblk = r >> 4, cblk = c >> 5) so each lane keeps one base per
// distinct (rlo, clo) and every block offset that is a compile-time constant
// folds into the LDS instruction's immediate (computing hoff whole left dozens
// of loop-invariant addresses in VGPRs).  tests/test_layout_cpu.py checks the
// identity for every call site's index pattern.
template <int LD = H>
__device__ __forceinline__ int hsplit(int rlo, int clo, int rblk, int cblk) {
    return hoff<LD>(rlo, clo) + 16 * LD * rblk + 256 * cblk;
}

// img[r0 + 8(l>>4) + e][c0 + (l&15)], e = 0..7 (two ds_read_b64_tr_b16);
// r0 % 32 == 0, c0 % 16 == 0.
template <int LD = H>
__device__ __forceinline__ half8 frag_tr_h(const h16 *img, int r0, int c0) {
    const int l = threadIdx.x & 63, i = l & 15, g = l >> 4;
    const h16 *p0 = img + hsplit<LD>(8 * (g & 1) + (i >> 2), (c0 & 16) + 4 * (i & 3), g >> 1, 0) +
                    (16 * LD * (r0 >> 4) + 256 * (c0 >> 5));
    v4s t0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s *)p0);
    v4s t1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s *)(p0 + 128));
    half8 r;
#pragma unroll
    for (int e = 0; e < 4; e++) {
        r[e] = __builtin_bit_cast(h16, (short)t0[e]);
        r[e + 4] = __builtin_bit_cast(h16, (short)t1[e]);
    }
    return r;
}

// frag_tr_h at this lane's first-read address p0 (the caller's hsplit base
// plus a compile-time offset).
__device__ __forceinline__ half8 frag_tr_p(const h16 *p0) {
    v4s t0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s *)p0);
    v4s t1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s *)(p0 + 128));
    half8 r;
#pragma unroll
    for (int e = 0; e < 4; e++) {
        r[e] = __builtin_bit_cast(h16, (short)t0[e]);
        r[e + 4] = __builtin_bit_cast(h16, (short)t1[e]);
    }
    return r;
}

// Same, plain row-major [rows][ld] image (the DQ image, ld 16).
__device__ __forceinline__ half8 frag_tr(const h16 *img, int ld, int r0, int c0) {
    const int l = threadIdx.x & 63, i = l & 15, g = l >> 4;
    const h16 *p0 = img + (r0 + 8 * g + (i >> 2)) * ld + c0 + 4 * (i & 3);
    v4s t0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s *)p0);
    v4s t1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s *)(p0 + 4 * ld));
    half8 r;
#pragma unroll
    for (int e = 0; e < 4; e++) {
        r[e] = __builtin_bit_cast(h16, (short)t0[e]);
        r[e + 4] = __builtin_bit_cast(h16, (short)t1[e]);
    }
    return r;
}

// ---------------------------------------------------------------- the network in LDS
// A-fragments, [tile][K-step][lane] x 16 B (each wave-instruction reads 1 KB
// contiguously):  W1: lane (i, g) = W1^T[16t + i][32s + 8g + e];
// W2: W2^T[16t + i][kperm(s, g, e)];  W3: [s][g][i < 4] = W3^T[i][kperm(s, g, e)]
// (lanes i >= 4 use zeros);  W2B (backward, dH1 = dZ2 W2^T):
// W2[j = 16t + i][kperm(s, g, e)] (Keras W2[in][out]);  W3R: W3^T [4][128]
// plain (dZ2);  biases f16.  All values are the f16 copy Keras computes with
// (the f32 variables cast to f16: params_h / target_h).
constexpr int W1_BYTES = 8 * 3 * 64 * 16, W2_BYTES = 8 * 4 * 64 * 16, W3_BYTES = 4 * 4 * 4 * 16;
constexpr int BIAS_BYTES = (2 * H + 8) * 2;
constexpr int NET_BYTES = W1_BYTES + W2_BYTES + W3_BYTES + BIAS_BYTES;  // 58896

struct Net {
    const half8 *w1, *w2, *w3;
    const h16 *b1, *b2, *b3;
};

__device__ __forceinline__ Net net_at(char *p) {
    Net n;
    n.w1 = reinterpret_cast<const half8 *>(p);
    n.w2 = reinterpret_cast<const half8 *>(p + W1_BYTES);
    n.w3 = reinterpret_cast<const half8 *>(p + W1_BYTES + W2_BYTES);
    n.b1 = reinterpret_cast<const h16 *>(p + W1_BYTES + W2_BYTES + W3_BYTES);
    n.b2 = n.b1 + H;
    n.b3 = n.b2 + H;
    return n;
}

// Stage one network from its f16 device-layout copy WH (qnet_layout.hpp) into
// LDS at p.  Every thread of the (NTH-thread) block takes part; the caller
// syncs.  Vector loads (an aligned group of 8 fan-in values is 16 contiguous
// bytes, a kperm run of 4 is 8), every one issued before the LDS stores and
// none under a branch (a per-element gather with a wait per entry made the
// prologue ~14 serial L2 round trips long).
template <int NTH>
__device__ void stage_net(const h16 *WH, char *p) {
    constexpr int N1 = 8 * 3 * 64, N2 = 8 * 4 * 64;
    constexpr int K1 = (N1 + NTH - 1) / NTH, K2 = (N2 + NTH - 1) / NTH;  // entries per thread
    half8 *w1 = reinterpret_cast<half8 *>(p);
    half8 *w2 = reinterpret_cast<half8 *>(p + W1_BYTES);
    half8 *w3 = reinterpret_cast<half8 *>(p + W1_BYTES + W2_BYTES);
    h16 *bb = reinterpret_cast<h16 *>(p + W1_BYTES + W2_BYTES + W3_BYTES);
    const int tid = threadIdx.x;
    half8 v1[K1];
    half4v v2[K2][2];
#pragma unroll
    for (int k = 0; k < K1; k++) {
        const int ent = min(tid + NTH * k, N1 - 1);  // (a clamped entry is loaded, not stored)
        const int t = ent / 192, s = (ent / 64) % 3, l = ent & 63, i = l & 15, g = l >> 4;
        const int n = 16 * t + i;
        const bool tile = s < 2 || g < 3;  // features 88..95: only 88 exists (the column)
        const half8 x = *reinterpret_cast<const half8 *>(WH + L::oW1T + qn_w1<H>(n, 32 * s + 8 * (tile ? g : 2)));
        const h16 c = WH[L::oW1X + n];
        v1[k][0] = tile ? x[0] : c;
#pragma unroll
        for (int e = 1; e < 8; e++) v1[k][e] = tile ? x[e] : (h16)0.0f;
    }
#pragma unroll
    for (int k = 0; k < K2; k++) {
        const int ent = min(tid + NTH * k, N2 - 1);
        const int t = ent / 256, s = (ent / 64) & 3, l = ent & 63, i = l & 15, g = l >> 4;
#pragma unroll
        for (int h = 0; h < 2; h++)
            v2[k][h] = *reinterpret_cast<const half4v *>(WH + L::oW2T + qn_wt(16 * t + i, kperm(s, g, 4 * h), H));
    }
    // W3 (64 entries) and the biases (264 halves): threads tid < 64 / tid < 264,
    // loads at clamped (valid) addresses by every thread, stores masked
    const int e3 = tid & 63, s3 = e3 >> 4, g3 = (e3 >> 2) & 3, i3 = e3 & 3;
    half4v v3[2];
#pragma unroll
    for (int h = 0; h < 2; h++)
        v3[h] = *reinterpret_cast<const half4v *>(WH + L::oW3T + i3 * H + kperm(s3, g3, 4 * h));
    const int jb = tid < 2 * H + NACT ? tid : 0;
    const h16 vb = WH[L::ob1 + jb];
#pragma unroll
    for (int k = 0; k < K1; k++)
        if (N1 % NTH == 0 || tid + NTH * k < N1) w1[tid + NTH * k] = v1[k];
#pragma unroll
    for (int k = 0; k < K2; k++) {
        if (N2 % NTH != 0 && tid + NTH * k >= N2) continue;
        half8 v;
#pragma unroll
        for (int e = 0; e < 4; e++) {
            v[e] = v2[k][0][e];
            v[e + 4] = v2[k][1][e];
        }
        w2[tid + NTH * k] = v;
    }
    if (tid < 64) {
        half8 v;
#pragma unroll
        for (int e = 0; e < 4; e++) {
            v[e] = v3[0][e];
            v[e + 4] = v3[1][e];
        }
        w3[tid] = v;
    }
    if (tid < 2 * H + NACT) bb[tid] = vb;
    static_assert(NTH >= 2 * H + NACT, "stage_net: one bias per thread");
}

// Diagnostics (tools/stamp_shared.py): when a stamps buffer is passed, lane 0
// of the wave (next) / thread 0 of the workgroup (grad) writes the phase ends
// of each agent it handles, s_memrealtime (100 MHz), into stamps[agent][k].
#define SH_STAMP(agent, k, who)                                                       \
    do {                                                                              \
        if (a.stamps && (who) == 0)                                                   \
            a.stamps[(size_t)(agent) * 16 + (k)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)

// ---------------------------------------------------------------- one 16-row tile
// X(S) / X(S') B-operands of a 16-row tile: lane (i, g) holds features
// 32s + 8g .. +7 of row i (int8 replay row -> f16, exact).
struct XTile {
    uint2 raw[3];
};

__device__ __forceinline__ void x_issue(const int8_t *row, XTile &x) {
    const int g = (threadIdx.x & 63) >> 4;
#pragma unroll
    for (int s = 0; s < 3; s++) x.raw[s] = reinterpret_cast<const uint2 *>(row)[4 * s + g];
}

// int8 -> f16 exactly, two values per v_perm + v_pk_add (as gx::xrows_commit):
// the byte b ^ 0x80 = v + 128 under a high byte 0x64 is the half 1024 + v + 128;
// subtracting 1152 leaves v.
__device__ __forceinline__ void x_frags(const XTile &x, half8 bx[3]) {
    typedef h16 h2v __attribute__((ext_vector_type(2)));
    const h2v bias = {(h16)-1152.0f, (h16)-1152.0f};
#pragma unroll
    for (int s = 0; s < 3; s++)
#pragma unroll
        for (int q = 0; q < 2; q++) {
            const uint32_t wv = (q ? x.raw[s].y : x.raw[s].x) ^ 0x80808080u;
            const h2v a0 = __builtin_bit_cast(h2v, __builtin_amdgcn_perm(0x64646464u, wv, 0x07010700u)) + bias;
            const h2v a1 = __builtin_bit_cast(h2v, __builtin_amdgcn_perm(0x64646464u, wv, 0x07030702u)) + bias;
            bx[s][4 * q + 0] = a0[0];
            bx[s][4 * q + 1] = a0[1];
            bx[s][4 * q + 2] = a1[0];
            bx[s][4 * q + 3] = a1[1];
        }
}

// relu(h16(h16(acc) + b)) of output tile t (bias b: the tile's 4 values of
// this lane) into the next layer's operand slot: tile t -> K-step t >> 1,
// elements 4 (t & 1) .. +3.
__device__ __forceinline__ void dense_out(f32x4 c, half4v b, int t, half8 *ops) {
    const half4v z = __builtin_convertvector(c, half4v) + b;
    const half4v zero = {(h16)0.0f, (h16)0.0f, (h16)0.0f, (h16)0.0f};
    const half4v r = z > zero ? z : zero;  // vector select: two v_pk_max_f16
#pragma unroll
    for (int e = 0; e < 4; e++) ops[t >> 1][4 * (t & 1) + e] = r[e];
}

__device__ __forceinline__ half4v bias4(const h16 *bias, int t) {
    return *reinterpret_cast<const half4v *>(bias + 16 * t + 4 * ((threadIdx.x & 63) >> 4));
}

// Forward of NT 16-row tiles through a net, every weight fragment read once
// from LDS and used for the NT tiles: hb1 / hb2 = the layer-1 / layer-2
// activations as next-layer operands (permuted K order); q = Q on the lanes
// g = 0 (Q[row i][0..3]; other lanes hold zeros).  Each output tile's weight
// fragments and bias are read from LDS one tile ahead (double-buffered, order
// pinned by scheduling barriers: the LDS latency hides behind the previous
// tile's MFMAs without the scheduler hoisting every read at once, and the
// epilogue never waits on a bias read).
template <int NT>
__device__ __forceinline__ void fwd_tiles(const Net &N, const half8 (&bx)[NT][3], half8 (&hb1)[NT][4],
                                          half8 (&hb2)[NT][4], f32x4 (&q)[NT]) {
    const int l = threadIdx.x & 63, i = l & 15, g = l >> 4;
    {
        half8 cur[3], nxt[3];
        half4v bc = bias4(N.b1, 0), bn = bc;
#pragma unroll
        for (int s = 0; s < 3; s++) cur[s] = N.w1[s * 64 + l];
#pragma unroll
        for (int t = 0; t < 8; t++) {
            if (t < 7) {
#pragma unroll
                for (int s = 0; s < 3; s++) nxt[s] = N.w1[((t + 1) * 3 + s) * 64 + l];
                bn = bias4(N.b1, t + 1);
            }
            f32x4 c[NT];
#pragma unroll
            for (int n = 0; n < NT; n++) c[n] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int s = 0; s < 3; s++)
#pragma unroll
                for (int n = 0; n < NT; n++) c[n] = mfma(cur[s], bx[n][s], c[n]);
#pragma unroll
            for (int n = 0; n < NT; n++) dense_out(c[n], bc, t, hb1[n]);
#pragma unroll
            for (int s = 0; s < 3; s++) cur[s] = nxt[s];
            bc = bn;
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    half8 cur[4], nxt[4];
    half4v bc = bias4(N.b2, 0), bn = bc;
#pragma unroll
    for (int s = 0; s < 4; s++) cur[s] = N.w2[s * 64 + l];
#pragma unroll
    for (int t = 0; t < 8; t++) {
        if (t < 7) {
#pragma unroll
            for (int s = 0; s < 4; s++) nxt[s] = N.w2[((t + 1) * 4 + s) * 64 + l];
            bn = bias4(N.b2, t + 1);
        } else {
#pragma unroll
            // lanes i >= 4 read row i & 3 (rows 4..15 of A only feed rows 4..15 of
            // the product, which no lane uses): no zero fill, no masked read
            for (int s = 0; s < 4; s++) nxt[s] = N.w3[(s * 4 + g) * 4 + (i & (NACT - 1))];
        }
        f32x4 c[NT];
#pragma unroll
        for (int n = 0; n < NT; n++) c[n] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < 4; s++)
#pragma unroll
            for (int n = 0; n < NT; n++) c[n] = mfma(cur[s], hb1[n][s], c[n]);
#pragma unroll
        for (int n = 0; n < NT; n++) dense_out(c[n], bc, t, hb2[n]);
#pragma unroll
        for (int s = 0; s < 4; s++) cur[s] = nxt[s];
        bc = bn;
        __builtin_amdgcn_sched_barrier(0);
    }
    f32x4 c[NT];
#pragma unroll
    for (int n = 0; n < NT; n++) c[n] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 4; s++)  // layer 3 (cur = W3 fragments)
#pragma unroll
        for (int n = 0; n < NT; n++) c[n] = mfma(cur[s], hb2[n][s], c[n]);
    // Q = h16(h16(acc) + b3) (a packed f16 add is the f32 add rounded once);
    // meaningful on lanes g = 0 (the callers read only those)
    const half4v b3 = *reinterpret_cast<const half4v *>(N.b3);
#pragma unroll
    for (int n = 0; n < NT; n++)
        q[n] = __builtin_convertvector(__builtin_convertvector(c[n], half4v) + b3, f32x4);
}

// ---------------------------------------------------------------- pass 1: S'
// LDS: both nets (2 x 58,896 B) + per wave: rewards f64 [128], ring slots
// [128], transition word (a | done << 8) [128], z-scored rewards f32 [128].
#ifndef SH_B4
#define SH_B4 0  // 1: the barrier between an agent's dW1 and the next agent's L1 (round 5)
#endif
#ifndef NEXT_NT
#define NEXT_NT 2  // 16-row tiles per weight read in k_shared_next
#endif
#ifndef NEXT_WAVES
#define NEXT_WAVES 8  // waves (agents in flight) per k_shared_next workgroup
#endif
constexpr int NEXT_WAVE_BYTES = B_ * 8 + B_ * 4 + B_ * 4 + B_ * 4;  // + the z-scored rewards
constexpr int NEXT_LDS = 2 * NET_BYTES + NEXT_WAVES * NEXT_WAVE_BYTES;
static_assert(NEXT_LDS <= 160 * 1024, "k_shared_next LDS");

__device__ __forceinline__ int ring_slot(const dmdqn_learn_args &a, int pos) {
    int s = a.start + pos;
    return s >= a.cap ? s - a.cap : s;
}

// One wave per agent at a time (8 agents in flight per workgroup).  HBM
// reads run ahead: the next agent's deque positions while this agent runs,
// this agent's row metadata (a, done, r) in one burst at its start, and each
// tile's X(S') one tile ahead.
__global__ void __launch_bounds__(64 * NEXT_WAVES, 1) k_shared_next(dmdqn_learn_args a, float *y_out,
                                                        uint8_t *act_out) {
    __shared__ __attribute__((aligned(16))) char smem[NEXT_LDS];
    stage_net<64 * NEXT_WAVES>(reinterpret_cast<const h16 *>(a.params_h), smem);
    stage_net<64 * NEXT_WAVES>(reinterpret_cast<const h16 *>(a.target_h), smem + NET_BYTES);
    __syncthreads();
    const Net on = net_at(smem), tg = net_at(smem + NET_BYTES);
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63, i = l & 15, g = l >> 4;
    char *wsc = smem + 2 * NET_BYTES + w * NEXT_WAVE_BYTES;
    double *r64 = reinterpret_cast<double *>(wsc);
    int *slots = reinterpret_cast<int *>(wsc + B_ * 8);
    uint32_t *tw = reinterpret_cast<uint32_t *>(wsc + B_ * 12);
    float *rnf = reinterpret_cast<float *>(wsc + B_ * 16);
    const int stride = gridDim.x * NEXT_WAVES;
    int agent = blockIdx.x * NEXT_WAVES + w;
    constexpr int RT = 16 * NEXT_NT;
    // deque positions of rows l and l + 64 (metadata) and 16n + i (the first
    // tiles' X)
    int p0 = 0, p1 = 0, pt[NEXT_NT];
#pragma unroll
    for (int n = 0; n < NEXT_NT; n++) pt[n] = 0;
    if (agent < a.NA) {
        p0 = a.idx[(size_t)agent * B_ + l];
        p1 = a.idx[(size_t)agent * B_ + l + 64];
#pragma unroll
        for (int n = 0; n < NEXT_NT; n++) pt[n] = a.idx[(size_t)agent * B_ + 16 * n + i];
    }
    for (; agent < a.NA; agent += stride) {
        SH_STAMP(agent, 10, l);
        const int8_t *base = a.ring_n + (size_t)agent * a.cap * DMDQN_ROW_BYTES;
        const int s0 = ring_slot(a, p0), s1 = ring_slot(a, p1);
        const uint4 m0 = *reinterpret_cast<const uint4 *>(base + (size_t)s0 * DMDQN_ROW_BYTES + DMDQN_ROW_A);
        const uint4 m1 = *reinterpret_cast<const uint4 *>(base + (size_t)s1 * DMDQN_ROW_BYTES + DMDQN_ROW_A);
        XTile xt[NEXT_NT];
#pragma unroll
        for (int n = 0; n < NEXT_NT; n++)
            x_issue(base + (size_t)ring_slot(a, pt[n]) * DMDQN_ROW_BYTES, xt[n]);
        // the next agent's positions, branch-free (the last agent's when none:
        // a branch here made later waits conservative, as in gx::pos3)
        const int nxt = agent + stride < a.NA ? agent + stride : a.NA - 1;
        p0 = a.idx[(size_t)nxt * B_ + l];
        p1 = a.idx[(size_t)nxt * B_ + l + 64];
#pragma unroll
        for (int n = 0; n < NEXT_NT; n++) pt[n] = a.idx[(size_t)nxt * B_ + 16 * n + i];
        slots[l] = s0;
        slots[l + 64] = s1;
        tw[l] = m0.x;
        tw[l + 64] = m1.x;
        r64[l] = __longlong_as_double((long long)(((unsigned long long)m0.w << 32) | m0.z));
        r64[l + 64] = __longlong_as_double((long long)(((unsigned long long)m1.w << 32) | m1.z));
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS writes landed
        __builtin_amdgcn_wave_barrier();
        // z-score of the batch rewards in numpy's pairwise order (learn_h16.hpp
        // zscore): 8 partial sums of 16
        double part = 0.0;
        if (l < 8) {
            part = r64[l];
            for (int k = 1; k < 16; k++) part = __dadd_rn(part, r64[8 * k + l]);
        }
        double p[8];
#pragma unroll
        for (int k = 0; k < 8; k++) p[k] = __shfl(part, k);
        const double mean = __ddiv_rn(__dadd_rn(0.0, __dadd_rn(__dadd_rn(__dadd_rn(p[0], p[1]),
                                                                         __dadd_rn(p[2], p[3])),
                                                               __dadd_rn(__dadd_rn(p[4], p[5]),
                                                                         __dadd_rn(p[6], p[7])))),
                                      128.0);
        part = 0.0;
        if (l < 8) {
            for (int k = 0; k < 16; k++) {
                const double d = __dsub_rn(r64[8 * k + l], mean);
                const double sq = __dmul_rn(d, d);
                part = k == 0 ? sq : __dadd_rn(part, sq);
            }
        }
#pragma unroll
        for (int k = 0; k < 8; k++) p[k] = __shfl(part, k);
        const double sd = __dadd_rn(
            __dsqrt_rn(__ddiv_rn(__dadd_rn(0.0, __dadd_rn(__dadd_rn(__dadd_rn(p[0], p[1]),
                                                                    __dadd_rn(p[2], p[3])),
                                                          __dadd_rn(__dadd_rn(p[4], p[5]),
                                                                    __dadd_rn(p[6], p[7])))),
                                 128.0)),
            1e-8);
        // the z-scored rewards of rows l and l + 64, by every lane (one f64
        // division per lane and row instead of per row in each tile's epilogue)
        rnf[l] = (float)__ddiv_rn(__dsub_rn(r64[l], mean), sd);
        rnf[l + 64] = (float)__ddiv_rn(__dsub_rn(r64[l + 64], mean), sd);
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the stores landed
        __builtin_amdgcn_wave_barrier();
        SH_STAMP(agent, 11, l);
#pragma unroll 1
        for (int rp = 0; rp < B_ / RT; rp++) {  // RT rows: NEXT_NT tiles share every weight read
            half8 bx[NEXT_NT][3], hb1[NEXT_NT][4], hb2[NEXT_NT][4];
#pragma unroll
            for (int n = 0; n < NEXT_NT; n++) x_frags(xt[n], bx[n]);
            if (rp + 1 < B_ / RT)  // the next rows, in flight behind these tiles
#pragma unroll
                for (int n = 0; n < NEXT_NT; n++)
                    x_issue(base + (size_t)slots[RT * (rp + 1) + 16 * n + i] * DMDQN_ROW_BYTES, xt[n]);
            f32x4 qt[NEXT_NT], qo[NEXT_NT];
            fwd_tiles<NEXT_NT>(tg, bx, hb1, hb2, qt);
            fwd_tiles<NEXT_NT>(on, bx, hb1, hb2, qo);
            if (g == 0) {
#pragma unroll
                for (int n = 0; n < NEXT_NT; n++) {
                    const int b = RT * rp + 16 * n + i;
                    // Double-DQN target (dqn_agent.py:342-347, first max on
                    // ties), each op rounded on its own as TF's
                    int best = 0;
                    float bq = qo[n][0];
                    if (qo[n][1] > bq) { best = 1; bq = qo[n][1]; }
                    if (qo[n][2] > bq) { best = 2; bq = qo[n][2]; }
                    if (qo[n][3] > bq) { best = 3; }
                    const float tq = best == 0 ? qt[n][0] : best == 1 ? qt[n][1] : best == 2 ? qt[n][2] : qt[n][3];
                    const uint32_t m = tw[b];
                    const float rn = rnf[b];
                    const float dn = ((m >> 8) & 0xffu) ? 1.0f : 0.0f;
                    const float gd = __fmul_rn(a.gamma, __fsub_rn(1.0f, dn));
                    y_out[(size_t)agent * B_ + b] = __fadd_rn(rn, __fmul_rn(gd, tq));
                    act_out[(size_t)agent * B_ + b] = (uint8_t)(m & 0xffu);
                    if (a.rn_out) a.rn_out[(size_t)agent * B_ + b] = rn;
                }
            }
        }
        __builtin_amdgcn_wave_barrier();  // every lane is done with this agent's scratch
        SH_STAMP(agent, 12, l);
    }
}

// ---------------------------------------------------------------- pass 2: gradients
// Per-row loss term and dL/dq (common.hpp loss_term), rounded as TF's ops.
__device__ __forceinline__ void row_loss(int kind, float diff, float &term, float &dq) {
#pragma clang fp contract(off)
    if (kind == DMDQN_LOSS_HUBER) {
        const float ae = fabsf(diff);
        term = ae <= 1.0f ? 0.5f * diff * diff : ae - 0.5f;
        dq = (ae <= 1.0f ? diff : copysignf(1.0f, diff)) * (1.0f / (float)B_);
    } else {
        term = diff * diff;
        dq = 2.0f * diff * (1.0f / (float)B_);
    }
}

// ---------------------------------------------------------------- pass 2: shared helpers
// (The round-3 neuron-owning gradient pass, k_shared_grad3, was an A/B
// template here until round 4; it lives on in git history -- rebuild it for a
// same-box A/B with tools/build_rev.py 2d71bef <name> -DSH_GRAD=3.  Round 5's
// one-wave-per-SIMD variant k_shared_grad6 (4 waves, two neuron tiles each;
// slower): tools/build_rev.py 21344f7 <name> -DSH_GRAD=6.  Round
// 6's k_shared_grad7 (half-agent chunks, forward of chunk q beside the
// backward of chunk q - 1, double-buffered images; bit-identical, 9 % slower):
// tools/build_rev.py f08126b <name>.)
namespace gx {
constexpr int X_BYTES = B_ * DP * 2;             // [128][96] f16
constexpr int IMG = B_ * H * 2;                  // [128][128] f16

// One agent's X(S) rows: 2 x 48 bytes per row over the workgroup's threads.
struct XRows {
    uint4 v[3];
};

template <int NTH>
__device__ __forceinline__ void xrows_issue(const dmdqn_learn_args &a, int agent, int pos,
                                            int part, XRows &x) {
    int s = a.start + pos;
    if (s >= a.cap) s -= a.cap;
    const uint4 *p = reinterpret_cast<const uint4 *>(
        a.ring_s + ((size_t)agent * a.cap + s) * DMDQN_ROW_BYTES + 48 * (part & 1));
#pragma unroll
    for (int c = 0; c < 3; c++) x.v[c] = p[c];
}

__device__ __forceinline__ void xrows_commit(const XRows &x, h16 *X, int part) {
    const int row = part >> 1, c0 = 48 * (part & 1);
    // int8 -> f16 exactly: byte b ^ 0x80 = x + 128 in the low byte of a half
    // whose high byte is 0x64 is 1024 + x + 128; subtract 1152 (v_perm, one xor
    // per 4 bytes, v_pk_add)
    typedef h16 h2v __attribute__((ext_vector_type(2)));
    const h2v bias = {(h16)-1152.0f, (h16)-1152.0f};
#pragma unroll
    for (int c = 0; c < 6; c++) {
        half8 h;
#pragma unroll
        for (int q = 0; q < 2; q++) {
            const uint32_t wv = (&x.v[c >> 1].x)[2 * (c & 1) + q] ^ 0x80808080u;
            // bytes {b0, 0x64, b1, 0x64} and {b2, 0x64, b3, 0x64}
            const uint32_t lo = __builtin_amdgcn_perm(0x64646464u, wv, 0x07010700u);
            const uint32_t hi = __builtin_amdgcn_perm(0x64646464u, wv, 0x07030702u);
            const h2v a0 = __builtin_bit_cast(h2v, lo) + bias, a1 = __builtin_bit_cast(h2v, hi) + bias;
            h[4 * q + 0] = a0[0];
            h[4 * q + 1] = a0[1];
            h[4 * q + 2] = a1[0];
            h[4 * q + 3] = a1[1];
        }
        *reinterpret_cast<half8 *>(X + hoff<DP>(row, c0 + 8 * c)) = h;
    }
}

// Deque position of the row of staging part `part` (2 parts per row) of
// `agent`, loaded unconditionally at a valid address (agent clamped to the last
// one, part wrapped): the look-ahead loads of the next agents sit on no branch,
// since the wait-count insertion is conservative at control-flow merges (a
// branch around them made the L1 phase wait for the next agent's X rows).
__device__ __forceinline__ int pos3(const dmdqn_learn_args &a, int agent, int part) {
    const int ag = agent < a.NA ? agent : a.NA - 1;
    return a.idx[(size_t)ag * B_ + ((part >> 1) & (B_ - 1))];
}

__device__ __forceinline__ float pickf4(float q0, float q1, float q2, float q3, int k) {
    // (bit selects on the values: an indexed pick of a float[4] went to scratch)
    const bool b0 = k & 1, b1 = k & 2;
    const float lo = b0 ? q1 : q0, hi = b0 ? q3 : q2;
    return b1 ? hi : lo;
}

__device__ __forceinline__ half4v relu4(f32x4 c, half4v b) {
    const half4v z = __builtin_convertvector(c, half4v) + b;
    // z > 0 ? z : +0 as a signed 16-bit max with 0 (v_pk_max_i16): a set sign
    // bit (negative, -0) is a negative integer; positive halves order as their
    // bits.  Same result for every non-NaN z.
    typedef short s4v __attribute__((ext_vector_type(4)));
    return __builtin_bit_cast(half4v, __builtin_elementwise_max(__builtin_bit_cast(s4v, z), (s4v)(0)));
}

}  // namespace gx

// ---------------------------------------------------------------- pass 2, v4
// Neuron-owning waves (round 3's k_shared_grad3: wave w owns layer-1 / layer-2
// neurons 16w..16w+15 with its W1^T / W2^T / W2 slice in registers for the
// launch, layers exchanging activations through LDS images), with the output
// layer, the loss and dZ2 moved to ROW-owning waves after the H2 image is
// complete: wave w takes batch rows 16w..16w+15,
// reads their H2 rows once (the B operand of Q^T = W3^T H2^T, four MFMAs over
// k = 0..127 from a W3^T LDS image), computes Q, the loss and dL/dQ on those
// rows, then dZ2 = h16(dq W3[k][a]) masked by H2 > 0 for every k of the rows
// straight from the same registers (the W3 row of the row's action from the
// image), and writes the dZ2 image rows.  That replaces the per-wave partial
// Q sums (8 waves' partials per row, summed by 16 lanes) and the separate
// dZ2 phase: four barriers per agent instead of five.
//   L1  Z1^T = W1^T X^T  (X image)          -> H1 image, own columns
//   L2  Z2^T = W2^T H1^T (H1 image)         -> H2 image, own columns
//   RQ  rows 16w..: Q, loss, dq ; dZ2 rows  -> DQ image, dZ2 image (rows)
//   G   dW3 (H2 own^T, DQ) ; dH1 own (dZ2 image) -> dZ1 own (over H2 own) ;
//       dW2 (H1^T, dZ2 own) ; dW1 (X^T, dZ1 own)
// Same rounding points as round 3's grad3 (Keras' mixed policy; same gradient bits).
namespace g4 {
using gx::X_BYTES;
using gx::IMG;
constexpr int OFF_X = 0;                          // two X buffers
constexpr int OFF_H1 = 2 * X_BYTES;
constexpr int OFF_Z2 = OFF_H1 + IMG;              // dZ2 [128][128], written by rows
constexpr int OFF_H2 = OFF_Z2 + IMG;              // H2 own columns, then dZ1 own columns
constexpr int OFF_DQ = OFF_H2 + IMG;              // [128][16]
// W3^T [4][W3LD] f16 (rows padded to 144 halves = 72 dwords, so the 4 rows start
// 8 banks apart): lane (i, g) of the Q MFMA reads row i & 3 (lanes of equal
// rows broadcast) and the dZ2 read takes row a -- both conflict-free.  Round 4's
// [16][128] image with repeated rows (rows 256 B apart, one bank set) made
// both reads 8-way / 4-way bank conflicts (tools/lds_banks.py).
constexpr int W3LD = H + 16, W3ROWS = NACT;
constexpr int OFF_W3 = OFF_DQ + B_ * 16 * 2;
constexpr int OFF_SC = OFF_W3 + W3ROWS * W3LD * 2;  // sloss [8]
constexpr int OFF_QS = OFF_SC + 32;                // Q statistics per row tile [8][6]
constexpr int LDS = OFF_QS + 8 * 6 * 4;
static_assert(LDS <= 160 * 1024, "k_shared_grad4 LDS");
static_assert(OFF_W3 % 16 == 0, "aligned W3 image");

// Sum over the 16 lanes of each DPP row (quad xor 1, xor 2, half-row mirror,
// row mirror): every lane of the row ends with the row's sum, in registers
// (no LDS round trip of a ds_bpermute shuffle).
__device__ __forceinline__ float row16_sum(float x) {
    x += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0xB1, 0xF, 0xF, false));
    x += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x4E, 0xF, 0xF, false));
    x += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x141, 0xF, 0xF, false));
    x += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x140, 0xF, 0xF, false));
    return x;
}

struct WSlice4 {
    half8 w1[3];   // lane (i, g): W1^T[16w + i][32s + 8g + e] (0 past feature 88)
    half8 w2[4];   // W2^T[16w + i][32s + 8g + e]
    half8 w2b[4];  // W2[16w + i][32s + 8g + e]  (= W2^T[k][j])
    half4v b1, b2, b3;
};

__device__ __forceinline__ void load_slice4(const h16 *WH, int w, WSlice4 &S) {
    const int l = threadIdx.x & 63, i = l & 15, g = l >> 4;
    const int j = 16 * w + i;
#pragma unroll
    for (int s = 0; s < 3; s++)
#pragma unroll
        for (int e = 0; e < 8; e++) {
            const int f = 32 * s + 8 * g + e;
            S.w1[s][e] = f < QN_D ? WH[L::oW1T + qn_w1<H>(j, f)] : (h16)0.0f;
        }
#pragma unroll
    for (int s = 0; s < 4; s++)
#pragma unroll
        for (int e = 0; e < 8; e++) {
            const int c = 32 * s + 8 * g + e;
            S.w2[s][e] = WH[L::oW2T + qn_wt(j, c, H)];
            S.w2b[s][e] = WH[L::oW2T + qn_wt(c, j, H)];
        }
#pragma unroll
    for (int e = 0; e < 4; e++) {
        const int k = 16 * w + 4 * g + e;
        S.b1[e] = WH[L::ob1 + k];
        S.b2[e] = WH[L::ob1 + H + k];
        S.b3[e] = WH[L::ob1 + 2 * H + e];
    }
}

template <bool QSTATS>
__global__ void __launch_bounds__(512, 1) k_shared_grad4(dmdqn_learn_args a, const float *y_in,
                                                       const uint8_t *act_in, float *slab) {
    constexpr int NTH = 512, RH = 4;  // row tiles per pass of L1 / L2 / dH1
    __shared__ __attribute__((aligned(16))) char smem[LDS];
    h16 *H1I = reinterpret_cast<h16 *>(smem + OFF_H1), *Z2I = reinterpret_cast<h16 *>(smem + OFF_Z2);
    h16 *H2I = reinterpret_cast<h16 *>(smem + OFF_H2), *DQI = reinterpret_cast<h16 *>(smem + OFF_DQ);
    h16 *W3I = reinterpret_cast<h16 *>(smem + OFF_W3);
    float *sloss = reinterpret_cast<float *>(smem + OFF_SC);
    float *sqs = reinterpret_cast<float *>(smem + OFF_QS);
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63, i = l & 15, g = l >> 4;
    const h16 *WH = reinterpret_cast<const h16 *>(a.params_h);
    WSlice4 W;
    load_slice4(WH, w, W);
    // W3^T image [16][128], row m = W3^T[m & 3]: the A operand of the Q MFMA,
    // read straight from it, puts row i's four Q values on every lane (i, g)
    for (int k = threadIdx.x; k < W3ROWS * H; k += NTH)
        W3I[(k / H) * W3LD + (k % H)] = WH[L::oW3T + (k & (NACT * H - 1))];
    half8 ones;
#pragma unroll
    for (int e = 0; e < 8; e++) ones[e] = (h16)1.0f;
    f32x4 G1[6], G2[8], G3, GB1, GB2, GB3;
    const f32x4 z4 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int f = 0; f < 6; f++) G1[f] = z4;
#pragma unroll
    for (int j = 0; j < 8; j++) G2[j] = z4;
    G3 = GB1 = GB2 = GB3 = z4;
    for (int k = threadIdx.x; k < B_ * 16; k += NTH) DQI[k] = (h16)0.0f;
    const int row = 16 * w + i;  // this lane's batch row in the RQ phase
    int wv = w;
    asm volatile("" : "+v"(wv));
    const int bR = hoff(i, 8 * g), bX = hoff<DP>(i, 8 * g);
    const int trH[2] = {hsplit(8 * (g & 1) + (i >> 2), 4 * (i & 3), g >> 1, 0),
                        hsplit(8 * (g & 1) + (i >> 2), 16 + 4 * (i & 3), g >> 1, 0)};
    const int trX[2] = {hsplit<DP>(8 * (g & 1) + (i >> 2), 4 * (i & 3), g >> 1, 0),
                        hsplit<DP>(8 * (g & 1) + (i >> 2), 16 + 4 * (i & 3), g >> 1, 0)};
    const int c0 = 16 * wv;  // own column block
    const int bW = hoff(i, (c0 & 16) + 4 * g) + 256 * (c0 >> 5);
    const int trO = hsplit(8 * (g & 1) + (i >> 2), (c0 & 16) + 4 * (i & 3), g >> 1, 0) + 256 * (c0 >> 5);
    // the partner wave's column tile (w ^ 1) and this wave's half of the row
    // tiles: dW2 j-tiles 4hh..4hh+3, dW1 f-tiles 3hh..3hh+2 (hh = w & 1)
    const int cP = 16 * (wv ^ 1), hh = wv & 1;
    const int trP = hsplit(8 * (g & 1) + (i >> 2), (cP & 16) + 4 * (i & 3), g >> 1, 0) + 256 * (cP >> 5);
    int hB[4], xB[3];
#pragma unroll
    for (int jj = 0; jj < 4; jj++) {
        const int jt = 4 * hh + jj;
        hB[jj] = (jj & 1 ? trH[1] : trH[0]) + 256 * (jt >> 1);
    }
#pragma unroll
    for (int ff = 0; ff < 3; ff++) {
        const int ft = 3 * hh + ff;
        xB[ff] = (ft & 1 ? trX[1] : trX[0]) + 256 * (ft >> 1);
    }
    const bool stager = threadIdx.x < 256;
    int agent = blockIdx.x;
    if (agent < a.NA && stager) {
        gx::XRows x0;
        gx::xrows_issue<NTH>(a, agent, gx::pos3(a, agent, threadIdx.x), threadIdx.x, x0);
        gx::xrows_commit(x0, reinterpret_cast<h16 *>(smem + OFF_X), threadIdx.x);
    }
    int npos = gx::pos3(a, agent + gridDim.x, threadIdx.x);
    float yv = 0.0f;
    int avl = 0;
    if (agent < a.NA) {
        yv = y_in[(size_t)agent * B_ + row];
        avl = act_in[(size_t)agent * B_ + row];
    }
    __syncthreads();
    int buf = 0;
    for (; agent < a.NA; agent += gridDim.x, buf ^= 1) {
        SH_STAMP(agent, 0, threadIdx.x);
        const h16 *X = reinterpret_cast<const h16 *>(smem + OFF_X + buf * X_BYTES);
        const int nxt = agent + gridDim.x;
        // look-ahead loads for the next agent, branch-free (pos3): every thread
        // loads (threads >= 256 repeat the first half's X parts), at the last
        // agent's rows when there is no next agent
        const int nxc = nxt < a.NA ? nxt : a.NA - 1;
        gx::XRows xn;
        gx::xrows_issue<NTH>(a, nxc, npos, threadIdx.x & 255, xn);
        const float yn = y_in[(size_t)nxc * B_ + row];
        const int an = act_in[(size_t)nxc * B_ + row];
        npos = gx::pos3(a, nxt + gridDim.x, threadIdx.x);
        // ---- L1: own neuron tile, row tiles in passes of RH -> H1 image
#pragma unroll
        for (int hf = 0; hf < 8 / RH; hf++) {
            f32x4 c[RH];
#pragma unroll
            for (int r = 0; r < RH; r++) c[r] = z4;
#pragma unroll
            for (int s = 0; s < 3; s++) {
                half8 xb[RH];
#pragma unroll
                for (int r = 0; r < RH; r++)
                    xb[r] = *reinterpret_cast<const half8 *>(X + bX + 16 * DP * (RH * hf + r) + 256 * s);
#pragma unroll
                for (int r = 0; r < RH; r++) c[r] = mfma(W.w1[s], xb[r], c[r]);
            }
#pragma unroll
            for (int r = 0; r < RH; r++)
                *reinterpret_cast<half4v *>(H1I + bW + 16 * H * (RH * hf + r)) = gx::relu4(c[r], W.b1);
        }
        SH_STAMP(agent, 1, threadIdx.x);
        __syncthreads();  // B1: H1 image
        // ---- L2: own tile -> H2 image
#pragma unroll
        for (int hf = 0; hf < 8 / RH; hf++) {
            f32x4 c[RH];
#pragma unroll
            for (int r = 0; r < RH; r++) c[r] = z4;
#pragma unroll
            for (int s = 0; s < 4; s++) {
                half8 hb[RH];
#pragma unroll
                for (int r = 0; r < RH; r++)
                    hb[r] = *reinterpret_cast<const half8 *>(H1I + bR + 16 * H * (RH * hf + r) + 256 * s);
#pragma unroll
                for (int r = 0; r < RH; r++) c[r] = mfma(W.w2[s], hb[r], c[r]);
            }
#pragma unroll
            for (int r = 0; r < RH; r++)
                *reinterpret_cast<half4v *>(H2I + bW + 16 * H * (RH * hf + r)) = gx::relu4(c[r], W.b2);
        }
        SH_STAMP(agent, 2, threadIdx.x);
        __syncthreads();  // B2: H2 image
        // ---- RQ: rows 16w + i.  Q^T = W3^T H2^T (K = k in four steps of 32)
        half8 h2r[4];
#pragma unroll
        for (int s = 0; s < 4; s++)
            h2r[s] = *reinterpret_cast<const half8 *>(H2I + bR + 16 * H * wv + 256 * s);
        f32x4 cq = z4;
#pragma unroll
        for (int s = 0; s < 4; s++)
            cq = mfma(*reinterpret_cast<const half8 *>(W3I + (i % W3ROWS) * W3LD + 32 * s + 8 * g),
                      h2r[s], cq);
        // every lane (i, g) holds Q[row][0..3] (the W3 image repeats its 4 rows):
        // the loss and dL/dQ of the row on every lane, stored by lanes g = 0
        float q[4];
#pragma unroll
        for (int e = 0; e < 4; e++) q[e] = r16(r16(cq[e]) + (float)W.b3[e]);
        const float qa = gx::pickf4(q[0], q[1], q[2], q[3], avl);
        float term, dq;
        row_loss(a.loss_kind, __fsub_rn(qa, yv), term, dq);
        dq = r16(dq);  // dL/dQ in f16 (the gradient of the learn's tf.cast)
        if (g == 0) {
            half4v d;
#pragma unroll
            for (int e = 0; e < 4; e++) d[e] = e == avl ? (h16)dq : (h16)0.0f;
            *reinterpret_cast<half4v *>(DQI + row * 16) = d;
        }
        if (QSTATS) {  // per row tile into LDS; summed in tile order after B3
            const float s1 = row16_sum((q[0] + q[1]) + (q[2] + q[3]));
            const float s2 = row16_sum((q[0] * q[0] + q[1] * q[1]) + (q[2] * q[2] + q[3] * q[3]));
            if (l == 0) {
                sqs[w * 6 + 0] = s1;
                sqs[w * 6 + 1] = s2;
            }
#pragma unroll
            for (int e = 0; e < NACT; e++) {  // every lane takes part in the ballot
                const float cnt = (float)__popcll(__ballot(g == 0 && avl == e));
                if (l == 0) sqs[w * 6 + 2 + e] = cnt;
            }
        }
        term = row16_sum(term);
        if (l == 0) sloss[w] = term;
        // dZ2 of the row for k = 32s + 8g + e: h16(dq W3[k][a]) where H2 > 0
        // (the W3 row of the action read first, then the stores)
        half8 w3[4];
#pragma unroll
        for (int s = 0; s < 4; s++) w3[s] = *reinterpret_cast<const half8 *>(W3I + avl * W3LD + 32 * s + 8 * g);
#pragma unroll
        for (int s = 0; s < 4; s++) {
            half8 o;
#pragma unroll
            for (int e = 0; e < 8; e++)
                o[e] = h2r[s][e] > (h16)0.0f ? (h16)(dq * (float)w3[s][e]) : (h16)0.0f;
            *reinterpret_cast<half8 *>(Z2I + bR + 16 * H * wv + 256 * s) = o;
        }
        // the next agent's X into the other buffer (last read two agents ago)
        if (nxt < a.NA && stager)
            gx::xrows_commit(xn, reinterpret_cast<h16 *>(smem + OFF_X + (buf ^ 1) * X_BYTES),
                             threadIdx.x);
        SH_STAMP(agent, 3, threadIdx.x);
        __syncthreads();  // B3: DQ, dZ2 image, loss partials, next X
        if (threadIdx.x == 0 && a.loss) {
            float ls = sloss[0];
            for (int v = 1; v < 8; v++) ls += sloss[v];
            a.loss[agent] = ls / (float)B_;
        }
        if (QSTATS && threadIdx.x < 6) {
            // the agent's Q statistics in row-tile order (one writer per agent:
            // deterministic, unlike float atomics from the eight waves)
            float t = sqs[threadIdx.x];
            for (int v = 1; v < 8; v++) t += sqs[v * 6 + threadIdx.x];
            a.qstats[(size_t)agent * 6 + threadIdx.x] += t;
        }
        // ---- dW3 (own k) and db3 (wave 0)
#pragma unroll
        for (int s = 0; s < 4; s++) {
            const half8 dqf = frag_tr(DQI, 16, 32 * s, 0);
            G3 = mfma(frag_tr_p(H2I + trO + 2 * 16 * H * s), dqf, G3);
            if (w == 0) GB3 = mfma(ones, dqf, GB3);
        }
        SH_STAMP(agent, 4, threadIdx.x);
        // ---- dH1 (own j) -> dZ1 own -> image (over this wave's H2 columns)
#pragma unroll
        for (int hf = 0; hf < 8 / RH; hf++) {
            f32x4 c[RH];
#pragma unroll
            for (int r = 0; r < RH; r++) c[r] = z4;
#pragma unroll
            for (int s = 0; s < 4; s++) {
                half8 zb[RH];
#pragma unroll
                for (int r = 0; r < RH; r++)
                    zb[r] = *reinterpret_cast<const half8 *>(Z2I + bR + 16 * H * (RH * hf + r) + 256 * s);
#pragma unroll
                for (int r = 0; r < RH; r++) c[r] = mfma(W.w2b[s], zb[r], c[r]);
            }
#pragma unroll
            for (int r = 0; r < RH; r++) {
                const int rt = RH * hf + r;
                half4v o;
                const half4v hv = *reinterpret_cast<const half4v *>(H1I + bW + 16 * H * rt);
#pragma unroll
                for (int e = 0; e < 4; e++) o[e] = hv[e] > (h16)0.0f ? (h16)c[r][e] : (h16)0.0f;
                *reinterpret_cast<half4v *>(H2I + bW + 16 * H * rt) = o;
            }
        }
        SH_STAMP(agent, 5, threadIdx.x);
        // ---- dW2[j][k] and db2 ; dW1[f][j] and db1 (K = rows), paired waves
        // (round 5): waves 2p and 2p+1 share their two column tiles (k of dW2,
        // j of dW1) and split the row tiles (j of dW2, f of dW1) in halves, so a
        // wave reads 4 H1 + 3 X + 4 own / partner fragments per K-step for 16
        // MFMAs instead of 8 + 6 + 2 (round 4: every wave read all eight H1 and
        // six X fragments for its one column tile).  Every gradient element is
        // the same MFMA chain as before: the slabs are bit-identical.
        // dW2 first: dZ2 (both column tiles) is complete since B3
#pragma unroll
        for (int s = 0; s < 4; s++) {
            const half8 bqA = frag_tr_p(Z2I + trO + 2 * 16 * H * s);
            const half8 bqB = frag_tr_p(Z2I + trP + 2 * 16 * H * s);
            GB2 = mfma(ones, bqA, GB2);
#pragma unroll
            for (int jj = 0; jj < 4; jj++) {
                const half8 av = frag_tr_p(H1I + hB[jj] + 2 * 16 * H * s);
                G2[2 * jj] = mfma(av, bqA, G2[2 * jj]);
                G2[2 * jj + 1] = mfma(av, bqB, G2[2 * jj + 1]);
            }
        }
        // the partner's dZ1 columns (written over its H2 columns in its dH1
        // phase) are complete only after this barrier
        __syncthreads();
#pragma unroll
        for (int s = 0; s < 4; s++) {
            const half8 bvA = frag_tr_p(H2I + trO + 2 * 16 * H * s);
            const half8 bvB = frag_tr_p(H2I + trP + 2 * 16 * H * s);
            GB1 = mfma(ones, bvA, GB1);
#pragma unroll
            for (int ff = 0; ff < 3; ff++) {
                const half8 xv = frag_tr_p(X + xB[ff] + 2 * 16 * DP * s);
                G1[2 * ff] = mfma(xv, bvA, G1[2 * ff]);
                G1[2 * ff + 1] = mfma(xv, bvB, G1[2 * ff + 1]);
            }
        }
        yv = yn;
        avl = an;
        SH_STAMP(agent, 6, threadIdx.x);
#if SH_B4
        __syncthreads();  // B4: the images are rewritten by the next agent
#endif
        // (round 6: no barrier here.  What the next agent's L1 writes, H1's
        // own columns, every wave last read in dW2 -- before the pair barrier
        // above; L1 reads the other X buffer, which RQ committed before B3.
        // The later writes wait for B1: L2's H2 columns, which dW1 reads; RQ's
        // X commit into this agent's buffer, dZ2 rows, DQ and loss partials.
        // So waves that finish dW1 early start the next agent's L1 MFMAs
        // beside the others' dW1.)
        SH_STAMP(agent, 7, threadIdx.x);
    }
    // partial sums of this workgroup, kernel layout (every index written once)
    float *G = slab + (size_t)blockIdx.x * L::P;
    const int n0 = 16 * w, n = n0 + i;  // this lane's neuron (C-tile column)
    if (i < NACT)  // G3: rows k = n0 + 4g + e, column a = i
        *reinterpret_cast<float4 *>(G + L::oW3T + i * H + n0 + 4 * g) =
            make_float4(G3[0], G3[1], G3[2], G3[3]);
    {
        const int hh = w & 1, nB = 16 * (w ^ 1) + i;  // the partner's column
#pragma unroll
        for (int jj = 0; jj < 4; jj++) {  // G2[2jj + c]: fan-in j = 16(4hh + jj) + 4g + e
            const int j0 = 16 * (4 * hh + jj) + 4 * g;
            *reinterpret_cast<float4 *>(G + L::oW2T + qn_wt(n, j0, H)) =
                make_float4(G2[2 * jj][0], G2[2 * jj][1], G2[2 * jj][2], G2[2 * jj][3]);
            *reinterpret_cast<float4 *>(G + L::oW2T + qn_wt(nB, j0, H)) =
                make_float4(G2[2 * jj + 1][0], G2[2 * jj + 1][1], G2[2 * jj + 1][2], G2[2 * jj + 1][3]);
        }
#pragma unroll
        for (int ff = 0; ff < 3; ff++) {  // G1[2ff + c]: features 16(3hh + ff) + 4g + e
            const int ft = 3 * hh + ff;
            if (ft < 5 || g < 2) {
                *reinterpret_cast<float4 *>(G + L::oW1T + qn_w1<H>(n, 16 * ft + 4 * g)) =
                    make_float4(G1[2 * ff][0], G1[2 * ff][1], G1[2 * ff][2], G1[2 * ff][3]);
                *reinterpret_cast<float4 *>(G + L::oW1T + qn_w1<H>(nB, 16 * ft + 4 * g)) =
                    make_float4(G1[2 * ff + 1][0], G1[2 * ff + 1][1], G1[2 * ff + 1][2],
                                G1[2 * ff + 1][3]);
            }
            if (ft == 5 && g == 2) {  // feature 88
                G[L::oW1X + n] = G1[2 * ff][0];
                G[L::oW1X + nB] = G1[2 * ff + 1][0];
            }
        }
    }
    if (g == 0) {
        G[L::ob2 + n] = GB2[0];
        G[L::ob1 + n] = GB1[0];
    }
    if (w == 0 && g == 0 && i < NACT) G[L::ob3 + i] = GB3[0];
}

}  // namespace g4




}  // namespace shk

// LDS of the S' pass's workgroup (one per CU): what it leaves of a CU's 160 KB
// is the budget of a sampler block running beside it (include/dmdqn.h).
extern "C" size_t dmdqn_learn_shared_lds_bytes(void) { return shk::NEXT_LDS; }

// Launch of the two passes (called by dmdqn_learn_shared_grad, learn_f16.hip).
int launch_shared_v2(const dmdqn_learn_args *a, float *y, uint8_t *act, float *slab, int n_slabs,
                     hipStream_t s) {
    using namespace shk;
    const int next_wg = (a->NA + NEXT_WAVES - 1) / NEXT_WAVES;
    const int next_blocks = next_wg < n_slabs ? next_wg : n_slabs;
    hipLaunchKernelGGL(k_shared_next, dim3(next_blocks), dim3(64 * NEXT_WAVES), 0, s, *a, y, act);
    DMDQN_LAUNCH_CHECK("k_shared_next");
    auto k = a->qstats ? g4::k_shared_grad4<true> : g4::k_shared_grad4<false>;
    hipLaunchKernelGGL(k, dim3(n_slabs), dim3(512), 0, s, *a, y, act, slab);
    DMDQN_LAUNCH_CHECK("k_shared_grad");
    return DMDQN_OK;
}

}  // namespace dmdqn
