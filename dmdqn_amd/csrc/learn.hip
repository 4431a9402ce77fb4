// learn.hip -- fused Double-DQN learn step, one workgroup (8 waves) per agent.
//
// Replaces src/agents/dqn_agent.py:328-380 (+ ReplayBuffer.sample's gather and
// reward z-score, :64-84, and the hard target sync :376-377):
//   gather S, S' rows (int8 replay rows -> LDS), z-score the f64 rewards with
//   numpy's pairwise order, a* = argmax online(S'), q_t = target(S')[a*],
//   y = r + gamma (1-d) q_t, q = online(S)[a], L = mean((y-q)^2), backward
//   through the 3 Dense layers, Keras-3 Adam, optional target <- online.
// All three GEMM chains run on MFMA (v_mfma_f32_16x16x4_f32: exact f32
// products, the strict-parity path).  Work split per layer: 8 waves x one
// 16-wide output-column tile each; the batch (128 rows) is the M dimension.
//
// LDS (H = 128): X f16 [128][96] (replay features are small integers, exact in
// f16) | H1 f32 [128][128] | H2 f32 [128][128] | per-row scratch.
#include <math.h>

#include <type_traits>

#include "common.hpp"
#include "qnet_layout.hpp"

namespace dmdqn {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int B_ = 128;     // batch (dqn_agent.py: batch_size 128)
constexpr int D_ = 89;      // observation dim
constexpr int DP = 96;      // padded feature stride of the X image in LDS
constexpr int NACT = 4;

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

template <int H>
struct Lay : QL<H> {
    using QL<H>::P;
    // LDS byte offsets
    static constexpr int X_OFF = 0;
    static constexpr int H1_OFF = B_ * DP * 2;
    static constexpr int H2_OFF = H1_OFF + B_ * H * 4;
    static constexpr int SC_OFF = H2_OFF + B_ * H * 4;
    static constexpr int LDS = SC_OFF + 6400;
};

struct Scratch {
    float *z3;    // [128][4]  target Q(S') then online Q(S)
    float *rn;    // [128] z-scored reward
    float *y;     // [128] TD target
    int *act;     // [128]
    float *dq;    // [128] dL/dq
    int *slot;    // [128]
    float *dn;    // [128] done
    double *r64;  // [128]
    double *red;  // [16]
};

// Y[b][n] = act(X[b][:] . W[:][n] + bias[n]) for the wave's 16-column tile.
// X rows come from LDS (f16 or f32), W^T [N][KS] (tiled, qn_wt; KS = 0: the
// layer-1 block, qn_w1) from global memory.
template <int H, int K, typename TX, bool RELU, int KS>
__device__ __forceinline__ void dense_tile(const TX *X, int ldx, const float *WT, const float *bias,
                                           float *Y, int ldy, int n0, int nvalid) {
    const int l = threadIdx.x & 63, lr = l & 15, lk = l >> 4;
    f32x4 acc[8];
#pragma unroll
    for (int t = 0; t < 8; t++) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int n = n0 + lr;
    for (int k0 = 0; k0 < K; k0 += 4) {
        const int kk = k0 + lk;
        const float bv =
            (kk < K && lr < nvalid) ? WT[KS == 0 ? qn_w1<H>(n, kk) : qn_wt(n, kk, KS)] : 0.0f;
#pragma unroll
        for (int t = 0; t < 8; t++) {
            const float av = (float)X[(16 * t + lr) * ldx + kk];
            acc[t] = mfma4(av, bv, acc[t]);
        }
    }
    if (lr < nvalid) {
        const float bb = bias[n];
#pragma unroll
        for (int t = 0; t < 8; t++)
#pragma unroll
            for (int j = 0; j < 4; j++) {
                float z = acc[t][j] + bb;
                if (RELU) z = z > 0.0f ? z : 0.0f;
                Y[(16 * t + 4 * lk + j) * ldy + n] = z;
            }
    }
}

// Full forward of one 128-row batch: H1, H2 (post-ReLU) in LDS, Q -> z3[128][4].
// X: the f16 LDS image (int8 rows) or the f32 pre-gathered rows (float rows).
template <int H, typename TX>
__device__ void forward(const float *P, const TX *X, float *H1, float *H2, float *z3) {
    using L = Lay<H>;
    const int w = threadIdx.x >> 6;
    constexpr int NT = H / 16;  // column tiles per layer
    for (int nt = w; nt < NT; nt += 8)
        dense_tile<H, D_, TX, true, 0>(X, DP, P + L::oW1T, P + L::ob1, H1, H, 16 * nt, 16);
    __syncthreads();
    for (int nt = w; nt < NT; nt += 8)
        dense_tile<H, H, float, true, H>(H1, H, P + L::oW2T, P + L::ob2, H2, H, 16 * nt, 16);
    __syncthreads();
    // output layer: 4 columns; wave w computes batch tile w (K = H)
    {
        const int l = threadIdx.x & 63, lr = l & 15, lk = l >> 4;
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
        const float *W3T = P + L::oW3T;
        for (int k0 = 0; k0 < H; k0 += 4) {
            const int kk = k0 + lk;
            const float bv = lr < NACT ? W3T[lr * H + kk] : 0.0f;
            const float av = H2[(16 * w + lr) * H + kk];
            acc = mfma4(av, bv, acc);
        }
        if (lr < NACT) {
            const float bb = P[L::ob3 + lr];
#pragma unroll
            for (int j = 0; j < 4; j++) z3[(16 * w + 4 * lk + j) * NACT + lr] = acc[j] + bb;
        }
    }
    __syncthreads();
}

struct AdamK {
    float alpha, c1, c2, eps;
};

// Keras-3 Adam (keras/src/optimizers/adam.py update_step) for one element.
__device__ __forceinline__ void adam_el(float *w, float *m, float *v, float *tgt, size_t i,
                                        float g, const AdamK &K, bool sync) {
    // each op rounded as TF's separate kernels (mul_rn: this file is built with
    // -ffp-contract=fast, which ignores the contract pragma)
    float mi = m[i], vi = v[i], wi = w[i];
    mi = mi + mul_rn(g - mi, K.c1);
    vi = vi + mul_rn(mul_rn(g, g) - vi, K.c2);
    wi = wi - (mi * K.alpha) / (sqrtf(vi) + K.eps);
    m[i] = mi;
    v[i] = vi;
    w[i] = wi;
    if (sync) tgt[i] = wi;
}

// XF: float replay rows (DMDQN_ROWS_F32): X(S') / X(S) are read as f32 from the
// pre-gathered a.xn / a.xs (global, batch order) instead of the f16 LDS image.
template <int H, bool XF>
__global__ void __launch_bounds__(512) k_learn_f32(dmdqn_learn_args a) {
    using L = Lay<H>;
    __shared__ __attribute__((aligned(16))) char smem[L::LDS];
    _Float16 *XL = (_Float16 *)(smem + L::X_OFF);
    using TX = typename std::conditional<XF, float, _Float16>::type;
    float *H1 = (float *)(smem + L::H1_OFF);
    float *H2 = (float *)(smem + L::H2_OFF);
    char *sc = smem + L::SC_OFF;
    Scratch S{(float *)sc,           (float *)(sc + 2048), (float *)(sc + 2560),
              (int *)(sc + 3072),    (float *)(sc + 3584), (int *)(sc + 4096),
              (float *)(sc + 4608),  (double *)(sc + 5120), (double *)(sc + 6144)};
    const int agent = blockIdx.x;
    const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
    const size_t P = (size_t)a.P;
    float *Wp = a.params + agent * P, *Mp = a.adam_m + agent * P, *Vp = a.adam_v + agent * P;
    float *Tp = a.target + agent * P;
    const bool sync = a.sync_target != 0;
    const AdamK AK{a.alpha, a.c1, a.c2, a.eps};

    // ---- P0: batch metadata (ReplayBuffer.sample :63-64 via deque positions)
    if (tid < B_) {
        int pos = a.idx[(size_t)agent * B_ + tid];
        DMDQN_DBG(pos >= 0 && pos < a.cap, DBG_LEARN_IDX);
#ifdef DMDQN_DEBUG_BOUNDS
        if (pos < 0 || pos >= a.cap) pos = 0;
#endif
        int s = a.start + pos;
        if (s >= a.cap) s -= a.cap;
        size_t r = (size_t)agent * a.cap + s;
        S.slot[tid] = s;
        S.act[tid] = a.ring_a[r];
        DMDQN_DBG(S.act[tid] < NACT, DBG_LEARN_ACT);
#ifdef DMDQN_DEBUG_BOUNDS
        if (S.act[tid] >= NACT) S.act[tid] = 0;
#endif
        S.r64[tid] = a.ring_r[r];
        S.dn[tid] = a.ring_d[r] ? 1.0f : 0.0f;
    }
    __syncthreads();
    // ---- reward z-score (dqn_agent.py:66-69): numpy pairwise sum of 128 f64
    // (8 interleaved accumulators, tree combine), population std, +1e-8.
    if (w == 0) {
        double acc = 0.0;
        if (l < 8) {
            acc = S.r64[l];
            for (int i = 1; i < 16; i++) acc = __dadd_rn(acc, S.r64[8 * i + l]);
            S.red[l] = acc;
        }
    }
    __syncthreads();
    if (tid == 0) {
        double *r = S.red;
        double sum = __dadd_rn(__dadd_rn(__dadd_rn(r[0], r[1]), __dadd_rn(r[2], r[3])),
                               __dadd_rn(__dadd_rn(r[4], r[5]), __dadd_rn(r[6], r[7])));
        sum = __dadd_rn(0.0, sum);
        S.red[8] = __ddiv_rn(sum, 128.0);
    }
    __syncthreads();
    if (w == 0 && l < 8) {
        const double mean = S.red[8];
        double acc = 0.0;
        for (int i = 0; i < 16; i++) {
            double d = __dsub_rn(S.r64[8 * i + l], mean);
            double sq = __dmul_rn(d, d);
            acc = i == 0 ? sq : __dadd_rn(acc, sq);
        }
        S.red[l] = acc;
    }
    __syncthreads();
    if (tid == 0) {
        double *r = S.red;
        double sum = __dadd_rn(__dadd_rn(__dadd_rn(r[0], r[1]), __dadd_rn(r[2], r[3])),
                               __dadd_rn(__dadd_rn(r[4], r[5]), __dadd_rn(r[6], r[7])));
        sum = __dadd_rn(0.0, sum);
        S.red[9] = __dadd_rn(__dsqrt_rn(__ddiv_rn(sum, 128.0)), 1e-8);
    }
    __syncthreads();
    if (tid < B_) {
        double z = __ddiv_rn(__dsub_rn(S.r64[tid], S.red[8]), S.red[9]);
        S.rn[tid] = (float)z;
        if (a.rn_out) a.rn_out[(size_t)agent * B_ + tid] = (float)z;
    }

    // ---- P1: gather S' rows
    auto gather = [&](const int8_t *ring) {
        for (int t = tid; t < B_ * (DP / 4); t += 512) {
            int b = t / (DP / 4), q = t - b * (DP / 4);
            const char4 c = reinterpret_cast<const char4 *>(
                ring + ((size_t)agent * a.cap + S.slot[b]) * DMDQN_ROW_BYTES)[q];
            _Float16 *dst = XL + b * DP + 4 * q;
            dst[0] = (_Float16)(float)c.x;
            dst[1] = (_Float16)(float)c.y;
            dst[2] = (_Float16)(float)c.z;
            dst[3] = (_Float16)(float)c.w;
        }
        __syncthreads();
    };
    const TX *X;
    if constexpr (XF) {
        X = a.xn + (size_t)agent * B_ * DP;
    } else {
        gather(a.ring_n);
        X = XL;
    }
    // ---- P2: target forward on S' -> z3 ; P3: online forward on S' -> a*, y
    forward<H>(a.target + agent * P, X, H1, H2, S.z3);
    // online forward on S': layer 3 reads H2 only, so its Q goes to the H1 region
    forward<H>(Wp, X, H1, H2, H1);
    if (tid < B_) {
        // y = r + (gamma (1 - d)) q_t, each op rounded as TF's (mul_rn: no fma)
        const float *qo = H1 + tid * NACT;
        int best = 0;
        for (int k = 1; k < NACT; k++)
            if (qo[k] > qo[best]) best = k;  // tf.argmax: first max
        float tq = S.z3[tid * NACT + best];
        float gd = a.gamma * (1.0f - S.dn[tid]);
        S.y[tid] = S.rn[tid] + mul_rn(gd, tq);
    }
    __syncthreads();
    // ---- P4/P5: gather S, online forward keeping H1, H2; q, loss, dq
    if constexpr (XF) {
        X = a.xs + (size_t)agent * B_ * DP;
    } else {
        gather(a.ring_s);
        X = XL;
    }
    forward<H>(Wp, X, H1, H2, S.z3);
    if (a.qstats) learn_qstats(a.qstats, agent, S.z3, S.act);
    float lsum = 0.0f;
    if (tid < B_) {
        float q = S.z3[tid * NACT + S.act[tid]];
        float dq;
        loss_term(a.loss_kind, q - S.y[tid], 1.0f / (float)B_, lsum, dq);
        S.dq[tid] = dq;
    }
    // loss: wave reductions then one lane
    if (w < 2) {
        for (int off = 32; off > 0; off >>= 1) lsum += __shfl_xor(lsum, off);
        if (l == 0) S.red[10 + w] = (double)lsum;
    }
    __syncthreads();
    if (tid == 0 && a.loss) a.loss[agent] = (float)(S.red[10] + S.red[11]) / (float)B_;

    // ---- backward
    // dW3[k][a] = sum_b H2[b][k] dq3[b][a] ; db3[a]  (VALU, one thread per element)
    float g3 = 0.0f, gb3 = 0.0f;
    for (int e = tid; e < H * NACT; e += 512) {
        int k = e >> 2, ac = e & 3;
        float s = 0.0f;
        for (int b = 0; b < B_; b++)
            if (S.act[b] == ac) s += H2[b * H + k] * S.dq[b];
        g3 = s;
    }
    if (tid < NACT) {
        float s = 0.0f;
        for (int b = 0; b < B_; b++)
            if (S.act[b] == tid) s += S.dq[b];
        gb3 = s;
    }
    __syncthreads();
    // dZ2 = dq * W3[:, a] masked by ReLU; overwrite H2 in place
    {
        const float *W3T = Wp + L::oW3T;
        for (int e = tid; e < B_ * H; e += 512) {
            int b = e / H, k = e - b * H;
            float h = H2[e];
            H2[e] = h > 0.0f ? S.dq[b] * W3T[S.act[b] * H + k] : 0.0f;
        }
    }
    __syncthreads();
    float gb2 = 0.0f;
    if (tid < H) {
        float s = 0.0f;
        for (int b = 0; b < B_; b++) s += H2[b * H + tid];
        gb2 = s;
    }
    // dW2[j][k] = sum_b H1[b][j] dZ2[b][k]: wave w owns j-tile(s), 8 k-tiles each
    constexpr int NT = H / 16;
    constexpr int QT = (NT + 7) / 8;  // j-tiles per wave
    f32x4 g2[QT][NT];
    {
        const int lr = l & 15, lk = l >> 4;
#pragma unroll
        for (int q = 0; q < QT; q++)
#pragma unroll
            for (int t = 0; t < NT; t++) g2[q][t] = f32x4{0.f, 0.f, 0.f, 0.f};
        for (int jt = w, q = 0; jt < NT; jt += 8, q++) {
            for (int b0 = 0; b0 < B_; b0 += 4) {
                const int b = b0 + lk;
                const float av = H1[b * H + 16 * jt + lr];
#pragma unroll
                for (int t = 0; t < NT; t++) g2[q][t] = mfma4(av, H2[b * H + 16 * t + lr], g2[q][t]);
            }
        }
    }
    // dH1[b][j] = sum_k dZ2[b][k] W2[j][k]: wave w owns batch tile w, all j tiles
    f32x4 d1[NT];
    {
        const int lr = l & 15, lk = l >> 4;
        const float *W2T = Wp + L::oW2T;
#pragma unroll
        for (int t = 0; t < NT; t++) d1[t] = f32x4{0.f, 0.f, 0.f, 0.f};
        for (int k0 = 0; k0 < H; k0 += 4) {
            const int k = k0 + lk;
            const float av = H2[(16 * w + lr) * H + k];
#pragma unroll
            for (int t = 0; t < NT; t++) d1[t] = mfma4(av, W2T[qn_wt(k, 16 * t + lr, H)], d1[t]);
        }
    }
    __syncthreads();  // everyone done reading H1 (dW2) and old W2 (dH1)
    // dZ1 = dH1 masked by ReLU(H1) -> H1 in place
    {
        const int lr = l & 15, lk = l >> 4;
#pragma unroll
        for (int t = 0; t < NT; t++)
#pragma unroll
            for (int j = 0; j < 4; j++) {
                int idx = (16 * w + 4 * lk + j) * H + 16 * t + lr;
                H1[idx] = H1[idx] > 0.0f ? d1[t][j] : 0.0f;
            }
    }
    // Adam on W2 from the dW2 accumulators (old W2 no longer read)
    {
        const int lr = l & 15, lk = l >> 4;
        for (int jt = w, q = 0; jt < NT; jt += 8, q++)
#pragma unroll
            for (int t = 0; t < NT; t++)
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    size_t i = L::oW2T + qn_wt(16 * t + lr, 16 * jt + 4 * lk + j, H);
                    adam_el(Wp, Mp, Vp, Tp, i, g2[q][t][j], AK, sync);
                }
    }
    __syncthreads();
    // db1 and dW1[i][j] = sum_b X[b][i] dZ1[b][j]; wave owns j-tile, 6 i-tiles
    float gb1 = 0.0f;
    if (tid < H) {
        float s = 0.0f;
        for (int b = 0; b < B_; b++) s += H1[b * H + tid];
        gb1 = s;
    }
    {
        const int lr = l & 15, lk = l >> 4;
        constexpr int IT = DP / 16;  // 6 tiles cover i < 96
        for (int jt = w; jt < NT; jt += 8) {
            f32x4 g1[IT];
#pragma unroll
            for (int t = 0; t < IT; t++) g1[t] = f32x4{0.f, 0.f, 0.f, 0.f};
            for (int b0 = 0; b0 < B_; b0 += 4) {
                const int b = b0 + lk;
                const float bv = H1[b * H + 16 * jt + lr];
#pragma unroll
                for (int t = 0; t < IT; t++)
                    g1[t] = mfma4((float)X[b * DP + 16 * t + lr], bv, g1[t]);
            }
#pragma unroll
            for (int t = 0; t < IT; t++)
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    int i = 16 * t + 4 * lk + j;
                    if (i < D_) adam_el(Wp, Mp, Vp, Tp, L::oW1T + qn_w1<H>(16 * jt + lr, i),
                                        g1[t][j], AK, sync);
                }
        }
    }
    // biases and W3
    if (tid < H) {
        adam_el(Wp, Mp, Vp, Tp, L::ob1 + tid, gb1, AK, sync);
        adam_el(Wp, Mp, Vp, Tp, L::ob2 + tid, gb2, AK, sync);
    }
    for (int e = tid; e < H * NACT; e += 512)
        adam_el(Wp, Mp, Vp, Tp, L::oW3T + (size_t)(e & 3) * H + (e >> 2), g3, AK, sync);
    if (tid < NACT) adam_el(Wp, Mp, Vp, Tp, L::ob3 + tid, gb3, AK, sync);
}

// ------------------------------------------------------------------ greedy act
// The online forward of select_action's greedy branch (dqn_agent.py:268-273)
// under the learn's precision policy: PREC 0 f32; 1 / 2 Keras mixed_float16 /
// mixed_bfloat16 (learn_h16.hpp): weights, biases and inputs cast to 16 bits,
// f32 sums, each matmul result rounded, the bias add rounded again, 16-bit
// Q values -- so the argmax (first max) sees the values Keras' would.
template <int PREC>
__device__ __forceinline__ float rq(float x) {
    if constexpr (PREC == 1) return (float)(_Float16)x;
    else if constexpr (PREC == 2) return (float)(__bf16)x;
    else return x;
}

template <int H, int PREC>
__global__ void __launch_bounds__(256) k_q_argmax(const float *params, size_t pstride,
                                                  const float *obs, int32_t *out, float *q_out) {
    using L = Lay<H>;
    __shared__ float x[D_], h1[H], h2[H], q[NACT];
    const int agent = blockIdx.x, tid = threadIdx.x;
    const float *Wp = params + (size_t)agent * pstride;  // pstride 0: one shared net
    for (int i = tid; i < D_; i += blockDim.x) x[i] = rq<PREC>(obs[(size_t)agent * D_ + i]);
    __syncthreads();
    for (int j = tid; j < H; j += blockDim.x) {
        float s = 0.0f;
        for (int i = 0; i < D_; i++) s += x[i] * rq<PREC>(Wp[L::oW1T + qn_w1<H>(j, i)]);
        s = rq<PREC>(rq<PREC>(s) + rq<PREC>(Wp[L::ob1 + j]));
        h1[j] = s > 0.0f ? s : 0.0f;
    }
    __syncthreads();
    for (int k = tid; k < H; k += blockDim.x) {
        float s = 0.0f;
        for (int j = 0; j < H; j++) s += h1[j] * rq<PREC>(Wp[L::oW2T + qn_wt(k, j, H)]);
        s = rq<PREC>(rq<PREC>(s) + rq<PREC>(Wp[L::ob2 + k]));
        h2[k] = s > 0.0f ? s : 0.0f;
    }
    __syncthreads();
    if (tid < NACT) {
        float s = 0.0f;
        for (int k = 0; k < H; k++) s += h2[k] * rq<PREC>(Wp[L::oW3T + tid * H + k]);
        q[tid] = rq<PREC>(rq<PREC>(s) + rq<PREC>(Wp[L::ob3 + tid]));
    }
    __syncthreads();
    if (tid == 0) {
        int best = 0;
        for (int k = 1; k < NACT; k++)
            if (q[k] > q[best]) best = k;
        out[agent] = best;
        if (q_out)
            for (int k = 0; k < NACT; k++) q_out[(size_t)agent * NACT + k] = q[k];
    }
}

int launch_learn_f16(const dmdqn_learn_args *a, hipStream_t s);   // learn_f16.hip
int launch_learn_bf16(const dmdqn_learn_args *a, hipStream_t s);  // learn_bf16.hip
int launch_learn_grad_f16(const dmdqn_learn_args *a, float *grad, hipStream_t s);
int launch_learn_grad_bf16(const dmdqn_learn_args *a, float *grad, hipStream_t s);
int launch_adam_agents_f16(const dmdqn_learn_args *a, const float *grad, hipStream_t s);
int launch_adam_agents_bf16(const dmdqn_learn_args *a, const float *grad, hipStream_t s);

DMDQN_DBG_READER(dbg_flags_learn)

}  // namespace dmdqn

using namespace dmdqn;

static int check_learn_args(const dmdqn_learn_args *a) {
    DMDQN_REQUIRE(a, "dmdqn_learn: null args");
    DMDQN_REQUIRE(a->NA > 0 && a->cap >= a->batch && a->start >= 0 && a->start < a->cap,
                  "dmdqn_learn: NA=%d cap=%d start=%d", a->NA, a->cap, a->start);
    DMDQN_REQUIRE(a->batch == B_, "dmdqn_learn: batch must be %d (got %d)", B_, a->batch);
    DMDQN_REQUIRE(a->row_format == DMDQN_ROWS_I8 || a->row_format == DMDQN_ROWS_F32,
                  "dmdqn_learn: row_format %d", a->row_format);
    DMDQN_REQUIRE((a->row_format == DMDQN_ROWS_F32 ? (a->xs && a->xn) : (a->ring_s && a->ring_n)) &&
                      a->ring_a && a->ring_d && a->ring_r && a->idx && a->params && a->adam_m &&
                      a->adam_v && a->target,
                  "dmdqn_learn: null pointer");
    DMDQN_REQUIRE(a->precision >= 0 && a->precision <= 2, "dmdqn_learn: precision %d",
                  a->precision);
    DMDQN_REQUIRE(a->loss_kind == DMDQN_LOSS_MSE || a->loss_kind == DMDQN_LOSS_HUBER,
                  "dmdqn_learn: loss_kind %d", a->loss_kind);
    return DMDQN_OK;
}

extern "C" int dmdqn_learn(const dmdqn_learn_args *a, void *stream) {
    if (int rc = check_learn_args(a)) return rc;
    if (a->precision == 1) return launch_learn_f16(a, as_stream(stream));
    if (a->precision == 2) return launch_learn_bf16(a, as_stream(stream));
    const bool xf = a->row_format == DMDQN_ROWS_F32;
    if (a->hidden == 128) {
        DMDQN_REQUIRE(a->P == Lay<128>::P, "dmdqn_learn: P=%d != %d", a->P, Lay<128>::P);
        auto k = xf ? k_learn_f32<128, true> : k_learn_f32<128, false>;
        hipLaunchKernelGGL(k, dim3(a->NA), dim3(512), 0, as_stream(stream), *a);
    } else if (a->hidden == 64) {
        DMDQN_REQUIRE(a->P == Lay<64>::P, "dmdqn_learn: P=%d != %d", a->P, Lay<64>::P);
        auto k = xf ? k_learn_f32<64, true> : k_learn_f32<64, false>;
        hipLaunchKernelGGL(k, dim3(a->NA), dim3(512), 0, as_stream(stream), *a);
    } else {
        DMDQN_REQUIRE(false, "dmdqn_learn: hidden must be 64 or 128 (got %d)", a->hidden);
    }
    DMDQN_LAUNCH_CHECK("k_learn");
    return DMDQN_OK;
}

extern "C" int dmdqn_learn_grad(const dmdqn_learn_args *a, float *grad, void *stream) {
    if (int rc = check_learn_args(a)) return rc;
    DMDQN_REQUIRE(grad, "dmdqn_learn_grad: null grad");
    DMDQN_REQUIRE(a->precision == 1 || a->precision == 2,
                  "dmdqn_learn_grad: precision %d (the split learn is fp16 / bf16 only)",
                  a->precision);
    return a->precision == 1 ? launch_learn_grad_f16(a, grad, as_stream(stream))
                             : launch_learn_grad_bf16(a, grad, as_stream(stream));
}

extern "C" int dmdqn_adam_agents(const dmdqn_learn_args *a, const float *grad, void *stream) {
    DMDQN_REQUIRE(a && grad && a->NA > 0 && a->params && a->adam_m && a->adam_v && a->target,
                  "dmdqn_adam_agents: null argument");
    DMDQN_REQUIRE(a->precision == 1 || a->precision == 2,
                  "dmdqn_adam_agents: precision %d (fp16 / bf16 only)", a->precision);
    return a->precision == 1 ? launch_adam_agents_f16(a, grad, as_stream(stream))
                             : launch_adam_agents_bf16(a, grad, as_stream(stream));
}

template <int H>
static void launch_q_argmax(int precision, int NA, const float *params, size_t pstride,
                            const float *obs, int32_t *out, float *q_out, void *stream) {
    auto k = precision == 1 ? k_q_argmax<H, 1> : precision == 2 ? k_q_argmax<H, 2> : k_q_argmax<H, 0>;
    hipLaunchKernelGGL(k, dim3(NA), dim3(H), 0, as_stream(stream), params, pstride, obs, out, q_out);
}

static int q_argmax(const float *params, size_t pstride, int NA, int P, int hidden, int precision,
                    const float *obs, int32_t *out, float *q_out, void *stream) {
    DMDQN_REQUIRE(params && obs && out && NA > 0, "dmdqn_q_argmax: bad args");
    DMDQN_REQUIRE(precision >= 0 && precision <= 2, "dmdqn_q_argmax: precision %d", precision);
    if (hidden == 128) {
        DMDQN_REQUIRE(P == Lay<128>::P, "dmdqn_q_argmax: P");
        launch_q_argmax<128>(precision, NA, params, pstride, obs, out, q_out, stream);
    } else if (hidden == 64) {
        DMDQN_REQUIRE(P == Lay<64>::P, "dmdqn_q_argmax: P");
        launch_q_argmax<64>(precision, NA, params, pstride, obs, out, q_out, stream);
    } else {
        DMDQN_REQUIRE(false, "dmdqn_q_argmax: hidden must be 64 or 128");
    }
    DMDQN_LAUNCH_CHECK("k_q_argmax");
    return DMDQN_OK;
}

extern "C" int dmdqn_q_argmax(const float *params, int NA, int P, int hidden, int precision,
                              const float *obs, int32_t *out, float *q_out, void *stream) {
    return q_argmax(params, (size_t)P, NA, P, hidden, precision, obs, out, q_out, stream);
}

extern "C" int dmdqn_q_argmax_shared(const float *params, int NA, int P, int hidden, int precision,
                                     const float *obs, int32_t *out, float *q_out, void *stream) {
    return q_argmax(params, 0, NA, P, hidden, precision, obs, out, q_out, stream);
}

// Hard target sync outside a learn (dqn_agent.py:382-387, update_target_network):
// target <- params for NW nets, and the 16-bit shadow the target forward reads
// (RNE; f16 or bf16) when target_h is given.
template <typename T16>
__global__ void __launch_bounds__(256) k_target_sync(const float *params, float *target,
                                                     T16 *target_h, int P, int Ph, long n) {
    const long i = (long)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const long w = i / P, k = i - w * P;
    const float x = params[i];
    target[i] = x;
    if (target_h) target_h[w * Ph + k] = (T16)x;
}

extern "C" int dmdqn_target_sync(const float *params, float *target, uint16_t *target_h, int NW,
                                 int P, int Ph, int precision, void *stream) {
    DMDQN_REQUIRE(params && target && NW > 0 && P > 0 && Ph >= P,
                  "dmdqn_target_sync: NW=%d P=%d Ph=%d", NW, P, Ph);
    DMDQN_REQUIRE(precision >= 0 && precision <= 2, "dmdqn_target_sync: precision %d", precision);
    DMDQN_REQUIRE(!target_h || precision != 0, "dmdqn_target_sync: fp32 has no 16-bit shadow");
    const long n = (long)NW * P;
    const dim3 grid((unsigned)((n + 255) / 256));
    if (precision == 2)
        hipLaunchKernelGGL(k_target_sync<__bf16>, grid, dim3(256), 0, as_stream(stream), params,
                           target, reinterpret_cast<__bf16 *>(target_h), P, Ph, n);
    else
        hipLaunchKernelGGL(k_target_sync<_Float16>, grid, dim3(256), 0, as_stream(stream), params,
                           target, reinterpret_cast<_Float16 *>(target_h), P, Ph, n);
    DMDQN_LAUNCH_CHECK("k_target_sync");
    return DMDQN_OK;
}
