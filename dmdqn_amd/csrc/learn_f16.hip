// learn_f16.hip -- fused Double-DQN learn step, mixed precision (the reference's
// tf.keras mixed_float16 policy, train.py:61): f16 operands on the MFMA
// (v_mfma_f32_16x16x32_f16, f32 accumulate), f32 master weights + Adam slots.
// One workgroup (8 waves) per agent, everything between the replay gather and
// the Adam update stays in LDS.
//
// GEMM orientation (C[M][N] = sum_k A[M][k] B[k][N], 16x16x32 fragments):
//   forward  Z^T[n][b] = W^T[n][k] . X[b][k]   A: W^T image rows, B: X rows
//            -> each lane holds 4 consecutive neurons of one batch row, stored
//               as one 8-byte write into the [b][n] activation image
//   dW3      C[k][a] = H2^T . DQ               (batch reduction: transposed reads)
//   dW2      C[j][k] = H1^T . dZ2              (transposed reads)
//   dH1^T    C[j][b] = W2 . dZ2^T              A: transposed read of W2^T image
//   dW1      C[i][j] = X^T . dZ1               (transposed reads)
// Gradient tiles come out in Keras [in][out] order: Adam runs straight from
// the accumulators with 64-byte contiguous row segments per 16 lanes.
//
// LDS (bytes): X f16[128][96] | W1T f16[128][96] | W2T f16[128][128] |
//   W3T f16[16][128] | H1 f16[128][128] | H2 f16[128][128] | biases f32 |
//   DQ f16[128][16] | scratch        = 162,976 B (1 workgroup / CU)
#include <math.h>

#include "common.hpp"

namespace dmdqn {
namespace f16k {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef _Float16 half4v __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short v4s __attribute__((vector_size(8)));
typedef __attribute__((address_space(3))) v4s lds_v4s;

constexpr int B_ = 128, D_ = 89, DP = 96, H = 128, NACT = 4;
constexpr int P = D_ * H + H + H * H + H + H * NACT + NACT;
constexpr int oW1 = 0, ob1 = D_ * H, oW2 = ob1 + H, ob2 = oW2 + H * H, oW3 = ob2 + H,
              ob3 = oW3 + H * NACT;

// LDS byte offsets
constexpr int X_OFF = 0;
constexpr int W1T_OFF = X_OFF + B_ * DP * 2;
constexpr int W2T_OFF = W1T_OFF + H * DP * 2;
constexpr int W3T_OFF = W2T_OFF + H * H * 2;
constexpr int H1_OFF = W3T_OFF + 16 * H * 2;
constexpr int H2_OFF = H1_OFF + B_ * H * 2;
constexpr int BIAS_OFF = H2_OFF + B_ * H * 2;       // b1[128] b2[128] b3[8] f32
constexpr int DQ_OFF = BIAS_OFF + (2 * H + 8) * 4;  // f16 [128][16]
constexpr int SC_OFF = DQ_OFF + B_ * 16 * 2;
constexpr int LDS_BYTES = SC_OFF + 6272;
static_assert(LDS_BYTES <= 163840, "LDS budget");

__device__ __forceinline__ f32x4 mfma(half8 a, half8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

// img[r0 + (l&15)][k0 + 8(l>>4) + e], e = 0..7: one 16-byte LDS read.
__device__ __forceinline__ half8 frag_row(const _Float16 *img, int ld, int r0, int k0) {
    const int l = threadIdx.x & 63;
    return *reinterpret_cast<const half8 *>(img + (r0 + (l & 15)) * ld + k0 + 8 * (l >> 4));
}

// img[r0 + 8(l>>4) + e][c0 + (l&15)], e = 0..7: two ds_read_b64_tr_b16.
// Lane 4q+p of each 16-lane group addresses row q, columns 4p..4p+3 of a
// 4-row block; lane i receives column i of the block (row q -> element q).
__device__ __forceinline__ half8 frag_tr(const _Float16 *img, int ld, int r0, int c0) {
    const int l = threadIdx.x & 63, i = l & 15, g = l >> 4;
    const _Float16 *p0 = img + (r0 + 8 * g + (i >> 2)) * ld + c0 + 4 * (i & 3);
    v4s t0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s *)p0);
    v4s t1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s *)(p0 + 4 * ld));
    half8 r;
#pragma unroll
    for (int e = 0; e < 4; e++) {
        r[e] = __builtin_bit_cast(_Float16, (short)t0[e]);
        r[e + 4] = __builtin_bit_cast(_Float16, (short)t1[e]);
    }
    return r;
}

struct Scratch {
    float *z3;    // [128][4]
    float *rn, *y, *dq, *dn;
    int *act, *slot;
    double *r64, *red;
};

// Forward of one 128-row batch: H1/H2 f16 images (post-ReLU), Q -> z3 (f32).
__device__ void forward(const _Float16 *X, const _Float16 *W1T, const _Float16 *W2T,
                        const _Float16 *W3T, const float *bias, _Float16 *H1, _Float16 *H2,
                        float *z3) {
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63, lr = l & 15, lg = l >> 4;
    const int n0 = 16 * w;  // this wave's 16 neurons
    // layer 1: K = 96 (3 k-steps)
    {
        f32x4 acc[8];
#pragma unroll
        for (int t = 0; t < 8; t++) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k0 = 0; k0 < DP; k0 += 32) {
            half8 a = frag_row(W1T, DP, n0, k0);
#pragma unroll
            for (int t = 0; t < 8; t++) acc[t] = mfma(a, frag_row(X, DP, 16 * t, k0), acc[t]);
        }
        const int n = n0 + 4 * lg;
#pragma unroll
        for (int t = 0; t < 8; t++) {
            half4v hv;
#pragma unroll
            for (int e = 0; e < 4; e++) {
                float z = acc[t][e] + bias[n + e];
                hv[e] = (_Float16)(z > 0.0f ? z : 0.0f);
            }
            *reinterpret_cast<half4v *>(H1 + (16 * t + lr) * H + n) = hv;
        }
    }
    __syncthreads();
    // layer 2: K = 128 (4 k-steps)
    {
        f32x4 acc[8];
#pragma unroll
        for (int t = 0; t < 8; t++) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k0 = 0; k0 < H; k0 += 32) {
            half8 a = frag_row(W2T, H, n0, k0);
#pragma unroll
            for (int t = 0; t < 8; t++) acc[t] = mfma(a, frag_row(H1, H, 16 * t, k0), acc[t]);
        }
        const int n = n0 + 4 * lg;
#pragma unroll
        for (int t = 0; t < 8; t++) {
            half4v hv;
#pragma unroll
            for (int e = 0; e < 4; e++) {
                float z = acc[t][e] + bias[H + n + e];
                hv[e] = (_Float16)(z > 0.0f ? z : 0.0f);
            }
            *reinterpret_cast<half4v *>(H2 + (16 * t + lr) * H + n) = hv;
        }
    }
    __syncthreads();
    // layer 3: Q^T[a][b], wave w -> batch tile w
    {
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k0 = 0; k0 < H; k0 += 32) acc = mfma(frag_row(W3T, H, 0, k0), frag_row(H2, H, 16 * w, k0), acc);
        if (lg == 0) {
            // (keras mixed_float16: the last Dense also outputs f16)
#pragma unroll
            for (int e = 0; e < 4; e++)
                z3[(16 * w + lr) * NACT + e] = (float)(_Float16)(acc[e] + bias[2 * H + e]);
        }
    }
    __syncthreads();
}

// Stage one network (fp32, Keras layout in global memory) into the f16 LDS
// images W1T[n][k], W2T[n][j], W3T[a][k] and the f32 biases.
__device__ void stage(const float *Wg, _Float16 *W1T, _Float16 *W2T, _Float16 *W3T, float *bias) {
    const int tid = threadIdx.x;
    // lanes of a wave: 16 consecutive k-quads x 4 neurons -> 8-byte LDS writes
    for (int t = tid; t < H * (DP / 4); t += 512) {   // W1T: 128 n x 24 k-quads
        int n = t / (DP / 4), kq = t - n * (DP / 4);
        half4v hv;
#pragma unroll
        for (int c = 0; c < 4; c++) {
            int k = 4 * kq + c;
            hv[c] = k < D_ ? (_Float16)Wg[oW1 + k * H + n] : (_Float16)0.0f;
        }
        *reinterpret_cast<half4v *>(W1T + n * DP + 4 * kq) = hv;
    }
    for (int t = tid; t < H * (H / 4); t += 512) {    // W2T: 128 n x 32 j-quads
        int n = t / (H / 4), jq = t - n * (H / 4);
        half4v hv;
#pragma unroll
        for (int c = 0; c < 4; c++) hv[c] = (_Float16)Wg[oW2 + (4 * jq + c) * H + n];
        *reinterpret_cast<half4v *>(W2T + n * H + 4 * jq) = hv;
    }
    for (int t = tid; t < 16 * H; t += 512) {         // W3T: 16 a (4 used) x 128 k
        int a = t / H, k = t - a * H;
        W3T[t] = a < NACT ? (_Float16)Wg[oW3 + k * NACT + a] : (_Float16)0.0f;
    }
    for (int t = tid; t < 2 * H + 8; t += 512)
        bias[t] = t < H ? Wg[ob1 + t] : t < 2 * H ? Wg[ob2 + t - H] : (t < 2 * H + NACT ? Wg[ob3 + t - 2 * H] : 0.0f);
    __syncthreads();
}

__device__ __forceinline__ void adam_el(float *w, float *m, float *v, float *tgt, size_t i, float g,
                                        float alpha, float c1, float c2, float eps, bool sync) {
    float mi = m[i], vi = v[i], wi = w[i];
    mi = mi + (g - mi) * c1;
    vi = vi + (g * g - vi) * c2;
    wi = wi - (mi * alpha) / (sqrtf(vi) + eps);
    m[i] = mi;
    v[i] = vi;
    w[i] = wi;
    if (sync) tgt[i] = wi;
}

__global__ void __launch_bounds__(512) k_learn_f16(dmdqn_learn_args a) {
    __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];
    _Float16 *X = (_Float16 *)(smem + X_OFF), *W1T = (_Float16 *)(smem + W1T_OFF);
    _Float16 *W2T = (_Float16 *)(smem + W2T_OFF), *W3T = (_Float16 *)(smem + W3T_OFF);
    _Float16 *H1 = (_Float16 *)(smem + H1_OFF), *H2 = (_Float16 *)(smem + H2_OFF);
    float *bias = (float *)(smem + BIAS_OFF);
    _Float16 *DQ = (_Float16 *)(smem + DQ_OFF);
    char *sc = smem + SC_OFF;
    Scratch S{(float *)sc,         (float *)(sc + 2048), (float *)(sc + 2560),
              (float *)(sc + 3072), (float *)(sc + 3584), (int *)(sc + 4096),
              (int *)(sc + 4608),   (double *)(sc + 5120), (double *)(sc + 6144)};
    const int agent = blockIdx.x;
    const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, lr = l & 15, lg = l >> 4;
    const size_t Pz = (size_t)P;
    float *Wp = a.params + agent * Pz, *Mp = a.adam_m + agent * Pz, *Vp = a.adam_v + agent * Pz;
    float *Tp = a.target + agent * Pz;
    const bool sync = a.sync_target != 0;
    const float alpha = a.alpha, c1 = a.c1, c2 = a.c2, eps = a.eps;

    // ---- batch metadata + reward z-score (numpy pairwise order, f64)
    if (tid < B_) {
        int pos = a.idx[(size_t)agent * B_ + tid];
        int s = a.start + pos;
        if (s >= a.cap) s -= a.cap;
        size_t r = (size_t)agent * a.cap + s;
        S.slot[tid] = s;
        S.act[tid] = a.ring_a[r];
        S.r64[tid] = a.ring_r[r];
        S.dn[tid] = a.ring_d[r] ? 1.0f : 0.0f;
    }
    __syncthreads();
    if (tid < 8) {
        double acc = S.r64[tid];
        for (int i = 1; i < 16; i++) acc = __dadd_rn(acc, S.r64[8 * i + tid]);
        S.red[tid] = acc;
    }
    __syncthreads();
    if (tid == 0) {
        double *r = S.red;
        double sum = __dadd_rn(__dadd_rn(__dadd_rn(r[0], r[1]), __dadd_rn(r[2], r[3])),
                               __dadd_rn(__dadd_rn(r[4], r[5]), __dadd_rn(r[6], r[7])));
        S.red[8] = __ddiv_rn(__dadd_rn(0.0, sum), 128.0);
    }
    __syncthreads();
    if (tid < 8) {
        const double mean = S.red[8];
        double acc = 0.0;
        for (int i = 0; i < 16; i++) {
            double d = __dsub_rn(S.r64[8 * i + tid], mean);
            double sq = __dmul_rn(d, d);
            acc = i == 0 ? sq : __dadd_rn(acc, sq);
        }
        S.red[tid] = acc;
    }
    __syncthreads();
    if (tid == 0) {
        double *r = S.red;
        double sum = __dadd_rn(__dadd_rn(__dadd_rn(r[0], r[1]), __dadd_rn(r[2], r[3])),
                               __dadd_rn(__dadd_rn(r[4], r[5]), __dadd_rn(r[6], r[7])));
        S.red[9] = __dadd_rn(__dsqrt_rn(__ddiv_rn(__dadd_rn(0.0, sum), 128.0)), 1e-8);
    }
    __syncthreads();
    if (tid < B_) S.rn[tid] = (float)__ddiv_rn(__dsub_rn(S.r64[tid], S.red[8]), S.red[9]);

    auto gather = [&](const int8_t *ring) {
        for (int t = tid; t < B_ * (DP / 4); t += 512) {
            int b = t / (DP / 4), q = t - b * (DP / 4);
            const char4 c = reinterpret_cast<const char4 *>(
                ring + ((size_t)agent * a.cap + S.slot[b]) * DP)[q];
            half4v hv;
            hv[0] = (_Float16)(float)c.x;
            hv[1] = (_Float16)(float)c.y;
            hv[2] = (_Float16)(float)c.z;
            hv[3] = (_Float16)(float)c.w;
            *reinterpret_cast<half4v *>(X + b * DP + 4 * q) = hv;
        }
    };

    // ---- target(S') then online(S') -> a*, y
    gather(a.ring_n);
    stage(a.target + agent * Pz, W1T, W2T, W3T, bias);
    forward(X, W1T, W2T, W3T, bias, H1, H2, S.z3);
    stage(Wp, W1T, W2T, W3T, bias);
    float *qo = (float *)H1;  // H1 is free while layer 3 runs
    forward(X, W1T, W2T, W3T, bias, H1, H2, qo);
    if (tid < B_) {
        int best = 0;
        for (int k = 1; k < NACT; k++)
            if (qo[tid * NACT + k] > qo[tid * NACT + best]) best = k;
        float tq = S.z3[tid * NACT + best];
        float gd = a.gamma * (1.0f - S.dn[tid]);
        S.y[tid] = S.rn[tid] + gd * tq;
    }
    __syncthreads();
    // ---- online(S) with activations kept; q, loss, dq
    gather(a.ring_s);
    __syncthreads();
    forward(X, W1T, W2T, W3T, bias, H1, H2, S.z3);
    float lsum = 0.0f;
    if (tid < B_) {
        float q = S.z3[tid * NACT + S.act[tid]];
        float diff = q - S.y[tid];
        float dq = 2.0f * diff / (float)B_;
        S.dq[tid] = dq;
        lsum = diff * diff;
        half8 z = {0, 0, 0, 0, 0, 0, 0, 0};
        *reinterpret_cast<half8 *>(DQ + tid * 16) = z;
        *reinterpret_cast<half8 *>(DQ + tid * 16 + 8) = z;
        DQ[tid * 16 + S.act[tid]] = (_Float16)dq;
    }
    if (w < 2) {
        for (int off = 32; off > 0; off >>= 1) lsum += __shfl_xor(lsum, off);
        if (l == 0) S.red[10 + w] = (double)lsum;
    }
    __syncthreads();
    if (tid == 0 && a.loss) a.loss[agent] = (float)(S.red[10] + S.red[11]) / (float)B_;

    // ---- dW3[k][a] = H2^T . DQ  (wave w: k-tile w) ; db3
    {
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int b0 = 0; b0 < B_; b0 += 32)
            acc = mfma(frag_tr(H2, H, b0, 16 * w), frag_tr(DQ, 16, b0, 0), acc);
        if (lr < NACT) {
#pragma unroll
            for (int e = 0; e < 4; e++)
                adam_el(Wp, Mp, Vp, Tp, oW3 + (size_t)(16 * w + 4 * lg + e) * NACT + lr, acc[e],
                        alpha, c1, c2, eps, sync);
        }
    }
    if (tid < NACT) {
        float s = 0.0f;
        for (int b = 0; b < B_; b++) s += (float)DQ[b * 16 + tid];
        adam_el(Wp, Mp, Vp, Tp, ob3 + tid, s, alpha, c1, c2, eps, sync);
    }
    __syncthreads();
    // ---- dZ2 = dq * W3[:, a] (ReLU mask), in place over H2
    for (int e = tid; e < B_ * H; e += 512) {
        int b = e >> 7, k = e & (H - 1);
        float h = (float)H2[e];
        float g = (float)DQ[b * 16 + S.act[b]] * (float)W3T[S.act[b] * H + k];
        H2[e] = (_Float16)(h > 0.0f ? g : 0.0f);
    }
    __syncthreads();
    float gb2 = 0.0f;
    if (tid < H) {
        for (int b = 0; b < B_; b++) gb2 += (float)H2[b * H + tid];
    }
    // ---- dW2[j][k] = H1^T . dZ2   (wave w: j-tile w, 8 k-tiles)
    f32x4 g2[8];
#pragma unroll
    for (int t = 0; t < 8; t++) g2[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int b0 = 0; b0 < B_; b0 += 32) {
        half8 av = frag_tr(H1, H, b0, 16 * w);
#pragma unroll
        for (int t = 0; t < 8; t++) g2[t] = mfma(av, frag_tr(H2, H, b0, 16 * t), g2[t]);
    }
    // ---- dH1^T[j][b] = W2[j][k] . dZ2^T  (A: transposed read of the W2T image)
    f32x4 d1[8];
#pragma unroll
    for (int t = 0; t < 8; t++) d1[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k0 = 0; k0 < H; k0 += 32) {
        half8 av = frag_tr(W2T, H, k0, 16 * w);
#pragma unroll
        for (int t = 0; t < 8; t++) d1[t] = mfma(av, frag_row(H2, H, 16 * t, k0), d1[t]);
    }
    __syncthreads();  // all reads of H1 (dW2) done
    // dZ1 = dH1 masked by ReLU(H1): lane holds neurons j..j+3 of batch row b
    {
        const int j = 16 * w + 4 * lg;
#pragma unroll
        for (int t = 0; t < 8; t++) {
            half4v *p = reinterpret_cast<half4v *>(H1 + (16 * t + lr) * H + j);
            half4v h = *p, o;
#pragma unroll
            for (int e = 0; e < 4; e++) o[e] = (float)h[e] > 0.0f ? (_Float16)d1[t][e] : (_Float16)0.0f;
            *p = o;
        }
    }
    // Adam on W2 (rows j = 16w + 4lg + e, cols k = 16t + lr) and b2
#pragma unroll
    for (int t = 0; t < 8; t++)
#pragma unroll
        for (int e = 0; e < 4; e++)
            adam_el(Wp, Mp, Vp, Tp, oW2 + (size_t)(16 * w + 4 * lg + e) * H + 16 * t + lr, g2[t][e],
                    alpha, c1, c2, eps, sync);
    if (tid < H) adam_el(Wp, Mp, Vp, Tp, ob2 + tid, gb2, alpha, c1, c2, eps, sync);
    __syncthreads();
    // ---- db1 ; dW1[i][j] = X^T . dZ1  (wave w: j-tile w, 6 i-tiles)
    if (tid < H) {
        float s = 0.0f;
        for (int b = 0; b < B_; b++) s += (float)H1[b * H + tid];
        adam_el(Wp, Mp, Vp, Tp, ob1 + tid, s, alpha, c1, c2, eps, sync);
    }
    {
        f32x4 g1[6];
#pragma unroll
        for (int t = 0; t < 6; t++) g1[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int b0 = 0; b0 < B_; b0 += 32) {
            half8 bv = frag_tr(H1, H, b0, 16 * w);
#pragma unroll
            for (int t = 0; t < 6; t++) g1[t] = mfma(frag_tr(X, DP, b0, 16 * t), bv, g1[t]);
        }
#pragma unroll
        for (int t = 0; t < 6; t++)
#pragma unroll
            for (int e = 0; e < 4; e++) {
                int i = 16 * t + 4 * lg + e;
                if (i < D_)
                    adam_el(Wp, Mp, Vp, Tp, oW1 + (size_t)i * H + 16 * w + lr, g1[t][e], alpha, c1,
                            c2, eps, sync);
            }
    }
}

}  // namespace f16k

int launch_learn_f16(const dmdqn_learn_args *a, hipStream_t s) {
    DMDQN_REQUIRE(a->hidden == 128 && a->P == f16k::P,
                  "dmdqn_learn: precision 1 (fp16) needs hidden=128 (P=%d)", f16k::P);
    hipLaunchKernelGGL(f16k::k_learn_f16, dim3(a->NA), dim3(512), 0, s, *a);
    DMDQN_LAUNCH_CHECK("k_learn_f16");
    return DMDQN_OK;
}

}  // namespace dmdqn
