// learn_f16.hip -- the f16 instantiation of learn_h16.hpp (the reference's
// tf.keras mixed_float16 policy, train.py:61: f16 MFMA operands, f32
// accumulate, f32 master weights + Adam), plus the shared-parameter learn
// (configuration C5) and the flat Keras-3 Adam it is followed by.
#define DMDQN_H16_BF16 0
#include "learn_h16.hpp"

namespace dmdqn {
namespace f16k {

// ----------------------------------------------------------------------------
// Shared-parameter DQN (not in the reference): ONE online /
// target network for every agent.  Persistent workgroups (one per CU, 256
// VGPRs) hold both networks' fragments in registers for the whole launch and
// loop over agents; each agent's batch runs the same forward/backward as the
// independent kernel, and its gradient tiles accumulate straight into MFMA
// accumulators that live across the agent loop.  Each workgroup then writes
// its partial sum (kernel layout, P floats) to slab[blockIdx.x].  No Adam
// here: k_reduce_slabs + (RCCL all-reduce across ranks) + k_adam follow.
template <bool QSTATS>
__global__ void __launch_bounds__(512, 2) k_learn_shared_f16(dmdqn_learn_args a, float *slab) {
    LEARN_SMEM_SETUP;
    const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, lr = l & 15, lg = l >> 4;
    const float *Wp = a.params;
    const _Float16 *TH = a.target_h ? reinterpret_cast<const _Float16 *>(a.target_h) : nullptr;
    const _Float16 *WH = reinterpret_cast<const _Float16 *>(a.params_h);
    Frags fr;
    stage_out(Wp, W3L, B3L);
    if (TH) stage_out(TH, W3L + NACT * H, B3L + NACT);
    else stage_out(a.target, W3L + NACT * H, B3L + NACT);
    const half8 ones = ones8();
    // dW2 accumulators (64 KB f32) live in LDS -- one workgroup per CU leaves
    // room -- laid out [wave][tile][lane] so each access is one contiguous
    // 1 KB wave row; the rest stay in registers.
    __shared__ f32x4 G2L[8 * 8 * 64];
    f32x4 G3 = {0.f, 0.f, 0.f, 0.f}, GB3 = G3, GB2 = G3, GB1 = G3, G1[6];
#pragma unroll
    for (int t = 0; t < 8; t++) G2L[(w * 8 + t) * 64 + l] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 6; t++) G1[t] = f32x4{0.f, 0.f, 0.f, 0.f};

    for (int agent = blockIdx.x; agent < a.NA; agent += gridDim.x) {
        // the shared nets are L2-resident: reload the fragments per agent (as
        // the independent kernel does from HBM) rather than pin 72 VGPRs
        if (TH) load_frags(TH, fr);
        else load_frags(a.target, fr);
        batch_head(a, agent, R2, S);  // X(S') in R2, metadata, z-score
        // buffer plan of k_learn_f16: the backward runs on (P1, P2) = (R2, R1)
        forward_x<true>(fr, tg, R2, R1, R1, S.z3, [WH](Frags &f) { load_w1(WH, f); },
                        [WH](Frags &f) { load_w2(WH, f); });  // X(S') stays in R2
        float *qo = (float *)DQ;
        Rows gs;
        forward_x<false>(fr, on, R2, R1, R2, qo,
                         [&](Frags &) { gather_issue(a.ring_s, a, agent, S.slot, gs); }, NoHook{},
                         [&]() { gather_commit(R1, gs); });
        ddqn_target(a, qo, S);
        forward_x<false>(fr, on, R1, R2, R1, S.z3);
        _Float16 *const P1 = R2, *const P2 = R1;
        loss_dq<QSTATS>(a, agent, DQ, S);
        // dW3 / db3
#pragma unroll
        for (int b0 = 0; b0 < B_; b0 += 32) {
            const half8 dqf = frag_tr(DQ, 16, b0, 0);
            G3 = mfma(frag_tr_h(P2, b0, 16 * w), dqf, G3);
            GB3 = mfma(ones, dqf, GB3);
        }
        __syncthreads();
        bwd_dz2(P2, on, S);
        h1_mask(P1, mask);
        // dW2 / db2 (tile by tile, accumulating into the LDS accumulators)
        {
            half8 av[4];
#pragma unroll
            for (int q = 0; q < 4; q++) {
                av[q] = frag_tr_h(P1, 32 * q, 16 * w);
                GB2 = mfma(ones, frag_tr_h(P2, 32 * q, 16 * w), GB2);
            }
#pragma unroll
            for (int t = 0; t < 8; t++) {
                f32x4 c = G2L[(w * 8 + t) * 64 + l];
#pragma unroll
                for (int q = 0; q < 4; q++) c = mfma(av[q], frag_tr_h(P2, 32 * q, 16 * t), c);
                G2L[(w * 8 + t) * 64 + l] = c;
            }
        }
        __syncthreads();
        f32x4 d1[8];
        bwd_dh1(P1, P2, fr, d1);
        {
            Rows gx;
            gather_issue(a.ring_s, a, agent, S.slot, gx);
            gather_commit(P2, gx);
        }
        bwd_dz1(P1, mask, d1);
        __syncthreads();
        // dW1 / db1
#pragma unroll
        for (int b0 = 0; b0 < B_; b0 += 32) {
            const half8 bv = frag_tr_h(P1, b0, 16 * w);
            GB1 = mfma(ones, bv, GB1);
#pragma unroll
            for (int t = 0; t < 6; t++) G1[t] = mfma(frag_tr_h<DP>(P2, b0, 16 * t), bv, G1[t]);
        }
        __syncthreads();  // P1 / P2 / scratch are rewritten by the next agent
    }
    // partial sums of this workgroup, kernel layout (every index written once)
    float *G = slab + (size_t)blockIdx.x * L::P;
    if (lr < NACT) {
        *reinterpret_cast<float4 *>(G + L::oW3T + lr * H + 16 * w + 4 * lg) =
            make_float4(G3[0], G3[1], G3[2], G3[3]);
        if (w == 0 && lg == 0) G[L::ob3 + lr] = GB3[0];
    }
#pragma unroll
    for (int t = 0; t < 8; t++) {
        const f32x4 c = G2L[(w * 8 + t) * 64 + l];
        *reinterpret_cast<float4 *>(G + L::oW2T + qn_wt(16 * t + lr, 16 * w + 4 * lg, H)) =
            make_float4(c[0], c[1], c[2], c[3]);
    }
    if (lg == 0) G[L::ob2 + 16 * w + lr] = GB2[0];
#pragma unroll
    for (int t = 0; t < 6; t++)
        if (t < 5 || lg < 2)  // tile 5: features 80..87 (89..95 do not exist)
            *reinterpret_cast<float4 *>(G + L::oW1T + qn_w1<H>(16 * w + lr, 16 * t + 4 * lg)) =
                make_float4(G1[t][0], G1[t][1], G1[t][2], G1[t][3]);
    if (lg == 0) G[L::ob1 + 16 * w + lr] = GB1[0];
    if (lg == 2) G[L::oW1X + 16 * w + lr] = G1[5][0];  // feature 88
}

// grad[i] = scale * sum_w slab[w][i] in a fixed order: wave v of a block sums
// slabs v, v + 8, v + 16, ... for 64 float4 columns, then the 8 partials are
// added in wave order.  (One thread per column walking all 256 slabs kept
// only 28 CUs busy on a chain of dependent loads: 72 us.)
__global__ void __launch_bounds__(512) k_reduce_slabs(const float *slab, int nw, float scale,
                                                      float *grad) {
    __shared__ float4 part[8][64];
    const int wv = threadIdx.x >> 6, l = threadIdx.x & 63;
    const int c = blockIdx.x * 64 + l;  // float4 column
    constexpr int NC = L::P / 4;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    if (c < NC) {
        const float4 *s4 = reinterpret_cast<const float4 *>(slab);
#pragma unroll 4
        for (int k = wv; k < nw; k += 8) {
            const float4 v = s4[(size_t)k * NC + c];
            acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
        }
    }
    part[wv][l] = acc;
    __syncthreads();
    if (wv == 0 && c < NC) {
        float4 t = part[0][l];
#pragma unroll
        for (int q = 1; q < 8; q++) {
            const float4 v = part[q][l];
            t.x += v.x; t.y += v.y; t.z += v.z; t.w += v.w;
        }
        t.x *= scale; t.y *= scale; t.z *= scale; t.w *= scale;
        reinterpret_cast<float4 *>(grad)[c] = t;
    }
}

}  // namespace f16k

// Keras-3 Adam over n flat parameters (A-11) with g = gscale * grad; on a
// target sync also writes the target copy and its f16 shadow.
__global__ void __launch_bounds__(256) k_adam(float *W, float *M, float *V, float *T,
                                              _Float16 *TH, _Float16 *WH, const float *G, int n,
                                              float gscale,
                                              float alpha, float c1, float c2, float eps, int sync) {
#pragma clang fp contract(off)  // each op rounded as TF's separate kernels
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const float g = G[i] * gscale;
    float m = M[i], v = V[i], w = W[i];
    m = m + (g - m) * c1;
    v = v + (g * g - v) * c2;
    w = w - (m * alpha) / (sqrtf(v) + eps);
    M[i] = m;
    V[i] = v;
    W[i] = w;
    if (WH) WH[i] = (_Float16)w;
    if (sync) {
        T[i] = w;
        if (TH) TH[i] = (_Float16)w;
    }
}


}  // namespace dmdqn

using namespace dmdqn;

namespace dmdqn {
int launch_shared_v2(const dmdqn_learn_args *a, float *y, uint8_t *act, float *slab, int n_slabs,
                     hipStream_t s);  // learn_shared.hip
}

extern "C" size_t dmdqn_learn_shared_work_bytes(int NA) {
    return NA > 0 ? (size_t)NA * f16k::B_ * (sizeof(float) + 1) : 0;
}

extern "C" int dmdqn_learn_shared_grad(const dmdqn_learn_args *a, float *slab, int n_slabs,
                                       float *grad, float scale, void *work, void *stream) {
    DMDQN_REQUIRE(a && slab && grad, "dmdqn_learn_shared_grad: null argument");
    DMDQN_REQUIRE(a->row_format == DMDQN_ROWS_I8, "dmdqn_learn_shared_grad: int8 replay rows only");
    DMDQN_REQUIRE(a->NA > 0 && a->cap >= a->batch && a->start >= 0 && a->start < a->cap,
                  "dmdqn_learn_shared_grad: NA=%d cap=%d start=%d", a->NA, a->cap, a->start);
    DMDQN_REQUIRE(a->batch == f16k::B_, "dmdqn_learn_shared_grad: batch must be %d", f16k::B_);
    DMDQN_REQUIRE(a->precision == 1 && a->hidden == 128 && a->P == f16k::L::P,
                  "dmdqn_learn_shared_grad: fp16 precision with hidden=128 (P=%d) only",
                  f16k::L::P);
    DMDQN_REQUIRE(a->ring_s && a->ring_n && a->ring_a && a->ring_d && a->ring_r && a->idx &&
                      a->params && a->target && a->params_h,
                  "dmdqn_learn_shared_grad: null array");
    DMDQN_REQUIRE(n_slabs >= 1, "dmdqn_learn_shared_grad: n_slabs must be >= 1");
    DMDQN_REQUIRE(a->loss_kind == DMDQN_LOSS_MSE || a->loss_kind == DMDQN_LOSS_HUBER,
                  "dmdqn_learn_shared_grad: loss_kind %d", a->loss_kind);
    DMDQN_REQUIRE(a->target_h, "dmdqn_learn_shared_grad: target_h (the f16 target) required");
    hipStream_t s = as_stream(stream);
    const char *v1 = getenv("DMDQN_SHARED_V1");  // A/B against the one-pass kernel
    if (work && !(v1 && v1[0] == '1')) {
        float *y = reinterpret_cast<float *>(work);
        uint8_t *act = reinterpret_cast<uint8_t *>(y + (size_t)a->NA * f16k::B_);
        int rc = launch_shared_v2(a, y, act, slab, n_slabs, s);
        if (rc) return rc;
    } else if (a->qstats) {
        hipLaunchKernelGGL(f16k::k_learn_shared_f16<true>, dim3(n_slabs), dim3(512), 0, s, *a, slab);
        DMDQN_LAUNCH_CHECK("k_learn_shared_f16");
    } else {
        hipLaunchKernelGGL(f16k::k_learn_shared_f16<false>, dim3(n_slabs), dim3(512), 0, s, *a,
                           slab);
        DMDQN_LAUNCH_CHECK("k_learn_shared_f16");
    }
    hipLaunchKernelGGL(f16k::k_reduce_slabs, dim3((f16k::L::P / 4 + 63) / 64), dim3(512), 0, s,
                       slab, n_slabs, scale, grad);
    DMDQN_LAUNCH_CHECK("k_reduce_slabs");
    return DMDQN_OK;
}

extern "C" int dmdqn_adam(float *params, float *adam_m, float *adam_v, float *target,
                          uint16_t *target_h, uint16_t *params_h, const float *grad, int n,
                          float gscale, float alpha, float c1, float c2, float eps, int sync,
                          void *stream) {
    DMDQN_REQUIRE(params && adam_m && adam_v && grad && n > 0, "dmdqn_adam: bad args");
    DMDQN_REQUIRE(!sync || target, "dmdqn_adam: target required on a sync");
    hipLaunchKernelGGL(k_adam, dim3((n + 255) / 256), dim3(256), 0, as_stream(stream), params,
                       adam_m, adam_v, target, reinterpret_cast<_Float16 *>(target_h),
                       reinterpret_cast<_Float16 *>(params_h), grad, n,
                       gscale, alpha, c1, c2, eps, sync);
    DMDQN_LAUNCH_CHECK("k_adam");
    return DMDQN_OK;
}
