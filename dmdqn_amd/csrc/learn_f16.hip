// learn_f16.hip -- the f16 instantiation of learn_h16.hpp (the reference's
// tf.keras mixed_float16 policy, train.py:61: f16 MFMA operands, f32
// accumulate, f32 master weights + Adam), plus the shared-parameter learn
// (configuration C5, SURVEY 8e: the two passes are in learn_shared.hip; the
// slab reduction is here) and the flat Keras-3 Adam it is followed by.
#define DMDQN_H16_BF16 0
#include "learn_h16.hpp"

namespace dmdqn {
namespace f16k {

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

// One Keras-3 Adam update (A-11) of parameter i with gradient gr, each op
// rounded as TF's separate kernels (mul_rn: this file is built with
// -ffp-contract=fast, which ignores the contract pragma); on a target sync
// also the target copy and its f16 shadow.  Shared by k_adam and
// k_reduce_adam, so both compute the same bits.
struct AdamK {
    float *W, *M, *V, *T;
    _Float16 *TH, *WH;
    float gscale, alpha, c1, c2, eps;
    int sync;
};
__device__ __forceinline__ void keras_adam1(const AdamK &k, int i, float gr, float w, float m, float v) {
    const float g = mul_rn(gr, k.gscale);
    m = m + mul_rn(g - m, k.c1);
    v = v + mul_rn(mul_rn(g, g) - v, k.c2);
    w = w - (m * k.alpha) / (sqrtf(v) + k.eps);
    k.M[i] = m;
    k.V[i] = v;
    k.W[i] = w;
    if (k.WH) k.WH[i] = (_Float16)w;
    if (k.sync) {
        k.T[i] = w;
        if (k.TH) k.TH[i] = (_Float16)w;
    }
}

// Keras-3 Adam over n flat parameters with g = gscale * grad.
__global__ void __launch_bounds__(256) k_adam(AdamK k, const float *G, int n) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    keras_adam1(k, i, G[i], k.W[i], k.M[i], k.V[i]);
}

namespace f16k {
// k_reduce_slabs and k_adam in one launch (one rank: nothing between them):
// the same sums in the same order (grad is still written), then the Adam step
// on them by the wave that formed them, its w / m / v loaded before the sums.
__global__ void __launch_bounds__(512) k_reduce_adam(const float *slab, int nw, float scale,
                                                     float *grad, AdamK k) {
    __shared__ float4 part[8][64];
    const int wv = threadIdx.x >> 6, l = threadIdx.x & 63;
    const int c = blockIdx.x * 64 + l;  // float4 column
    constexpr int NC = L::P / 4;
    const int cc = c < NC ? c : NC - 1;
    float4 w4 = make_float4(0.f, 0.f, 0.f, 0.f), m4 = w4, v4 = w4;
    if (wv == 0) {
        w4 = reinterpret_cast<const float4 *>(k.W)[cc];
        m4 = reinterpret_cast<const float4 *>(k.M)[cc];
        v4 = reinterpret_cast<const float4 *>(k.V)[cc];
    }
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    if (c < NC) {
        const float4 *s4 = reinterpret_cast<const float4 *>(slab);
#pragma unroll 4
        for (int q = wv; q < nw; q += 8) {
            const float4 v = s4[(size_t)q * NC + c];
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
        keras_adam1(k, 4 * c + 0, t.x, w4.x, m4.x, v4.x);
        keras_adam1(k, 4 * c + 1, t.y, w4.y, m4.y, v4.y);
        keras_adam1(k, 4 * c + 2, t.z, w4.z, m4.z, v4.z);
        keras_adam1(k, 4 * c + 3, t.w, w4.w, m4.w, v4.w);
    }
}
}  // namespace f16k


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
    DMDQN_REQUIRE(a && slab, "dmdqn_learn_shared_grad: null argument");
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
    DMDQN_REQUIRE(work, "dmdqn_learn_shared_grad: work (dmdqn_learn_shared_work_bytes) required");
    hipStream_t s = as_stream(stream);
    float *y = reinterpret_cast<float *>(work);
    uint8_t *act = reinterpret_cast<uint8_t *>(y + (size_t)a->NA * f16k::B_);
    const int rc = launch_shared_v2(a, y, act, slab, n_slabs, s);
    if (rc) return rc;
    if (!grad) return DMDQN_OK;  // the slabs are reduced by dmdqn_adam_slabs
    hipLaunchKernelGGL(f16k::k_reduce_slabs, dim3((f16k::L::P / 4 + 63) / 64), dim3(512), 0, s,
                       slab, n_slabs, scale, grad);
    DMDQN_LAUNCH_CHECK("k_reduce_slabs");
    return DMDQN_OK;
}

extern "C" int dmdqn_adam_slabs(float *params, float *adam_m, float *adam_v, float *target,
                                uint16_t *target_h, uint16_t *params_h, const float *slab,
                                int n_slabs, float *grad, float scale, int n, float gscale,
                                float alpha, float c1, float c2, float eps, int sync, void *stream) {
    DMDQN_REQUIRE(params && adam_m && adam_v && slab && grad && n_slabs >= 1,
                  "dmdqn_adam_slabs: bad args");
    DMDQN_REQUIRE(n == f16k::L::P, "dmdqn_adam_slabs: n=%d (the shared net's %d parameters)", n,
                  f16k::L::P);
    DMDQN_REQUIRE(!sync || target, "dmdqn_adam_slabs: target required on a sync");
    const AdamK k{params, adam_m, adam_v, target, reinterpret_cast<_Float16 *>(target_h),
                  reinterpret_cast<_Float16 *>(params_h), gscale, alpha, c1, c2, eps, sync};
    hipLaunchKernelGGL(f16k::k_reduce_adam, dim3((f16k::L::P / 4 + 63) / 64), dim3(512), 0,
                       as_stream(stream), slab, n_slabs, scale, grad, k);
    DMDQN_LAUNCH_CHECK("k_reduce_adam");
    return DMDQN_OK;
}

extern "C" int dmdqn_adam(float *params, float *adam_m, float *adam_v, float *target,
                          uint16_t *target_h, uint16_t *params_h, const float *grad, int n,
                          float gscale, float alpha, float c1, float c2, float eps, int sync,
                          void *stream) {
    DMDQN_REQUIRE(params && adam_m && adam_v && grad && n > 0, "dmdqn_adam: bad args");
    DMDQN_REQUIRE(!sync || target, "dmdqn_adam: target required on a sync");
    const AdamK k{params, adam_m, adam_v, target, reinterpret_cast<_Float16 *>(target_h),
                  reinterpret_cast<_Float16 *>(params_h), gscale, alpha, c1, c2, eps, sync};
    hipLaunchKernelGGL(k_adam, dim3((n + 255) / 256), dim3(256), 0, as_stream(stream), k, grad, n);
    DMDQN_LAUNCH_CHECK("k_adam");
    return DMDQN_OK;
}
