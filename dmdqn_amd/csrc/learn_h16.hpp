// learn_h16.hpp -- fused Double-DQN learn step with 16-bit MFMA operands,
// instantiated twice: learn_f16.hip (f16, v_mfma_f32_16x16x32_f16: the
// reference's tf.keras mixed_float16 policy, train.py:61) and learn_bf16.hip
// (bf16, v_mfma_f32_16x16x32_bf16: the same algorithm under a mixed_bfloat16
// policy, BASELINE config C2).  Both keep f32 accumulation and f32 master
// weights + Adam slots, and round where Keras 3 / TF do under the mixed
// policy (tests/golden/tf_shim.py states the sources; tests/golden/
// learn_mixed.npz is the reference's own learn run that way):
//   * weights and biases: the f32 variables cast to h16 at each use;
//   * Dense: z = h16(h16(x W) + b) -- the matmul result is rounded, then the
//     16-bit bias add rounds again; relu; Q is the h16 output of layer 3;
//   * dL/dQ rounded to h16 (the gradient of the learn's tf.cast);
//   * dH = h16(dZ W^T) masked by relu; dW = h16(X^T dZ), db = h16(sum dZ):
//     the gradients Adam receives are 16-bit values (no loss scaling).
// The includer defines DMDQN_H16_BF16 (0 or 1) first.
//
// One workgroup (8 waves) per agent, TWO workgroups per CU: 74 KB of LDS and
// <= 128 VGPRs, so one agent's HBM phases (weight fragments, replay gather,
// Adam read-modify-write) overlap the other agent's MFMA phases.
//
// Weights never pass through LDS: each wave owns 16 output neurons and reads
// their fan-in rows (transposed layout, qnet_layout.hpp) straight from HBM
// into MFMA A-fragments (32 contiguous bytes per lane, converted f32 -> f16).
// LDS holds only activations:   R1 = H1 / dZ1 (f16 [128][128])
//                               R2 = X / H2 / dZ2 (f16 [128][128])
//                               DQ (f16 [128][16]) + per-row scratch
//
// GEMM orientation (C[M][N] = sum_k A[M][k] B[k][N], 16x16x32 fragments):
//   forward  Z^T[n][b] = W^T[n][k] . X[b][k]   -> lane holds 4 consecutive
//            neurons of one batch row: one 8-byte store into the [b][n] image
//   dW3      C[k][a] = H2^T . DQ       (batch reductions use ds_read_b64_tr_b16)
//   dW2      C[j][k] = H1^T . dZ2
//   dH1^T    C[j][b] = W2[j][k] . dZ2^T
//   dW1      C[i][j] = X^T . dZ1
//   bias grads: the same MFMAs with an all-ones operand (column sums).
// Gradient tiles C[in][out] hold 4 consecutive fan-in values per lane, which
// is 16 contiguous bytes of the transposed parameter layout: Adam is one
// float4 read-modify-write of w, m, v per lane straight from the accumulators.

#include <math.h>

#include "common.hpp"
#include "qnet_layout.hpp"

#if DMDQN_H16_BF16
#define H16K bf16k
#define H16_T __bf16
#define H16_MFMA __builtin_amdgcn_mfma_f32_16x16x32_bf16
#define H16_LEARN_KERNEL k_learn_bf16
#define H16_LAUNCH launch_learn_bf16
#define H16_LAUNCH_GRAD launch_learn_grad_bf16
#define H16_LAUNCH_ADAM launch_adam_agents_bf16
#define H16_ADAM_KERNEL k_adam_agents_bf16
#define H16_NAME "bf16"
#else
#define H16K f16k
#define H16_T _Float16
#define H16_MFMA __builtin_amdgcn_mfma_f32_16x16x32_f16
#define H16_LEARN_KERNEL k_learn_f16
#define H16_LAUNCH launch_learn_f16
#define H16_LAUNCH_GRAD launch_learn_grad_f16
#define H16_LAUNCH_ADAM launch_adam_agents_f16
#define H16_ADAM_KERNEL k_adam_agents_f16
#define H16_NAME "fp16"
#endif

namespace dmdqn {
namespace H16K {

typedef H16_T h16;  // the MFMA operand type (f16 or bf16)

typedef h16 half8 __attribute__((ext_vector_type(8)));
typedef h16 half4v __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short v4s __attribute__((vector_size(8)));
typedef __attribute__((address_space(3))) v4s lds_v4s;

constexpr int B_ = 128, DP = QN_DP, H = 128, NACT = QN_NA;
using L = QL<H>;

// LDS byte offsets
constexpr int R1_OFF = 0;
constexpr int R2_OFF = R1_OFF + B_ * H * 2;
constexpr int DQ_OFF = R2_OFF + B_ * H * 2;
constexpr int SC_OFF = DQ_OFF + B_ * 16 * 2;
constexpr int W3_OFF = SC_OFF + 6272;          // f16 W3T images [2][4][128]: online, target
constexpr int B3_OFF = W3_OFF + 2 * NACT * H * 2; // f32 b3 [2][4]
constexpr int LDS_BYTES = B3_OFF + 2 * NACT * 4;
static_assert(LDS_BYTES <= 81920, "two workgroups per CU");

__device__ __forceinline__ f32x4 mfma(half8 a, half8 b, f32x4 c) {
    return H16_MFMA(a, b, c, 0, 0, 0);
}

// threadIdx.x behind an empty asm: the per-thread addresses derived from it
// are recomputed at each use instead of being common-subexpressioned across
// the whole kernel (the three gathers share their slot-read and LDS-store
// addresses; kept live from the first to the last they spilled to scratch --
// 18 KB of scratch writes per workgroup reaching HBM, and vmcnt(0) reloads).
__device__ __forceinline__ int fresh_tid() {
    int t = threadIdx.x;
    asm volatile("" : "+v"(t));
    return t;
}

// img[r0 + (l&15)][k0 + 8(l>>4) + e], e = 0..7: one 16-byte LDS read.
__device__ __forceinline__ half8 frag_row(const h16 *img, int ld, int r0, int k0) {
    const int l = threadIdx.x & 63;
    return *reinterpret_cast<const half8 *>(img + (r0 + (l & 15)) * ld + k0 + 8 * (l >> 4));
}

// img[r0 + 8(l>>4) + e][c0 + (l&15)], e = 0..7: two ds_read_b64_tr_b16.
// Lane 4q+p of each 16-lane group addresses row q, columns 4p..4p+3 of a
// 4-row block; lane i receives column i of the block (row q -> element q).
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

// The activation images -- [128][128] H1, H2, dZ2, dZ1, the W2^T image and
// the [128][96] X -- are stored in 8-row x 32-column blocks of 512 B (a band
// of 8 rows is LD/32 blocks, a multiple of 256 B),
// row r's 16-byte chunks within a block XOR-permuted by bit 1 and bit 3 of r
// (a search over the linear permutations of row bits 0, 1, 3):
//   * row-fragment reads (ds_read_b128 of rows r0..r0+15, chunk 4s+lg): each
//     16-lane bank group {0-3,12-15 | 20-27} covers all 16 bank slots;
//   * transposed reads (ds_read_b64_tr_b16 of rows r0+8g+q, chunks 2c..2c+1):
//     each 32-lane half covers all 32 eight-byte slots;
// so both are conflict-free (the plain 256-B rows were 8-way on both), the
// 8-byte MFMA-output stores are 2-way (the least any permutation of whole
// 16-byte chunks allows for 16 rows at one column), and
// every address is a lane constant plus an immediate.  (The 2-way conflicts
// of the 192-B X rows go too.)
template <int LD = H>
__device__ __forceinline__ int hoff(int r, int c) {
    static_assert(LD % 32 == 0, "whole blocks per band");
    const int ch = c >> 3;
    return 8 * LD * (r >> 3) + 256 * (ch >> 2) + 32 * (r & 7) +
           8 * ((ch & 3) ^ (((r >> 1) & 1) | ((r >> 2) & 2))) + (c & 7);
}

// frag_row on a blocked image (r0 a multiple of 16, k0 of 32).
template <int LD = H>
__device__ __forceinline__ half8 frag_row_h(const h16 *img, int r0, int k0, int tid = threadIdx.x) {
    const int l = tid & 63;
    return *reinterpret_cast<const half8 *>(img + hoff<LD>(r0 + (l & 15), k0 + 8 * (l >> 4)));
}

// frag_tr on a blocked image (r0 a multiple of 8, c0 of 16); rows +4 share
// the row's permutation and sit 128 elements further.
template <int LD = H>
__device__ __forceinline__ half8 frag_tr_h(const h16 *img, int r0, int c0) {
    const int l = threadIdx.x & 63, i = l & 15, g = l >> 4;
    const h16 *p0 = img + hoff<LD>(r0 + 8 * g + (i >> 2), c0 + 4 * (i & 3));
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

// A-fragment of a transposed f32 weight matrix WT[N][ld] (tiled, qn_wt)
// straight from HBM: WT[n0 + (l&15)][k0 + 8(l>>4) + e] -> f16, 32 contiguous
// bytes per lane.  nvalid masks padded rows.
__device__ __forceinline__ half8 wfrag(const float *WT, int ld, int n0, int k0, int nvalid = 16) {
    const int l = threadIdx.x & 63, lr = l & 15;
    half8 r;
    if (lr < nvalid) {
        const float4 *p = reinterpret_cast<const float4 *>(WT + qn_wt(n0 + lr, k0 + 8 * (l >> 4), ld));
        float4 x = p[0], y = p[1];
        r[0] = (h16)x.x; r[1] = (h16)x.y; r[2] = (h16)x.z; r[3] = (h16)x.w;
        r[4] = (h16)y.x; r[5] = (h16)y.y; r[6] = (h16)y.z; r[7] = (h16)y.w;
    } else {
#pragma unroll
        for (int e = 0; e < 8; e++) r[e] = (h16)0.0f;
    }
    return r;
}

// Same fragment from an f16 copy (16-byte loads, no conversion).
__device__ __forceinline__ half8 wfrag(const h16 *WT, int ld, int n0, int k0, int nvalid = 16) {
    const int l = threadIdx.x & 63, lr = l & 15;
    half8 r;
    if (lr < nvalid) {
        r = *reinterpret_cast<const half8 *>(WT + qn_wt(n0 + lr, k0 + 8 * (l >> 4), ld));
    } else {
#pragma unroll
        for (int e = 0; e < 8; e++) r[e] = (h16)0.0f;
    }
    return r;
}

// Layer-1 A-fragment s (features 32s..32s+31) of neurons n0..n0+15 from the
// W1 block (qn_w1): 8 consecutive features per lane.  Fragment 2's lanes
// lg = 3 cover features 88..95, of which only 88 exists (the W1T column;
// 89..95 are zero weights, not stored).
__device__ __forceinline__ half8 w1frag(const float *W1, int n0, int s) {
    const int l = threadIdx.x & 63, lg = l >> 4, n = n0 + (l & 15);
    const bool tile = s < 2 || lg < 3;
    // branch-free: every lane loads a valid tile address (fragment 2's lane
    // group 3 re-reads group 2's) and, for fragment 2, the feature-88 column;
    // the select follows (a branch around the loads made the head wait)
    const float4 *p = reinterpret_cast<const float4 *>(W1 + qn_w1<H>(n, 32 * s + 8 * (tile ? lg : 2)));
    const float4 x = p[0], y = p[1];
    const float c = s == 2 ? W1[qn_w1<H>(n, QN_DT)] : 0.0f;
    half8 r;
    r[0] = (h16)(tile ? x.x : c); r[1] = (h16)(tile ? x.y : 0.0f);
    r[2] = (h16)(tile ? x.z : 0.0f); r[3] = (h16)(tile ? x.w : 0.0f);
    r[4] = (h16)(tile ? y.x : 0.0f); r[5] = (h16)(tile ? y.y : 0.0f);
    r[6] = (h16)(tile ? y.z : 0.0f); r[7] = (h16)(tile ? y.w : 0.0f);
    return r;
}

__device__ __forceinline__ half8 w1frag(const h16 *W1, int n0, int s) {
    const int l = threadIdx.x & 63, lg = l >> 4, n = n0 + (l & 15);
    const bool tile = s < 2 || lg < 3;
    const half8 t = *reinterpret_cast<const half8 *>(W1 + qn_w1<H>(n, 32 * s + 8 * (tile ? lg : 2)));
    const h16 c = s == 2 ? W1[qn_w1<H>(n, QN_DT)] : (h16)0.0f;
    half8 r;
    r[0] = tile ? t[0] : c;
#pragma unroll
    for (int e = 1; e < 8; e++) r[e] = tile ? t[e] : (h16)0.0f;
    return r;
}

__device__ __forceinline__ float4 ld_bias4(const float *p) { return *reinterpret_cast<const float4 *>(p); }
__device__ __forceinline__ float r16(float x) { return (float)(h16)x; }
// A bias read for a forward: the f32 variable cast to h16 (Keras' autocast),
// kept packed (2 VGPRs for 4 neurons).
__device__ __forceinline__ half4v ld_bias4_h(const float *p) {
    return __builtin_convertvector(*reinterpret_cast<const f32x4 *>(p), half4v);
}
__device__ __forceinline__ float4 ld_bias4(const h16 *p) {
    const half4v h = *reinterpret_cast<const half4v *>(p);
    return make_float4((float)h[0], (float)h[1], (float)h[2], (float)h[3]);
}
__device__ __forceinline__ half4v ld_bias4_h(const h16 *p) {
    return *reinterpret_cast<const half4v *>(p);
}

__device__ __forceinline__ half8 ones8() {
    half8 r;
#pragma unroll
    for (int e = 0; e < 8; e++) r[e] = (h16)1.0f;
    return r;
}

struct Scratch {
    float *z3;  // [128][4]
    float *rn, *y, *dq, *dn;
    int *act, *slot;
    double *r64, *red;
};

// Per-wave register copy of one network's weights: the A-fragments of the
// wave's 16 neurons for layers 1 and 2, the (4-row) output layer, and the
// lane's biases.  Loaded once per network and reused by every forward that
// network runs (the online net serves both the S' and the S forward).
struct Frags {
    half8 w1[3], w2[4];
    half4v b1, b2;
};

// The output layer (4 x 128) of a network as an f16 LDS image + f32 bias,
// staged once per launch: the forwards' layer 3 and dZ2 read it from LDS, so
// they never wait behind fragment prefetches in the in-order vmcnt queue, and
// dZ2 sees the pre-update W3 (Adam on W3 runs before dZ2).
struct OutL {
    const h16 *w3;  // [4][128]
    const float *b3;     // [4]
};

template <typename T>
__device__ __forceinline__ void load_w1(const T *Wg, Frags &f) {
    const int w = threadIdx.x >> 6, lg = (threadIdx.x & 63) >> 4;
#pragma unroll
    for (int s = 0; s < 3; s++) f.w1[s] = w1frag(Wg + L::oW1T, 16 * w, s);
    f.b1 = ld_bias4_h(Wg + L::ob1 + 16 * w + 4 * lg);
}

template <typename T>
__device__ __forceinline__ void load_w2(const T *Wg, Frags &f) {
    const int w = threadIdx.x >> 6, lg = (threadIdx.x & 63) >> 4;
#pragma unroll
    for (int s = 0; s < 4; s++) f.w2[s] = wfrag(Wg + L::oW2T, H, 16 * w, 32 * s);
    f.b2 = ld_bias4_h(Wg + L::ob2 + 16 * w + 4 * lg);
}

// The output layer (W3T f16 image + b3) of one network into LDS, in two
// halves: the loads (into registers, issued early) and the LDS stores (once
// they land; the caller syncs).  Thread t < 128: W3T[4t..4t+3]; t in 128..131:
// b3[t - 128] (in v.x).
// The loads are issued by every thread at valid addresses (no divergent
// branch around a load: the wait-count insertion is conservative at control
// flow, and a branch there made the head wait for each load in turn).
struct OutStage {
    float4 v;
    float b;
};

template <typename T>
__device__ __forceinline__ OutStage stage_out_load(const T *Wg) {
    const int t = threadIdx.x;
    OutStage o;
    o.v = ld_bias4(Wg + L::oW3T + 4 * (t & (NACT * H / 4 - 1)));
    o.b = (float)(h16)Wg[L::ob3 + (t & (NACT - 1))];
    return o;
}

__device__ __forceinline__ void stage_out_store(const OutStage &o, h16 *w3, float *b3) {
    const int t = threadIdx.x;
    if (t < NACT * H / 4) {
        half4v hv;
        hv[0] = (h16)o.v.x; hv[1] = (h16)o.v.y; hv[2] = (h16)o.v.z; hv[3] = (h16)o.v.w;
        *reinterpret_cast<half4v *>(w3 + 4 * t) = hv;
    } else if (t < NACT * H / 4 + NACT) {
        b3[t - NACT * H / 4] = o.b;
    }
}

template <typename T>
__device__ __forceinline__ void load_frags(const T *Wg, Frags &f) {
    load_w1(Wg, f);
    load_w2(Wg, f);
}

struct NoHook {
    __device__ void operator()(Frags &) const {}
};

// Dense + relu under the mixed policy: relu(h16(h16(acc) + b)) -- the
// matmul result rounded, then the correctly rounded 16-bit bias add (f16:
// packed v_pk_add_f16; bf16: an f32 add rounded once, the same value).
__device__ __forceinline__ half4v relu_h4(f32x4 acc, half4v b) {
    const half4v z = __builtin_convertvector(acc, half4v) + b;
    const half4v zero = {(h16)0.0f, (h16)0.0f, (h16)0.0f, (h16)0.0f};
    return z > zero ? z : zero;  // vector select (packed max; the build has no SLP)
}

struct NoHook0 {
    __device__ void operator()() const {}
};

// Forward with explicit buffers: X (rows, stride DP) -> H1b -> H2b -> qout.
//   HOLD = true : H2b == H1b -- layer 2 keeps its 8 output tiles in registers
//                 across a barrier before overwriting H1 (X survives).
//   HOLD = false: H2b != H1b -- each layer-2 tile is written as soon as it is
//                 computed (H2b may be X's buffer: X is dead after layer 1).
// Hooks: after_l1(f) / after_l2(f) as in forward(); after_sync2() runs after
// the barrier that follows layer 2 (every wave is done reading H1b).
template <bool HOLD, typename H1k = NoHook, typename H2k = NoHook, typename S2k = NoHook0>
__device__ void forward_x(Frags &f, const OutL o, const h16 *X, h16 *H1b, h16 *H2b,
                          float *qout, H1k after_l1 = {}, H2k after_l2 = {},
                          S2k after_sync2 = {}) {
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63, lr = l & 15, lg = l >> 4;
    const int n = 16 * w + 4 * lg;
    // the X-row addresses from a fresh lane id: shared across the three
    // forwards they were kept live through the kernel and spilled (round 5)
    const int tx = fresh_tid();
#pragma unroll
    for (int t = 0; t < 8; t++) {
        f32x4 c = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < 3; s++) c = mfma(f.w1[s], frag_row_h<DP>(X, 16 * t, 32 * s, tx), c);
        *reinterpret_cast<half4v *>(H1b + hoff(16 * t + lr, n)) = relu_h4(c, f.b1);
    }
    after_l1(f);
    __syncthreads();
    if constexpr (HOLD) {
        f32x4 acc[8];
#pragma unroll
        for (int t = 0; t < 8; t++) {
            f32x4 c = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int s = 0; s < 4; s++) c = mfma(f.w2[s], frag_row_h(H1b, 16 * t, 32 * s), c);
            acc[t] = c;
        }
        const half4v b2 = f.b2;
        after_l2(f);
        __syncthreads();  // every wave has read H1
#pragma unroll
        for (int t = 0; t < 8; t++)
            *reinterpret_cast<half4v *>(H2b + hoff(16 * t + lr, n)) = relu_h4(acc[t], b2);
    } else {
#pragma unroll
        for (int t = 0; t < 8; t++) {
            f32x4 c = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int s = 0; s < 4; s++) c = mfma(f.w2[s], frag_row_h(H1b, 16 * t, 32 * s), c);
            *reinterpret_cast<half4v *>(H2b + hoff(16 * t + lr, n)) = relu_h4(c, f.b2);
        }
        after_l2(f);
    }
    __syncthreads();
    after_sync2();
    {
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < 4; s++) {
            half8 a3;
            if (lr < NACT) a3 = frag_row(o.w3, H, 0, 32 * s);
            else
#pragma unroll
                for (int e = 0; e < 8; e++) a3[e] = (h16)0.0f;
            acc = mfma(a3, frag_row_h(H2b, 16 * w, 32 * s), acc);
        }
        if (lg == 0) {
            float4 q;
            q.x = r16(r16(acc[0]) + o.b3[0]);
            q.y = r16(r16(acc[1]) + o.b3[1]);
            q.z = r16(r16(acc[2]) + o.b3[2]);
            q.w = r16(r16(acc[3]) + o.b3[3]);
            *reinterpret_cast<float4 *>(qout + (16 * w + lr) * NACT) = q;
        }
    }
    __syncthreads();
}

// A gradient entry as Adam receives it under the mixed policy: 16-bit.
__device__ __forceinline__ float gval(const f32x4 &g, int e) { return r16(g[e]); }

// Keras-3 Adam (keras/src/optimizers/adam.py update_step) on one parameter,
// every op rounded on its own as TF's separate elementwise kernels do: no fma
// contraction (mul_rn: this file is built with -ffp-contract=fast for the
// MFMA epilogues, which ignores the contract pragma), correctly rounded sqrt
// and divide (HIP's default).
__device__ __forceinline__ void adam_el(float &w, float &m, float &v, float g, float alpha,
                                        float c1, float c2, float eps) {
    m = m + mul_rn(g - m, c1);
    v = v + mul_rn(mul_rn(g, g) - v, c2);
    w = w - (m * alpha) / (sqrtf(v) + eps);
}

struct AdamC {
    float alpha, c1, c2, eps;
    bool sync;
    h16 *TH;    // f16 target copy written on syncs (or null)
    bool gout;  // compile-time: write the 16-bit gradient to G instead of the
    float *G;   // Adam step (split learn: dmdqn_learn_grad + dmdqn_adam_agents)
};

// Keras-3 Adam on NT groups of 4 consecutive parameters (one 16-byte lane
// access each).  All w, m, v loads of the NT groups are issued before any
// store, so one memory round trip covers NT tiles.
template <int NT>
__device__ __forceinline__ void adam4n(float *W, float *M, float *V, float *T, const size_t *idx,
                                       const f32x4 *g, const AdamC &k) {
    if (k.gout) {
#pragma unroll
        for (int q = 0; q < NT; q++)
            *reinterpret_cast<float4 *>(k.G + idx[q]) =
                make_float4(gval(g[q], 0), gval(g[q], 1), gval(g[q], 2), gval(g[q], 3));
        return;
    }
    float4 w[NT], m[NT], v[NT];
#pragma unroll
    for (int q = 0; q < NT; q++) {
        w[q] = *reinterpret_cast<const float4 *>(W + idx[q]);
        m[q] = *reinterpret_cast<const float4 *>(M + idx[q]);
        v[q] = *reinterpret_cast<const float4 *>(V + idx[q]);
    }
    // keep all 3*NT loads in flight together: under VGPR pressure the
    // scheduler would otherwise sink each load to its use (one round trip each)
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int q = 0; q < NT; q++) {
        float *pw = &w[q].x, *pm = &m[q].x, *pv = &v[q].x;
#pragma unroll
        for (int e = 0; e < 4; e++)
            adam_el(pw[e], pm[e], pv[e], gval(g[q], e), k.alpha, k.c1, k.c2, k.eps);
    }
#pragma unroll
    for (int q = 0; q < NT; q++) {
        *reinterpret_cast<float4 *>(W + idx[q]) = w[q];
        *reinterpret_cast<float4 *>(M + idx[q]) = m[q];
        *reinterpret_cast<float4 *>(V + idx[q]) = v[q];
        if (k.sync) {
            *reinterpret_cast<float4 *>(T + idx[q]) = w[q];
            if (k.TH) {
                half4v hv;
                hv[0] = (h16)w[q].x; hv[1] = (h16)w[q].y;
                hv[2] = (h16)w[q].z; hv[3] = (h16)w[q].w;
                *reinterpret_cast<half4v *>(k.TH + idx[q]) = hv;
            }
        }
    }
}

// Keras-3 Adam over NB batches of NT gradient tiles, double-buffered: the
// w, m, v loads of batch h+1 are issued BEFORE the stores of batch h.  Loads
// and stores share the in-order vmcnt counter, so with the plain order every
// batch's loads would also wait for the previous batch's stores to land.
// Each batch's loads are pinned together by a scheduling barrier (without it
// the scheduler, under the 128-VGPR cap, sinks loads to their uses).  Measured
// (one box): W2 4x2 + W1 2x3 tiles, 4.18 ms vs 4.36 ms for the plain order.
// `grad()` runs after the first batch's loads are issued and produces g[]:
// the w, m, v loads do not depend on the gradient, so their latency hides
// behind the gradient MFMAs.
// Issue the first Adam batch before the gradient MFMAs: for W1 (measured
// 1-2 % faster); not for W2, where the 24 extra live VGPRs next to the dW2
// accumulators and the W2 fragments spill (10 -> 28) and cost 10 %.
#ifndef DMDQN_EARLY_W3
#define DMDQN_EARLY_W3 0
#endif
#ifndef DMDQN_GX_EARLY
#define DMDQN_GX_EARLY 0
#endif
#ifndef DMDQN_EARLY_W2
#define DMDQN_EARLY_W2 0
#endif
#ifndef DMDQN_EARLY_W1
#define DMDQN_EARLY_W1 1
#endif
// `valid(tile)` says whether the lane's 4 parameters of that tile exist (the
// W1 block stores only features 0..88; a lane with nothing to update keeps its
// registers and touches no memory).
struct AllValid {
    __device__ constexpr bool operator()(int) const { return true; }
};

template <int NB, int NT, bool EARLY, typename Index, typename GT, typename Grad,
          typename Valid = AllValid>
__device__ __forceinline__ void adam_pipe(float *W, float *M, float *V, float *T, Index ix,
                                          const GT *g, const AdamC &k, Grad grad,
                                          Valid valid = {}) {
    if (k.gout) {  // the same index map, the gradient stored instead
        grad();
#pragma unroll
        for (int t = 0; t < NB * NT; t++)
            if (valid(t))
                *reinterpret_cast<float4 *>(k.G + ix(t)) =
                    make_float4(gval(g[t], 0), gval(g[t], 1), gval(g[t], 2), gval(g[t], 3));
        return;
    }
    float4 w[2][NT], m[2][NT], v[2][NT];
    if constexpr (!EARLY) grad();
#pragma unroll
    for (int q = 0; q < NT; q++) {
        const size_t i = ix(q);
        w[0][q] = m[0][q] = v[0][q] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (valid(q)) {
            w[0][q] = *reinterpret_cast<const float4 *>(W + i);
            m[0][q] = *reinterpret_cast<const float4 *>(M + i);
            v[0][q] = *reinterpret_cast<const float4 *>(V + i);
        }
    }
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (EARLY) {
        grad();
        __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int h = 0; h < NB; h++) {
        const int c = h & 1, n = c ^ 1;
        if (h + 1 < NB) {
#pragma unroll
            for (int q = 0; q < NT; q++) {
                const size_t i = ix((h + 1) * NT + q);
                w[n][q] = m[n][q] = v[n][q] = make_float4(0.f, 0.f, 0.f, 0.f);
                if (valid((h + 1) * NT + q)) {
                    w[n][q] = *reinterpret_cast<const float4 *>(W + i);
                    m[n][q] = *reinterpret_cast<const float4 *>(M + i);
                    v[n][q] = *reinterpret_cast<const float4 *>(V + i);
                }
            }
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int q = 0; q < NT; q++) {
            float *pw = &w[c][q].x, *pm = &m[c][q].x, *pv = &v[c][q].x;
            const GT gq = g[h * NT + q];
#pragma unroll
            for (int e = 0; e < 4; e++)
                adam_el(pw[e], pm[e], pv[e], gval(gq, e), k.alpha, k.c1, k.c2, k.eps);
        }
#pragma unroll
        for (int q = 0; q < NT; q++) {
            const size_t i = ix(h * NT + q);
            if (!valid(h * NT + q)) continue;
            *reinterpret_cast<float4 *>(W + i) = w[c][q];
            *reinterpret_cast<float4 *>(M + i) = m[c][q];
            *reinterpret_cast<float4 *>(V + i) = v[c][q];
            if (k.sync) {
                *reinterpret_cast<float4 *>(T + i) = w[c][q];
                if (k.TH) {
                    half4v hv;
                    hv[0] = (h16)w[c][q].x; hv[1] = (h16)w[c][q].y;
                    hv[2] = (h16)w[c][q].z; hv[3] = (h16)w[c][q].w;
                    *reinterpret_cast<half4v *>(k.TH + i) = hv;
                }
            }
        }
    }
}

__device__ __forceinline__ void adam4(float *W, float *M, float *V, float *T, size_t i, f32x4 g,
                                      const AdamC &k) {
    adam4n<1>(W, M, V, T, &i, &g, k);
}

__device__ __forceinline__ void adam1(float *W, float *M, float *V, float *T, size_t i, float g,
                                      const AdamC &k) {
    if (k.gout) {
        k.G[i] = r16(g);
        return;
    }
    float m = M[i], v = V[i], w = W[i];
    adam_el(w, m, v, r16(g), k.alpha, k.c1, k.c2, k.eps);  // the 16-bit gradient
    M[i] = m;
    V[i] = v;
    W[i] = w;
    if (k.sync) {
        T[i] = w;
        if (k.TH) k.TH[i] = (h16)w;
    }
}

// ----------------------------------------------------------------------------
// Per-agent pieces shared by the independent kernel (k_learn_f16) and the
// shared-parameter kernel (k_learn_shared_f16).  All are called by every
// thread of the 512-thread workgroup.

template <bool XF> struct RowsT { uint2 v[3]; };        // int8 rows: 3 x 8 features per thread
template <> struct RowsT<true> { float4 v[6]; };        // float rows: the same 24 features
using Rows = RowsT<false>;


// Replay rows (int8, DMDQN_ROW_BYTES = one 128-B line each) of one agent's
// batch -> X f16 [128][96] in R2, in two halves so the loads can be in flight
// across other work: issue (3 x 8 bytes per thread into registers), then
// commit (convert + LDS store) once R2 is free.
__device__ __forceinline__ void gather_issue(const int8_t *ring, const dmdqn_learn_args &a,
                                             int agent, const int *slot, Rows &g) {
    const int tid = fresh_tid();
#pragma unroll
    for (int i = 0; i < 3; i++) {
        const int t = tid + 512 * i, b = t / 12, q = t - 12 * (t / 12);
        g.v[i] = reinterpret_cast<const uint2 *>(ring + ((size_t)agent * a.cap + slot[b]) *
                                                            DMDQN_ROW_BYTES)[q];
    }
}

__device__ __forceinline__ void gather_commit(h16 *R2, const Rows &g) {
    const int tid = fresh_tid();
#pragma unroll
    for (int i = 0; i < 3; i++) {
        const int t = tid + 512 * i, b = t / 12, q = t - 12 * (t / 12);
        half8 hv;
#pragma unroll
        for (int e = 0; e < 4; e++) {
            hv[e] = (h16)(float)(int8_t)(g.v[i].x >> (8 * e));
            hv[e + 4] = (h16)(float)(int8_t)(g.v[i].y >> (8 * e));
        }
        *reinterpret_cast<half8 *>(R2 + hoff<DP>(b, 8 * q)) = hv;
    }
}

// X(S) / X(S') of either row format into an f16 [128][96] image: int8 ring rows
// through the slots (gather_issue / gather_commit), or the float rows
// pre-gathered in batch order (a.xs / a.xn, DMDQN_ROWS_F32) cast to 16 bits
// as Keras' mixed policy casts the layer input.
template <bool XF>
__device__ __forceinline__ void gather_x(const dmdqn_learn_args &a, int agent, bool next,
                                         const int *slot, RowsT<XF> &g) {
    if constexpr (XF) {
        const float *X = (next ? a.xn : a.xs) + (size_t)agent * B_ * DP;
        const int tid = fresh_tid();
#pragma unroll
        for (int i = 0; i < 3; i++) {
            const int t = tid + 512 * i, b = t / 12, q = t - 12 * (t / 12);
            g.v[2 * i] = *reinterpret_cast<const float4 *>(X + b * DP + 8 * q);
            g.v[2 * i + 1] = *reinterpret_cast<const float4 *>(X + b * DP + 8 * q + 4);
        }
    } else {
        gather_issue(next ? a.ring_n : a.ring_s, a, agent, slot, g);
    }
}

template <bool XF>
__device__ __forceinline__ void commit_x(h16 *R, const RowsT<XF> &g) {
    if constexpr (XF) {
        const int tid = fresh_tid();
#pragma unroll
        for (int i = 0; i < 3; i++) {
            const int t = tid + 512 * i, b = t / 12, q = t - 12 * (t / 12);
            const float *f0 = &g.v[2 * i].x, *f1 = &g.v[2 * i + 1].x;
            half8 hv;
#pragma unroll
            for (int e = 0; e < 4; e++) {
                hv[e] = (h16)f0[e];
                hv[e + 4] = (h16)f1[e];
            }
            *reinterpret_cast<half8 *>(R + hoff<DP>(b, 8 * q)) = hv;
        }
    } else {
        gather_commit(R, g);
    }
}

// The batch's deque positions (thread tid < 128: position tid).  Loaded first
// in the kernel: the slot computation then waits only for them (vmcnt is
// in-order, so a load issued after the weight fragments would wait for those).
__device__ __forceinline__ int batch_pos(const dmdqn_learn_args &a, int agent) {
    return a.idx[(size_t)agent * B_ + (threadIdx.x & (B_ - 1))];
}

// Ring slots of the batch (deque positions -> slots).  Ends with a barrier.
__device__ __forceinline__ void batch_slots(const dmdqn_learn_args &a, int pos, const Scratch &S) {
    // every thread stores (the 4 lane groups of 128 store the same values):
    // a store under tid < B_ let the compiler sink the idx load into that
    // branch, behind the fragment loads, and wait for all of them
    DMDQN_DBG(pos >= 0 && pos < a.cap, DBG_LEARN_IDX);
#ifdef DMDQN_DEBUG_BOUNDS
    if (pos < 0 || pos >= a.cap) pos = 0;
#endif
    int s = a.start + pos;
    if (s >= a.cap) s -= a.cap;
    S.slot[threadIdx.x & (B_ - 1)] = s;
    __syncthreads();
}

// The transition metadata (a, done, r) from the s' rows (bytes 96..111 of the
// line gather_issue(ring_n) reads: the same HBM line, in flight together).
struct Meta { uint4 v; };

__device__ __forceinline__ void meta_issue(const dmdqn_learn_args &a, int agent, const int *slot,
                                           Meta &m) {
    const int tid = threadIdx.x;
    if (tid < B_)
        m.v = *reinterpret_cast<const uint4 *>(a.ring_n + ((size_t)agent * a.cap + slot[tid]) *
                                                                DMDQN_ROW_BYTES + DMDQN_ROW_A);
}

__device__ __forceinline__ void meta_commit(const Meta &m, const Scratch &S) {
    static_assert(DMDQN_ROW_D == DMDQN_ROW_A + 1 && DMDQN_ROW_R == DMDQN_ROW_A + 8, "row tail");
    const int tid = threadIdx.x;
    if (tid < B_) {
        S.act[tid] = m.v.x & 0xffu;
        DMDQN_DBG(S.act[tid] < NACT, DBG_LEARN_ACT);
#ifdef DMDQN_DEBUG_BOUNDS
        if (S.act[tid] >= NACT) S.act[tid] = 0;
#endif
        S.dn[tid] = (m.v.x >> 8) & 0xffu ? 1.0f : 0.0f;
        S.r64[tid] = __longlong_as_double((long long)(((unsigned long long)m.v.w << 32) | m.v.z));
    }
}

// The reward z-score of ReplayBuffer.sample (dqn_agent.py:64-69) over S.r64:
// f64 mean and population std over the 128 rewards in numpy's pairwise order
// (8 partial sums of 16), + 1e-8.  Starts with a barrier (S.r64 complete).
__device__ __forceinline__ void zscore(const Scratch &S) {
    const int tid = threadIdx.x;
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
}

// Slots, then the s' rows -> X(S') in R2 plus the metadata, then the z-score.
// X(S') is visible to every thread on return (zscore's barriers).  XF: float
// rows, the metadata from the per-slot arrays.  issued() runs once the row
// loads are in flight (the caller's LDS stores of earlier loads).
template <bool XF = false, typename Issued>
__device__ __forceinline__ void batch_head(const dmdqn_learn_args &a, int agent, int pos, h16 *R2,
                                           const Scratch &S, Issued issued) {
    batch_slots(a, pos, S);
    RowsT<XF> gn;
    gather_x<XF>(a, agent, true, S.slot, gn);
    issued();
    if constexpr (XF) {
        const int tid = threadIdx.x;
        if (tid < B_) {
            const size_t r = (size_t)agent * a.cap + S.slot[tid];
            S.act[tid] = a.ring_a[r] < NACT ? a.ring_a[r] : 0;
            S.dn[tid] = a.ring_d[r] ? 1.0f : 0.0f;
            S.r64[tid] = a.ring_r[r];
        }
        commit_x<XF>(R2, gn);
    } else {
        Meta mt;
        meta_issue(a, agent, S.slot, mt);
        gather_commit(R2, gn);
        meta_commit(mt, S);
    }
    zscore(S);
    if (a.rn_out && threadIdx.x < B_) a.rn_out[(size_t)agent * B_ + threadIdx.x] = S.rn[threadIdx.x];
}

// Double-DQN target y = r^ + gamma (1 - d) Q_target(S')[argmax Q_online(S')]
// (dqn_agent.py:342-347; first max on ties).  qo: online Q(S') [128][4];
// S.z3: target Q(S').  Ends with a barrier.
__device__ __forceinline__ void ddqn_target(const dmdqn_learn_args &a, const float *qo,
                                            const Scratch &S) {
    const int tid = threadIdx.x;
    if (tid < B_) {
        // y = r + (gamma (1 - d)) q_t, each op rounded as TF's (mul_rn: no fma)
        const float4 q = *reinterpret_cast<const float4 *>(qo + tid * NACT);
        int best = 0;
        float bq = q.x;
        if (q.y > bq) { best = 1; bq = q.y; }
        if (q.z > bq) { best = 2; bq = q.z; }
        if (q.w > bq) { best = 3; }
        float tq = S.z3[tid * NACT + best];
        float gd = a.gamma * (1.0f - S.dn[tid]);
        S.y[tid] = S.rn[tid] + mul_rn(gd, tq);
    }
    __syncthreads();
}

// MSE (dqn_agent.py:350-352) or Huber loss (loss_term) of Q_online(S) in S.z3 at
// the taken actions, written to a.loss[agent]; dL/dQ (f16) into DQ [128][16] and
// S.dq.  Ends with a barrier.
template <bool QSTATS>
__device__ __forceinline__ void loss_dq(const dmdqn_learn_args &a, int agent, h16 *DQ,
                                        const Scratch &S) {
    const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
    if (QSTATS) learn_qstats(a.qstats, agent, S.z3, S.act);
    float lsum = 0.0f;
    if (tid < B_) {
        float q = S.z3[tid * NACT + S.act[tid]];
        float dq;
        loss_term(a.loss_kind, q - S.y[tid], 1.0f / (float)B_, lsum, dq);
        half8 z;
#pragma unroll
        for (int e = 0; e < 8; e++) z[e] = (h16)0.0f;
        *reinterpret_cast<half8 *>(DQ + tid * 16) = z;
        *reinterpret_cast<half8 *>(DQ + tid * 16 + 8) = z;
        DQ[tid * 16 + S.act[tid]] = (h16)dq;
        S.dq[tid] = (float)(h16)dq;
    }
    if (w < 2) {
        for (int off = 32; off > 0; off >>= 1) lsum += __shfl_xor(lsum, off);
        if (l == 0) S.red[10 + w] = (double)lsum;
    }
    __syncthreads();
    if (tid == 0 && a.loss) a.loss[agent] = (float)(S.red[10] + S.red[11]) / (float)B_;
}

// dZ2 = dq * W3[:, a] masked by ReLU(H2), in place over H2 in R2 (8 columns
// per task); `on` holds the pre-update W3.  Ends with a barrier.
__device__ __forceinline__ void bwd_dz2(h16 *R2, const OutL on, const Scratch &S) {
    for (int t = threadIdx.x; t < B_ * (H / 8); t += 512) {
        const int b = t >> 4, k8 = (t & 15) * 8, ac = S.act[b];
        half8 *p = reinterpret_cast<half8 *>(R2 + hoff(b, k8));
        half8 h = *p, o;
        const half8 wv = *reinterpret_cast<const half8 *>(on.w3 + ac * H + k8);
        const float dq = S.dq[b];
#pragma unroll
        for (int e = 0; e < 8; e++)
            o[e] = (float)h[e] > 0.0f ? (h16)(dq * (float)wv[e]) : (h16)0.0f;
        *p = o;
    }
    __syncthreads();
}

// ReLU mask of H1 (R1) as bits: mask[b][j/32] (128 x 4 words).
__device__ __forceinline__ void h1_mask(const h16 *R1, uint32_t *mask) {
    const int tid = threadIdx.x, b = tid >> 2, q = tid & 3;
    uint32_t bits = 0;
#pragma unroll
    for (int c = 0; c < 4; c++) {
        const half8 hv = *reinterpret_cast<const half8 *>(R1 + hoff(b, 32 * q + 8 * c));
#pragma unroll
        for (int e = 0; e < 8; e++) bits |= ((float)hv[e] > 0.0f ? 1u : 0u) << (8 * c + e);
    }
    mask[b * 4 + q] = bits;
}

// dH1^T[j][b] = W2[j][k] . dZ2^T.  The caller has synced after the last use of
// H1; the W2^T f16 image [k][j] goes into R1 from the wave-owned forward
// fragments (the exact f16 operand of the forward), and the A operand is its
// transposed read.  Ends with a barrier (image and dZ2 consumed).
__device__ __forceinline__ void w2t_image(h16 *R1, const Frags &fr) {
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63, lr = l & 15, lg = l >> 4;
#pragma unroll
    for (int s2 = 0; s2 < 4; s2++)
        *reinterpret_cast<half8 *>(R1 + hoff(16 * w + lr, 32 * s2 + 8 * lg)) = fr.w2[s2];
}

__device__ __forceinline__ void bwd_dh1_from_image(const h16 *R1, const h16 *R2,
                                                   f32x4 d1[8]) {
    const int w = threadIdx.x >> 6;
#pragma unroll
    for (int t = 0; t < 8; t++) d1[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s2 = 0; s2 < 4; s2++) {
        const half8 av = frag_tr_h(R1, 32 * s2, 16 * w);
#pragma unroll
        for (int t = 0; t < 8; t++) d1[t] = mfma(av, frag_row_h(R2, 16 * t, 32 * s2), d1[t]);
    }
    __syncthreads();
}

__device__ __forceinline__ void bwd_dh1(h16 *R1, const h16 *R2, const Frags &fr,
                                        f32x4 d1[8]) {
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63, lr = l & 15, lg = l >> 4;
#pragma unroll
    for (int s2 = 0; s2 < 4; s2++)
        *reinterpret_cast<half8 *>(R1 + hoff(16 * w + lr, 32 * s2 + 8 * lg)) = fr.w2[s2];
    __syncthreads();
#pragma unroll
    for (int t = 0; t < 8; t++) d1[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s2 = 0; s2 < 4; s2++) {
        const half8 av = frag_tr_h(R1, 32 * s2, 16 * w);
#pragma unroll
        for (int t = 0; t < 8; t++) d1[t] = mfma(av, frag_row_h(R2, 16 * t, 32 * s2), d1[t]);
    }
    __syncthreads();
}

// dZ1 = dH1 masked by ReLU(H1) -> R1 (lane: neurons j..j+3 of row b).
__device__ __forceinline__ void bwd_dz1(h16 *R1, const uint32_t *mask, const f32x4 d1[8]) {
    // lane ids from fresh_tid: the addresses are recomputed here instead of
    // being kept (or spilled) from the forwards that use the same expressions
    const int tx = fresh_tid(), w = tx >> 6, l = tx & 63, lr = l & 15, lg = l >> 4;
    const int j = 16 * w + 4 * lg;
#pragma unroll
    for (int t = 0; t < 8; t++) {
        const int b = 16 * t + lr;
        const uint32_t bits = (mask[b * 4 + (j >> 5)] >> (j & 31)) & 0xfu;
        half4v o;
#pragma unroll
        for (int e = 0; e < 4; e++) o[e] = ((bits >> e) & 1u) ? (h16)d1[t][e] : (h16)0.0f;
        *reinterpret_cast<half4v *>(R1 + hoff(b, j)) = o;
    }
}

#define LEARN_SMEM_SETUP                                                                       \
    __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];                              \
    h16 *R1 = (h16 *)(smem + R1_OFF), *R2 = (h16 *)(smem + R2_OFF);                            \
    h16 *DQ = (h16 *)(smem + DQ_OFF);                                                          \
    char *sc = smem + SC_OFF;                                                                  \
    Scratch S{(float *)sc,          (float *)(sc + 2048), (float *)(sc + 2560),                \
              (float *)(sc + 3072), (float *)(sc + 3584), (int *)(sc + 4096),                  \
              (int *)(sc + 4608),   (double *)(sc + 5120), (double *)(sc + 6144)};             \
    h16 *W3L = (h16 *)(smem + W3_OFF);                                                         \
    float *B3L = (float *)(smem + B3_OFF);                                                     \
    const OutL on{W3L, B3L}, tg{W3L + NACT * H, B3L + NACT};                                   \
    uint32_t *mask = reinterpret_cast<uint32_t *>(DQ)

// Diagnostics: block-level phase end time (after a barrier), only when a
// stamps buffer is passed.  s_memrealtime ticks at 100 MHz.
#define STAMP(i)                                                              \
    do {                                                                      \
        if (a.stamps && threadIdx.x == 0)                                     \
            a.stamps[(size_t)blockIdx.x * 16 + (i)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)

// ----------------------------------------------------------------------------
// Independent agents: one workgroup per agent, Adam fused on the gradient tiles.
// QSTATS: also emit the learn metrics (a.qstats != NULL).  SYNC: this learn
// ends with the hard target copy (a.sync_target): a compile-time constant, so
// the Adam streams of the other 499 of 500 learns carry no branch (a branch
// there makes the vmcnt waits conservative).  GOUT: the split learn -- every
// gradient entry goes to gout[agent][P] (the 16-bit value Adam would receive)
// and dmdqn_adam_agents applies the identical Adam step in a second launch,
// which can share the chip with the next step's side-stream work.
// TS: the 16-bit target shadow is given (a.target_h != NULL, the normal case):
// a compile-time choice, because a run-time branch between the two fragment
// sources made the loaded registers meet at a control-flow merge, where the
// compiler waits for every load (round 5).
template <bool QSTATS, bool SYNC, bool GOUT, bool XF = false, bool TS = true>
__global__ void __launch_bounds__(512, 4) H16_LEARN_KERNEL(dmdqn_learn_args a, float *gout) {
    LEARN_SMEM_SETUP;
    const int agent = blockIdx.x;
    const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, lr = l & 15, lg = l >> 4;
    const size_t Pz = (size_t)L::P;
    float *Wp = a.params + agent * Pz, *Mp = a.adam_m + agent * Pz, *Vp = a.adam_v + agent * Pz;
    float *Tp = a.target + agent * Pz;
    const size_t Ph = (Pz + 7) / 8 * 8;
    h16 *TH = TS ? reinterpret_cast<h16 *>(a.target_h) + agent * Ph : nullptr;
    const AdamC AK{a.alpha, a.c1, a.c2, a.eps, SYNC && !GOUT, TH, GOUT,
                   GOUT ? gout + agent * Pz : nullptr};
    STAMP(0);
    // Issue order (vmcnt is in-order): the deque positions, the output layers,
    // then the target's fragments -- so the slot computation waits only for
    // the positions and the S' row gather goes out while the fragments land
    // (round 4 stored the output layers to LDS right after issuing the
    // fragments: the head then waited for every fragment before the gather)
    const int pos = batch_pos(a, agent);
    const OutStage so_on = stage_out_load(Wp);
    OutStage so_tg;
    if constexpr (TS) so_tg = stage_out_load(TH);
    else so_tg = stage_out_load(Tp);
    Frags fr;
    if constexpr (TS) load_frags(TH, fr);  // in flight during the z-score + gather
    else load_frags(Tp, fr);

    // ---- slots, X(S') + metadata from the s' rows, z-score (the output
    // layers' LDS images are synced by its barriers)
    batch_head<XF>(a, agent, pos, R2, S, [&]() {
        stage_out_store(so_on, W3L, B3L);
        stage_out_store(so_tg, W3L + NACT * H, B3L + NACT);
    });
    STAMP(1);
    STAMP(2);
    // ---- target(S') -> z3 ; online(S') -> Q ; y
    // target forward keeps X(S') in R2; the online net's fragments (reused by
    // both online forwards) load layer by layer as the target's die
    const float *Wpc = Wp;
    // Buffer plan: target X=R2 -> H1 R1 -> H2 R1 (hold; X survives) ;
    // online S': X=R2 -> H1 R1 -> H2 R2 over the dead X (no hold), the S rows
    // issued after layer 1 land in R1 once layer 2 is done ; training forward:
    // X=R1 -> H1 R2 -> H2 R1 over X (no hold).  The backward then finds H1 in R2
    // and H2 in R1: it runs on the swapped pair (P1, P2) = (R2, R1).
    forward_x<true>(fr, tg, R2, R1, R1, S.z3, [Wpc](Frags &f) { load_w1(Wpc, f); },
                    [Wpc](Frags &f) { load_w2(Wpc, f); });
    STAMP(3);
    float *qo = (float *)DQ;
    RowsT<XF> gs;
    forward_x<false>(fr, on, R2, R1, R2, qo,
                     [&](Frags &) { gather_x<XF>(a, agent, false, S.slot, gs); }, NoHook{},
                     [&]() { commit_x<XF>(R1, gs); });
    STAMP(4);
    STAMP(5);
    ddqn_target(a, qo, S);
    STAMP(6);
    forward_x<false>(fr, on, R1, R2, R1, S.z3);
    h16 *const P1 = R2, *const P2 = R1;
    STAMP(7);
    const half8 ones = ones8();
#if DMDQN_EARLY_W3
    static_assert(!GOUT, "the early-W3 variant has no split form");
    // ---- dW3[k][a] = H2^T . DQ (wave w: k-tile w) ; db3 (wave 0).  W3's
    // Adam loads (lanes lr < 4: rows k = 16w + 4lg + e, column a -> W3T[a][k..k+3])
    // are issued before the loss, so their latency hides behind it.
    {
        const size_t i3 = L::oW3T + (size_t)(lr & 3) * H + 16 * w + 4 * lg;
        float4 w3 = {}, m3 = {}, v3 = {};
        if (lr < NACT) {
            w3 = *reinterpret_cast<const float4 *>(Wp + i3);
            m3 = *reinterpret_cast<const float4 *>(Mp + i3);
            v3 = *reinterpret_cast<const float4 *>(Vp + i3);
        }
        __builtin_amdgcn_sched_barrier(0);
        loss_dq<QSTATS>(a, agent, DQ, S);
        f32x4 acc = {0.f, 0.f, 0.f, 0.f}, gb = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int b0 = 0; b0 < B_; b0 += 32) {
            half8 dqf = frag_tr(DQ, 16, b0, 0);
            acc = mfma(frag_tr_h(P2, b0, 16 * w), dqf, acc);
            gb = mfma(ones, dqf, gb);  // every wave (no MFMA under divergent control)
        }
        if (lr < NACT) {
            float *pw = &w3.x, *pm = &m3.x, *pv = &v3.x;
#pragma unroll
            for (int e = 0; e < 4; e++)
                adam_el(pw[e], pm[e], pv[e], r16(acc[e]), AK.alpha, AK.c1, AK.c2, AK.eps);
            *reinterpret_cast<float4 *>(Wp + i3) = w3;
            *reinterpret_cast<float4 *>(Mp + i3) = m3;
            *reinterpret_cast<float4 *>(Vp + i3) = v3;
            if (SYNC) {
                *reinterpret_cast<float4 *>(Tp + i3) = w3;
                if (TH) {
                    half4v hv;
                    hv[0] = (h16)w3.x; hv[1] = (h16)w3.y;
                    hv[2] = (h16)w3.z; hv[3] = (h16)w3.w;
                    *reinterpret_cast<half4v *>(TH + i3) = hv;
                }
            }
            if (w == 0 && lg == 0) adam1(Wp, Mp, Vp, Tp, L::ob3 + lr, gb[0], AK);
        }
    }
#else
    loss_dq<QSTATS>(a, agent, DQ, S);
    // ---- dW3[k][a] = H2^T . DQ (wave w: k-tile w) ; db3 (wave 0)
    {
        f32x4 acc = {0.f, 0.f, 0.f, 0.f}, gb = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int b0 = 0; b0 < B_; b0 += 32) {
            half8 dqf = frag_tr(DQ, 16, b0, 0);
            acc = mfma(frag_tr_h(P2, b0, 16 * w), dqf, acc);
            gb = mfma(ones, dqf, gb);  // every wave (no MFMA under divergent control)
        }
        if (lr < NACT) {
            // rows k = 16w + 4lg + e (consecutive), column a: W3T[a][k..k+3]
            adam4(Wp, Mp, Vp, Tp, L::oW3T + (size_t)lr * H + 16 * w + 4 * lg, acc, AK);
            if (w == 0 && lg == 0) adam1(Wp, Mp, Vp, Tp, L::ob3 + lr, gb[0], AK);
        }
    }
#endif
    __syncthreads();  // dW3 read H2; dZ2 overwrites it
    STAMP(8);
    bwd_dz2(P2, on, S);
    STAMP(9);
    h1_mask(P1, mask);  // the DQ region is free now
    // ---- dW2[j][k] = H1^T . dZ2 (wave w: j-tile w, 8 k-tiles) ; db2 (k-tile w) ; Adam
    {
        f32x4 g2[8], gb = {0.f, 0.f, 0.f, 0.f};
        // rows j = 16w + 4lg + e, column k = 16t + lr  ->  W2T[k][j..j+3]
        adam_pipe<4, 2, DMDQN_EARLY_W2>(
            Wp, Mp, Vp, Tp,
            [&](int t) { return (size_t)L::oW2T + qn_wt(16 * t + lr, 16 * w + 4 * lg, H); }, g2,
            AK, [&]() {
#pragma unroll
                for (int t = 0; t < 8; t++) g2[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int b0 = 0; b0 < B_; b0 += 32) {
                    const half8 av = frag_tr_h(P1, b0, 16 * w);
                    gb = mfma(ones, frag_tr_h(P2, b0, 16 * w), gb);
#pragma unroll
                    for (int t = 0; t < 8; t++) g2[t] = mfma(av, frag_tr_h(P2, b0, 16 * t), g2[t]);
                }
                // H1 fully consumed (dW2, mask): P1 becomes the W2^T image now,
                // from the register copy of old W2 (fr.w2), dead during Adam
                __syncthreads();
                w2t_image(P1, fr);
            });
        const int tx = fresh_tid();  // (16w + lr kept from the head spilled)
        if ((tx & 63) < 16) adam1(Wp, Mp, Vp, Tp, L::ob2 + (tx >> 6) * 16 + (tx & 15), gb[0], AK);
    }
    __syncthreads();  // W2^T image complete
    f32x4 d1[8];
#if DMDQN_GX_EARLY
    {
        RowsT<XF> gx;  // X(S) again for dW1: issued before dH1, lands in P2 once dZ2 is consumed
        gather_x<XF>(a, agent, false, S.slot, gx);
        __builtin_amdgcn_sched_barrier(0);
        bwd_dh1_from_image(P1, P2, d1);
        commit_x<XF>(P2, gx);
    }
#else
    bwd_dh1_from_image(P1, P2, d1);
    {
        RowsT<XF> gx;  // X(S) again for dW1 (P2 is free)
        gather_x<XF>(a, agent, false, S.slot, gx);
        commit_x<XF>(P2, gx);
    }
#endif
    STAMP(10);
    bwd_dz1(P1, mask, d1);
    __syncthreads();
    STAMP(11);
    // ---- dW1[i][j] = X^T . dZ1 (wave w: j-tile w, 6 i-tiles) ; db1 (j-tile w)
    {
        const int tx = fresh_tid(), lr = tx & 15, lg = (tx & 63) >> 4;
        f32x4 g1[6], gb = {0.f, 0.f, 0.f, 0.f};
        // rows i = 16t + 4lg + e, column j = 16w + lr -> W1T[j][i..i+3]; tile 5
        // holds features 80..95: lanes lg < 2 (80..87) update in the pipe, lane
        // lg = 2's first row is feature 88 (the W1T column, below), the rest
        // (89..95) do not exist
        adam_pipe<2, 3, DMDQN_EARLY_W1>(
            Wp, Mp, Vp, Tp,
            [&](int t) { return (size_t)L::oW1T + qn_w1<H>(16 * w + lr, t < 5 || lg < 2 ? 16 * t + 4 * lg : 0); },
            g1, AK, [&]() {
#pragma unroll
                for (int t = 0; t < 6; t++) g1[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int b0 = 0; b0 < B_; b0 += 32) {
                    const half8 bv = frag_tr_h(P1, b0, 16 * w);
                    gb = mfma(ones, bv, gb);
#pragma unroll
                    for (int t = 0; t < 6; t++)
                        g1[t] = mfma(frag_tr_h<DP>(P2, b0, 16 * t), bv, g1[t]);
                }
            },
            [&](int t) { return t < 5 || lg < 2; });
        // b1[j] (lanes lg = 0: every row of the ones-MFMA holds the column sum)
        // and W1T[j][88] (lanes lg = 2, row 88 of tile 5)
        if (lg == 0 || lg == 2)
            adam1(Wp, Mp, Vp, Tp, (lg == 0 ? L::ob1 : L::oW1X) + 16 * w + lr,
                  lg == 0 ? gb[0] : g1[5][0], AK);
    }
    if (a.stamps) {
        __syncthreads();
        STAMP(12);
    }
}

// The split learn's second launch: Keras-3 Adam (adam_el, the fused kernel's
// arithmetic) on every agent's P parameters from grad[NA][P]; on a sync also
// the f32 target and its 16-bit shadow (agent stride Ph).  One lane per 4
// consecutive parameters, blockIdx.y = agent.
template <bool SYNC>
__global__ void __launch_bounds__(256) H16_ADAM_KERNEL(float *W, float *M, float *V, float *T,
                                                       h16 *TH, const float *G, float alpha,
                                                       float c1, float c2, float eps) {
    constexpr int P4 = L::P / 4;
    const int q = blockIdx.x * 256 + threadIdx.x;
    if (q >= P4) return;
    const size_t Ph = ((size_t)L::P + 7) / 8 * 8;
    const size_t i = (size_t)blockIdx.y * L::P + 4 * (size_t)q;
    float4 w = *reinterpret_cast<const float4 *>(W + i), m = *reinterpret_cast<const float4 *>(M + i);
    float4 v = *reinterpret_cast<const float4 *>(V + i);
    const float4 g = *reinterpret_cast<const float4 *>(G + i);
    float *pw = &w.x, *pm = &m.x, *pv = &v.x;
    const float *pg = &g.x;
#pragma unroll
    for (int e = 0; e < 4; e++) adam_el(pw[e], pm[e], pv[e], pg[e], alpha, c1, c2, eps);
    *reinterpret_cast<float4 *>(W + i) = w;
    *reinterpret_cast<float4 *>(M + i) = m;
    *reinterpret_cast<float4 *>(V + i) = v;
    if (SYNC) {
        *reinterpret_cast<float4 *>(T + i) = w;
        if (TH) {
            half4v hv;
            hv[0] = (h16)w.x; hv[1] = (h16)w.y;
            hv[2] = (h16)w.z; hv[3] = (h16)w.w;
            *reinterpret_cast<half4v *>(TH + (size_t)blockIdx.y * Ph + 4 * (size_t)q) = hv;
        }
    }
}

DMDQN_DBG_READER(dbg_flags)

// The kernel instance for a run-time target-shadow flag (TS above).
template <bool QSTATS, bool SYNC, bool GOUT, bool XF>
void (*pick_learn(bool ts))(dmdqn_learn_args, float *) {
    return ts ? H16_LEARN_KERNEL<QSTATS, SYNC, GOUT, XF, true>
              : H16_LEARN_KERNEL<QSTATS, SYNC, GOUT, XF, false>;
}

}  // namespace H16K

int H16_LAUNCH(const dmdqn_learn_args *a, hipStream_t s) {
    DMDQN_REQUIRE(a->hidden == 128 && a->P == H16K::L::P,
                  "dmdqn_learn: precision %d (" H16_NAME ") needs hidden=128 (P=%d)", a->precision,
                  H16K::L::P);
    using namespace H16K;
    const bool ts = a->target_h != nullptr;
    auto kern = a->qstats ? (a->sync_target ? pick_learn<true, true, false, false>(ts)
                                            : pick_learn<true, false, false, false>(ts))
                          : (a->sync_target ? pick_learn<false, true, false, false>(ts)
                                            : pick_learn<false, false, false, false>(ts));
    if (a->row_format == DMDQN_ROWS_F32)  // float rows (the drop-in surface): X from a.xs / a.xn
        kern = a->qstats ? (a->sync_target ? pick_learn<true, true, false, true>(ts)
                                           : pick_learn<true, false, false, true>(ts))
                         : (a->sync_target ? pick_learn<false, true, false, true>(ts)
                                           : pick_learn<false, false, false, true>(ts));
    hipLaunchKernelGGL(kern, dim3(a->NA), dim3(512), 0, s, *a, (float *)nullptr);
    DMDQN_LAUNCH_CHECK("k_learn_" H16_NAME);
    return DMDQN_OK;
}

// The split learn's first launch: forward/backward, gradient -> grad[NA][P].
int H16_LAUNCH_GRAD(const dmdqn_learn_args *a, float *grad, hipStream_t s) {
    DMDQN_REQUIRE(a->hidden == 128 && a->P == H16K::L::P,
                  "dmdqn_learn_grad: precision %d (" H16_NAME ") needs hidden=128 (P=%d)",
                  a->precision, H16K::L::P);
    using namespace H16K;
    DMDQN_REQUIRE(a->row_format == DMDQN_ROWS_I8, "dmdqn_learn_grad: int8 replay rows only");
    const bool ts = a->target_h != nullptr;
    auto kern = a->qstats ? pick_learn<true, false, true, false>(ts)
                          : pick_learn<false, false, true, false>(ts);
    hipLaunchKernelGGL(kern, dim3(a->NA), dim3(512), 0, s, *a, grad);
    DMDQN_LAUNCH_CHECK("k_learn_" H16_NAME " (gradient)");
    return DMDQN_OK;
}

// The split learn's second launch (a's Adam constants and sync_target).
int H16_LAUNCH_ADAM(const dmdqn_learn_args *a, const float *grad, hipStream_t s) {
    using namespace H16K;
    DMDQN_REQUIRE(a->P == L::P, "dmdqn_adam_agents: P=%d != %d", a->P, L::P);
    const dim3 grid((L::P / 4 + 255) / 256, a->NA);
    h16 *TH = reinterpret_cast<h16 *>(a->target_h);
    if (a->sync_target)
        hipLaunchKernelGGL(H16_ADAM_KERNEL<true>, grid, dim3(256), 0, s, a->params, a->adam_m,
                           a->adam_v, a->target, TH, grad, a->alpha, a->c1, a->c2, a->eps);
    else
        hipLaunchKernelGGL(H16_ADAM_KERNEL<false>, grid, dim3(256), 0, s, a->params, a->adam_m,
                           a->adam_v, a->target, TH, grad, a->alpha, a->c1, a->c2, a->eps);
    DMDQN_LAUNCH_CHECK("k_adam_agents_" H16_NAME);
    return DMDQN_OK;
}

}  // namespace dmdqn
