// Diagnostic micro-test: does a packed-f32 VALU op read the value written by
// the VALU instruction just before it, while another wave on the same SIMD
// runs MFMAs?  (The pattern found in the sim: v_mov_b32 v4, s36 followed by
// v_pk_mul_f32 v[4:5], v[4:5], v[8:9] op_sel:[0,1].)
//
// 512-thread blocks: waves 0-3 run back-to-back MFMAs when `mfma` is set (one
// per SIMD), waves 4-7 run the probe sequence `iters` times and count results
// that differ from the value the program order defines.  Modes:
//   0: v_mov_b32 vLo, <vgpr>  -> v_pk_mul_f32 (reads the pair)
//   1: v_mov_b32 vLo, <sgpr>  -> v_pk_mul_f32
//   2: v_add_f32 vLo, ...     -> v_pk_mul_f32
//   3: v_mov_b32 vLo, <sgpr>  -> s_nop 0 -> v_pk_mul_f32
//   4: v_mov_b32 vLo, <sgpr>  -> s_nop 1 -> v_pk_mul_f32
//   5: v_mov_b32 vLo, <sgpr>  -> v_pk_add_f32
//   6: v_mov_b32 vLo, <sgpr>  -> v_pk_fma_f32
//   7: v_mov_b32 vHi, <sgpr>  -> v_pk_mul_f32 (the high half just written)
//   8: v_mov_b32 vLo, <sgpr>  -> v_mul_f32 (plain VALU, control)
// The sim's sequence -- a packed op WRITING the pair just before the v_mov:
//   9: v_pk_add_f32 v[40:41] -> s_nop 0 -> v_mov_b32 v40, <sgpr> -> v_pk_mul_f32
//  10: v_pk_add_f32 v[40:41] -> s_nop 0 -> v_mov_b32 v40, <sgpr> -> s_nop 7 -> v_mul_f32
//  11: as 9 with s_nop 1      12: as 9 with s_nop 2      13: as 10 with s_nop 1
//  14: v_pk_mul_f32 v[40:41] -> s_nop 0 -> v_mov_b32 v40, <sgpr> -> s_nop 7 -> v_mul_f32
//  15: the sim's four instructions verbatim (pk_add with neg modifiers, s_nop 0,
//      v_mov from an SGPR, pk_mul with op_sel:[0,1])
//  16: as 15, the pk_mul without op_sel      17: as 15, the pk_add without neg
//  18: as 15 with s_nop 1                     19: as 15 with s_nop 2
//  20: as 15 without the v_mov (pk_mul op_sel reads the pk_add result)
//  21: as 15 with the v_mov writing the HIGH half (v47) and pk_mul reading it
// mfma = 2: no MFMA waves (the caller runs the fp16 learn on another stream).
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define PROBE(PRE, OP)                                                                \
    asm volatile("v_mov_b32 v40, %1\n"                                                \
                 "v_mov_b32 v41, %2\n"                                                \
                 "v_mov_b32 v42, %2\n"                                                \
                 "v_mov_b32 v43, %2\n"                                                \
                 "s_nop 7\n" PRE OP                                                   \
                 "s_nop 7\n"                                                          \
                 "v_mov_b32 %0, v44\n"                                                \
                 : "=v"(r)                                                            \
                 : "v"(old), "v"(other), "s"(neu), "v"(neu_v)                         \
                 : "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47")

// Single packed op on operands written long before (s_nop 7); both result
// lanes returned.  v40 = old (per lane), v41 = 7, v42 = 2, v43 = 4.
#define PROBE2(OP)                                                                    \
    asm volatile("v_mov_b32 v40, %2\n"                                                \
                 "v_mov_b32 v41, %3\n"                                                \
                 "v_mov_b32 v42, %4\n"                                                \
                 "v_mov_b32 v43, %5\n"                                                \
                 "s_nop 7\n" OP                                                       \
                 "s_nop 7\n"                                                          \
                 "v_mov_b32 %0, v44\n"                                                \
                 "v_mov_b32 %1, v45\n"                                                \
                 : "=v"(r), "=v"(r2)                                                  \
                 : "v"(old), "v"(c7), "v"(c2), "v"(c4)                                \
                 : "v40", "v41", "v42", "v43", "v44", "v45")

__global__ void __launch_bounds__(512) k_pk_probe(int iters, int mode, int mfma, float sval,
                                                  uint32_t *err, float *sink) {
    const int w = threadIdx.x >> 6;
    if (w < 4) {
        if (mfma != 1) return;
        half8 a, b;
        for (int e = 0; e < 8; e++) {
            a[e] = (_Float16)(threadIdx.x * 0.001f + e);
            b[e] = (_Float16)(e * 0.5f);
        }
        f32x4 c = {0.f, 0.f, 0.f, 0.f};
        for (int i = 0; i < iters * 2; i++) c = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
        if (c[0] == 1234.5f) sink[threadIdx.x] = c[1];
        return;
    }
    const float old = 3.0f + (float)(threadIdx.x & 7), other = 2.0f;
    uint32_t bad = 0;
    for (int i = 0; i < iters; i++) {
        const float neu = sval;                      // kernel argument: an SGPR
        const float neu_v = sval + (float)(i & 1) * 0.0f + (float)(threadIdx.x >> 10);  // a VGPR
        float r, want, r2 = 0.0f, want2 = 0.0f;
        const float c7 = 7.0f + (float)(threadIdx.x >> 10), c2 = c7 - 5.0f, c4 = c7 - 3.0f;
        switch (mode) {
            case 22: PROBE2("v_pk_mul_f32 v[44:45], v[40:41], v[42:43] op_sel_hi:[0,1]\n");
                     want = old * 2.0f; want2 = old * 4.0f; break;
            case 23: PROBE2("v_pk_mul_f32 v[44:45], v[40:41], v[42:43] op_sel:[1,0]\n");
                     want = 7.0f * 2.0f; want2 = 7.0f * 4.0f; break;
            case 24: PROBE2("v_pk_mul_f32 v[44:45], v[40:41], v[42:43] op_sel_hi:[1,0]\n");
                     want = old * 2.0f; want2 = 7.0f * 2.0f; break;
            case 25: PROBE2("v_pk_add_f32 v[44:45], v[40:41], v[42:43] op_sel_hi:[0,1]\n");
                     want = old + 2.0f; want2 = old + 4.0f; break;
            case 26: PROBE2("v_pk_add_f32 v[44:45], v[40:41], v[42:43] neg_lo:[0,1] neg_hi:[0,1]\n");
                     want = old - 2.0f; want2 = 7.0f - 4.0f; break;
            case 27: PROBE2("v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n");
                     want = old * 2.0f; want2 = 7.0f * 4.0f; break;
            case 28: PROBE2("v_pk_mul_f32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n");
                     want = old * 4.0f; want2 = 7.0f * 4.0f; break;
            case 29: PROBE2("v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[42:43] op_sel_hi:[0,1,1]\n");
                     want = old * 2.0f + 2.0f; want2 = old * 4.0f + 4.0f; break;
            case 0: PROBE("v_mov_b32 v40, %4\n", "v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n");
                    want = neu * other; break;
            case 1: PROBE("v_mov_b32 v40, %3\n", "v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n");
                    want = neu * other; break;
            case 2: PROBE("v_add_f32 v40, %3, %4\n", "v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n");
                    want = (neu + neu) * other; break;
            case 3: PROBE("v_mov_b32 v40, %3\ns_nop 0\n", "v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n");
                    want = neu * other; break;
            case 4: PROBE("v_mov_b32 v40, %3\ns_nop 1\n", "v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n");
                    want = neu * other; break;
            case 5: PROBE("v_mov_b32 v40, %3\n", "v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n");
                    want = neu + other; break;
            case 6: PROBE("v_mov_b32 v40, %3\n", "v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[42:43]\n");
                    want = neu * other + other; break;
            case 7: PROBE("v_mov_b32 v41, %3\n", "v_pk_mul_f32 v[44:45], v[40:41], v[42:43] op_sel:[1,0] op_sel_hi:[0,1]\n");
                    want = neu * other; break;
            case 9: PROBE("v_pk_add_f32 v[40:41], v[42:43], v[42:43]\ns_nop 0\nv_mov_b32 v40, %3\n",
                          "v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n");
                    want = neu * other; break;
            case 10: PROBE("v_pk_add_f32 v[40:41], v[42:43], v[42:43]\ns_nop 0\nv_mov_b32 v40, %3\n",
                           "s_nop 7\nv_mul_f32 v44, v40, v42\n");
                    want = neu * other; break;
            case 11: PROBE("v_pk_add_f32 v[40:41], v[42:43], v[42:43]\ns_nop 1\nv_mov_b32 v40, %3\n",
                           "v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n");
                    want = neu * other; break;
            case 12: PROBE("v_pk_add_f32 v[40:41], v[42:43], v[42:43]\ns_nop 2\nv_mov_b32 v40, %3\n",
                           "v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n");
                    want = neu * other; break;
            case 13: PROBE("v_pk_add_f32 v[40:41], v[42:43], v[42:43]\ns_nop 1\nv_mov_b32 v40, %3\n",
                           "s_nop 7\nv_mul_f32 v44, v40, v42\n");
                    want = neu * other; break;
            case 14: PROBE("v_pk_mul_f32 v[40:41], v[42:43], v[42:43]\ns_nop 0\nv_mov_b32 v40, %3\n",
                           "s_nop 7\nv_mul_f32 v44, v40, v42\n");
                    want = neu * other; break;
            case 15: PROBE("v_pk_add_f32 v[46:47], v[40:41], v[42:43] neg_lo:[0,1] neg_hi:[0,1]\n"
                           "s_nop 0\nv_mov_b32 v46, %3\n",
                           "v_pk_mul_f32 v[44:45], v[46:47], v[40:41] op_sel:[0,1]\n");
                    want = neu * other; break;
            case 16: PROBE("v_pk_add_f32 v[46:47], v[40:41], v[42:43] neg_lo:[0,1] neg_hi:[0,1]\n"
                           "s_nop 0\nv_mov_b32 v46, %3\n",
                           "v_pk_mul_f32 v[44:45], v[46:47], v[40:41]\n");
                    want = neu * old; break;
            case 17: PROBE("v_pk_add_f32 v[46:47], v[40:41], v[42:43]\n"
                           "s_nop 0\nv_mov_b32 v46, %3\n",
                           "v_pk_mul_f32 v[44:45], v[46:47], v[40:41] op_sel:[0,1]\n");
                    want = neu * other; break;
            case 18: PROBE("v_pk_add_f32 v[46:47], v[40:41], v[42:43] neg_lo:[0,1] neg_hi:[0,1]\n"
                           "s_nop 1\nv_mov_b32 v46, %3\n",
                           "v_pk_mul_f32 v[44:45], v[46:47], v[40:41] op_sel:[0,1]\n");
                    want = neu * other; break;
            case 19: PROBE("v_pk_add_f32 v[46:47], v[40:41], v[42:43] neg_lo:[0,1] neg_hi:[0,1]\n"
                           "s_nop 2\nv_mov_b32 v46, %3\n",
                           "v_pk_mul_f32 v[44:45], v[46:47], v[40:41] op_sel:[0,1]\n");
                    want = neu * other; break;
            case 20: PROBE("v_pk_add_f32 v[46:47], v[40:41], v[42:43] neg_lo:[0,1] neg_hi:[0,1]\n"
                           "s_nop 0\n",
                           "v_pk_mul_f32 v[44:45], v[46:47], v[40:41] op_sel:[0,1]\n");
                    want = (old - other) * other; break;
            case 21: PROBE("v_pk_add_f32 v[46:47], v[40:41], v[42:43] neg_lo:[0,1] neg_hi:[0,1]\n"
                           "s_nop 0\nv_mov_b32 v47, %3\n",
                           "v_pk_mul_f32 v[44:45], v[46:47], v[40:41] op_sel:[1,1]\n");
                    want = neu * other; break;
            default: PROBE("v_mov_b32 v40, %3\n", "v_mul_f32 v44, v40, v42\n");
                    want = neu * other; break;
        }
        if (r != want || r2 != want2) {
            bad++;
            err[1] = __float_as_uint(r != want ? r : r2);  // one observed wrong value
            err[2] = __float_as_uint(old);
        }
    }
    if (bad) atomicAdd(err, bad);
}

extern "C" int pk_probe(int blocks, int iters, int mode, int mfma, uint32_t *err, float *sink,
                        void *stream) {
    hipLaunchKernelGGL(k_pk_probe, dim3(blocks), dim3(512), 0, (hipStream_t)stream, iters, mode,
                       mfma, 5.0f, err, sink);
    return (int)hipGetLastError();
}
