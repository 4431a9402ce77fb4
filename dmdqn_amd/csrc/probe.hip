// probe.hip -- HBM streaming probe (dmdqn_stream_probe, include/dmdqn.h).
//
// Not part of the reference loop: bench.py runs it once, outside the timed
// region and on the stream the learn runs on, so the learn's roofline
// fraction can be read against what THIS box's HBM streams in the same
// process (boxes of the pool differ by up to ~15 % on the same binary).
//
// Two shapes, 16 B per lane, every byte touched once:
//   mode 0  copy   dst[i] = src[i]                (1 read : 1 write)
//   mode 1  triad  dst[i] = src[i] + src[i + n]   (2 reads : 1 write -- close
//           to the learn's own mix, ~1.6 reads per write: w, m, v, the forward
//           fragments and the replay lines in; w, m, v out)
// Grid: 8 workgroups of 256 threads per CU, grid-stride, four 16-B loads in
// flight per lane per iteration.
#include "common.hpp"

namespace {

constexpr int PROBE_THREADS = 256;
constexpr int PROBE_UNROLL = 4;

__global__ __launch_bounds__(PROBE_THREADS) void k_probe_copy(float4 *__restrict__ dst,
                                                              const float4 *__restrict__ src,
                                                              size_t n) {
    const size_t stride = (size_t)gridDim.x * PROBE_THREADS;
    size_t i = (size_t)blockIdx.x * PROBE_THREADS + threadIdx.x;
    for (; i + (PROBE_UNROLL - 1) * stride < n; i += PROBE_UNROLL * stride) {
        float4 r[PROBE_UNROLL];
#pragma unroll
        for (int u = 0; u < PROBE_UNROLL; u++) r[u] = src[i + u * stride];
#pragma unroll
        for (int u = 0; u < PROBE_UNROLL; u++) dst[i + u * stride] = r[u];
    }
    for (; i < n; i += stride) dst[i] = src[i];
}

__global__ __launch_bounds__(PROBE_THREADS) void k_probe_triad(float4 *__restrict__ dst,
                                                               const float4 *__restrict__ src,
                                                               size_t n) {
    const size_t stride = (size_t)gridDim.x * PROBE_THREADS;
    const float4 *__restrict__ b = src + n;
    size_t i = (size_t)blockIdx.x * PROBE_THREADS + threadIdx.x;
    for (; i + (PROBE_UNROLL - 1) * stride < n; i += PROBE_UNROLL * stride) {
        float4 x[PROBE_UNROLL], y[PROBE_UNROLL];
#pragma unroll
        for (int u = 0; u < PROBE_UNROLL; u++) {
            x[u] = src[i + u * stride];
            y[u] = b[i + u * stride];
        }
#pragma unroll
        for (int u = 0; u < PROBE_UNROLL; u++) {
            float4 s;
            s.x = x[u].x + y[u].x;
            s.y = x[u].y + y[u].y;
            s.z = x[u].z + y[u].z;
            s.w = x[u].w + y[u].w;
            dst[i + u * stride] = s;
        }
    }
    for (; i < n; i += stride) {
        const float4 x = src[i], y = b[i];
        dst[i] = make_float4(x.x + y.x, x.y + y.y, x.z + y.z, x.w + y.w);
    }
}

}  // namespace

extern "C" int dmdqn_stream_probe(void *dst, const void *src, size_t n_bytes, int mode,
                                  void *stream) {
    DMDQN_REQUIRE(dst && src, "dmdqn_stream_probe: null buffer");
    DMDQN_REQUIRE(mode == 0 || mode == 1, "dmdqn_stream_probe: mode %d (0 copy, 1 triad)", mode);
    DMDQN_REQUIRE(n_bytes > 0 && n_bytes % 16 == 0, "dmdqn_stream_probe: n_bytes %zu (multiple of 16)",
                  n_bytes);
    DMDQN_REQUIRE(((uintptr_t)dst | (uintptr_t)src) % 16 == 0, "dmdqn_stream_probe: 16-B alignment");
    int dev = 0, n_cu = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        n_cu = 256;
    const size_t n = n_bytes / 16;
    const int blocks = 8 * (n_cu > 0 ? n_cu : 256);
    hipStream_t s = dmdqn::as_stream(stream);
    if (mode == 0)
        hipLaunchKernelGGL(k_probe_copy, dim3(blocks), dim3(PROBE_THREADS), 0, s,
                           reinterpret_cast<float4 *>(dst), reinterpret_cast<const float4 *>(src), n);
    else
        hipLaunchKernelGGL(k_probe_triad, dim3(blocks), dim3(PROBE_THREADS), 0, s,
                           reinterpret_cast<float4 *>(dst), reinterpret_cast<const float4 *>(src), n);
    DMDQN_LAUNCH_CHECK("k_probe");
    return DMDQN_OK;
}
