// probe.hip -- HBM streaming probe (dmdqn_stream_probe, include/dmdqn.h).
//
// Not part of the reference loop: bench.py runs it once, outside the timed
// region and on the stream the learn runs on, so the learn's roofline
// fraction can be read against what THIS box's HBM streams in the same
// process (boxes of the pool differ by up to ~15 % on the same binary).
//
// Shapes, 16 B per lane, every byte touched once (n = n_bytes / 16 vectors):
//   copy   dst[i] = src[i]                (1 read : 1 write)
//   triad  dst[i] = src[i] + src[n + i]   (2 reads : 1 write -- close to the
//          learn's own mix, ~1.6 reads per write: w, m, v, the forward
//          fragments and the replay lines in; w, m, v out)
//   read   every src[i] read, one 16-B sum per thread written (reads only)
// each with plain or non-temporal (nt) loads and stores.  Grid: 8 workgroups
// of 256 threads per CU, grid-stride, four 16-B loads in flight per lane.
#include "common.hpp"

namespace {

typedef float f4 __attribute__((ext_vector_type(4)));
constexpr int PROBE_THREADS = 256;
constexpr int PROBE_UNROLL = 4;

template <bool NT>
__device__ __forceinline__ f4 ld(const f4 *p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    return *p;
}
template <bool NT>
__device__ __forceinline__ void st(f4 *p, f4 v) {
    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// KIND 0 copy, 1 triad, 2 read
template <int KIND, bool NT>
__global__ __launch_bounds__(PROBE_THREADS) void k_probe(f4 *__restrict__ dst,
                                                         const f4 *__restrict__ src, size_t n) {
    const size_t stride = (size_t)gridDim.x * PROBE_THREADS;
    const f4 *__restrict__ b = src + n;
    size_t i = (size_t)blockIdx.x * PROBE_THREADS + threadIdx.x;
    const size_t me = i;
    f4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
    for (; i + (PROBE_UNROLL - 1) * stride < n; i += PROBE_UNROLL * stride) {
        f4 x[PROBE_UNROLL], y[PROBE_UNROLL];
#pragma unroll
        for (int u = 0; u < PROBE_UNROLL; u++) {
            x[u] = ld<NT>(src + i + u * stride);
            if constexpr (KIND == 1) y[u] = ld<NT>(b + i + u * stride);
        }
#pragma unroll
        for (int u = 0; u < PROBE_UNROLL; u++) {
            if constexpr (KIND == 0) st<NT>(dst + i + u * stride, x[u]);
            if constexpr (KIND == 1) st<NT>(dst + i + u * stride, x[u] + y[u]);
            if constexpr (KIND == 2) acc += x[u];
        }
    }
    for (; i < n; i += stride) {
        const f4 x = ld<NT>(src + i);
        if constexpr (KIND == 0) st<NT>(dst + i, x);
        if constexpr (KIND == 1) st<NT>(dst + i, x + ld<NT>(b + i));
        if constexpr (KIND == 2) acc += x;
    }
    if constexpr (KIND == 2) dst[me] = acc;
}

}  // namespace

extern "C" int dmdqn_stream_probe(void *dst, const void *src, size_t n_bytes, int mode,
                                  void *stream) {
    DMDQN_REQUIRE(dst && src, "dmdqn_stream_probe: null buffer");
    DMDQN_REQUIRE(mode >= 0 && mode <= 5,
                  "dmdqn_stream_probe: mode %d (0 copy, 1 triad, 2 read; +3 non-temporal)", mode);
    DMDQN_REQUIRE(n_bytes > 0 && n_bytes % 16 == 0,
                  "dmdqn_stream_probe: n_bytes %zu (multiple of 16)", n_bytes);
    DMDQN_REQUIRE(((uintptr_t)dst | (uintptr_t)src) % 16 == 0, "dmdqn_stream_probe: 16-B alignment");
    int dev = 0, n_cu = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        n_cu <= 0)
        n_cu = 256;
    const size_t n = n_bytes / 16;
    const int blocks = 8 * n_cu;
    hipStream_t s = dmdqn::as_stream(stream);
    f4 *d = reinterpret_cast<f4 *>(dst);
    const f4 *x = reinterpret_cast<const f4 *>(src);
    switch (mode) {
        case 0: hipLaunchKernelGGL((k_probe<0, false>), dim3(blocks), dim3(PROBE_THREADS), 0, s, d, x, n); break;
        case 1: hipLaunchKernelGGL((k_probe<1, false>), dim3(blocks), dim3(PROBE_THREADS), 0, s, d, x, n); break;
        case 2: hipLaunchKernelGGL((k_probe<2, false>), dim3(blocks), dim3(PROBE_THREADS), 0, s, d, x, n); break;
        case 3: hipLaunchKernelGGL((k_probe<0, true>), dim3(blocks), dim3(PROBE_THREADS), 0, s, d, x, n); break;
        case 4: hipLaunchKernelGGL((k_probe<1, true>), dim3(blocks), dim3(PROBE_THREADS), 0, s, d, x, n); break;
        default: hipLaunchKernelGGL((k_probe<2, true>), dim3(blocks), dim3(PROBE_THREADS), 0, s, d, x, n); break;
    }
    DMDQN_LAUNCH_CHECK("k_probe");
    return DMDQN_OK;
}
