// observe.hip -- local-state / observation / reward assembly, one block per env.
//
// Restates (bit-exactly; pinned by tests/golden/observe_*.npz through the oracle):
//   src/experimental/order_lanes.py:430-499  get_own_state -> local[17]
//   src/experimental/order_lanes.py:392-427  _get_neighbor_info (J_r_c arithmetic)
//   src/experimental/order_lanes.py:502-555  build_state_vector -> obs[89]
//   src/scripts/train.py:159-165, :254       r = 0.3*local + 0.7*global (f64)
// Built with -ffp-contract=off so 0.3*l + 0.7*g is two roundings + one add, as
// in CPython.
#include "observe.hpp"

namespace dmdqn {

__global__ void k_observe(int R, int C, const int32_t *halt, const int32_t *phase,
                          const int32_t *tspent, int mode, float *local, float *obs,
                          const float *prev_local, double *reward) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    const int A = R * C;
    const int e = blockIdx.x;
    float *loc = sm;                      // [A][17]
    double *sums = (double *)(sm + ((A * 17 + 3) & ~3));  // [A]
    const size_t eo = (size_t)e * A;
    for (int t = threadIdx.x; t < A * 17; t += blockDim.x) {
        int a = t / 17, f = t - a * 17;
        float v = local_feature(f, halt + (eo + a) * 12, phase[eo + a], tspent[eo + a], mode);
        loc[t] = v;
        if (local) local[eo * 17 + t] = v;
    }
    __syncthreads();
    if (obs) {
        for (int t = threadIdx.x; t < A * 89; t += blockDim.x) {
            int a = t / 89, i = t - a * 89;
            obs[eo * 89 + t] = obs_feature(R, C, a, i, loc);
        }
    }
    if (reward && prev_local) {
        const float *pl = prev_local + eo * 17;
        for (int a = threadIdx.x; a < A; a += blockDim.x) {
            double s = 0.0;
            for (int k = 0; k < 12; k++) s += (double)pl[a * 17 + k];
            sums[a] = s;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            double g = 0.0;
            for (int a = 0; a < A; a++) g += sums[a];
            sums[A] = -1.0 * g;
        }
        __syncthreads();
        const double g = sums[A];
        for (int a = threadIdx.x; a < A; a += blockDim.x)
            reward[eo + a] = combine_reward(-1.0 * sums[a], g);
    }
}

}  // namespace dmdqn

using namespace dmdqn;

extern "C" int dmdqn_observe(int R, int C, int E, const int32_t *halt, const int32_t *phase,
                             const int32_t *tspent, int mode, float *local, float *obs,
                             const float *prev_local, double *reward, void *stream) {
    DMDQN_REQUIRE(R >= 1 && C >= 1 && R <= 10 && C <= 10 && E > 0,
                  "dmdqn_observe: grid %dx%d / E=%d out of range (J_r_c ids need r,c<10)", R, C, E);
    DMDQN_REQUIRE(halt && phase && tspent, "dmdqn_observe: null input");
    DMDQN_REQUIRE(mode == 0 || mode == 1, "dmdqn_observe: mode must be 0 or 1");
    DMDQN_REQUIRE(!reward || prev_local, "dmdqn_observe: reward needs prev_local");
    const int A = R * C;
    size_t lds = (size_t)((A * 17 + 3) & ~3) * sizeof(float) + (size_t)(A + 1) * sizeof(double);
    hipLaunchKernelGGL(k_observe, dim3(E), dim3(256), lds, as_stream(stream), R, C, halt, phase,
                       tspent, mode, local, obs, prev_local, reward);
    DMDQN_LAUNCH_CHECK("k_observe");
    return DMDQN_OK;
}
