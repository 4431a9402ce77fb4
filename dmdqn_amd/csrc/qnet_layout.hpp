// qnet_layout.hpp -- per-agent parameter layout of the Q-network in HBM.
//
// The reference's Keras model (src/agents/dqn_agent.py:153-184) keeps
// kernels as [fan_in][fan_out].  On the device every agent's parameters (and
// its target copy and Adam m / v) are stored TRANSPOSED, [fan_out][fan_in],
// with the 89 input features padded to 96:
//   W1T[H][96] | W2T[H][H] | W3T[4][H] | b1[H] | b2[H] | b3[4]
// W1T and W2T are TILED (qn_wt): 16 x 16 (fan-out x fan-in) tiles of 1 KB in
// row-major tile order, each stored as [fan-in / 8 (2)][fan-out (16)][fan-in % 8 (8)]:
//   (a) a forward MFMA A-fragment (8 consecutive fan-in values of one neuron)
//       is 32 contiguous bytes;
//   (b) a weight-gradient tile C[in][out] produced by MFMA holds 4 consecutive
//       fan-in values per lane, and the 64 lanes' 16-byte Adam accesses cover
//       the tile's 1 KB contiguously (row-major [fan_out][fan_in] gave 16
//       separate 64-byte pieces per wave-instruction: 17 % slower learn).
// W3T stays row-major.  Padding entries (features 89..95) have zero weights
// and receive zero gradients, so Adam keeps them at zero.  Host helpers
// (dmdqn_amd/agent.py) convert to/from the Keras get_weights order.
#pragma once

namespace dmdqn {

constexpr int QN_D = 89;    // observation dim (order_lanes.py:554)
constexpr int QN_DP = 96;   // padded fan-in of layer 1
constexpr int QN_NA = 4;    // actions

// Offset of W^T[out][in] in a tiled [N][K] block (K = padded fan-in, N and K
// multiples of 16).
__host__ __device__ constexpr int qn_wt(int out, int in, int K) {
    return (((out >> 4) * (K >> 4) + (in >> 4)) << 8) + (((in >> 3) & 1) << 7) + ((out & 15) << 3) +
           (in & 7);
}

template <int H>
struct QL {
    static constexpr int oW1T = 0;
    static constexpr int oW2T = oW1T + H * QN_DP;
    static constexpr int oW3T = oW2T + H * H;
    static constexpr int ob1 = oW3T + QN_NA * H;
    static constexpr int ob2 = ob1 + H;
    static constexpr int ob3 = ob2 + H;
    static constexpr int P = ob3 + QN_NA;  // floats per agent (multiple of 4)
    static_assert(P % 4 == 0, "16-byte aligned agent rows");
};

}  // namespace dmdqn
